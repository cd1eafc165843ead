// gpu_backend.h — GpuBackend_t: wtf's Backend_t over the MI355X engine
// (include/wtfgpu.h). The drop-in sibling of BochscpuBackend_t
// (src/wtf/bochscpu_backend.h:61-327).
//
// Two ways to run:
//  * Backend_t::Run / Restore — the reference contract, one testcase at a time
//    on lane 0, so the unchanged client loop (RunTestcaseAndRestore,
//    client.cc:88-180) works as is;
//  * RunBatch — N testcases at once, one per lane. Breakpoint hits of a whole
//    round are serviced on the host lane by lane with g_Backend = this and the
//    lane selected; fuzzer modules keep per-lane state through ModuleSlots
//    (SURVEY H2). Register and memory accesses of handlers go to a host view of
//    the lane (registers gathered in bulk, pages fetched on demand or
//    prefetched for the stack, writes staged and applied in bulk).
#pragma once
#include "unimpl_hist.h"
#include <atomic>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/wtfgpu.h"
#include "kdmp.h"
#include "module_slots.h"
#include "runner.h"
#include "wtf_api.h"

namespace wtfgpu_host {

struct BatchStats {
  uint64_t rounds = 0, breakpoint_hits = 0, kernel_launches = 0, retired = 0, group_steps = 0;
  uint64_t page_fetches = 0, prefetched_pages = 0, batches = 0, testcases = 0, staged_pages = 0, stack_windows = 0;
  uint64_t prepared = 0;  // streaming: testcases whose prepared insert the backend took (no InsertTestcase call)
  double kernel_ms = 0, service_ms = 0, total_ms = 0;
  // service_ms split: bulk reads (regs, dirty lists), stack/learned prefetch,
  // module handlers (incl. on-demand page fetches), flush (writes + resume/stop)
  double bulk_ms = 0, prefetch_ms = 0, handler_ms = 0, fetch_ms = 0, flush_ms = 0;
  // RunBatch outside the run loop: restore + InsertTestcase + flush, coverage attribution, Target.Restore
  double insert_ms = 0, coverage_ms = 0, target_restore_ms = 0;
  // algorithmic bytes the lanes moved (instruction bytes + data
  // bytes read + written, counted per lane by k_run)
  uint64_t alg_bytes = 0;
  // insert_ms split: device restore + host views, module InsertTestcase calls,
  // register / memory / feed uploads
  double restore_ms = 0, module_ms = 0, upload_ms = 0;
  // upload split: write-record preparation on the host, register upload,
  // memory-write apply, feed upload; device restore within restore_ms
  double up_prep_ms = 0, up_regs_ms = 0, up_apply_ms = 0, up_feed_ms = 0, restore_dev_ms = 0;
  double out_ms = 0, fresh_ms = 0, occ_ms = 0, harvest_ms = 0;  // streaming: result hand-over, refill list, slice list, whole harvest
  // streaming harvest split: per-lane byte counters, coverage logs, attribution
  double bytes_ms = 0, covlog_ms = 0, attrib_ms = 0;
  uint64_t cov_entries = 0;  // (lane, rip) new-coverage log entries collected
  // run loop split: wtfgpu_run wall (launches + syncs), exit read-back + classification, final registers
  double run_ms = 0, exits_ms = 0, regs_ms = 0;
  // engine errors by exit status, the last unimplemented opcode and its rip
  std::atomic<uint64_t> err_unimpl{0}, err_overlay{0}, err_other{0}, err_handler{0};
  UnimplHist unimpl_ops;  // opcode histogram of the UNIMPLEMENTED exits
  std::atomic<uint64_t> last_unimpl_op{0}, last_unimpl_rip{0};
};

class GpuBackend_t final : public Backend_t, public Executor_t {
 public:
  GpuBackend_t();
  ~GpuBackend_t() override;

  // snapshot: the parsed dump backs the host view of every lane
  bool LoadDump(const std::string &dump_path);

  // ---- Backend_t
  bool Initialize(const Options_t &Opts, const CpuState_t &CpuState) override;
  std::optional<TestcaseResult_t> Run(const uint8_t *Buffer, const uint64_t BufferSize) override;
  bool Restore(const CpuState_t &CpuState) override;
  void Stop(const TestcaseResult_t &Res) override;
  void SetLimit(const uint64_t Limit) override;
  uint64_t GetReg(const Registers_t Reg) override;
  uint64_t SetReg(const Registers_t Reg, const uint64_t Value) override;
  uint64_t Rdrand() override;
  void PrintRunStats() override;
  bool SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler) override;
  // also declares the handler's device-side action (wtfgpu_set_breakpoint_actions);
  // WTFGPU_DEVICE_BP_ACTIONS=0 in the environment keeps every hit on the host
  bool SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler, const BreakpointAction_t &Action) override;
  bool DirtyGpa(const Gpa_t Gpa) override;
  bool VirtTranslate(const Gva_t Gva, Gpa_t &Gpa, const MemoryValidate_t Validate) const override;
  uint8_t *PhysTranslate(const Gpa_t Gpa) const override;
  bool PageFaultsMemoryIfNeeded(const Gva_t Gva, const uint64_t Size) override;
  bool PhysWriteDirect(const Gpa_t Gpa, const uint8_t *Buffer, const uint64_t Size) override;
  bool PhysReadDirect(const Gpa_t Gpa, uint8_t *Buffer, const uint64_t Size) const override;
  bool SetFeed(const uint8_t *Data, const uint64_t Size) override;
  bool DeclareInsert(const InsertAction_t &Action) override;
  bool SetInsert(const uint8_t *Data, const uint64_t Size) override;
  const std::unordered_set<Gva_t> &LastNewCoverage() const override;
  bool RevokeLastNewCoverage() override;
  using Backend_t::SetBreakpoint;

  // ---- batched path
  // Runs testcases [0, n) on lanes [0, n) (n <= lanes), servicing breakpoints,
  // then restores every lane. `slots` (optional) gives each lane its own module
  // state. Coverage is attributed in lane order against the aggregate set.
  bool RunBatch(const Target_t &Target, const std::vector<std::pair<const uint8_t *, size_t>> &Testcases,
                std::vector<LaneResult> &Out, ModuleSlots *Slots) override;
  Backend_t *AsBackend() override { return this; }
  // streaming (continuous batching): see Executor_t
  bool CanStream() const override { return true; }
  bool TakesPrepared() const override { return feed_action_ || insert_action_; }
  uint32_t FreeLanes() const override;
  bool StreamStep(const Target_t &Target, const std::vector<StreamTestcase_t> &In, uint64_t Slice,
                  std::vector<StreamResult_t> &Out, ModuleSlots *Slots, size_t *Taken) override;
  void ResetCoverage() override;
  void SetFullCoverage(bool On) override { full_coverage_ = On; }
  void SetWantRegisters(bool On) override { want_gprs_ = On; }
  uint64_t LastIcount() const override { return last_icount_; }
  bool LastError() const override { return last_error_; }
  bool LastHandlerFault() const override { return last_run_.handler_fault; }
  void LastRunStats(LaneResult &L) const override {
    L.bytes = last_run_.bytes;
    L.dirty = last_run_.dirty;
    L.edges = last_run_.edges;
    L.edges_new = last_run_.edges_new;
  }
  size_t CoverageSize() const override { return aggregate_.size(); }
  void TakeNewExtra(std::vector<uint64_t> &Out) override;
  size_t AbsorbExtra(const std::vector<uint64_t> &All) override;
  std::string StatsJson() const override;
  bool CoverageMap(uint8_t **Map, uint64_t *Bytes, bool *Device) override;
  size_t AbsorbCoverageMap() override;
  size_t MergeCoverageMap(const uint8_t *Merged, uint64_t Bytes, bool Device) override {
    if (!Device || wtfgpu_coverage_merge_in(ctx_, Merged, Bytes) != WTFGPU_OK) return 0;
    return AbsorbCoverageMap();
  }
  bool EnableTrace(uint32_t PerLane) override {
    trace_cap_ = PerLane;
    return ctx_ && wtfgpu_set_trace(ctx_, PerLane) == WTFGPU_OK;
  }
  bool LaneTrace(uint32_t Lane, std::vector<uint64_t> &Rips, bool &Truncated) override;
  bool EnableTenet(uint64_t BytesPerLane) override {
    tenet_cap_ = BytesPerLane;
    return ctx_ && wtfgpu_set_tenet(ctx_, BytesPerLane) == WTFGPU_OK;
  }
  bool LaneTenet(uint32_t Lane, std::vector<uint8_t> &Bytes, bool &Truncated) override;
  const BatchStats &Stats() const { return stats_; }
  uint32_t Lanes() const override { return nlanes_; }
  wtfgpu_ctx *Engine() const { return ctx_; }
  const std::unordered_set<uint64_t> &AggregateCoverage() const { return aggregate_; }

 private:
  // A page of a lane's view staged on the host: `data` is what handlers see and
  // may write through PhysTranslate, `orig` its content when staged (flush
  // diffs the two). Both live in the staging arena.
  struct Staged {
    uint64_t gpfn;
    uint8_t *data;
    const uint8_t *orig;
  };
  struct LaneView {
    uint64_t gpr[18] = {};  // wtfgpu order: 16 gprs, rip, rflags
    bool regs_dirty = false;
    // cr2 / cr3 (GetReg / SetReg): bit 0 = cr2, bit 1 = cr3; fetched from the
    // device on first use after a run, written back at flush when dirty
    uint64_t cr[2] = {};
    uint8_t cr_known = 0, cr_dirty = 0;
    std::optional<TestcaseResult_t> result;
    // a handler or InsertTestcase access did not translate (HandlerFault_t):
    // the testcase ends as an engine error (DESIGN U43)
    bool handler_fault = false;
    uint64_t seed = 0;
    uint64_t inject = ~0ull;  // PageFaultsMemoryIfNeeded: page to #PF after the handler
    bool has_feed = false;    // SetFeed / SetInsert: chunks for the device Feed action / insert
    std::vector<uint8_t> feed;
    bool dirty_known = false;
    std::vector<uint32_t> dirty;  // gpfns the lane's overlay holds
    std::vector<Staged> pages;    // staged pages (few per lane: linear search)
    // writes to pages that are not staged, logged instead of fetching the
    // page (PhysWriteDirect); merged into a page if it gets staged later
    struct Logged {
      uint64_t gpa;
      uint32_t len, off;
    };
    std::vector<Logged> wlog;
    std::vector<uint8_t> wdata;
    // stack window: kWin bytes at [rsp] gathered for handlers that read their
    // return address / stack arguments (sub-page prefetch, valid one round)
    static constexpr uint32_t kWin = 128;
    uint64_t win_gpa = 0;
    uint32_t win_len = 0;
    uint8_t win[kWin];
  };

  // a lane's view for the host to read or change: marks it touched, so the
  // lane's next refill resets it (reset_view); the per-lane loops of the
  // harvest and refill read views_ directly and treat an untouched view as
  // reset (no result, no feed) without pulling its cache lines in
  LaneView &view(uint32_t lane) const {
    touched_[lane] = 1;
    return views_[lane];
  }
  LaneView &cur() const { return view(cur_); }
  void reset_view(uint32_t lane);
  uint8_t *lane_page(uint32_t lane, uint64_t gpfn) const;
  // read-only view for page walks: the dump page when the lane's overlay does
  // not hold the frame (no staging copy)
  const uint8_t *lane_page_ro(uint32_t lane, uint64_t gpfn) const;
  Staged *find_staged(uint32_t lane, uint64_t gpfn) const;
  // n consecutive staging slots (one block): pinned orig pages + data pages
  size_t alloc_slots(size_t n, uint8_t **orig, uint8_t **data) const;
  // stage a page whose original content is `orig` (kept alive by the caller:
  // a dump page, the zero page or a pinned staging slot)
  uint8_t *stage(uint32_t lane, uint64_t gpfn, const uint8_t *orig, uint8_t *data) const;
  uint8_t *stage_copy(uint32_t lane, uint64_t gpfn, const uint8_t *orig) const;
  void drop_staged(LaneView &v) const;
  bool in_overlay(const LaneView &v, uint64_t gpfn) const;
  int flush_lanes(const std::vector<uint32_t> &lanes);
  // until every lane has a result
  bool run_lanes(const std::vector<uint32_t> &lanes, std::vector<LaneResult> *out, ModuleSlots *slots,
                 bool per_lane_state);
  // stop_args: the range's prefetched StopWithArgs arguments (6 per lane from
  // `first`), else they are read for the lanes that need them
  bool classify(const std::vector<uint32_t> &pending, uint32_t first, const wtfgpu_exit_t *ex,
                std::vector<uint8_t> &done, std::vector<LaneResult> *out, std::vector<uint32_t> &hits,
                const uint64_t *stop_args = nullptr);
  bool fill_results(const std::vector<uint32_t> &lanes, uint32_t first, const wtfgpu_exit_t *ex,
                    const std::vector<uint8_t> &done, std::vector<LaneResult> *out, std::vector<uint32_t> *finished);
  bool stop_prestopped(const std::vector<uint32_t> &lanes);
  void account_run(const wtfgpu_run_stats_t &rs);
  bool service_hits(const std::vector<uint32_t> &hits, uint32_t first, std::vector<uint8_t> &done, ModuleSlots *slots,
                    bool per_lane_state);
  // InsertTestcase for `lanes` (restored views), module state per lane, on all
  // host threads when the module allows it
  void insert_lanes(const Target_t &Target, const std::vector<uint32_t> &lanes,
                    const std::vector<std::pair<const uint8_t *, size_t>> &tcs, ModuleSlots *Slots,
                    std::vector<uint8_t> &ok);
  void target_restore(const Target_t &Target, const std::vector<uint32_t> &lanes, ModuleSlots *Slots);
  // coverage of finished lanes, attributed in the order given (LastNewCoverage)
  // (pf_hdr: a part's prefetched entry count; the entries of other lanes
  // than `lanes` are skipped)
  void collect_coverage(const std::vector<uint32_t> &lanes, std::vector<LaneResult> &res,
                        const uint64_t *pf_hdr = nullptr);
  // streaming state: slot occupancy, the caller's tag per lane, results
  std::vector<uint8_t> busy_;
  std::vector<uint64_t> tag_;
  std::vector<uint64_t> tc_bytes_;  // the testcase size in each lane (B_exec)
  std::vector<LaneResult> lres_;
  std::vector<uint8_t> lres_stale_;  // lres_[l] still holds a handed-out result: reset at the lane's next harvest
  std::vector<uint32_t> cov_lanes_;  // coverage collection buffers (streaming)
  std::vector<uint64_t> cov_rips_;
  std::vector<uint8_t> cov_want_;  // lanes whose prefetched entries count (collect_coverage)
  std::vector<std::pair<uint32_t, uint64_t>> cov_sorted_;  // the same, sorted by (lane, rip)
  bool cov_ovf_warned_ = false;
  bool want_gprs_ = true;
  uint64_t last_icount_ = 0;  // of the last Run
  LaneResult last_run_;       // the last Run's result and run stats (PrintRunStats)
  bool last_error_ = false;
  // streaming parts (see parts_n): lane range, slice in flight, its occupied
  // lanes, exit read-back, pinned staging of the part's feeds
  struct Part {
    uint32_t lo = 0, hi = 0;
    bool launched = false;
    // the part's occupied and free lanes, ascending, kept as lanes finish and
    // are refilled (the refill takes the lowest free lanes first)
    std::vector<uint32_t> occ, free;
    wtfgpu_exit_t *ex = nullptr;  // the slice's exit records: pinned (one DMA of 40 B per lane)
    uint64_t ex_cap = 0;
    uint8_t *pin = nullptr;
    uint64_t pin_cap = 0;
    // the slice's read-back queued behind it (wtfgpu_prefetch_results /
    // _coverage), pinned: byte and dirty-page counts, StopWithArgs
    // arguments, the coverage entry count
    bool pf = false, pf_cov = false;
    uint64_t *nb = nullptr, *sargs = nullptr, *cov_hdr = nullptr;
    uint32_t *dc = nullptr;
  };
  bool prefetch_part(Part &P);
  std::vector<Part> parts_;
  uint8_t *wpin_ = nullptr;  // pinned staging of host-handler writes (flush_lanes; applied synchronously)
  uint64_t wpin_cap_ = 0;
  uint32_t next_part_ = 0;
  uint32_t parts_n() const;
  bool harvest_part(Part &P, const Target_t &Target, std::vector<StreamResult_t> &Out, ModuleSlots *Slots);
  void finish_coverage(uint32_t n, std::vector<LaneResult> *out, std::vector<uint32_t> *timedout);
  bool set_code_pages();

  wtfgpu_ctx *ctx_ = nullptr;
  KernelDump dump_;
  CpuState_t initial_{};
  wtfgpu_regs_t initial_regs_{};
  uint32_t nlanes_ = 0, overlay_pages_ = 0;
  uint64_t limit_ = 0;
  mutable std::vector<LaneView> views_;
  mutable std::vector<uint8_t> touched_;  // view(lane) was taken since the lane's last reset_view
  // a prepared insert's bytes for the lane's feed upload (StreamTestcase_t::prep,
  // valid during the StreamStep call): the feed itself, or with ins the testcase
  // the feed's one chunk (u32 size, bytes) holds
  struct PrepFeed {
    const uint8_t *p = nullptr;
    uint32_t len = 0;
    uint8_t has = 0, ins = 0;
  };
  std::vector<PrepFeed> pf_;
  // the lane the calling thread services (handlers of different lanes run on
  // several threads when the module state is thread_local, module_slots.h)
  static thread_local uint32_t cur_;
  std::unordered_map<uint64_t, BreakpointHandler_t> breakpoints_;
  std::vector<wtfgpu_bp_action_t> bp_actions_;  // device-side equivalents of some handlers
  uint32_t trace_cap_ = 0;                       // rip-trace capacity per lane (EnableTrace)
  uint64_t tenet_cap_ = 0;                       // Tenet stream bytes per lane (EnableTenet)
  std::unordered_map<uint64_t, BreakpointAction_t::ArgsResult_t> args_results_;  // StopWithArgs, by gva
  bool feed_action_ = false;                     // a Feed action is on the device
  bool insert_action_ = false;                   // the declared insert is on the device (wtfgpu_set_insert)
  int upload_feed(uint32_t n);                   // lanes [0, n)
  std::unordered_set<uint64_t> aggregate_;
  std::unordered_set<uint64_t> code_vpns_;  // the map's pages (set_code_pages)
  std::vector<uint64_t> extra_new_;         // aggregate values outside them since TakeNewExtra
  void commit_fresh(const std::vector<uint64_t> &fresh);
  std::unordered_set<Gva_t> last_new_coverage_;
  mutable BatchStats stats_;
  // staging arena: blocks of slots, each slot a pinned 4 KiB page (device
  // gathers land there directly) + a 4 KiB data page handed to handlers;
  // recycled once no lane holds a staged page
  struct Block {
    uint8_t *orig = nullptr;
    std::unique_ptr<uint8_t[]> data;
    size_t cap = 0, used = 0;
  };
  struct Arena {  // one per host thread
    std::vector<Block> blocks;
    size_t cur = 0;
  };
  mutable std::vector<Arena> arenas_;  // [0, Threads()): HostPool threads in a loop; the last: calls outside loops
  mutable std::mutex spare_mu_;        // the last arena's lock
  mutable std::shared_mutex recycle_mu_;  // allocations (shared) vs recycle_arenas (exclusive)
  void release_slots(size_t n) const;     // slots alloc_slots reserved that were never staged
  std::unordered_map<uint64_t, uint64_t> covlog_count_;  // WTFGPU_COVLOG_TOP diagnostic
  uint64_t covlog_calls_ = 0;
  void recycle_arenas() const;
  mutable std::atomic<size_t> live_staged_{0};
  // serialises engine calls made from handler threads (shared scratch buffers)
  // and the learned-prefetch tables
  mutable std::mutex engine_mu_;
  bool parallel_service(const ModuleSlots *slots) const;
  // learned prefetch: overlay frames a breakpoint's handler fetched on demand
  // (e.g. the tlv packet buffer); fetched in bulk for that breakpoint's next hits
  mutable std::unordered_map<uint64_t, std::vector<uint64_t>> bp_pages_;
  mutable std::unordered_map<uint64_t, uint64_t> fetch_by_bp_;  // on-demand fetches per breakpoint (stats)
  mutable std::unordered_set<uint64_t> bp_stack_;
  std::unordered_set<uint64_t> bp_seen_;  // breakpoints serviced at least once (scouting)  // breakpoints whose handler reads the stack page
  static thread_local uint64_t servicing_bp_, servicing_sp_;
  static thread_local bool scouting_;
  void learn(uint64_t gpfn) const;
  bool full_coverage_ = false;
};


}  // namespace wtfgpu_host
