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
#include <memory>
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
  uint64_t rounds = 0, breakpoint_hits = 0, kernel_launches = 0, retired = 0;
  uint64_t page_fetches = 0, prefetched_pages = 0, batches = 0, testcases = 0;
  double kernel_ms = 0, service_ms = 0, total_ms = 0;
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
  bool DirtyGpa(const Gpa_t Gpa) override;
  bool VirtTranslate(const Gva_t Gva, Gpa_t &Gpa, const MemoryValidate_t Validate) const override;
  uint8_t *PhysTranslate(const Gpa_t Gpa) const override;
  bool PageFaultsMemoryIfNeeded(const Gva_t Gva, const uint64_t Size) override;
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
  void ResetCoverage() override;
  void SetFullCoverage(bool On) override { full_coverage_ = On; }
  size_t CoverageSize() const override { return aggregate_.size(); }
  std::string StatsJson() const override;
  const BatchStats &Stats() const { return stats_; }
  uint32_t Lanes() const override { return nlanes_; }
  wtfgpu_ctx *Engine() const { return ctx_; }
  const std::unordered_set<uint64_t> &AggregateCoverage() const { return aggregate_; }

 private:
  struct HostPage {
    std::unique_ptr<uint8_t[]> data, orig;
  };
  struct LaneView {
    uint64_t gpr[18] = {};  // wtfgpu order: 16 gprs, rip, rflags
    bool regs_dirty = false;
    std::optional<TestcaseResult_t> result;
    uint64_t seed = 0;
    bool dirty_known = false;
    std::vector<uint32_t> dirty;  // gpfns the lane's overlay holds
    std::unordered_map<uint64_t, HostPage> pages;  // gpfn -> host copy (mutable through PhysTranslate)
  };

  LaneView &cur() const { return views_[cur_]; }
  void reset_view(uint32_t lane);
  uint8_t *lane_page(uint32_t lane, uint64_t gpfn) const;
  int flush_lanes(const std::vector<uint32_t> &lanes);
  bool run_lanes(const std::vector<uint32_t> &lanes, std::vector<LaneResult> *out, ModuleSlots *slots,
                 bool per_lane_state);
  void finish_coverage(uint32_t n, std::vector<LaneResult> *out, std::vector<uint32_t> *timedout);
  bool set_code_pages();

  wtfgpu_ctx *ctx_ = nullptr;
  KernelDump dump_;
  CpuState_t initial_{};
  wtfgpu_regs_t initial_regs_{};
  uint32_t nlanes_ = 0, overlay_pages_ = 0;
  uint64_t limit_ = 0;
  mutable std::vector<LaneView> views_;
  uint32_t cur_ = 0;
  std::unordered_map<uint64_t, BreakpointHandler_t> breakpoints_;
  std::unordered_set<uint64_t> aggregate_;
  std::unordered_set<Gva_t> last_new_coverage_;
  mutable BatchStats stats_;
  bool full_coverage_ = false;
};


}  // namespace wtfgpu_host
