// runner.h — the batched client loop over an executor:
// `run` replays inputs (wtf run, subcommands.cc:20-75) and `fuzz` is the
// node loop with an in-process master (client.cc:187-258 + server.h:720-886:
// mutate, run, keep testcases that found new coverage, save crashes), both
// batched N testcases per executor call.
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <filesystem>
#include <mutex>
#include <thread>
#include <cstdint>
#include <deque>
#include <unordered_map>
#include <future>
#include <random>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

#include "../../include/wtfgpu.h"
#include "merge_block.h"
#include "wtf_api.h"

namespace wtfgpu_host {

struct LaneResult {
  TestcaseResult_t result;
  bool error = false;        // the engine could not finish the testcase (unimplemented opcode, overlay full)
  bool handler_fault = false;  // ... because a handler's guest access did not translate (DESIGN U43)
  uint32_t exit_status = 0;  // last engine exit status (wtfgpu_status)
  uint64_t icount = 0;       // retired instructions
  uint64_t rip = 0;
  uint64_t gprs[18] = {};    // final gprs (wtfgpu order) + rip + rflags
  std::vector<uint64_t> new_coverage;  // LastNewCoverage, attributed in lane order
  // run stats (BochscpuRunStats_t, bochscpu_backend.h:17-45), filled when the
  // executor is asked for registers (run mode): instruction + data bytes
  // (B_insn), dirty pages, RecordEdge calls and those new to the testcase's set
  uint64_t bytes = 0, edges = 0, edges_new = 0;
  uint32_t dirty = 0;
};

struct StreamTestcase_t {
  const uint8_t *data;
  size_t size;
  uint64_t tag;  // the caller's name for it, returned with its result
  // Target_t::PrepareInsert's outcome for it, when the node prepared it
  // (PreparedInsert_t; Call = not prepared) and its bytes (Feed)
  PreparedInsert_t prep = PreparedInsert_t::Call;
  const uint8_t *prep_data = nullptr;
  size_t prep_size = 0;
};
// A finished testcase: its tag and its result, which stays in the executor's
// storage and is valid until the executor's next StreamStep (no per-result
// copies of the ~250-byte LaneResult on the step's thread).
struct StreamResult_t {
  uint64_t tag;
  LaneResult *r;
};

// A backend that runs many testcases per call (GpuBackend_t; the oracle twin
// runs them one after the other).
class Executor_t {
 public:
  // ---- streaming (continuous batching): lanes are slots. StreamStep puts
  // testcases into free lanes (In[0, *Taken): at most FreeLanes(), which is
  // an upper bound), runs occupied lanes for one slice of `Slice` wave-steps
  // and returns the testcases that finished, in lane order. A testcase's data
  // is only read during the call. (A pipelined executor returns a slice's
  // results one call later: its lanes run while the host serves others.)
  virtual bool CanStream() const { return false; }
  // StreamStep uses prepared inserts (StreamTestcase_t::prep)
  virtual bool TakesPrepared() const { return false; }
  virtual uint32_t FreeLanes() const { return 0; }
  virtual bool StreamStep(const Target_t &, const std::vector<StreamTestcase_t> &, uint64_t,
                          std::vector<StreamResult_t> &, ModuleSlots *, size_t *Taken) {
    if (Taken) *Taken = 0;
    return false;
  }

  virtual ~Executor_t() = default;
  virtual Backend_t *AsBackend() = 0;
  virtual uint32_t Lanes() const = 0;
  // testcases [0, n) -> out[0, n): restore, insert, run, service, attribute coverage
  virtual bool RunBatch(const Target_t &Target, const std::vector<std::pair<const uint8_t *, size_t>> &Testcases,
                        std::vector<LaneResult> &Out, ModuleSlots *Slots) = 0;
  // forget the aggregate coverage
  virtual void ResetCoverage() = 0;
  // parity mode: LaneResult::new_coverage holds each testcase's full rip set
  // (as if it ran first), not the lane-order delta
  virtual void SetFullCoverage(bool On) = 0;
  // LaneResult::gprs filled (run mode prints them; the fuzz loop does not read them)
  virtual void SetWantRegisters(bool) {}
  // the retired count / engine-error flag of the last Backend_t::Run
  virtual uint64_t LastIcount() const { return 0; }
  virtual bool LastError() const { return false; }
  virtual bool LastHandlerFault() const { return false; }
  // the run stats (LaneResult::bytes / dirty / edges / edges_new) of the last Backend_t::Run
  virtual void LastRunStats(LaneResult &) const {}
  virtual size_t CoverageSize() const = 0;
  virtual std::string StatsJson() const { return "{}"; }
  // The coverage map over the executable-page slot table (one byte per code
  // byte of every executable page reachable from the snapshot cr3; identical
  // on every shard): host or device memory.
  virtual bool CoverageMap(uint8_t **Map, uint64_t *Bytes, bool *Device) {
    *Map = nullptr;
    *Bytes = 0;
    *Device = false;
    return true;
  }
  // Rips set in the map (after a merge) that the aggregate lacks join it;
  // returns how many.
  virtual size_t AbsorbCoverageMap() { return 0; }
  // A merged map (CoverageExchange_t::MergeEnd: host or device memory, as
  // CoverageMap's) is MAX-ed into this executor's map, then absorbed as above.
  virtual size_t MergeCoverageMap(const uint8_t *, uint64_t, bool) { return 0; }
  // Coverage values outside the map (rips on pages outside the slot table,
  // --edges values; SURVEY 8(e)'s overflow list): the ones this shard added
  // to its aggregate since the last call are moved into Out; AbsorbExtra adds
  // other shards' to the aggregate (and returns how many were new).
  virtual void TakeNewExtra(std::vector<uint64_t> &Out) { Out.clear(); }
  virtual size_t AbsorbExtra(const std::vector<uint64_t> &) { return 0; }
  // Rip traces (wtf run --trace-type rip / cov, SetTraceFile,
  // bochscpu_backend.cc:506-520): every testcase of the next RunBatch logs
  // the rips it is about to execute, PerLane at most; LaneTrace(i) is
  // testcase i's (Truncated: it logged more than PerLane).
  virtual bool EnableTrace(uint32_t) { return false; }
  virtual bool LaneTrace(uint32_t, std::vector<uint64_t> &, bool &) { return false; }
  // Tenet traces (wtf run --trace-type tenet, bochscpu_backend.cc:1215-1323):
  // every testcase of the next RunBatch logs the entry stream wtfgpu_set_tenet
  // documents (include/wtfgpu.h), BytesPerLane at most; LaneTenet(i) is
  // testcase i's (Truncated: it logged more). FormatTenet (runner.cc) turns it
  // into the reference's text.
  virtual bool EnableTenet(uint64_t) { return false; }
  virtual bool LaneTenet(uint32_t, std::vector<uint8_t> &, bool &) { return false; }
};

// The collective between shards (one node per GPU): an in-place MAX
// all-reduce of every shard's coverage map. RCCL over xGMI on the GPU node
// (main_gpu.cc, node_capi.cc); TCP on the CPU (net_exchange.cc) for the twin.
class CoverageExchange_t {
 public:
  virtual ~CoverageExchange_t() = default;
  virtual int Rank() const = 0;
  virtual int World() const = 0;
  // whether the session runs the per-step merge at all: across shards, or on
  // one shard when the exchange is told to take its collective path anyway
  // (RcclExchange_t's --rccl-force, a test of the RCCL calls at world 1)
  virtual bool Exchanging() const { return World() > 1; }
  virtual bool AllReduceMax(uint8_t *Map, uint64_t Bytes, bool Device) = 0;
  // *All = every shard's Mine is true
  virtual bool AllDone(bool Mine, bool *All) = 0;
  // All = the concatenation of every shard's Mine, in rank order (the
  // overflow list of coverage values outside the map)
  virtual bool AllGatherV(const std::vector<uint64_t> &Mine, std::vector<uint64_t> &All) = 0;

  // The deferred merge of one node step (collective, every shard every step):
  // MergeBegin starts the MAX all-reduce of Map into the exchange's own buffer
  // and the all-gather of (Done, Extras); MergeEnd, called before the next
  // MergeBegin, waits for them and hands out the merged map (host or device
  // memory like Map, valid until the next MergeBegin), every shard's extras
  // in rank order and whether every shard was done. Nothing waits in the step
  // that starts a merge; its result is absorbed one step later. The overflow
  // values and the done flags travel as MergeBlocks blocks (merge_block.h: at
  // most kMergeCap values per shard per merge, done only once a shard's queue
  // is empty). This default runs the synchronous collectives above inside
  // MergeBegin on a copy of the map (the TCP twins); RcclExchange_t overlaps
  // them with the step on a stream of their own.
  virtual bool MergeBegin(const uint8_t *Map, uint64_t Bytes, bool Device, const std::vector<uint64_t> &Extras,
                          bool Done);
  virtual bool MergeEnd(const uint8_t **Merged, uint64_t *Bytes, std::vector<uint64_t> &AllExtras, bool *AllDone);

 protected:
  std::vector<uint8_t> merged_;       // the default MergeBegin's result
  std::vector<uint64_t> merged_extra_;
  bool merged_done_ = false, merged_device_ = false;
  MergeBlocks blocks_{kMergeCap};
};

// BochscpuRunStats_t::Print (bochscpu_backend.h:25-37; NumberToHuman /
// BytesToHuman, human.cc:38-72): one testcase's instructions (the aggregate's
// size as the unique count), dirty pages, memory-access bytes and edges.
void PrintTestcaseRunStats(const LaneResult &L, size_t AggregateCoverage);

struct RunnerOptions {
  std::string mode = "run";  // run | fuzz | master
  std::string name;          // target name
  std::string target;        // dir with state/, inputs/, outputs/, crashes/
  std::string input;         // run: file or directory (default <target>/inputs)
  std::string results;       // run: JSON-lines output path
  uint64_t limit = 0;
  uint32_t lanes = 1;
  uint32_t overlay_pages = 32;
  uint64_t runs = 0;         // fuzz: testcases; run: repetitions of each input (subcommands.cc:85-88)
  double seconds = 0;        // fuzz: wall-clock budget (0 = none)
  uint64_t seed = 1337;
  uint64_t max_len = 0x1000;
  int device = 0;
  bool full_coverage = false;
  bool edges = false;        // --edges: branch edges join the coverage (RecordEdge)
  std::string trace_path;    // run: --trace-path dir (one <input>.trace per input, subcommands.cc:52-74)
  std::string trace_type = "rip";  // run: --trace-type rip | cov | tenet (wtf.cc:197-200)
  uint32_t trace_cap = 1u << 20;   // run: rips kept per testcase
  uint64_t tenet_cap = 0;          // run: Tenet stream bytes per testcase (0: 16 MiB, at most 32 GiB / lanes)
  bool quiet = false;
  bool serial_mutation = false;  // one mutator, in order: the reference master's stream exactly
  // fuzz: continuous batching on executors that stream (the gpu node): every
  // occupied lane runs `slice` wave-steps per step, finished lanes are
  // refilled at once; 0 = whole batches (every lane runs to its end)
  uint64_t slice = 4096;
  // GPU: k_run launches of this many wave-steps with the lanes regrouped by
  // rip between them (wtfgpu_set_regroup); 0 = fixed lane order, ~0 = the
  // engine's default (WTFGPU_REGROUP_STEPS)
  uint64_t regroup = ~0ull;
  bool stream_run = false;  // run: replay the inputs through the streaming path
  // run: the reference client's RunTestcaseAndRestore (client.cc:88-180), one
  // testcase at a time through Backend_t::Run / Restore (no batching)
  bool serial = false;
  std::string module_so;  // an unchanged module built as a shared object, one copy per lane
  int rank = 0, world = 1;         // fuzz: shard rank of world (one node per GPU)
  std::string exchange = "127.0.0.1:31337";  // TCP coverage exchange (CPU shards): rank 0 listens here
  std::string nccl_id_file;        // GPU shards: RCCL unique id file (rank 0 writes it)
  // GPU, test switch (also WTF_RCCL_FORCE=1): a world-1 node still builds the
  // RCCL communicator and runs every step's merge through it (frozen copy,
  // fused all-reduce + all-gather, unpack, absorb) instead of skipping it
  bool rccl_force = false;
  // the wire protocol (remote.h, wire.h): `master` listens, `fuzz` dials
  std::string address;             // tcp://ip:port or unix://path
  int nodes = 1;                   // master: nodes to wait for
  bool batched = false;            // N testcases per round trip (else the reference's one)
  // fuzz: every sample_every-th testcase (in accounting order) is written to
  // `sample` as a JSON line (testcase bytes, result, crash name, retired
  // count, final GPRs, new coverage) so a run at the bench's configuration
  // can be replayed on the twin (tests/test_gpu_bench_parity.py)
  std::string sample;
  uint64_t sample_every = 0;
};

struct FuzzStats {
  uint64_t execs = 0, retired = 0, crashes = 0, timeouts = 0, cr3 = 0, errors = 0, batches = 0, merged_rips = 0;
  uint64_t merges = 0, merged_map_bytes = 0;  // merges absorbed; merged-map bytes they carried
  uint64_t error_retired = 0;  // instructions retired by testcases the engine could not finish
  double run_s = 0, merge_ms = 0;
  double produce_wait_ms = 0, account_ms = 0;  // streaming: waiting on the mutator, master bookkeeping
  double make_ms = 0, step_ms = 0;             // streaming: mutation on the step's own thread, whole steps
  double fill_ms = 0;                          // streaming: taking the step's testcases (make_ms included)
  double call_ms = 0;                          // streaming: whole StreamStep calls, destructors included
  double newcov_ms = 0, crashsave_ms = 0;      // account_ms split: corpus admissions, new crash names
};

// Testcases stored back to back: one allocation per chunk of mutations, so
// handing 64K+ testcases per step to the lanes allocates and frees nothing
// per testcase on the step's thread.
struct TcArena {
  std::vector<uint8_t> Data;
  std::vector<uint64_t> Off{0};
  size_t Live = 0;  // streaming: testcases of this arena not yet accounted
  // prepared inserts (Target_t::PrepareInsert), one per testcase when present
  std::vector<PreparedInsert_t> Prep;
  std::vector<uint8_t> PrepData;
  std::vector<uint64_t> PrepOff{0};
  void Add(const void *P, size_t N) {
    const uint8_t *B = (const uint8_t *)P;
    Data.insert(Data.end(), B, B + N);
    Off.push_back(Data.size());
  }
  // the last testcase added, prepared by F (every testcase of a prepared arena is)
  void Prepare(PrepareInsert_t F, std::vector<uint8_t> &Scratch) {
    const size_t I = Count() - 1;
    Scratch.clear();
    const PreparedInsert_t K = F(Ptr(I), Len(I), Scratch);
    Prep.push_back(K);
    if (K == PreparedInsert_t::Feed) PrepData.insert(PrepData.end(), Scratch.begin(), Scratch.end());
    PrepOff.push_back(PrepData.size());
  }
  size_t Count() const { return Off.size() - 1; }
  const uint8_t *Ptr(size_t I) const { return Data.data() + Off[I]; }
  size_t Len(size_t I) const { return Off[I + 1] - Off[I]; }
};
using TcBatch = std::vector<std::unique_ptr<TcArena>>;
struct TcRef {
  TcArena *A = nullptr;
  uint32_t I = 0;
  const uint8_t *data() const { return A->Ptr(I); }
  size_t size() const { return A->Len(I); }
  PreparedInsert_t prep() const { return I < A->Prep.size() ? A->Prep[I] : PreparedInsert_t::Call; }
  const uint8_t *prep_data() const { return A->PrepData.data() + A->PrepOff[I]; }
  size_t prep_size() const { return A->PrepOff[I + 1] - A->PrepOff[I]; }
};

// The fuzz loop of one node / shard, one batch per Step(): an in-process
// master (corpus, mutator, crash saving: server.h:629-886) feeding the
// executor N testcases at a time (client.cc:187-258, batched). With a
// CoverageExchange_t of world > 1, shard r mutates with seed + r and merges
// coverage maps after every batch.
// Saves files on a background thread in the order given (the master's
// crashes/ writes, server.h:839-847: off the bookkeeping thread; flushed
// before the session ends).
class FileWriter {
 public:
  FileWriter();
  ~FileWriter();
  void Save(std::filesystem::path Path, const uint8_t *Data, size_t Size);
  void Flush();

 private:
  void Loop();
  std::mutex Mu_;
  std::condition_variable Cv_, Idle_;
  std::deque<std::pair<std::filesystem::path, std::vector<uint8_t>>> Q_;
  bool Stop_ = false, Busy_ = false;
  std::thread Th_;
};

class FuzzSession {
 public:
  FuzzSession(const RunnerOptions &O, Executor_t &Exec, Target_t &Target, ModuleSlots &Slots,
              CoverageExchange_t *X);
  ~FuzzSession();
  bool Start();      // corpus inputs + the first batch; false = nothing to run
  bool Step();       // one batch; false = the executor failed
  bool Done() const;
  // shards (world > 1): every shard was done as of the last merge absorbed
  // (the loop's collective stop decision); FinishMerge absorbs the merge
  // still in flight (collective: every shard calls it once, at the end)
  bool AllDone() const { return AllDone_; }
  bool FinishMerge();
  const FuzzStats &Stats() const { return S_; }
  size_t CorpusSize() const { return Corpus_.Size(); }
  double WallSeconds() const;
  std::string SummaryJson() const;
  void FlushFiles() { Writer_.Flush(); }  // crash files written so far are on disk

 private:
  TcBatch MakeBatch(uint64_t n);
  PrepareInsert_t Prepare_ = nullptr;  // the target's PrepareInsert when the executor takes it
  std::atomic<uint64_t> MutateCpuNs_{0};  // CPU time of the parallel mutation (and preparation) threads
  void Adopt(TcBatch &&B);  // streaming: the batch's testcases join the ready queue
  uint64_t Budget(uint64_t n) const;
  bool More(uint64_t done) const;
  bool MergeCoverage(bool Done);
  bool AbsorbMerge();  // MergeEnd of the merge in flight, absorbed
  bool MergePending_ = false, AllDone_ = false;
  void WriteSample(const uint8_t *Tc, size_t Size, const LaneResult &L);
  FILE *Sample_ = nullptr;
  bool StreamStep(bool Done);
  void Account(const uint8_t *Tc, size_t Size, const LaneResult &L, bool KnownCrash = false);
  void AccountStep(std::vector<StreamResult_t> &Out);
  // arenas: a released one (every testcase accounted) is kept for the next
  // batch (its buffers keep their capacity: no allocation and no first-touch
  // page faults per batch)
  void ReleaseArena(TcArena *A);
  std::unique_ptr<TcArena> NewArena();
  std::mutex ArenaPoolMu_;
  std::vector<std::unique_ptr<TcArena>> ArenaPool_;

  const RunnerOptions O_;
  Executor_t &Exec_;
  Target_t &Target_;
  ModuleSlots &Slots_;
  CoverageExchange_t *X_;
  std::mt19937_64 Rng_;
  fs::path T_;
  Corpus_t Corpus_;
  std::unique_ptr<Mutator_t> Mutator_;
  std::vector<std::string> Pending_;
  TcBatch Batch_;                // batch mode: the batch in the lanes
  std::vector<TcRef> BatchRefs_;
  std::string LastNewCov_;  // the testcase last passed to Mutator_->OnNewCoverage
  bool HaveNewCov_ = false;
  std::future<TcBatch> Next_;
  FileWriter Writer_;
  std::unordered_set<std::string> CrashNames_;
  std::unordered_set<uint64_t> Coverage_;  // the master's aggregate (server.h:816-854)
  FuzzStats S_;
  std::chrono::steady_clock::time_point t0_;
  // streaming (RunnerOptions::slice != 0 on an executor that streams)
  bool stream_ = false;
  std::deque<TcRef> Ready_;                                      // mutated, not yet in a lane
  std::unordered_map<TcArena *, std::unique_ptr<TcArena>> Arenas_;  // owners of Ready_ / Slot_ testcases
  std::vector<TcRef> Slot_;  // tag -> testcase in a lane (tags are slot indices)
  std::vector<uint64_t> FreeSlot_;
  size_t InFlight_ = 0;
};

bool ParseRunnerArgs(int argc, char **argv, RunnerOptions &O);
// A Tenet entry stream (include/wtfgpu.h wtfgpu_set_tenet) as the reference's
// text (BochscpuBackend_t::DumpTenetDelta, bochscpu_backend.cc:1215-1323): the
// first REGS entry sets every register, each later one the registers that
// changed since the previous one, then the accesses logged before it as
// ,mr= / ,mw= / ,mrw= 0x<va>:<HEX>; a line only when something was printed.
// Stops at a truncated or incomplete entry.
void FormatTenet(const uint8_t *Stream, size_t Bytes, FILE *F);
// Loads the snapshot, initialises the executor and the module, runs the mode.
// make_executor is called after the options are parsed; returns the exit code.
int RunnerMain(const RunnerOptions &O, Executor_t &Exec, const Options_t &Opts, const CpuState_t &State,
               CoverageExchange_t *X = nullptr);
// Options_t + CpuState_t from <target>/state (regs.json, symbol store) and the runner options.
bool LoadTarget(const RunnerOptions &O, Options_t &Opts, CpuState_t &State);

// A lane's FAULT exit named as the guest would report it: ring 3 as the user-mode
// crash detection does, ring 0 as the bugcheck the kernel raises
// (crash_detection_umode.cc:53-129 + backend.cc:204-212).
TestcaseResult_t FaultToResult(uint32_t vector, uint32_t error, uint64_t rip, uint64_t addr, uint32_t cpl);

// The CpuState_t -> wtfgpu_regs_t mapping (LoadState, bochscpu_backend.cc:1026-1122).
wtfgpu_regs_t RegsFromCpuState(const CpuState_t &S);

}  // namespace wtfgpu_host
