// runner.h — the batched client loop over an executor:
// `run` replays inputs (wtf run, subcommands.cc:20-75) and `fuzz` is the
// node loop with an in-process master (client.cc:187-258 + server.h:720-886:
// mutate, run, keep testcases that found new coverage, save crashes), both
// batched N testcases per executor call.
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/wtfgpu.h"
#include "wtf_api.h"

namespace wtfgpu_host {

struct LaneResult {
  TestcaseResult_t result;
  bool error = false;        // the engine could not finish the testcase (unimplemented opcode, overlay full)
  uint32_t exit_status = 0;  // last engine exit status (wtfgpu_status)
  uint64_t icount = 0;       // retired instructions
  uint64_t rip = 0;
  uint64_t gprs[18] = {};    // final gprs (wtfgpu order) + rip + rflags
  std::vector<uint64_t> new_coverage;  // LastNewCoverage, attributed in lane order
};

// A backend that runs many testcases per call (GpuBackend_t; the oracle twin
// runs them one after the other).
class Executor_t {
 public:
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
  virtual size_t CoverageSize() const = 0;
  virtual std::string StatsJson() const { return "{}"; }
};

struct RunnerOptions {
  std::string mode = "run";  // run | fuzz
  std::string name;          // target name
  std::string target;        // dir with state/, inputs/, outputs/, crashes/
  std::string input;         // run: file or directory (default <target>/inputs)
  std::string results;       // run: JSON-lines output path
  uint64_t limit = 0;
  uint32_t lanes = 1;
  uint32_t overlay_pages = 32;
  uint64_t runs = 0;         // fuzz: testcases
  double seconds = 0;        // fuzz: wall-clock budget (0 = none)
  uint64_t seed = 1337;
  uint64_t max_len = 0x1000;
  int device = 0;
  bool full_coverage = false;
  bool quiet = false;
  bool serial_mutation = false;  // one mutator, in order: the reference master's stream exactly
};

bool ParseRunnerArgs(int argc, char **argv, RunnerOptions &O);
// Loads the snapshot, initialises the executor and the module, runs the mode.
// make_executor is called after the options are parsed; returns the exit code.
int RunnerMain(const RunnerOptions &O, Executor_t &Exec, const Options_t &Opts, const CpuState_t &State);
// Options_t + CpuState_t from <target>/state (regs.json, symbol store) and the runner options.
bool LoadTarget(const RunnerOptions &O, Options_t &Opts, CpuState_t &State);

// A lane's FAULT exit named as the guest would report it: ring 3 as the user-mode
// crash detection does, ring 0 as the bugcheck the kernel raises
// (crash_detection_umode.cc:53-129 + backend.cc:204-212).
TestcaseResult_t FaultToResult(uint32_t vector, uint32_t error, uint64_t rip, uint64_t addr, uint32_t cpl);

// The CpuState_t -> wtfgpu_regs_t mapping (LoadState, bochscpu_backend.cc:1026-1122).
wtfgpu_regs_t RegsFromCpuState(const CpuState_t &S);

}  // namespace wtfgpu_host
