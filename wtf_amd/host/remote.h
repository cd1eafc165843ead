// remote.h — the master and the node over the wire protocol (wire.h).
//
//   <node> master --name T --target D --address tcp://127.0.0.1:31337 --nodes K [--batched]
//                 [--runs N] [--seconds S] [--seed S] [--max_len L]
//       The reference master (server.h:629-886: corpus, mutator, crash
//       saving) as a FuzzSession whose executor is the connected nodes: with
//       --batched every node announces its lanes and gets that many testcases
//       per round trip; without it, the reference protocol (one testcase per
//       round trip, so reference clients can connect).
//   <node> fuzz --name T --target D --address A [--batched] [--lanes N] ...
//       The client loop (client.cc:187-258) on this node's executor: every
//       Batch (or Testcase) the master sends runs through RunBatch and the
//       results go back in order; coverage of a timed-out testcase is revoked
//       before it is sent (client.cc:122-133).
#pragma once
#include "runner.h"

namespace wtfgpu_host {

// The master's view of the nodes (one socket each), as an executor.
class RemoteExecutor_t final : public Executor_t {
 public:
  ~RemoteExecutor_t() override;
  // Waits for `Nodes` connections on ListenFd; batched nodes say hello first.
  bool Accept(int ListenFd, int Nodes, bool Batched);
  Backend_t *AsBackend() override { return nullptr; }
  uint32_t Lanes() const override { return Lanes_; }
  bool RunBatch(const Target_t &, const std::vector<std::pair<const uint8_t *, size_t>> &Testcases,
                std::vector<LaneResult> &Out, ModuleSlots *) override;
  void ResetCoverage() override {}
  void SetFullCoverage(bool) override {}
  size_t CoverageSize() const override { return Seen_.size(); }
  std::string StatsJson() const override;

 private:
  struct Node {
    int Fd = -1;
    uint64_t Lanes = 1;
  };
  std::vector<Node> Nodes_;
  bool Batched_ = false;
  uint32_t Lanes_ = 0;
  std::unordered_set<uint64_t> Seen_;  // union of the coverage the nodes reported
  uint64_t Frames_ = 0, BytesOut_ = 0, BytesIn_ = 0;
  double WireMs_ = 0;
};

// `master` mode (no backend, no snapshot: the mutator and the corpus only).
int MasterMain(const RunnerOptions &O);
// `fuzz --address`: the node's client loop on Exec (the target initialised).
int NodeMain(const RunnerOptions &O, Executor_t &Exec, Target_t &Target, ModuleSlots &Slots);

}  // namespace wtfgpu_host
