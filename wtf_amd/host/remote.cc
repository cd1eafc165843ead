// remote.cc — see remote.h.
#include "remote.h"

#include <chrono>
#include <cstdio>

#include "wire.h"

namespace wtfgpu_host {

namespace {
using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }
}  // namespace

RemoteExecutor_t::~RemoteExecutor_t() {
  for (Node &N : Nodes_) wire::Close(N.Fd);
}

bool RemoteExecutor_t::Accept(int ListenFd, int Nodes, bool Batched) {
  Batched_ = Batched;
  for (int i = 0; i < Nodes; i++) {
    Node N;
    N.Fd = wire::Accept(ListenFd);
    if (N.Fd < 0) return false;
    if (Batched) {
      std::string Msg;
      if (!wire::ReceiveFrame(N.Fd, Msg, 4096) || !wire::DecodeHello(Msg, N.Lanes)) {
        printf("node %d: no batched hello\n", i);
        return false;
      }
    }
    Lanes_ += (uint32_t)N.Lanes;
    Nodes_.push_back(N);
  }
  return true;
}

// The batch is cut in node order (node k gets the next Lanes(k) testcases);
// every frame is sent before the first answer is read, so the nodes run in
// parallel; results come back in the batch's order.
bool RemoteExecutor_t::RunBatch(const Target_t &, const std::vector<std::pair<const uint8_t *, size_t>> &Testcases,
                                std::vector<LaneResult> &Out, ModuleSlots *) {
  const auto t0 = Clock::now();
  Out.assign(Testcases.size(), LaneResult{});
  std::vector<std::pair<size_t, size_t>> Part(Nodes_.size(), {0, 0});
  size_t Off = 0;
  for (size_t k = 0; k < Nodes_.size() && Off < Testcases.size(); k++) {
    const size_t n = std::min<size_t>(Nodes_[k].Lanes, Testcases.size() - Off);
    Part[k] = {Off, n};
    Off += n;
  }
  if (Off != Testcases.size()) return false;  // more testcases than lanes
  for (size_t k = 0; k < Nodes_.size(); k++) {
    const auto [o, n] = Part[k];
    if (!n) continue;
    std::string Msg;
    if (Batched_) {
      Msg = wire::EncodeBatch({Testcases.begin() + o, Testcases.begin() + o + n});
    } else {
      Msg = wire::EncodeTestcase(Testcases[o].first, Testcases[o].second);
    }
    if (!wire::SendFrame(Nodes_[k].Fd, Msg)) return false;
    BytesOut_ += Msg.size() + 4;
    Frames_++;
  }
  for (size_t k = 0; k < Nodes_.size(); k++) {
    const auto [o, n] = Part[k];
    if (!n) continue;
    std::string Msg;
    if (!wire::ReceiveFrame(Nodes_[k].Fd, Msg)) return false;
    BytesIn_ += Msg.size() + 4;
    if (Batched_) {
      std::vector<wire::WireResult> R;
      if (!wire::DecodeBatchResult(Msg, R) || R.size() != n) return false;
      for (size_t i = 0; i < n; i++) {
        LaneResult &L = Out[o + i];
        L.result = std::move(R[i].Result);
        L.icount = R[i].Retired;
        L.error = R[i].Error;
        L.new_coverage = std::move(R[i].Coverage);
      }
    } else {  // the reference Result message: the testcase comes back with it
      std::string Tc;
      LaneResult &L = Out[o];
      if (!wire::DecodeResult(Msg, Tc, L.new_coverage, L.result)) return false;
      if (Tc.size() != Testcases[o].second || memcmp(Tc.data(), Testcases[o].first, Tc.size()) != 0) return false;
    }
  }
  for (const LaneResult &L : Out) Seen_.insert(L.new_coverage.begin(), L.new_coverage.end());
  WireMs_ += ms_since(t0);
  return true;
}

std::string RemoteExecutor_t::StatsJson() const {
  char b[256];
  snprintf(b, sizeof(b),
           "{\"kind\":\"remote\",\"nodes\":%zu,\"batched\":%d,\"frames\":%llu,\"bytes_out\":%llu,\"bytes_in\":%llu,"
           "\"round_trip_ms\":%.3f}",
           Nodes_.size(), (int)Batched_, (unsigned long long)Frames_, (unsigned long long)BytesOut_,
           (unsigned long long)BytesIn_, WireMs_);
  return b;
}

int MasterMain(const RunnerOptions &O) {
  Target_t *Target = Targets_t::Instance().Get(O.name);
  if (!Target) {
    printf("Target %s not found\n", O.name.c_str());
    return 1;
  }
  const int L = wire::Listen(O.address);
  if (L < 0) {
    printf("Listen on %s failed\n", O.address.c_str());
    return 1;
  }
  RemoteExecutor_t Exec;
  const bool ok = Exec.Accept(L, O.nodes, O.batched);
  wire::Close(L);
  if (!ok) return 1;
  ModuleSlots Slots;
  FuzzSession F(O, Exec, *Target, Slots, nullptr);
  if (!F.Start()) {
    printf("Nothing to run: empty corpus and no inputs\n");
    return 1;
  }
  while (!F.Done())
    if (!F.Step()) {
      printf("a node failed\n");
      return 1;
    }
  F.FlushFiles();
  printf("%s\n", F.SummaryJson().c_str());
  return 0;  // the node sockets close with Exec: the nodes' loops end
}

int NodeMain(const RunnerOptions &O, Executor_t &Exec, Target_t &Target, ModuleSlots &Slots) {
  const int Fd = wire::Dial(O.address);
  if (Fd < 0) {
    printf("Dial %s failed\n", O.address.c_str());
    return 1;
  }
  Exec.SetWantRegisters(false);
  if (O.batched && !wire::SendFrame(Fd, wire::EncodeHello(Exec.Lanes()))) return 1;
  uint64_t Received = 0, Retired = 0;
  const auto t0 = Clock::now();
  std::string Msg;
  std::vector<std::string> Tc;
  while (wire::ReceiveFrame(Fd, Msg)) {
    if (O.batched) {
      if (!wire::DecodeBatch(Msg, Tc)) return 1;
    } else {
      Tc.resize(1);
      if (!wire::DecodeTestcase(Msg, Tc[0])) return 1;
    }
    std::vector<wire::WireResult> W(Tc.size());
    for (size_t b = 0; b < Tc.size(); b += Exec.Lanes()) {
      const size_t n = std::min<size_t>(Exec.Lanes(), Tc.size() - b);
      std::vector<std::pair<const uint8_t *, size_t>> In(n);
      for (size_t i = 0; i < n; i++) In[i] = {(const uint8_t *)Tc[b + i].data(), Tc[b + i].size()};
      std::vector<LaneResult> R;
      if (!Exec.RunBatch(Target, In, R, &Slots)) {
        printf("RunBatch failed\n");
        return 1;
      }
      for (size_t i = 0; i < n; i++) {
        wire::WireResult &X = W[b + i];
        X.Result = R[i].result;
        X.Retired = R[i].icount;
        X.Error = R[i].error;
        // RevokeLastNewCoverage on a timeout before the result is sent (client.cc:122-133)
        if (!std::holds_alternative<Timedout_t>(R[i].result)) X.Coverage = std::move(R[i].new_coverage);
        Retired += R[i].icount;
      }
    }
    Received += Tc.size();
    const std::string Out =
        O.batched ? wire::EncodeBatchResult(W)
                  : wire::EncodeResult((const uint8_t *)Tc[0].data(), Tc[0].size(), W[0].Coverage, W[0].Result);
    if (!wire::SendFrame(Fd, Out)) break;
  }
  wire::Close(Fd);
  const double s = std::chrono::duration<double>(Clock::now() - t0).count();
  printf("{\"mode\":\"node\",\"target\":\"%s\",\"lanes\":%u,\"batched\":%d,\"execs\":%llu,\"retired\":%llu,\"wall_s\":%.6f,"
         "\"backend\":%s}\n",
         O.name.c_str(), Exec.Lanes(), (int)O.batched, (unsigned long long)Received, (unsigned long long)Retired, s,
         Exec.StatsJson().c_str());
  return 0;
}

}  // namespace wtfgpu_host
