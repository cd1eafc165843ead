// rccl_exchange.cc — CoverageExchange_t for GPU shards: one RCCL
// communicator over the node's GPUs (xGMI). Each node step's merge
// (MergeBegin / MergeEnd) copies the device coverage map into a frozen
// buffer, then runs one fused group on the exchange's own stream: an
// out-of-place ncclAllReduce(uint8, ncclMax) of the frozen copy into `merged`
//  and an ncclAllGather of every rank's MergeBlocks block (the
// values outside the map plus the done flag). The next step's kernels run
// meanwhile; the result is absorbed one step later. The host waits for the
// D2D frozen copy before MergeBegin returns (a map-sized copy, tens of
// microseconds: it orders the copy before the next step's commits on every
// engine queue without an event per queue) and never for a k_run slice.
// A world-1 node skips all of this unless it is forced (--rccl-force /
// WTF_RCCL_FORCE=1), which runs every call against a one-rank communicator:
// the GPU test of the RCCL path on a one-GPU box. The unique id travels out
// of band: through a file (`wtfgpu fuzz --world n --rank r --nccl-id-file f`,
// rank 0 writes it) or from the caller (libwtfnode, bench.py broadcasts it).
// A failed hip / nccl call fails the merge, and the session with it.
#include "rccl_exchange.h"

#include "merge_block.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <thread>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

namespace wtfgpu_host {

struct RcclExchange_t::Impl {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;  // the collectives' own stream
  uint8_t *flag = nullptr;       // device byte for AllDone
  uint64_t *gbuf = nullptr;      // AllGatherV staging: world counts, then world * cap values
  uint64_t gcap = 0;             // u64 slots in gbuf
  // deferred merge: the frozen copy of the map and the reduced map, the
  // MergeBlocks blocks sent / received (device and pinned host), the event
  // MergeEnd waits for, and the overflow values still to send
  uint8_t *frozen = nullptr, *merged = nullptr;
  uint64_t merged_bytes = 0, merged_cap = 0;
  uint64_t *dsend = nullptr, *drecv = nullptr, *hsend = nullptr, *hrecv = nullptr;
  hipEvent_t ev = nullptr;
  bool inflight = false;
  MergeBlocks blocks{kMergeCap};
};

bool RcclUniqueId(uint8_t Out[kRcclIdBytes]) {
  static_assert(sizeof(ncclUniqueId) == kRcclIdBytes, "ncclUniqueId size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return false;
  memcpy(Out, &id, sizeof(id));
  return true;
}

bool RcclIdViaFile(const std::string &Path, int Rank, uint8_t Id[kRcclIdBytes], double TimeoutS) {
  if (Rank == 0) {
    if (!RcclUniqueId(Id)) return false;
    const std::string tmp = Path + ".tmp";
    {
      std::ofstream f(tmp, std::ios::binary);
      f.write((const char *)Id, kRcclIdBytes);
      if (!f) return false;
    }
    std::filesystem::rename(tmp, Path);
    return true;
  }
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < TimeoutS) {
    std::ifstream f(Path, std::ios::binary);
    if (f && f.read((char *)Id, kRcclIdBytes)) return true;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  return false;
}

RcclExchange_t::RcclExchange_t(int Rank, int World, bool Force)
    : rank_(Rank), world_(World), force_(Force), impl_(new Impl) {}

RcclExchange_t::~RcclExchange_t() {
  if (impl_->stream) (void)hipStreamSynchronize(impl_->stream);  // a merge still in flight completes (every rank issued it)
  if (impl_->comm) ncclCommDestroy(impl_->comm);
  if (impl_->merged) (void)hipFree(impl_->merged);
  if (impl_->frozen) (void)hipFree(impl_->frozen);
  if (impl_->dsend) (void)hipFree(impl_->dsend);
  if (impl_->drecv) (void)hipFree(impl_->drecv);
  if (impl_->hsend) (void)hipHostFree(impl_->hsend);
  if (impl_->hrecv) (void)hipHostFree(impl_->hrecv);
  if (impl_->ev) (void)hipEventDestroy(impl_->ev);
  if (impl_->flag) (void)hipFree(impl_->flag);
  if (impl_->gbuf) (void)hipFree(impl_->gbuf);
  if (impl_->stream) (void)hipStreamDestroy(impl_->stream);
  delete impl_;
}

bool RcclExchange_t::Init(const uint8_t Id[kRcclIdBytes], void *Stream) {
  (void)Stream;  // the engine's stream: the collectives use their own (see above)
  if (!Exchanging()) return true;
  if (hipStreamCreateWithFlags(&impl_->stream, hipStreamNonBlocking) != hipSuccess) return false;
  ncclUniqueId id;
  memcpy(&id, Id, sizeof(id));
  const ncclResult_t r = ncclCommInitRank(&impl_->comm, world_, id, rank_);
  if (r != ncclSuccess) {
    fprintf(stderr, "ncclCommInitRank(rank %d of %d): %s\n", rank_, world_, ncclGetErrorString(r));
    return false;
  }
  return true;
}

bool RcclExchange_t::AllReduceMax(uint8_t *Map, uint64_t Bytes, bool Device) {
  if (!Exchanging()) return true;
  if (!Device || !impl_->comm) return false;
  if (ncclAllReduce(Map, Map, Bytes, ncclUint8, ncclMax, impl_->comm, impl_->stream) != ncclSuccess) return false;
  return hipStreamSynchronize(impl_->stream) == hipSuccess;
}

bool RcclExchange_t::AllDone(bool Mine, bool *All) {
  if (!Exchanging()) {
    *All = Mine;
    return true;
  }
  if (!impl_->flag && hipMalloc((void **)&impl_->flag, 1) != hipSuccess) return false;
  uint8_t notdone = Mine ? 0 : 1;
  if (hipMemcpyAsync(impl_->flag, &notdone, 1, hipMemcpyHostToDevice, impl_->stream) != hipSuccess) return false;
  if (!AllReduceMax(impl_->flag, 1, true)) return false;
  if (hipMemcpyAsync(&notdone, impl_->flag, 1, hipMemcpyDeviceToHost, impl_->stream) != hipSuccess ||
      hipStreamSynchronize(impl_->stream) != hipSuccess)
    return false;
  *All = notdone == 0;
  return true;
}

// counts first (one u64 per rank), then every list padded to the longest
bool RcclExchange_t::AllGatherV(const std::vector<uint64_t> &Mine, std::vector<uint64_t> &All) {
  All = Mine;
  if (!Exchanging()) return true;
  if (!impl_->comm) return false;
  auto grow = [&](uint64_t slots) {
    if (slots <= impl_->gcap) return true;
    if (impl_->gbuf) (void)hipFree(impl_->gbuf);
    impl_->gbuf = nullptr;
    impl_->gcap = 0;
    if (hipMalloc((void **)&impl_->gbuf, slots * 8) != hipSuccess) return false;
    impl_->gcap = slots;
    return true;
  };
  const uint64_t W = (uint64_t)world_;
  std::vector<uint64_t> counts(W, 0);
  uint64_t mine = Mine.size();
  if (!grow(W + 1)) return false;
  if (hipMemcpyAsync(impl_->gbuf + W, &mine, 8, hipMemcpyHostToDevice, impl_->stream) != hipSuccess ||
      ncclAllGather(impl_->gbuf + W, impl_->gbuf, 1, ncclUint64, impl_->comm, impl_->stream) != ncclSuccess ||
      hipMemcpyAsync(counts.data(), impl_->gbuf, W * 8, hipMemcpyDeviceToHost, impl_->stream) != hipSuccess ||
      hipStreamSynchronize(impl_->stream) != hipSuccess)
    return false;
  uint64_t cap = 0;
  for (uint64_t c : counts) cap = std::max(cap, c);
  if (cap == 0) return true;  // every rank sees the same counts: all skip together
  if (!grow(W * cap + cap)) return false;
  uint64_t *send = impl_->gbuf + W * cap;
  if ((mine && hipMemcpyAsync(send, Mine.data(), mine * 8, hipMemcpyHostToDevice, impl_->stream) != hipSuccess) ||
      ncclAllGather(send, impl_->gbuf, cap, ncclUint64, impl_->comm, impl_->stream) != ncclSuccess)
    return false;
  std::vector<uint64_t> got(W * cap);
  if (hipMemcpyAsync(got.data(), impl_->gbuf, W * cap * 8, hipMemcpyDeviceToHost, impl_->stream) != hipSuccess ||
      hipStreamSynchronize(impl_->stream) != hipSuccess)
    return false;
  All.clear();
  for (uint64_t r = 0; r < W; r++) All.insert(All.end(), got.begin() + r * cap, got.begin() + r * cap + counts[r]);
  return true;
}

bool RcclExchange_t::MergeBegin(const uint8_t *Map, uint64_t Bytes, bool Device, const std::vector<uint64_t> &Extras,
                                bool Done) {
  Impl &I = *impl_;
  if (!Exchanging()) {  // nothing to exchange: the result is this shard's own
    merged_extra_ = Extras;
    merged_done_ = Done;
    I.merged_bytes = 0;
    I.inflight = true;
    return true;
  }
  if (!Device || !I.comm || I.inflight) return false;
  const uint64_t W = (uint64_t)world_, B = kMergeCap + 1;
  if (!I.dsend) {  // sized once: no allocation (and no device-wide sync) during a run
    if (hipMalloc((void **)&I.dsend, B * 8) != hipSuccess || hipMalloc((void **)&I.drecv, W * B * 8) != hipSuccess ||
        hipHostMalloc((void **)&I.hsend, B * 8) != hipSuccess || hipHostMalloc((void **)&I.hrecv, W * B * 8) != hipSuccess ||
        hipEventCreateWithFlags(&I.ev, hipEventDisableTiming) != hipSuccess)
      return false;
  }
  if (Bytes > I.merged_cap) {  // the map's size is fixed after set_code_pages: the first merge sizes it
    if (I.merged) (void)hipFree(I.merged);
    if (I.frozen) (void)hipFree(I.frozen);
    I.merged = I.frozen = nullptr;
    I.merged_cap = 0;
    if (hipMalloc((void **)&I.merged, Bytes) != hipSuccess || hipMalloc((void **)&I.frozen, Bytes) != hipSuccess)
      return false;
    I.merged_cap = Bytes;
  }
  I.merged_bytes = Bytes;
  // The map as of this step, frozen before the call returns: the engine's
  // coverage commits are synchronous (so the live map is final here), and the
  // next step's commits may write it while the all-reduce below still runs.
  // Every shard reduces what it had at the same step: a fixed-seed campaign
  // merges the same maps whatever the collective's timing (DESIGN U44).
  if (Bytes && (hipMemcpyAsync(I.frozen, Map, Bytes, hipMemcpyDeviceToDevice, I.stream) != hipSuccess ||
                hipStreamSynchronize(I.stream) != hipSuccess))
    return false;
  const uint64_t words = I.blocks.Pack(Extras, Done, I.hsend);
  if (hipMemcpyAsync(I.dsend, I.hsend, words * 8, hipMemcpyHostToDevice, I.stream) != hipSuccess) return false;
  if (ncclGroupStart() != ncclSuccess) return false;
  if (Bytes && ncclAllReduce(I.frozen, I.merged, Bytes, ncclUint8, ncclMax, I.comm, I.stream) != ncclSuccess) return false;
  if (ncclAllGather(I.dsend, I.drecv, B, ncclUint64, I.comm, I.stream) != ncclSuccess) return false;
  if (ncclGroupEnd() != ncclSuccess) return false;
  if (hipMemcpyAsync(I.hrecv, I.drecv, W * B * 8, hipMemcpyDeviceToHost, I.stream) != hipSuccess ||
      hipEventRecord(I.ev, I.stream) != hipSuccess)
    return false;
  I.inflight = true;
  return true;
}

bool RcclExchange_t::MergeEnd(const uint8_t **Merged, uint64_t *Bytes, std::vector<uint64_t> &AllExtras,
                              bool *AllDone) {
  Impl &I = *impl_;
  if (!I.inflight) return false;
  I.inflight = false;
  if (!Exchanging()) {
    AllExtras.swap(merged_extra_);
    merged_extra_.clear();
    *AllDone = merged_done_;
    *Merged = nullptr;
    *Bytes = 0;
    return true;
  }
  if (hipEventSynchronize(I.ev) != hipSuccess) return false;
  const uint64_t W = (uint64_t)world_, B = kMergeCap + 1;
  if (!MergeBlocks::Unpack(I.hrecv, W * B, W, B, kMergeCap, AllExtras, AllDone)) return false;
  *Merged = I.merged;
  *Bytes = I.merged_bytes;
  return true;
}

}  // namespace wtfgpu_host
