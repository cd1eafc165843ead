// rccl_exchange.cc — CoverageExchange_t for GPU shards: one RCCL
// communicator over the node's GPUs (xGMI), an in-place
// ncclAllReduce(uint8, ncclMax) of the device coverage map on the engine's
// stream. The unique id travels out of band: through a file
// (`wtfgpu fuzz --world n --rank r --nccl-id-file f`, rank 0 writes it) or
// from the caller (libwtfnode, bench.py broadcasts it).
#include "rccl_exchange.h"

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
  hipStream_t stream = nullptr;
  uint8_t *flag = nullptr;  // device byte for AllDone
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

RcclExchange_t::RcclExchange_t(int Rank, int World) : rank_(Rank), world_(World), impl_(new Impl) {}

RcclExchange_t::~RcclExchange_t() {
  if (impl_->comm) ncclCommDestroy(impl_->comm);
  if (impl_->flag) (void)hipFree(impl_->flag);
  delete impl_;
}

bool RcclExchange_t::Init(const uint8_t Id[kRcclIdBytes], void *Stream) {
  impl_->stream = (hipStream_t)Stream;
  if (world_ <= 1) return true;
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
  if (world_ <= 1) return true;
  if (!Device || !impl_->comm) return false;
  if (ncclAllReduce(Map, Map, Bytes, ncclUint8, ncclMax, impl_->comm, impl_->stream) != ncclSuccess) return false;
  return hipStreamSynchronize(impl_->stream) == hipSuccess;
}

bool RcclExchange_t::AllDone(bool Mine, bool *All) {
  if (world_ <= 1) {
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

}  // namespace wtfgpu_host
