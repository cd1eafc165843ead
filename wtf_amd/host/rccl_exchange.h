// rccl_exchange.h — CoverageExchange_t over RCCL (see rccl_exchange.cc).
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "runner.h"

namespace wtfgpu_host {

constexpr size_t kRcclIdBytes = 128;  // sizeof(ncclUniqueId)

// a fresh communicator id (rank 0)
bool RcclUniqueId(uint8_t Out[kRcclIdBytes]);
// rank 0 makes the id and writes it to Path; the others wait for the file
bool RcclIdViaFile(const std::string &Path, int Rank, uint8_t Id[kRcclIdBytes], double TimeoutS = 120);

class RcclExchange_t final : public CoverageExchange_t {
 public:
  // Force: take the collective path at world 1 too (a one-rank communicator)
  RcclExchange_t(int Rank, int World, bool Force = false);
  ~RcclExchange_t() override;
  // Stream: the engine's HIP stream (wtfgpu_stream); collective on every rank
  bool Init(const uint8_t Id[kRcclIdBytes], void *Stream);
  int Rank() const override { return rank_; }
  int World() const override { return world_; }
  bool Exchanging() const override { return world_ > 1 || force_; }
  bool AllReduceMax(uint8_t *Map, uint64_t Bytes, bool Device) override;
  bool AllDone(bool Mine, bool *All) override;
  bool AllGatherV(const std::vector<uint64_t> &Mine, std::vector<uint64_t> &All) override;
  // the deferred merge on the exchange's stream: a frozen copy of the map (the
  // next step's commits write the live one), MAX all-reduce of that copy into
  // a buffer of its own, one all-gather of every rank's MergeBlocks block
  // (merge_block.h), fused in one group; nothing waits on the collectives
  // before MergeEnd
  bool MergeBegin(const uint8_t *Map, uint64_t Bytes, bool Device, const std::vector<uint64_t> &Extras,
                  bool Done) override;
  bool MergeEnd(const uint8_t **Merged, uint64_t *Bytes, std::vector<uint64_t> &AllExtras, bool *AllDone) override;

 private:
  struct Impl;
  int rank_, world_;
  bool force_;
  Impl *impl_;
};

}  // namespace wtfgpu_host
