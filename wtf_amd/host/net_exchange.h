// net_exchange.h — CoverageExchange_t over TCP (see net_exchange.cc).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "runner.h"

namespace wtfgpu_host {

class TcpExchange_t final : public CoverageExchange_t {
 public:
  TcpExchange_t(int Rank, int World) : rank_(Rank), world_(World) {}
  ~TcpExchange_t() override;
  // rank 0 binds Host:Port and waits for the others; they retry until TimeoutS
  bool Connect(const std::string &Host, uint16_t Port, double TimeoutS = 60);
  int Rank() const override { return rank_; }
  int World() const override { return world_; }
  bool AllReduceMax(uint8_t *Map, uint64_t Bytes, bool Device) override;
  bool AllDone(bool Mine, bool *All) override;
  bool AllGatherV(const std::vector<uint64_t> &Mine, std::vector<uint64_t> &All) override;

 private:
  int rank_, world_;
  int listen_ = -1;
  std::vector<int> peers_;  // rank 0: fd per rank (index 0 unused); others: [0] = rank 0
};

}  // namespace wtfgpu_host
