// module_slots.cc — see module_slots.h.
#include "module_slots.h"

#include <cstdio>
#include <cstdlib>

namespace wtfgpu_host {

std::vector<LaneStateOps> &LaneStateRegistry() {
  static std::vector<LaneStateOps> R;
  return R;
}

namespace {
thread_local int64_t t_in = -1;  // lane swapped in on this thread
}

ModuleSlots::~ModuleSlots() { release(); }

bool ModuleSlots::ThreadSafe() const {
  for (const auto &ops : LaneStateRegistry())
    if (!ops.tls) return false;
  return inst_ || !LaneStateRegistry().empty();
}

void ModuleSlots::release() {
  const auto &R = LaneStateRegistry();
  for (size_t k = 0; k < lanes_.size(); k++)
    if (lanes_[k]) R[k % R.size()].destroy(lanes_[k]);
  for (size_t i = 0; i < initial_.size(); i++) R[i].destroy(initial_[i]);
  lanes_.clear();
  initial_.clear();
  dirty_.clear();
}

void ModuleSlots::Capture(uint32_t lanes) {
  release();
  const auto &R = LaneStateRegistry();
  for (const auto &ops : R) initial_.push_back(ops.clone(ops.object()));
  lanes_.assign((size_t)lanes * R.size(), nullptr);
  dirty_.assign(lanes, 0);
  t_in = -1;
}

void ModuleSlots::ResetAll() {
  for (size_t l = 0; l < dirty_.size(); l++) ResetLane((uint32_t)l);
}

void ModuleSlots::ResetLane(uint32_t l) {
  if (l >= dirty_.size() || !dirty_[l]) return;
  const auto &R = LaneStateRegistry();
  void **objs = lanes_.data() + (size_t)l * R.size();
  for (size_t i = 0; i < R.size(); i++)
    if (objs[i]) R[i].assign(objs[i], initial_[i]);
  dirty_[l] = 0;
}

void ModuleSlots::SwapIn(uint32_t lane) {
  if (t_in >= 0) {
    fprintf(stderr, "ModuleSlots: lane %lld still swapped in\n", (long long)t_in);
    std::abort();
  }
  const auto &R = LaneStateRegistry();
  if (lane >= dirty_.size()) {
    fprintf(stderr, "ModuleSlots: lane %u out of range\n", lane);
    std::abort();
  }
  void **objs = lanes_.data() + (size_t)lane * R.size();
  for (size_t i = 0; i < R.size(); i++) {
    if (!objs[i]) objs[i] = R[i].clone(initial_[i]);
    R[i].swap(R[i].object(), objs[i]);
  }
  dirty_[lane] = 1;
  t_in = lane;
}

void ModuleSlots::SwapOut(uint32_t lane) {
  if (t_in != (int64_t)lane) {
    fprintf(stderr, "ModuleSlots: swap-out of lane %u, lane %lld is in\n", lane, (long long)t_in);
    std::abort();
  }
  const auto &R = LaneStateRegistry();
  void **objs = lanes_.data() + (size_t)lane * R.size();
  for (size_t i = 0; i < R.size(); i++) R[i].swap(R[i].object(), objs[i]);
  t_in = -1;
}

}  // namespace wtfgpu_host
