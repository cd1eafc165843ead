// module_instances.h — per-lane instances of an unchanged fuzzer module
// (option (b)).
//
// An upstream module keeps its testcase state in plain globals
// (fuzzer_tlv_server.cc:42-65: the packet deque the ProcessPacket breakpoint
// pops) and assumes one testcase in flight. Without the one-line
// WTF_LANE_STATE annotation (module_slots.h) it can still run batched: the
// module is built as a shared object and loaded once per lane, each copy from
// its own (then unlinked) file, so the dynamic loader gives every copy its own data segment
// (its globals, its static Target_t, its handler functions). Lane l then runs
// copy l: its InsertTestcase / Restore, and the breakpoint handlers copy l set
// during its Init.
//
// The copies share everything outside the module (g_Backend, g_Dbg, the
// backend itself): the shared object leaves those undefined and binds them to
// the executable's exported definitions; its own definitions bind inside the
// copy (-Bsymbolic), so an executable that also links the module cannot
// capture the copies' globals. The count is bounded (kMaxInstances): every
// copy costs its code and data pages.
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "wtf_api.h"

namespace wtfgpu_host {

class ModuleInstances {
 public:
  static constexpr uint32_t kMaxInstances = 4096;

  // Count private copies of the module shared object SoPath; each registers a
  // Target_t named Name (targets.cc:11-38), kept here and taken back out of
  // Targets_t so the registry holds no duplicates.
  bool Load(const std::string &SoPath, const std::string &Name, uint32_t Count);
  // Target.Init of every copy (g_Backend must be set): the breakpoints copy k
  // sets while its Init runs are recorded as copy k's handlers.
  bool InitAll(const Options_t &Opts, const CpuState_t &State);
  uint32_t Count() const { return (uint32_t)targets_.size(); }
  const Target_t &TargetOf(uint32_t Lane) const { return targets_.at(Lane); }
  // the handler lane `Lane`'s copy set at Rip, or null
  BreakpointHandler_t HandlerOf(uint32_t Lane, uint64_t Rip) const;

  // The instances whose copy is running Init on this thread (a backend's
  // SetBreakpoint routes the handler here), or null; RegisteringIndex() is
  // that copy. Copy 0's breakpoints also go through the backend's own path
  // (device breakpoint list, device actions); later copies must hook the same
  // rips.
  static ModuleInstances *Registering();
  int RegisteringIndex() const { return reg_; }
  void AddHandler(uint64_t Rip, BreakpointHandler_t Handler);

 private:
  std::vector<void *> handles_;  // dlopen handles (process lifetime, never closed)
  std::vector<Target_t> targets_;
  std::vector<std::unordered_map<uint64_t, BreakpointHandler_t>> handlers_;
  int reg_ = -1;
};

}  // namespace wtfgpu_host
