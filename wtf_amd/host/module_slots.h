// module_slots.h — per-lane state for fuzzer modules.
//
// wtf modules keep testcase state in globals (fuzzer_tlv_server.cc:42-65 holds
// the packet deque the ProcessPacket breakpoint consumes) and assume one
// testcase runs at a time. A batch runs N testcases at once, so each lane needs
// its own copy of that state while its handlers run.
//
// A module names its per-testcase global once, next to its definition:
//
//     struct { std::deque<Packet_t> Packets; CpuState_t Context; } GlobalState;
//     WTF_LANE_STATE(GlobalState);
//
// That one line is the only addition a module needs for batching; everything
// else (Init, InsertTestcase, Restore, the handlers) is unchanged. Upstream wtf
// defines the macro as nothing.
//
// A module whose per-testcase global is `thread_local` names it with
// WTF_LANE_STATE_TLS instead: the gpu backend then services breakpoint hits of
// different lanes on several host threads at once (each thread swaps the lane
// it services into its own instance of the global). g_Backend is thread_local
// in this build for the same reason; module code is unchanged by it.
//
// ModuleSlots keeps one typed copy of every registered object per lane. The
// lane's copy is swapped into the global (std::swap: container pointers are
// exchanged, no element copies) around every call into the module for that
// lane, and swapped back out afterwards. A lane's first swap-in starts from a
// deep copy of the state as Init left it. Raw byte copies of the module's data
// segment are NOT used: containers built during Init (a deque's first node)
// would then be shared between lanes and clobbered by the first insert.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <type_traits>
#include <utility>
#include <vector>

namespace wtfgpu_host {

class ModuleInstances;

// Type-erased operations over one registered global.
struct LaneStateOps {
  void *(*object)();                     // the calling thread's instance
  bool tls;                              // declared thread_local
  void *(*clone)(const void *);          // new T(copy)
  void (*assign)(void *, const void *);  // dst = src
  void (*swap)(void *, void *);
  void (*destroy)(void *);
};

// Registry of WTF_LANE_STATE objects (filled by static initialisers).
std::vector<LaneStateOps> &LaneStateRegistry();

template <typename T>
struct LaneStateRegistrar {
  LaneStateRegistrar(void *(*Object)(), bool Tls) {
    LaneStateRegistry().push_back(LaneStateOps{
        Object, Tls, [](const void *S) -> void * { return new T(*(const T *)S); },
        [](void *D, const void *S) { *(T *)D = *(const T *)S; },
        [](void *A, void *B) {
          using std::swap;
          swap(*(T *)A, *(T *)B);
        },
        [](void *P) { delete (T *)P; }});
  }
};

class ModuleSlots {
 public:
  ModuleSlots() = default;
  ~ModuleSlots();
  ModuleSlots(const ModuleSlots &) = delete;
  ModuleSlots &operator=(const ModuleSlots &) = delete;

  // The current module state becomes every lane's initial state (call after Init).
  void Capture(uint32_t lanes);
  // Every lane's copy back to the captured state (start of a batch).
  void ResetAll();
  // ResetAll for one lane (lanes are independent: callers may reset
  // different lanes on different threads)
  void ResetLane(uint32_t lane);
  void SwapIn(uint32_t lane);
  void SwapOut(uint32_t lane);
  size_t Objects() const { return initial_.size(); }
  // every registered object is thread_local (or every lane runs its own copy
  // of the module, module_instances.h): lanes may be serviced in parallel
  bool ThreadSafe() const;
  // per-lane module copies: lane l runs copy l's Target_t and handlers
  void AttachInstances(ModuleInstances *I) { inst_ = I; }
  ModuleInstances *Instances() const { return inst_; }

 private:
  void release();
  std::vector<void *> initial_;             // per registered object
  std::vector<void *> lanes_;  // [lane * objects + object], nullptr = not materialised
  std::vector<uint8_t> dirty_;              // lane copy differs from initial
  ModuleInstances *inst_ = nullptr;
};

}  // namespace wtfgpu_host

#define WTF_LANE_STATE_CAT2(a, b) a##b
#define WTF_LANE_STATE_CAT(a, b) WTF_LANE_STATE_CAT2(a, b)
#define WTF_LANE_STATE_REG(Object, Tls)                                                          \
  static ::wtfgpu_host::LaneStateRegistrar<std::remove_reference_t<decltype(Object)>> WTF_LANE_STATE_CAT( \
      LaneStateReg_, __LINE__)([]() -> void * { return &Object; }, Tls)
#define WTF_LANE_STATE(Object) WTF_LANE_STATE_REG(Object, false)
#define WTF_LANE_STATE_TLS(Object) WTF_LANE_STATE_REG(Object, true)
