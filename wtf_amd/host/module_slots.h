// module_slots.h — per-lane state for unchanged fuzzer modules.
//
// wtf modules keep testcase state in globals (fuzzer_tlv_server.cc:42-65 holds
// the packet deque the ProcessPacket breakpoint consumes) and assume one
// testcase runs at a time. A batch runs N testcases at once, so each lane needs
// its own copy of that state. A module is built as its own shared object; its
// writable data (the RW PT_LOAD segments minus the RELRO part: .data, .bss) is
// the module state. ModuleSlots keeps one copy of those bytes per lane and swaps
// the lane's copy in around every call into the module for that lane (Insert,
// breakpoint handlers, Restore). Heap objects the state points to belong to that
// lane's copy (the module allocates and frees them through its own globals), so
// they need no copying.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace wtfgpu_host {

class ModuleSlots {
 public:
  // Loads the module (dlopen). Its static Target_t registers itself.
  bool Load(const std::string &so_path);
  // The current module state becomes every lane's initial state (call after Init).
  void Capture(uint32_t lanes);
  void SwapIn(uint32_t lane);
  void SwapOut(uint32_t lane);
  size_t StateBytes() const;
  void *Handle() const { return handle_; }

 private:
  struct Segment {
    uint8_t *addr;
    size_t size;
  };
  void *handle_ = nullptr;
  std::vector<Segment> segs_;
  std::vector<uint8_t> initial_;
  std::vector<std::vector<uint8_t>> slots_;  // lazily materialised from initial_
  std::vector<uint8_t> touched_;
  int32_t in_ = -1;
};

}  // namespace wtfgpu_host
