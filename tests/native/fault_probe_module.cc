// fault_probe_module.cc — TEST ONLY: a fuzzer module (loaded with
// --module-so, one copy per lane) whose handlers make the guest accesses a
// handler may fail, to pin U43: a failed translation under a Backend_t helper
// ends that testcase as an engine error on every backend (the reference node
// stops at the same access, backend.cc:39-42 / 101-104, backend.h:352-356),
// and the other testcases of the batch are unaffected.
//
// Target "fault_probe" on the tlv snapshot (rip = tlv_server!ProcessPacket):
// the first testcase byte picks what the ProcessPacket handler does.
//   0 Stop(Ok_t())                       3 VirtWriteDirty to GVA 0x10
//   1 VirtRead8(GVA 0)                   4 InsertTestcase writes GVA 0x10
//   2 VirtReadString running off the stack page into an unmapped one
//   5 SimulateReturnFromFunction(7) then Stop(Crash_t("probe-done")) at the
//     return address (the helper works on a translating address)
//   6 GetArg(4) (stack read) then Stop(Crash_t("probe-arg"))
#include "wtf_api.h"

namespace {
int Mode = 0;

void OnProcessPacket(Backend_t *B) {
  switch (Mode) {
    case 0: B->Stop(Ok_t()); return;
    case 1: (void)B->VirtRead8(Gva_t(0)); break;
    case 2: {
      // the stack's top page is followed by an unmapped one (tlv.py STACK_TOP)
      uint64_t Top = (B->Rsp() | 0xfff) + 1;
      while (true) {
        Gpa_t G;
        if (!B->VirtTranslate(Gva_t(Top), G, MemoryValidate_t::ValidateRead)) break;
        Top += 0x1000;
      }
      const uint8_t Fill[16] = {'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x', 'x'};
      B->VirtWriteDirty(Gva_t(Top - 16), Fill, sizeof(Fill));
      (void)B->VirtReadString(Gva_t(Top - 16), 64);
      break;
    }
    case 3: {
      const uint64_t V = 1;
      B->VirtWriteStructDirty(Gva_t(0x10), &V);
      break;
    }
    case 5: B->SimulateReturnFromFunction(7); return;
    case 6: (void)B->GetArg(4); B->Stop(Crash_t("probe-arg")); return;
    default: break;
  }
  B->Stop(Crash_t("probe-survived"));  // never reached in modes 1-3: the helper ends the handler
}

bool Init(const Options_t &, const CpuState_t &State) {
  const Gva_t Ret = Gva_t(g_Backend->VirtRead8(Gva_t(State.Rsp)));
  if (!g_Backend->SetBreakpoint("tlv_server!ProcessPacket", OnProcessPacket)) return false;
  return g_Backend->SetBreakpoint(Ret, [](Backend_t *B) { B->Stop(Crash_t("probe-done")); });
}

bool InsertTestcase(const uint8_t *Buffer, const size_t BufferSize) {
  Mode = BufferSize ? Buffer[0] : 0;
  if (Mode == 4) {
    const uint64_t V = 1;
    g_Backend->VirtWriteStructDirty(Gva_t(0x10), &V);
  }
  return true;
}

bool Restore() { return true; }

Target_t FaultProbe("fault_probe", Init, InsertTestcase, Restore);
}  // namespace
