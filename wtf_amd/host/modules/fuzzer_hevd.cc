// fuzzer_hevd.cc — the hevd fuzzer module (reference src/wtf/fuzzer_hevd.cc),
// written against wtf_api.h with the same handlers, symbols and result names:
//  * InsertTestcase (:20-59): u32 IOCTL code -> rdx, the rest (<= 1024 bytes)
//    -> the user buffer at r8, its size -> r9 and GetArgAddress(5) (also
//    declared as InsertAction_t, which the gpu backend applies on the device);
//  * the instruction after the 6-byte call to DeviceIoControl stops the
//    testcase with Ok (:64-73; also declared as BreakpointAction_t::StopOk);
//  * nt!DbgPrintEx is skipped (return 0) after reading its format (:78-88);
//  * nt!ExGenRandom: right after its `rdrand rdx` (+0xe0) rdx := Rdrand()
//    (:96-108, the BLAKE3 chain of Backend_t::Rdrand; also declared as data,
//    BreakpointAction_t::Rdrand, which the gpu backend runs on the device);
//  * nt!KeBugCheck2 -> Crash_t("crash-<code>-<p0>-<p1>-<p2>-<p3>-<p4>") (:114-128; also
//    declared as BreakpointAction_t::StopWithArgs, named from the device-kept arguments);
//  * nt!SwapContext -> Cr3Change_t (:134-139).
// The module keeps no per-testcase state, so nothing is registered with
// WTF_LANE_STATE.
#include <cstdio>
#include <string>

#include "../wtf_api.h"

namespace Hevd {

// fmt's {:#x}: "0x" + lowercase hex, "0x0" for zero
static void AppendHex(std::string &S, uint64_t V) {
  char B[18];
  int N = 0;
  do {
    B[N++] = "0123456789abcdef"[V & 15];
    V >>= 4;
  } while (V);
  S += "0x";
  while (N) S += B[--N];
}

// nt!KeBugCheck2(BCode, B0, B1, B2, B3, B4) -> the crash name (:114-128)
TestcaseResult_t BugCheckResult(const uint64_t *A) {
  std::string Name = "crash";
  Name.reserve(6 * 19 + 5);
  for (int i = 0; i < 6; i++) {
    Name += '-';
    AppendHex(Name, A[i]);
  }
  return Crash_t(std::move(Name));
}

bool InsertTestcase(const uint8_t *Buffer, const size_t BufferSize) {
  if (BufferSize < sizeof(uint32_t)) return true;
  uint32_t Ioctl;
  memcpy(&Ioctl, Buffer, sizeof(Ioctl));
  const size_t IoctlBufferSize = BufferSize - sizeof(uint32_t);
  const uint8_t *IoctlBuffer = Buffer + sizeof(uint32_t);
  if (IoctlBufferSize > 1024) return false;
  // the declared form below (Init): a backend that applies it on the device
  // takes the whole testcase
  if (g_Backend->SetInsert(Buffer, BufferSize)) return true;
  g_Backend->Rdx(Ioctl);
  const Gva_t IoctlBufferPtr = Gva_t(g_Backend->R8());
  if (!g_Backend->VirtWriteDirty(IoctlBufferPtr, IoctlBuffer, IoctlBufferSize)) return false;
  g_Backend->R9(IoctlBufferSize);
  const Gva_t OutBufferSizePtr = g_Backend->GetArgAddress(5);
  if (!g_Backend->VirtWriteStructDirty(OutBufferSizePtr, &IoctlBufferSize)) return false;
  return true;
}

// InsertTestcase ahead of time (PrepareInsert_t): its size checks, then the
// declared insert of the whole testcase
PreparedInsert_t PrepareInsert(const uint8_t *, const size_t BufferSize, std::vector<uint8_t> &) {
  if (BufferSize < sizeof(uint32_t)) return PreparedInsert_t::Nothing;
  if (BufferSize - sizeof(uint32_t) > 1024) return PreparedInsert_t::Failed;
  return PreparedInsert_t::Insert;
}

bool Init(const Options_t &, const CpuState_t &) {
  // InsertTestcase as data (device-side on the gpu backend)
  g_Backend->DeclareInsert(
      InsertAction_t::HeadAndPayload(Registers_t::Rdx, Registers_t::R8, Registers_t::R9, /*LenArg=*/5));
  const Gva_t Rip = Gva_t(g_Backend->Rip());
  const Gva_t AfterCall = Rip + Gva_t(6);
  if (!g_Backend->SetBreakpoint(
          AfterCall, [](Backend_t *Backend) { Backend->Stop(Ok_t()); },
          BreakpointAction_t::StopOk()))  // device-side on the gpu backend
    return false;
  if (!g_Backend->SetBreakpoint("nt!DbgPrintEx", [](Backend_t *Backend) {
        const Gva_t FormatPtr = Backend->GetArgGva(2);
        const std::string Format = Backend->VirtReadString(FormatPtr);
        (void)Format;
        Backend->SimulateReturnFromFunction(0);
      },
      BreakpointAction_t::SimulateReturn(0).AfterReadingString(Registers_t::R8)))  // device-side on the gpu backend
    return false;
  const Gva_t ExGenRandom = Gva_t(g_Dbg.GetSymbol("nt!ExGenRandom") + 0xe0 + 4);
  if (g_Backend->VirtRead4(ExGenRandom - Gva_t(4)) != 0xf2c70f48) {
    printf("It seems that nt!ExGenRandom's code has changed, update the offset!\n");
    return false;
  }
  if (!g_Backend->SetBreakpoint(
          ExGenRandom, [](Backend_t *Backend) { Backend->Rdx(Backend->Rdrand()); },
          BreakpointAction_t::Rdrand(Registers_t::Rdx)))  // device-side on the gpu backend
    return false;
  if (!g_Backend->SetBreakpoint("nt!KeBugCheck2", [](Backend_t *Backend) {
        const uint64_t A[6] = {Backend->GetArg(0), Backend->GetArg(1), Backend->GetArg(2),
                               Backend->GetArg(3), Backend->GetArg(4), Backend->GetArg(5)};
        Backend->Stop(BugCheckResult(A));
      },
      BreakpointAction_t::StopWithArgs(6, BugCheckResult)))  // device-side on the gpu backend
    return false;
  if (!g_Backend->SetBreakpoint("nt!SwapContext", [](Backend_t *Backend) { Backend->Stop(Cr3Change_t()); }))
    return false;
  return true;
}

Target_t Hevd("hevd", Init, InsertTestcase, []() { return true; }, LibfuzzerMutator_t::Create, PrepareInsert);

}  // namespace Hevd
