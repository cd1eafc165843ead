// crash_detection_umode.cc — the user-mode crash detection hooks every
// user-mode module installs (crash_detection_umode.cc:20-167): a perf
// interrupt ends the testcase as a timeout, a bugcheck is a crash, a context
// switch is a cr3 change, an exception dispatched to user mode is a crash
// named after its code and address, a fast-fail is a stack-buffer-overrun
// crash, an application-verifier stop is a heap-corruption crash.
#include "crash_detection_umode.h"

#include <cstdio>
#include <cstdlib>

#include "../wtf_api.h"

namespace {
constexpr uint32_t kCppException = 0xE06D7363;
constexpr uint32_t kDbgPrintException = 0x40010006;
constexpr uint32_t kDbgPrintExceptionWide = 0x4001000A;

// EXCEPTION_RECORD64 (nt.h)
struct ExceptionRecord_t {
  uint32_t ExceptionCode;
  uint32_t ExceptionFlags;
  uint64_t ExceptionRecord;
  uint64_t ExceptionAddress;
  uint32_t NumberParameters;
  uint32_t Pad;
  uint64_t ExceptionInformation[15];
};
}  // namespace

bool SetupUsermodeCrashDetectionHooks() {
  if (!g_Backend->SetBreakpoint("hal!HalpPerfInterrupt", [](Backend_t *B) { B->Stop(Timedout_t()); }))
    printf("Failed to set breakpoint on HalpPerfInterrupt, but ignoring..\n");

  if (!g_Backend->SetCrashBreakpoint("nt!KeBugCheck2")) {
    printf("Failed to SetBreakpoint on KeBugCheck2\n");
    return false;
  }

  if (!g_Backend->SetBreakpoint("nt!SwapContext", [](Backend_t *B) { B->Stop(Cr3Change_t()); })) {
    printf("Failed to SetBreakpoint on SwapContext\n");
    return false;
  }

  // RtlDispatchException(PEXCEPTION_RECORD, PCONTEXT)
  if (!g_Backend->SetBreakpoint("ntdll!RtlDispatchException", [](Backend_t *B) {
        ExceptionRecord_t R{};
        if (!B->VirtReadStruct(B->GetArgGva(0), &R)) std::abort();
        if (R.ExceptionCode == kCppException || R.ExceptionCode == kDbgPrintException ||
            R.ExceptionCode == kDbgPrintExceptionWide)
          return;  // C++ throws and DbgPrint are not crashes
        uint32_t Code = R.ExceptionCode;
        if (Code == EXCEPTION_ACCESS_VIOLATION && R.NumberParameters > 1) {
          switch (R.ExceptionInformation[0]) {  // 0 read, 1 write, 8 DEP
            case 0: Code = EXCEPTION_ACCESS_VIOLATION_READ; break;
            case 1: Code = EXCEPTION_ACCESS_VIOLATION_WRITE; break;
            case 8: Code = EXCEPTION_ACCESS_VIOLATION_EXECUTE; break;
            default: break;
          }
        }
        B->SaveCrash(Gva_t(R.ExceptionAddress), Code);
      })) {
    printf("Failed to SetBreakpoint on RtlDispatchException\n");
    return false;
  }

  // int 0x29 (__fastfail) lands here with the faulting address at [rsp]
  if (!g_Backend->SetBreakpoint("nt!KiRaiseSecurityCheckFailure", [](Backend_t *B) {
        B->SaveCrash(B->VirtReadGva(Gva_t(B->Rsp())), STATUS_STACK_BUFFER_OVERRUN);
      })) {
    printf("Failed to SetBreakpoint on KiRaiseSecurityCheckFailure\n");
    return false;
  }

  if (g_Dbg.GetModuleBase("verifier") > 0) {
    if (!g_Backend->SetBreakpoint("verifier!VerifierStopMessage", [](Backend_t *B) {
          B->SaveCrash(Gva_t(B->Rsp()), STATUS_HEAP_CORRUPTION);
        })) {
      printf("Failed to SetBreakpoint on VerifierStopMessage\n");
      return false;
    }
  }
  return true;
}
