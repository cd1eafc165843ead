// wtf_api.cc — the backend-independent half of the wtf host interface:
// Backend_t helpers, target registry, symbol store, regs.json loading.
// Semantics follow the reference functions cited per definition.
#include "wtf_api.h"

#include <cstdio>
#include <fstream>
#include <sstream>

#include "blake3_lite.h"
#include "json_lite.h"

thread_local Backend_t *g_Backend = nullptr;
Debugger_t g_Dbg;

// backend.cc:11-14
bool Backend_t::SetTraceFile(const fs::path &, const TraceType_t) {
  printf("SetTraceFile not implemented.\n");
  return true;
}

// backend.cc:16-28
bool Backend_t::PhysWrite(const Gpa_t Gpa, const uint8_t *Buffer, const uint64_t BufferSize, const bool Dirty) {
  if (PhysWriteDirect(Gpa, Buffer, BufferSize)) return true;  // the backend dirties what it writes
  uint8_t *Dst = PhysTranslate(Gpa);
  if (!Dst) return false;
  memcpy(Dst, Buffer, BufferSize);
  if (Dirty) {
    for (uint64_t Cur = Gpa.U64(); Cur < Gpa.U64() + BufferSize; Cur += Page::Size) DirtyGpa(Gpa_t(Cur));
  }
  return true;
}

// A failed translation under a helper: the reference's __debugbreak
// (backend.cc:39-42), here the end of the calling handler (HandlerFault_t).
[[noreturn]] static void handler_fault(const uint64_t Gva) {
  printf("Translation of GVA %#llx failed\n", (unsigned long long)Gva);
  throw HandlerFault_t{Gva};
}

// backend.cc:30-56: page-chunked translate + copy; a failed translation ends
// the handler (HandlerFault_t), it never returns false
bool Backend_t::VirtRead(const Gva_t Gva, uint8_t *Buffer, const uint64_t BufferSize) const {
  uint64_t Left = BufferSize, Cur = Gva.U64();
  while (Left) {
    Gpa_t Gpa;
    if (!VirtTranslate(Gva_t(Cur), Gpa, MemoryValidate_t::ValidateRead)) handler_fault(Cur);
    const uint64_t Chunk = std::min<uint64_t>(Left, Page::Size - (Cur & 0xfff));
    if (!PhysReadDirect(Gpa, Buffer, Chunk)) {
      const uint8_t *Hva = PhysTranslate(Gpa);
      if (!Hva) return false;
      memcpy(Buffer, Hva, Chunk);
    }
    Buffer += Chunk;
    Cur += Chunk;
    Left -= Chunk;
  }
  return true;
}

uint32_t Backend_t::VirtRead4(const Gva_t Gva) const {
  uint32_t V = 0;
  VirtReadStruct(Gva, &V);
  return V;
}
uint64_t Backend_t::VirtRead8(const Gva_t Gva) const {
  uint64_t V = 0;
  VirtReadStruct(Gva, &V);
  return V;
}
Gva_t Backend_t::VirtReadGva(const Gva_t Gva) const { return Gva_t(VirtRead8(Gva)); }
Gpa_t Backend_t::VirtReadGpa(const Gva_t Gva) const { return Gpa_t(VirtRead8(Gva)); }

// backend.h:333-430: read up to MaxLength bytes, stop at the terminator; a
// page the string reaches that does not translate ends the handler
// (:352-356, HandlerFault_t)
template <typename Ch>
static std::basic_string<Ch> read_cstring(const Backend_t *B, const Gva_t Gva, const uint64_t MaxLength) {
  std::basic_string<Ch> S;
  uint64_t Cur = Gva.U64();
  for (uint64_t i = 0; i + sizeof(Ch) <= MaxLength; i += sizeof(Ch), Cur += sizeof(Ch)) {
    Ch C = 0;
    if (!B->VirtRead(Gva_t(Cur), (uint8_t *)&C, sizeof(Ch))) break;  // PhysTranslate failed (no frame)
    if (C == 0) break;
    S.push_back(C);
  }
  return S;
}
std::string Backend_t::VirtReadString(const Gva_t Gva, const uint64_t MaxLength) const {
  return read_cstring<char>(this, Gva, MaxLength);
}
std::u16string Backend_t::VirtReadWideString(const Gva_t Gva, const uint64_t MaxLength) const {
  return read_cstring<char16_t>(this, Gva, MaxLength);
}

// backend.cc:91-122
bool Backend_t::VirtWrite(const Gva_t Gva, const uint8_t *Buffer, const uint64_t BufferSize, const bool Dirty) {
  uint64_t Left = BufferSize, Cur = Gva.U64();
  while (Left) {
    Gpa_t Gpa;
    if (!VirtTranslate(Gva_t(Cur), Gpa, MemoryValidate_t::ValidateRead)) handler_fault(Cur);
    const uint64_t Chunk = std::min<uint64_t>(Left, Page::Size - (Cur & 0xfff));
    if (!PhysWrite(Gpa, Buffer, Chunk, Dirty)) return false;
    Buffer += Chunk;
    Cur += Chunk;
    Left -= Chunk;
  }
  return true;
}
bool Backend_t::VirtWriteDirty(const Gva_t Gva, const uint8_t *Buffer, const uint64_t BufferSize) {
  return VirtWrite(Gva, Buffer, BufferSize, true);
}

// backend.cc:129-166
bool Backend_t::SimulateReturnFromFunction(const uint64_t Return) {
  Rax(Return);
  const uint64_t Stack = Rsp();
  const uint64_t Saved = VirtRead8(Gva_t(Stack));
  Rsp(Stack + 8);
  Rip(Saved);
  return true;
}
bool Backend_t::SimulateReturnFrom32bitFunction(const uint32_t Return, const uint32_t StdcallArgsCount) {
  Rax(Return);
  const uint64_t Stack = Rsp();
  const uint32_t Saved = VirtRead4(Gva_t(Stack));
  Rsp(Stack + 4 + 4 * uint64_t(StdcallArgsCount));
  Rip(Saved);
  return true;
}

// backend.cc:168-202: Win64 calling convention
Gva_t Backend_t::GetArgAddress(const uint64_t Idx) {
  if (Idx <= 3) {
    printf("The first four arguments are stored in registers (@rcx, @rdx, @r8, @r9) which means you cannot get "
           "their addresses.\n");
    std::abort();
  }
  return Gva_t(Rsp() + 8 + Idx * 8);
}
uint64_t Backend_t::GetArg(const uint64_t Idx) {
  switch (Idx) {
    case 0: return Rcx();
    case 1: return Rdx();
    case 2: return R8();
    case 3: return R9();
    default: return VirtRead8(GetArgAddress(Idx));
  }
}
Gva_t Backend_t::GetArgGva(const uint64_t Idx) { return Gva_t(GetArg(Idx)); }
std::pair<uint64_t, Gva_t> Backend_t::GetArgAndAddress(const uint64_t Idx) { return {GetArg(Idx), GetArgAddress(Idx)}; }
std::pair<Gva_t, Gva_t> Backend_t::GetArgAndAddressGva(const uint64_t Idx) {
  return {GetArgGva(Idx), GetArgAddress(Idx)};
}

// backend.cc:204-212: crash-<EXCEPTION_NAME>-<address>
bool Backend_t::SaveCrash(const Gva_t ExceptionAddress, const uint32_t ExceptionCode) {
  char Name[160];
  snprintf(Name, sizeof(Name), "crash-%s-%#llx", std::string(ExceptionCodeToStr(ExceptionCode)).c_str(),
           (unsigned long long)ExceptionAddress.U64());
  Stop(Crash_t(Name));
  return true;
}

// backend.cc:214-239
bool Backend_t::SetBreakpoint(const char *Symbol, const BreakpointHandler_t Handler) {
  const Gva_t Gva = Gva_t(g_Dbg.GetSymbol(Symbol));
  if (Gva == Gva_t(0)) {
    printf("Could not set a breakpoint at %s.\n", Symbol);
    return false;
  }
  return SetBreakpoint(Gva, Handler);
}
bool Backend_t::SetBreakpoint(const char *Symbol, const BreakpointHandler_t Handler,
                              const BreakpointAction_t &Action) {
  const Gva_t Gva = Gva_t(g_Dbg.GetSymbol(Symbol));
  if (Gva == Gva_t(0)) {
    printf("Could not set a breakpoint at %s.\n", Symbol);
    return false;
  }
  return SetBreakpoint(Gva, Handler, Action);
}
BreakpointAction_t BreakpointAction_t::SetGprs(const CpuState_t &C) {
  BreakpointAction_t A;
  A.Kind = Kind_t::SetGprs;
  const uint64_t G[17] = {C.Rax, C.Rcx, C.Rdx, C.Rbx, C.Rsp, C.Rbp, C.Rsi, C.Rdi, C.R8,
                          C.R9,  C.R10, C.R11, C.R12, C.R13, C.R14, C.R15, C.Rip};
  for (int i = 0; i < 17; i++) A.Gprs[i] = G[i];
  return A;
}
bool Backend_t::SetCrashBreakpoint(const Gva_t Gva) {
  return SetBreakpoint(Gva, [](Backend_t *B) { B->Stop(Crash_t()); });
}
bool Backend_t::SetCrashBreakpoint(const char *Symbol) {
  return SetBreakpoint(Symbol, [](Backend_t *B) { B->Stop(Crash_t()); });
}

void Backend_t::PrintRegisters() {
  printf("rax=%016llx rbx=%016llx rcx=%016llx\n", (unsigned long long)Rax(), (unsigned long long)Rbx(),
         (unsigned long long)Rcx());
  printf("rdx=%016llx rsi=%016llx rdi=%016llx\n", (unsigned long long)Rdx(), (unsigned long long)Rsi(),
         (unsigned long long)Rdi());
  printf("rip=%016llx rsp=%016llx rbp=%016llx\n", (unsigned long long)Rip(), (unsigned long long)Rsp(),
         (unsigned long long)Rbp());
}

// ------------------------------------------------------------------ targets (targets.cc:11-38)
Target_t::Target_t(const std::string &Name_, const Init_t Init_, const InsertTestcase_t InsertTestcase_,
                   const Restore_t Restore_, const CreateMutator_t CreateMutator_,
                   const PrepareInsert_t PrepareInsert_)
    : Name(Name_), Init(Init_), InsertTestcase(InsertTestcase_), Restore(Restore_), CreateMutator(CreateMutator_),
      PrepareInsert(PrepareInsert_) {
  Targets_t::Instance().Registers(*this);
}
Targets_t &Targets_t::Instance() {
  static Targets_t T;
  return T;
}
void Targets_t::Registers(const Target_t &Target) { Targets.emplace_back(Target); }
Target_t *Targets_t::Get(const std::string &Name) {
  for (auto &T : Targets)
    if (T.Name == Name) return &T;
  return nullptr;
}
void Targets_t::DisplayRegisteredTargets() {
  printf("Existing targets:\n");
  for (const auto &T : Targets) printf("  - Name: %s\n", T.Name.c_str());
}

// ------------------------------------------------------------------ symbol store (debugger.h:346-388)
static std::string slurp(const fs::path &P) {
  std::ifstream F(P, std::ios::binary);
  std::stringstream S;
  S << F.rdbuf();
  return S.str();
}

bool Debugger_t::Init(const fs::path &, const fs::path &SymbolFilePath) {
  const jsonl::Value J = jsonl::parse(slurp(SymbolFilePath));
  for (const auto &[K, V] : J.obj) Symbols_[K] = V.u64();
  return true;
}
bool Debugger_t::AddSymbol(const std::string &Name, const uint64_t Address) {
  Symbols_[Name] = Address;
  return true;
}
uint64_t Debugger_t::GetSymbol(const char *Name) const {
  auto It = Symbols_.find(Name);
  if (It == Symbols_.end()) {
    printf("%s could not be found in the symbol store\n", Name);
    exit(0);
  }
  return It->second;
}

// ------------------------------------------------------------------ utils (utils.cc:57-258, 417-472)
std::string_view ExceptionCodeToStr(const uint32_t Code) {
  switch (Code) {
    case EXCEPTION_ACCESS_VIOLATION: return "EXCEPTION_ACCESS_VIOLATION";
    case EXCEPTION_BREAKPOINT: return "EXCEPTION_BREAKPOINT";
    case EXCEPTION_ILLEGAL_INSTRUCTION: return "EXCEPTION_ILLEGAL_INSTRUCTION";
    case EXCEPTION_INT_DIVIDE_BY_ZERO: return "EXCEPTION_INT_DIVIDE_BY_ZERO";
    case EXCEPTION_PRIV_INSTRUCTION: return "EXCEPTION_PRIV_INSTRUCTION";
    case STATUS_STACK_BUFFER_OVERRUN: return "EXCEPTION_STACK_BUFFER_OVERRUN";
    case STATUS_HEAP_CORRUPTION: return "STATUS_HEAP_CORRUPTION";
    case EXCEPTION_ACCESS_VIOLATION_READ: return "EXCEPTION_ACCESS_VIOLATION_READ";
    case EXCEPTION_ACCESS_VIOLATION_WRITE: return "EXCEPTION_ACCESS_VIOLATION_WRITE";
    case EXCEPTION_ACCESS_VIOLATION_EXECUTE: return "EXCEPTION_ACCESS_VIOLATION_EXECUTE";
    default: return "UNKNOWN";
  }
}

bool LoadCpuStateFromJSON(CpuState_t &S, const fs::path &Path) {
  const jsonl::Value J = jsonl::parse(slurp(Path));
  S = CpuState_t{};
  auto R = [&](const char *K) { return J.at(K).u64(); };
  S.Rax = R("rax"), S.Rbx = R("rbx"), S.Rcx = R("rcx"), S.Rdx = R("rdx"), S.Rsi = R("rsi"), S.Rdi = R("rdi");
  S.Rip = R("rip"), S.Rsp = R("rsp"), S.Rbp = R("rbp");
  S.R8 = R("r8"), S.R9 = R("r9"), S.R10 = R("r10"), S.R11 = R("r11"), S.R12 = R("r12"), S.R13 = R("r13");
  S.R14 = R("r14"), S.R15 = R("r15"), S.Rflags = R("rflags");
  S.Tsc = R("tsc"), S.ApicBase = R("apic_base"), S.SysenterCs = R("sysenter_cs"), S.SysenterEsp = R("sysenter_esp");
  S.SysenterEip = R("sysenter_eip"), S.Pat = R("pat"), S.Efer.Flags = R("efer"), S.Star = R("star");
  S.Lstar = R("lstar"), S.Cstar = R("cstar"), S.Sfmask = R("sfmask"), S.KernelGsBase = R("kernel_gs_base");
  S.TscAux = R("tsc_aux"), S.Fpcw = (uint16_t)R("fpcw"), S.Fpsw = (uint16_t)R("fpsw"), S.Fptw = (uint16_t)R("fptw");
  S.Cr0.Flags = R("cr0"), S.Cr2 = R("cr2"), S.Cr3 = R("cr3"), S.Cr4.Flags = R("cr4"), S.Cr8 = R("cr8");
  S.Xcr0 = (uint32_t)R("xcr0"), S.Dr0 = R("dr0"), S.Dr1 = R("dr1"), S.Dr2 = R("dr2"), S.Dr3 = R("dr3");
  S.Dr6 = (uint32_t)R("dr6"), S.Dr7 = (uint32_t)R("dr7"), S.Mxcsr = (uint32_t)R("mxcsr");
  S.MxcsrMask = (uint32_t)R("mxcsr_mask"), S.Fpop = (uint16_t)R("fpop");
  auto Seg = [&](const char *K, Seg_t &D) {
    const jsonl::Value &V = J.at(K);
    D.Present = V.at("present").b;
    D.Selector = (uint16_t)V.at("selector").u64();
    D.Base = V.at("base").u64();
    D.Limit = (uint32_t)V.at("limit").u64();
    D.Attr = (uint16_t)V.at("attr").u64();
    // the reference's Present is bit 7 of the Attr union (globals.h:33-51), so
    // the attr write overrides the JSON "present" flag (utils.cc:116-129)
    D.Present = (D.Attr >> 7) & 1;
  };
  Seg("es", S.Es), Seg("cs", S.Cs), Seg("ss", S.Ss), Seg("ds", S.Ds), Seg("fs", S.Fs), Seg("gs", S.Gs);
  Seg("tr", S.Tr), Seg("ldtr", S.Ldtr);
  S.Gdtr.Base = J.at("gdtr").at("base").u64(), S.Gdtr.Limit = (uint16_t)J.at("gdtr").at("limit").u64();
  S.Idtr.Base = J.at("idtr").at("base").u64(), S.Idtr.Limit = (uint16_t)J.at("idtr").at("limit").u64();
  // an empty-looking x87 stack is forced empty (utils.cc:170-190)
  bool AllInfinity = true;
  const jsonl::Value &Fpst = J.at("fpst");
  for (size_t i = 0; i < 8 && i < Fpst.arr.size(); i++) {
    const std::string &V = Fpst.arr[i].str;
    const bool Inf = V.find("Infinity") != std::string::npos;
    AllInfinity = AllInfinity && Inf;
    S.Fpst[i] = Inf ? 0 : std::strtoull(V.c_str(), nullptr, 0);
  }
  if (S.Fptw == 0 && AllInfinity) S.Fptw = 0xffff;
  return true;
}

bool SanitizeCpuState(CpuState_t &S) {
  if (S.Rip < 0x7fffffff0000ull && S.Cr8 != 0) S.Cr8 = 0;
  S.Dr0 = S.Dr1 = S.Dr2 = S.Dr3 = 0;
  S.Dr6 = S.Dr7 = 0;
  for (const Seg_t *G : {&S.Es, &S.Fs, &S.Cs, &S.Gs, &S.Ss, &S.Ds}) {
    if (G->Reserved() != ((G->Limit >> 16) & 0xf)) {
      printf("Segment with selector %x has invalid attributes.\n", G->Selector);
      return false;
    }
  }
  if (S.MxcsrMask == 0) S.MxcsrMask = 0xffbf;
  return true;
}

// ------------------------------------------------------------------ corpus / files
std::string TestcaseResultName(const TestcaseResult_t &Res) {
  return std::string(std::visit([](const auto &R) { return std::string_view(R.Name()); }, Res));
}

// utils.cc:279-300: 16-byte BLAKE3 digest as hex, low nibble first per byte
// (the reference's order, so saved file names match)
std::string Blake3HexDigest(const uint8_t *Data, const size_t DataSize) {
  uint8_t H[16];
  wtfgpu_host::blake3_hash(Data, DataSize, H, sizeof(H));
  static const char *Hex = "0123456789abcdef";
  std::string S;
  for (uint8_t B : H) {
    S.push_back(Hex[B & 15]);
    S.push_back(Hex[B >> 4]);
  }
  return S;
}

bool SaveFile(const fs::path &Path, const uint8_t *Buffer, const size_t BufferSize) {
  std::ofstream F(Path, std::ios::binary);
  if (!F) return false;
  F.write((const char *)Buffer, BufferSize);
  return bool(F);
}

std::vector<uint8_t> ReadFile(const fs::path &Path) {
  std::ifstream F(Path, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(F)), std::istreambuf_iterator<char>());
}

// corpus.h:56-86
bool Corpus_t::SaveTestcase(const TestcaseResult_t &Result, Testcase_t Testcase) {
  const std::string Hash = Blake3HexDigest(Testcase.Buffer_.get(), Testcase.BufferSize_);
  std::string Name = Hash;
  if (!std::holds_alternative<Ok_t>(Result)) Name = TestcaseResultName(Result) + "-" + Hash;
  if (!OutputsPath_.empty()) {
    const fs::path Out = OutputsPath_ / Name;
    if (!fs::exists(Out) && !SaveFile(Out, Testcase.Buffer_.get(), Testcase.BufferSize_)) {
      printf("Could not create the destination file.\n");
      return false;
    }
  }
  Bytes_ += Testcase.BufferSize_;
  Testcases_.emplace_back(std::move(Testcase));
  return true;
}
