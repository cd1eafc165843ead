// wtf_api.h — the wtf host interface the gpu backend and fuzzer modules are
// written against, restated for building this repository on its own.
//
// The names, member signatures and semantics follow the reference so that a
// module source written for wtf compiles unchanged against this header and a
// maintainer can drop `gpu_backend.{h,cc}` into upstream wtf next to
// `bochscpu_backend`:
//   Gva_t / Gpa_t               src/wtf/gxa.h:10-53
//   TestcaseResult_t            src/wtf/backend.h:12-31
//   Registers_t, MemoryValidate_t, BreakpointHandler_t   backend.h:110-154
//   Backend_t                   backend.h:161-602, helpers backend.cc:16-332
//   CpuState_t, Options_t       src/wtf/globals.h:1020-1385 (fields this path uses)
//   Target_t / Targets_t        src/wtf/targets.h:14-48, targets.cc:11-38
//   Debugger_t (Linux)          src/wtf/debugger.h:346-388 (symbol-store.json)
// Coverage sets use std::unordered_set where the reference uses tsl::robin_set
// (same interface for the members modules call).
#pragma once
#include <cstdint>
#include <cstring>
#include <filesystem>
#include <functional>
#include <memory>
#include <optional>
#include <random>
#include <span>
#include <string>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <variant>
#include <vector>

#include "module_slots.h"

namespace fs = std::filesystem;

namespace Page {
constexpr uint64_t Size = 0x1000;
}

// ------------------------------------------------------------------ addresses
template <typename Tag>
class Address_t {
  uint64_t v_ = 0;

 public:
  Address_t() = default;
  explicit Address_t(const uint64_t V) : v_(V) {}
  uint64_t U64() const { return v_; }
  Address_t Offset() const { return Address_t(v_ & 0xfff); }
  Address_t Align() const { return Address_t(v_ & ~0xfffull); }
  explicit operator bool() const { return v_ != 0; }
  bool operator==(const Address_t &O) const { return v_ == O.v_; }
  bool operator!=(const Address_t &O) const { return v_ != O.v_; }
  bool operator<(const Address_t &O) const { return v_ < O.v_; }
  Address_t operator+(const Address_t &O) const { return Address_t(v_ + O.v_); }
  Address_t operator-(const Address_t &O) const { return Address_t(v_ - O.v_); }
  Address_t operator*(const Address_t &O) const { return Address_t(v_ * O.v_); }
  Address_t &operator+=(const Address_t &O) {
    v_ += O.v_;
    return *this;
  }
  uint64_t *operator&() { return &v_; }
};
using Gva_t = Address_t<struct GvaTag_t>;
using Gpa_t = Address_t<struct GpaTag_t>;

template <typename Tag>
struct std::hash<Address_t<Tag>> {
  size_t operator()(const Address_t<Tag> &A) const noexcept { return std::hash<uint64_t>()(A.U64()); }
};

// ------------------------------------------------------------------ results
struct Ok_t {
  constexpr std::string_view Name() const { return "ok"; }
};
struct Timedout_t {
  constexpr std::string_view Name() const { return "timedout"; }
};
struct Cr3Change_t {
  constexpr std::string_view Name() const { return "cr3"; }
};
struct Crash_t {
  std::string CrashName;
  Crash_t() = default;
  explicit Crash_t(const std::string &Name) : CrashName(Name) {}
  std::string_view Name() const { return "crash"; }
};
using TestcaseResult_t = std::variant<Ok_t, Timedout_t, Cr3Change_t, Crash_t>;

enum PfError_t {
  ErrorPresent = 1 << 0,
  ErrorWrite = 1 << 1,
  ErrorUser = 1 << 2,
  ErrorReservedWrite = 1 << 3,
  ErrorInstructionFetch = 1 << 4
};

enum class MemoryValidate_t : uint32_t {
  ValidateRead = 1,
  ValidateWrite = 2,
  ValidateExecute = 4,
  ValidateReadWrite = 3,
  ValidateReadExecute = 5
};
inline bool operator&(const MemoryValidate_t &A, const MemoryValidate_t &B) {
  return (uint32_t(A) & uint32_t(B)) != 0;
}

// Order as in the reference (backend.h:133-154).
enum class Registers_t : uint32_t {
  Rax, Rbx, Rcx, Rdx, Rsi, Rdi, Rip, Rsp, Rbp,
  R8, R9, R10, R11, R12, R13, R14, R15, Rflags, Cr2, Cr3
};

enum class TraceType_t { NoTrace, Rip, UniqueRip, Tenet };
enum class BackendType_t { Bochscpu, Whv, Kvm, Gpu };

// ------------------------------------------------------------------ cpu state
struct Seg_t {
  bool Present = false;
  uint16_t Selector = 0;
  uint64_t Base = 0;
  uint32_t Limit = 0;
  uint16_t Attr = 0;
  // bits 8-11 of Attr mirror Limit bits 16-19 (utils.cc:234-243)
  uint16_t Reserved() const { return (Attr >> 8) & 0xf; }
  bool operator==(const Seg_t &) const = default;
};
struct GlobalSeg_t {
  uint64_t Base = 0;
  uint16_t Limit = 0;
  bool operator==(const GlobalSeg_t &) const = default;
};
struct FlagsReg_t {  // Cr0_t / Cr4_t / Efer_t expose .Flags (globals.h)
  uint64_t Flags = 0;
  bool operator==(const FlagsReg_t &) const = default;
};
struct Zmm_t {
  uint64_t Q[8] = {};
  bool operator==(const Zmm_t &) const = default;
};

struct CpuState_t {
  uint64_t Seed = 0;
  uint64_t Rax = 0, Rcx = 0, Rdx = 0, Rbx = 0, Rsp = 0, Rbp = 0, Rsi = 0, Rdi = 0;
  uint64_t R8 = 0, R9 = 0, R10 = 0, R11 = 0, R12 = 0, R13 = 0, R14 = 0, R15 = 0;
  uint64_t Rip = 0, Rflags = 0;
  Seg_t Es, Cs, Ss, Ds, Fs, Gs, Ldtr, Tr;
  GlobalSeg_t Gdtr, Idtr;
  FlagsReg_t Cr0;
  uint64_t Cr2 = 0, Cr3 = 0;
  FlagsReg_t Cr4;
  uint64_t Cr8 = 0;
  uint64_t Dr0 = 0, Dr1 = 0, Dr2 = 0, Dr3 = 0;
  uint32_t Dr6 = 0, Dr7 = 0;
  uint32_t Xcr0 = 0;
  Zmm_t Zmm[32];
  uint16_t Fpcw = 0, Fpsw = 0, Fptw = 0, Fpop = 0;
  uint64_t Fpst[8] = {};
  uint32_t Mxcsr = 0, MxcsrMask = 0;
  uint64_t Tsc = 0;
  FlagsReg_t Efer;
  uint64_t KernelGsBase = 0, ApicBase = 0, Pat = 0;
  uint64_t SysenterCs = 0, SysenterEip = 0, SysenterEsp = 0;
  uint64_t Star = 0, Lstar = 0, Cstar = 0, Sfmask = 0, TscAux = 0;
  bool operator==(const CpuState_t &) const = default;
};

struct RunOptions_t {
  fs::path BaseTracePath;
  TraceType_t TraceType = TraceType_t::NoTrace;
  fs::path InputPath;
  uint64_t Runs = 0;
};
struct FuzzOptions_t {
  fs::path TargetPath;
  uint32_t Seed = 0;
  std::string Address;
};

struct Options_t {
  bool Verbose = false;
  BackendType_t Backend = BackendType_t::Gpu;
  std::string TargetName;
  fs::path StatePath, DumpPath, CpuStatePath, SymbolFilePath, GuestFilesPath, CoveragePath;
  uint64_t Limit = 0;
  CpuState_t CpuState;
  bool Edges = false;
  RunOptions_t Run;
  FuzzOptions_t Fuzz;
  // gpu backend knobs (new): device, lanes per batch, copy-on-write pages per lane
  int GpuDevice = 0;
  uint32_t GpuLanes = 1;
  uint32_t GpuOverlayPages = 32;
  // per-lane new-coverage set entries (wtfgpu_alloc_lanes; 3/4 usable): a
  // testcase's rips not yet in the aggregate; --full-coverage (parity mode,
  // every rip of the testcase) takes the larger set
  uint32_t GpuCoverageSet = 2048;
};

// ------------------------------------------------------------------ backend
class Backend_t;
using BreakpointHandler_t = void (*)(Backend_t *);

// A guest access of a handler (VirtRead / VirtWrite / the string readers) whose
// translation failed. The reference stops the whole node there: it prints the
// GVA and executes `int3` (__debugbreak, platform.h:35; backend.cc:39-42,
// 58-72, 101-104; backend.h:352-356). Here the helper throws this instead, and
// the backend that called the handler (or InsertTestcase) catches it: the
// handler is abandoned at that access, exactly where the reference stops, and
// only that testcase ends, as an engine error (DESIGN U43; a batched node must
// not lose its other lanes to one testcase).
struct HandlerFault_t {
  uint64_t Gva;
};

// What a breakpoint handler does, stated as data (this repository's
// extension; the reference only has the handler). A backend that can apply it
// without leaving the execution engine (the gpu backend does it on the device,
// wtfgpu_set_breakpoint_actions) may do so instead of calling the handler; any
// other backend calls the handler. The module guarantees the two are the same
// register effect; the GPU-vs-twin parity tests check it testcase by testcase.
struct BreakpointAction_t {
  enum class Kind_t { Host, SimulateReturn, SetGprs, Feed, Rdrand, StopOk, StopWithArgs };
  Kind_t Kind = Kind_t::Host;
  uint64_t Return = 0;  // SimulateReturn: SimulateReturnFromFunction(Return)
  uint64_t Gprs[17] = {};  // SetGprs: rax, rcx, rdx, rbx, rsp, rbp, rsi, rdi, r8..r15, rip
  using ArgsResult_t = TestcaseResult_t (*)(const uint64_t *Args);
  ArgsResult_t ArgsResult = nullptr;  // StopWithArgs

  static BreakpointAction_t SimulateReturn(const uint64_t Value) {
    BreakpointAction_t A;
    A.Kind = Kind_t::SimulateReturn;
    A.Return = Value;
    return A;
  }
  // ... after a VirtReadString(Reg, MaxLength) whose result the handler drops
  // (tlv printf's format): the read's translations are part of the handler
  // (a failing one ends the testcase, U43), so the backend checks them too
  BreakpointAction_t AfterReadingString(const Registers_t Reg, const uint64_t MaxLength = 256) const {
    BreakpointAction_t A = *this;
    A.StringReg = (int)Reg;
    A.StringMax = MaxLength;
    return A;
  }
  int StringReg = -1;  // SimulateReturn: Registers_t of the string read first, -1 none
  uint64_t StringMax = 0;
  // the 16 GPRs and rip of a CpuState_t (registers only; rflags untouched)
  static BreakpointAction_t SetGprs(const struct CpuState_t &State);
  // pop the testcase's next input chunk (Backend_t::SetFeed): none left, or
  // Size >= Window -> Stop(Ok_t()); else write it so that it ends at
  // Base + Window (dirty), Base = its address, Len = its size; the hooked
  // instruction then runs (Gprs[0] / Gprs[1] hold the two Registers_t)
  // Stop(Ok_t())
  static BreakpointAction_t StopOk() {
    BreakpointAction_t A;
    A.Kind = Kind_t::StopOk;
    return A;
  }
  // Reg := Backend_t::Rdrand() (the testcase's BLAKE3 chain); the hooked
  // instruction then runs
  static BreakpointAction_t Rdrand(const Registers_t Reg) {
    BreakpointAction_t A;
    A.Kind = Kind_t::Rdrand;
    A.Gprs[0] = (uint64_t)Reg;
    return A;
  }
  // Stop(Result(Args)), Args = GetArg(0 .. NArgs - 1) of the hooked function
  // (NArgs <= 6): a handler that only names the testcase's end from its
  // arguments (nt!KeBugCheck2 -> Crash_t, fuzzer_hevd.cc:114-128)
  static BreakpointAction_t StopWithArgs(const uint32_t NArgs, const ArgsResult_t Result) {
    BreakpointAction_t A;
    A.Kind = Kind_t::StopWithArgs;
    A.Return = NArgs;
    A.ArgsResult = Result;
    return A;
  }
  static BreakpointAction_t Feed(const Registers_t Base, const Registers_t Len,
                                 const uint64_t Window) {
    BreakpointAction_t A;
    A.Kind = Kind_t::Feed;
    A.Return = Window;
    A.Gprs[0] = (uint64_t)Base;
    A.Gprs[1] = (uint64_t)Len;
    return A;
  }
};

// What an InsertTestcase does, stated as data (this repository's extension,
// like BreakpointAction_t): the testcase's first 4 bytes (u32) go to HeadReg,
// the rest (the payload) is written, dirty, at the address in PtrReg, its size
// goes to LenReg and, with LenArg != 0, as a u64 to GetArgAddress(LenArg)
// (fuzzer_hevd.cc:20-59 exactly). A backend that applies it on the device says
// so from DeclareInsert at Init; the module's InsertTestcase then hands it the
// testcase (SetInsert) instead of writing it itself. The module keeps its own
// size checks (what it rejects is never handed over).
struct InsertAction_t {
  Registers_t HeadReg = Registers_t::Rdx;
  Registers_t PtrReg = Registers_t::R8;
  Registers_t LenReg = Registers_t::R9;
  uint32_t LenArg = 0;
  static InsertAction_t HeadAndPayload(const Registers_t Head, const Registers_t Ptr, const Registers_t Len,
                                       const uint32_t LenArg) {
    InsertAction_t A;
    A.HeadReg = Head;
    A.PtrReg = Ptr;
    A.LenReg = Len;
    A.LenArg = LenArg;
    return A;
  }
};

class Backend_t {
 public:
  virtual ~Backend_t() = default;

  // pure virtuals (backend.h:171-263, 583-589)
  virtual bool Initialize(const Options_t &Opts, const CpuState_t &CpuState) = 0;
  virtual std::optional<TestcaseResult_t> Run(const uint8_t *Buffer, const uint64_t BufferSize) = 0;
  virtual bool Restore(const CpuState_t &CpuState) = 0;
  virtual void Stop(const TestcaseResult_t &Res) = 0;
  virtual void SetLimit(const uint64_t Limit) = 0;
  virtual uint64_t GetReg(const Registers_t Reg) = 0;
  virtual uint64_t SetReg(const Registers_t Reg, const uint64_t Value) = 0;
  virtual uint64_t Rdrand() = 0;
  virtual void PrintRunStats() = 0;
  virtual bool SetTraceFile(const fs::path &TestcaseTracePath, const TraceType_t TraceType);
  virtual bool SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler) = 0;
  virtual bool DirtyGpa(const Gpa_t Gpa) = 0;
  virtual bool VirtTranslate(const Gva_t Gva, Gpa_t &Gpa, const MemoryValidate_t Validate) const = 0;
  virtual uint8_t *PhysTranslate(const Gpa_t Gpa) const = 0;
  virtual bool PageFaultsMemoryIfNeeded(const Gva_t Gva, const uint64_t Size) = 0;
  virtual const std::unordered_set<Gva_t> &LastNewCoverage() const = 0;
  virtual bool RevokeLastNewCoverage() = 0;
  // Optional fast paths under PhysWrite / VirtRead (not in the reference, whose
  // helpers always go through PhysTranslate, backend.cc:16-56): a backend that
  // does not hold guest memory in host pages serves a physical read or write
  // without materialising the page. false = not handled, use PhysTranslate.
  virtual bool PhysWriteDirect(const Gpa_t, const uint8_t *, const uint64_t) { return false; }
  virtual bool PhysReadDirect(const Gpa_t, uint8_t *, const uint64_t) const { return false; }
  // The current testcase's input chunks for a Feed breakpoint action, as
  // (u32 little-endian size, bytes) records. true = the backend serves that
  // breakpoint from them; false (default) = its handler runs.
  virtual bool SetFeed(const uint8_t *, const uint64_t) { return false; }
  // The declared insert (InsertAction_t): true = this backend applies it to
  // every testcase the module hands over with SetInsert (which then returns
  // true); false (default) = InsertTestcase writes the testcase itself.
  virtual bool DeclareInsert(const InsertAction_t &) { return false; }
  virtual bool SetInsert(const uint8_t *, const uint64_t) { return false; }

  // helpers implemented on top of the virtuals (backend.cc)
  bool SaveCrash(const Gva_t ExceptionAddress, const uint32_t ExceptionCode);
  bool SetBreakpoint(const char *Symbol, const BreakpointHandler_t Handler);
  // Handler + its data-form equivalent (BreakpointAction_t). Default: the
  // action is ignored and the handler is the breakpoint.
  virtual bool SetBreakpoint(const Gva_t Gva, const BreakpointHandler_t Handler, const BreakpointAction_t &) {
    return SetBreakpoint(Gva, Handler);
  }
  bool SetBreakpoint(const char *Symbol, const BreakpointHandler_t Handler, const BreakpointAction_t &Action);
  bool SetCrashBreakpoint(const char *Symbol);
  bool SetCrashBreakpoint(const Gva_t Gva);
  bool PhysWrite(const Gpa_t Gpa, const uint8_t *Buffer, const uint64_t BufferSize, const bool Dirty = false);
  bool VirtRead(const Gva_t Gva, uint8_t *Buffer, const uint64_t BufferSize) const;
  template <typename Ty>
  bool VirtReadStruct(const Gva_t Gva, const Ty *Buffer) const {
    return VirtRead(Gva, (uint8_t *)Buffer, sizeof(Ty));
  }
  uint32_t VirtRead4(const Gva_t Gva) const;
  uint64_t VirtRead8(const Gva_t Gva) const;
  Gva_t VirtReadGva(const Gva_t Gva) const;
  Gpa_t VirtReadGpa(const Gva_t Gva) const;
  std::string VirtReadString(const Gva_t Gva, const uint64_t MaxLength = 256) const;
  std::u16string VirtReadWideString(const Gva_t Gva, const uint64_t MaxLength = 256) const;
  bool VirtWrite(const Gva_t Gva, const uint8_t *Buffer, const uint64_t BufferSize, const bool Dirty = false);
  template <typename Ty>
  bool VirtWriteStruct(const Gva_t Gva, const Ty *Buffer) {
    return VirtWrite(Gva, (uint8_t *)Buffer, sizeof(Ty));
  }
  bool VirtWriteDirty(const Gva_t Gva, const uint8_t *Buffer, const uint64_t BufferSize);
  template <typename Ty>
  bool VirtWriteStructDirty(const Gva_t Gva, const Ty *Buffer) {
    return VirtWriteDirty(Gva, (uint8_t *)Buffer, sizeof(Ty));
  }
  bool SimulateReturnFromFunction(const uint64_t Return);
  bool SimulateReturnFrom32bitFunction(const uint32_t Return, const uint32_t StdcallArgsCount = 0);
  uint64_t GetArg(const uint64_t Idx);
  Gva_t GetArgGva(const uint64_t Idx);
  Gva_t GetArgAddress(const uint64_t Idx);
  std::pair<uint64_t, Gva_t> GetArgAndAddress(const uint64_t Idx);
  std::pair<Gva_t, Gva_t> GetArgAndAddressGva(const uint64_t Idx);

#define WTF_REG_ACCESSORS(Name)                                   \
  uint64_t Name() { return GetReg(Registers_t::Name); }           \
  void Name(const uint64_t V) { SetReg(Registers_t::Name, V); }   \
  void Name(const Gva_t V) { SetReg(Registers_t::Name, V.U64()); }
  WTF_REG_ACCESSORS(Rsp)
  WTF_REG_ACCESSORS(Rbp)
  WTF_REG_ACCESSORS(Rip)
  WTF_REG_ACCESSORS(Rax)
  WTF_REG_ACCESSORS(Rbx)
  WTF_REG_ACCESSORS(Rcx)
  WTF_REG_ACCESSORS(Rdx)
  WTF_REG_ACCESSORS(Rsi)
  WTF_REG_ACCESSORS(Rdi)
  WTF_REG_ACCESSORS(R8)
  WTF_REG_ACCESSORS(R9)
  WTF_REG_ACCESSORS(R10)
  WTF_REG_ACCESSORS(R11)
  WTF_REG_ACCESSORS(R12)
  WTF_REG_ACCESSORS(R13)
  WTF_REG_ACCESSORS(R14)
  WTF_REG_ACCESSORS(R15)
#undef WTF_REG_ACCESSORS
  void PrintRegisters();
};

// thread_local: the gpu backend services lanes on several host threads
// (module_slots.h); module code reads it exactly as upstream's global.
extern thread_local Backend_t *g_Backend;

// ------------------------------------------------------------------ corpus / mutators
// corpus.h:17-38 (Testcase_t), :40-103 (Corpus_t); mutator.h:10-20 (Mutator_t).
struct Testcase_t {
  std::unique_ptr<uint8_t[]> Buffer_;
  size_t BufferSize_ = 0;
  Testcase_t(const uint8_t *Buffer, const size_t BufferSize)
      : Buffer_(new uint8_t[BufferSize ? BufferSize : 1]), BufferSize_(BufferSize) {
    if (BufferSize) memcpy(Buffer_.get(), Buffer, BufferSize);
  }
  Testcase_t(Testcase_t &&) = default;
  Testcase_t &operator=(Testcase_t &&) = default;
};

class Corpus_t {
  std::vector<Testcase_t> Testcases_;
  fs::path OutputsPath_;
  uint64_t Bytes_ = 0;
  std::mt19937_64 &Rng_;
  const std::vector<Testcase_t> *View_ = nullptr;  // read-only view of another corpus

 public:
  Corpus_t(const fs::path &OutputsPath, std::mt19937_64 &Rng) : OutputsPath_(OutputsPath), Rng_(Rng) {}
  // a read-only view of Base's testcases that picks with its own generator
  // (parallel mutation; Base must not change while the view is used)
  Corpus_t(const Corpus_t &Base, std::mt19937_64 &Rng)
      : OutputsPath_(Base.OutputsPath_), Rng_(Rng), View_(Base.View_ ? Base.View_ : &Base.Testcases_) {}
  Corpus_t(const Corpus_t &) = delete;
  Corpus_t &operator=(const Corpus_t &) = delete;
  size_t Size() const { return View_ ? View_->size() : Testcases_.size(); }
  // Saved as <result>-<blake3 hex> ("ok" results unprefixed) under OutputsPath (corpus.h:56-86).
  bool SaveTestcase(const TestcaseResult_t &Result, Testcase_t Testcase);
  const Testcase_t *PickTestcase() const {
    const std::vector<Testcase_t> &T = View_ ? *View_ : Testcases_;
    if (T.empty()) return nullptr;
    return &T[std::uniform_int_distribution<size_t>(0, T.size() - 1)(Rng_)];
  }
  uint64_t Bytes() const { return Bytes_; }
};

class Mutator_t {
 public:
  Mutator_t() = default;
  virtual ~Mutator_t() = default;
  virtual std::string GetNewTestcase(const Corpus_t &Corpus) = 0;
  virtual void OnNewCoverage(const Testcase_t &) {}
};

// The default mutator of a target (targets.h:25; mutator.cc:8-54): one
// mutation of a corpus pick per testcase by libFuzzer's MutationDispatcher
// (src/libs/libfuzzer/FuzzerMutate.cpp, vendored by the reference), restated
// in mutator_lite.cc with the same generator (std::minstd_rand seeded with the
// low 32 bits of one draw of the master's mt19937_64), the same 12 mutators in
// the same order, the same draw order and the same persistent scratch state;
// its output stream for a seed is the reference's, bit for bit
// (tests/test_host_parity.py against the reference build).
class LibfuzzerMutator_t : public Mutator_t {
  std::minstd_rand Rand_;                 // fuzzer::Random (FuzzerMutate.h:212-228)
  size_t MaxSize_;
  std::vector<uint8_t> Scratch_;          // ScratchBuffer_ (mutator.cc:17-18)
  std::vector<uint8_t> InPlace_;          // MutationDispatcher::MutateInPlaceHere
  std::vector<uint8_t> CrossOverWith_;    // last new-coverage testcase
  bool HasCrossOver_ = false;
  size_t R(size_t N) { return N ? size_t(Rand_()) % N : 0; }
  bool RB() { return size_t(Rand_()) % 2; }
  uint8_t RandCh();
  size_t Apply(size_t Which, uint8_t *Data, size_t Size);
  size_t CopyPartOf(const uint8_t *From, size_t FromSize, uint8_t *To, size_t ToSize);
  size_t InsertPartOf(const uint8_t *From, size_t FromSize, uint8_t *To, size_t ToSize, size_t MaxToSize);
  size_t CrossOver(const uint8_t *A, size_t SizeA, const uint8_t *B, size_t SizeB, uint8_t *Out, size_t MaxOut);
  template <typename T>
  size_t ChangeBinaryInteger(uint8_t *Data, size_t Size);

 public:
  LibfuzzerMutator_t(std::mt19937_64 &Rng, const size_t MaxSize)
      : Rand_((unsigned int)Rng()), MaxSize_(MaxSize), Scratch_(MaxSize) {}
  static std::unique_ptr<Mutator_t> Create(std::mt19937_64 &Rng, const size_t MaxSize) {
    return std::make_unique<LibfuzzerMutator_t>(Rng, MaxSize);
  }
  std::string GetNewTestcase(const Corpus_t &Corpus) override;
  void OnNewCoverage(const Testcase_t &T) override {
    CrossOverWith_.assign(T.Buffer_.get(), T.Buffer_.get() + T.BufferSize_);
    HasCrossOver_ = true;
  }
};

// ------------------------------------------------------------------ targets

// InsertTestcase prepared ahead (this repository's extension, like
// InsertAction_t): what a module's InsertTestcase does on a backend that takes
// the testcase as data (Backend_t::SetFeed / SetInsert returning true), as a
// function of the testcase bytes alone. The fuzz node runs it on the threads
// that make the testcases; the backend then takes its bytes for the lane
// without calling InsertTestcase (and calls InsertTestcase after all if it
// would refuse them). The lane's module state must be what a reset left.
enum class PreparedInsert_t : int8_t {
  Failed = -1,   // InsertTestcase returns false
  Call = 0,      // not preparable: call InsertTestcase
  Nothing = 1,   // InsertTestcase returns true and hands the backend nothing
  Feed = 2,      // ... does only SetFeed(Out) and returns true
  Insert = 3,    // ... does only SetInsert(testcase) and returns true (Out unused)
};
using PrepareInsert_t = PreparedInsert_t (*)(const uint8_t *, size_t, std::vector<uint8_t> &Out);

struct Target_t {
  using Init_t = bool (*)(const Options_t &, const CpuState_t &);
  using InsertTestcase_t = bool (*)(const uint8_t *, const size_t);
  using Restore_t = bool (*)();
  using CreateMutator_t = std::unique_ptr<Mutator_t> (*)(std::mt19937_64 &, const size_t);

  explicit Target_t(const std::string &Name, const Init_t Init, const InsertTestcase_t InsertTestcase,
                    const Restore_t Restore = []() { return true; },
                    const CreateMutator_t CreateMutator = LibfuzzerMutator_t::Create,
                    const PrepareInsert_t PrepareInsert = nullptr);

  std::string Name;
  Init_t Init = nullptr;
  InsertTestcase_t InsertTestcase = nullptr;
  Restore_t Restore = nullptr;
  CreateMutator_t CreateMutator = nullptr;
  PrepareInsert_t PrepareInsert = nullptr;  // optional (above)
};

struct Targets_t {
  std::vector<Target_t> Targets;
  Target_t *Get(const std::string &Name);
  void DisplayRegisteredTargets();
  void Registers(const Target_t &Target);
  static Targets_t &Instance();
};

// ------------------------------------------------------------------ symbols
class Debugger_t {
  std::unordered_map<std::string, uint64_t> Symbols_;

 public:
  bool Init(const fs::path &DumpPath, const fs::path &SymbolFilePath);
  bool AddSymbol(const std::string &Name, const uint64_t Address);
  uint64_t GetModuleBase(const char *Name) const { return GetSymbol(Name); }
  // Like the reference, a missing symbol ends the process (debugger.h:368-376).
  uint64_t GetSymbol(const char *Name) const;
};
extern Debugger_t g_Dbg;

// ------------------------------------------------------------------ utils
// utils.h:19, 226-227
using span_u8 = std::span<uint8_t>;
const uint64_t _1KB = 1024;
const uint64_t _1MB = _1KB * _1KB;

std::string_view ExceptionCodeToStr(const uint32_t ExceptionCode);
std::string TestcaseResultName(const TestcaseResult_t &Res);
std::string Blake3HexDigest(const uint8_t *Data, const size_t DataSize);
bool SaveFile(const fs::path &Path, const uint8_t *Buffer, const size_t BufferSize);
std::vector<uint8_t> ReadFile(const fs::path &Path);
bool LoadCpuStateFromJSON(CpuState_t &CpuState, const fs::path &CpuStatePath);
bool SanitizeCpuState(CpuState_t &CpuState);

// NT status codes used by crash naming (nt.h:256-258 plus the standard ones).
constexpr uint32_t EXCEPTION_ACCESS_VIOLATION = 0xC0000005;
constexpr uint32_t EXCEPTION_INT_DIVIDE_BY_ZERO = 0xC0000094;
constexpr uint32_t EXCEPTION_ILLEGAL_INSTRUCTION = 0xC000001D;
constexpr uint32_t EXCEPTION_PRIV_INSTRUCTION = 0xC0000096;
constexpr uint32_t EXCEPTION_BREAKPOINT = 0x80000003;
constexpr uint32_t STATUS_STACK_BUFFER_OVERRUN = 0xC0000409;
constexpr uint32_t STATUS_HEAP_CORRUPTION = 0xC0000374;
constexpr uint32_t EXCEPTION_ACCESS_VIOLATION_READ = 0xCFFFFFFF;
constexpr uint32_t EXCEPTION_ACCESS_VIOLATION_WRITE = 0xCFFFFFFE;
constexpr uint32_t EXCEPTION_ACCESS_VIOLATION_EXECUTE = 0xCFFFFFFD;
