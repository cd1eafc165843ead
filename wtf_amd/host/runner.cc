// runner.cc — see runner.h.
#include "runner.h"
#include "remote.h"
#include "host_pool.h"
#include "module_instances.h"

#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <future>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <thread>

#include "../../include/wtfgpu.h"

namespace wtfgpu_host {

namespace {

// parallel mutation of a fuzz batch (make_batch): batches of at least
// kParMutateMin new testcases, kMutateChunk testcases per generator
constexpr size_t kParMutateMin = 8192, kMutateChunk = 2048;
// CPU time of the calling thread (ns)
uint64_t ThreadCpuNs() {
  timespec t{};
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}


using Clock = std::chrono::steady_clock;
double secs_since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

std::string crash_name(const TestcaseResult_t &R) {
  if (const Crash_t *C = std::get_if<Crash_t>(&R)) return C->CrashName;
  return "";
}

std::string json_escape(const std::string &S) {
  std::string O;
  for (char c : S) {
    if (c == '"' || c == '\\') O += '\\';
    O += c;
  }
  return O;
}

std::vector<fs::path> list_inputs(const fs::path &P) {
  std::vector<fs::path> V;
  if (fs::is_directory(P)) {
    for (const auto &E : fs::directory_iterator(P))
      if (E.is_regular_file()) V.push_back(E.path());
    std::sort(V.begin(), V.end());
  } else if (fs::exists(P)) {
    V.push_back(P);
  }
  return V;
}
  void seg(wtfgpu_seg_t &d, const Seg_t &s) {
  d.base = s.Base;
  d.limit = s.Limit;
  d.selector = s.Selector;
  d.attr = s.Attr;
  d.present = s.Present;
}
}  // namespace

void FormatTenet(const uint8_t *S, size_t Bytes, FILE *F) {
  // reference print order (rax, rbx, rcx, rdx, rbp, rsp, rsi, rdi, r8..r15)
  // over the stream's x86 order (rax, rcx, rdx, rbx, rsp, rbp, rsi, rdi, ...)
  static const int Order[16] = {0, 3, 1, 2, 5, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
  static const char *Name[17] = {"rax", "rcx", "rdx", "rbx", "rsp", "rbp", "rsi", "rdi", "r8",
                                 "r9",  "r10", "r11", "r12", "r13", "r14", "r15", "rip"};
  static const char *Type[4] = {"", "mr", "mw", "mrw"};
  static const char Hex[] = "0123456789ABCDEF";
  uint64_t Prev[17] = {};
  bool First = true;
  std::string Line, Mem;
  auto word = [&](size_t q) {
    uint64_t v;
    memcpy(&v, S + q, 8);
    return v;
  };
  size_t q = 0;
  while (q + 16 <= Bytes) {
    const uint64_t w0 = word(q), w1 = word(q + 8);
    if (w0 == 2ull << 56) {  // REGS
      if (q + 8 + 17 * 8 > Bytes) break;
      uint64_t Cur[17];
      memcpy(Cur, S + q + 8, sizeof(Cur));
      Line.clear();
      char Buf[48];
      for (int k = 0; k < 17; k++) {
        const int r = k < 16 ? Order[k] : 16;
        if (!First && Cur[r] == Prev[r]) continue;
        snprintf(Buf, sizeof(Buf), "%s=0x%llx%s", Name[r], (unsigned long long)Cur[r], k < 16 ? "," : "");
        Line += Buf;
      }
      Line += Mem;
      if (!Line.empty()) {
        Line += '\n';
        fwrite(Line.data(), 1, Line.size(), F);
      }
      Mem.clear();
      memcpy(Prev, Cur, sizeof(Prev));
      First = false;
      q += 8 + 17 * 8;
      continue;
    }
    const uint32_t Ty = (uint32_t)(w1 >> 32) & 0xff, Len = (uint32_t)w1;
    if (w1 >> 56 != 1 || Ty == 0 || Ty > 3) break;  // a truncation mark
    const size_t n = 16 + ((size_t)Len + 7) / 8 * 8;
    if (q + n > Bytes) break;
    char Buf[40];
    snprintf(Buf, sizeof(Buf), ",%s=0x%llx:", Type[Ty], (unsigned long long)w0);
    Mem += Buf;
    for (uint32_t i = 0; i < Len; i++) {
      Mem += Hex[S[q + 16 + i] >> 4];
      Mem += Hex[S[q + 16 + i] & 15];
    }
    q += n;
  }
  if (!Mem.empty()) {  // accesses of a truncated stream's last instruction
    Mem += '\n';
    fwrite(Mem.data(), 1, Mem.size(), F);
  }
}

// The ring-3 CpuState_t -> wtfgpu_regs_t mapping (LoadState, bochscpu_backend.cc:1026-1122).
wtfgpu_regs_t RegsFromCpuState(const CpuState_t &S) {
  wtfgpu_regs_t r{};
  const uint64_t g[16] = {S.Rax, S.Rcx, S.Rdx, S.Rbx, S.Rsp, S.Rbp, S.Rsi, S.Rdi,
                          S.R8, S.R9, S.R10, S.R11, S.R12, S.R13, S.R14, S.R15};
  memcpy(r.gpr, g, sizeof(g));
  r.rip = S.Rip;
  r.rflags = S.Rflags;
  r.cr0 = S.Cr0.Flags, r.cr2 = S.Cr2, r.cr3 = S.Cr3, r.cr4 = S.Cr4.Flags, r.cr8 = S.Cr8;
  r.efer = S.Efer.Flags, r.xcr0 = S.Xcr0, r.kernel_gs_base = S.KernelGsBase;
  r.star = S.Star, r.lstar = S.Lstar, r.cstar = S.Cstar, r.sfmask = S.Sfmask;
  r.tsc = S.Tsc, r.tsc_aux = S.TscAux, r.apic_base = S.ApicBase, r.pat = S.Pat;
  r.sysenter_cs = S.SysenterCs, r.sysenter_eip = S.SysenterEip, r.sysenter_esp = S.SysenterEsp;
  seg(r.seg[WTFGPU_ES], S.Es), seg(r.seg[WTFGPU_CS], S.Cs), seg(r.seg[WTFGPU_SS], S.Ss);
  seg(r.seg[WTFGPU_DS], S.Ds), seg(r.seg[WTFGPU_FS], S.Fs), seg(r.seg[WTFGPU_GS], S.Gs);
  seg(r.seg[WTFGPU_TR], S.Tr), seg(r.seg[WTFGPU_LDTR], S.Ldtr);
  r.gdtr_base = S.Gdtr.Base, r.gdtr_limit = S.Gdtr.Limit, r.idtr_base = S.Idtr.Base, r.idtr_limit = S.Idtr.Limit;
  r.mxcsr = S.Mxcsr, r.mxcsr_mask = S.MxcsrMask;
  r.fpcw = S.Fpcw, r.fpsw = S.Fpsw, r.fptw = S.Fptw, r.fpop = S.Fpop;
  memcpy(r.fpst, S.Fpst, sizeof(r.fpst));
  for (int i = 0; i < 16; i++) {
    r.xmm[i][0] = S.Zmm[i].Q[0], r.xmm[i][1] = S.Zmm[i].Q[1];
    r.ymmh[i][0] = S.Zmm[i].Q[2], r.ymmh[i][1] = S.Zmm[i].Q[3];
    for (int q = 0; q < 4; q++) r.zmmh[i][q] = S.Zmm[i].Q[4 + q];
    for (int q = 0; q < 8; q++) r.zmm_hi[i][q] = S.Zmm[16 + i].Q[q];
  }
  return r;
}

TestcaseResult_t FaultToResult(uint32_t vector, uint32_t error, uint64_t rip, uint64_t addr, uint32_t cpl) {
  uint32_t code = EXCEPTION_ACCESS_VIOLATION_READ;
  switch (vector) {
    case WTFGPU_VEC_DE: code = EXCEPTION_INT_DIVIDE_BY_ZERO; break;
    case WTFGPU_VEC_UD: code = EXCEPTION_ILLEGAL_INSTRUCTION; break;
    case WTFGPU_VEC_GP: code = EXCEPTION_ACCESS_VIOLATION_READ; break;
    case WTFGPU_VEC_PF:
      code = (error & ErrorInstructionFetch) ? EXCEPTION_ACCESS_VIOLATION_EXECUTE
             : (error & ErrorWrite)          ? EXCEPTION_ACCESS_VIOLATION_WRITE
                                             : EXCEPTION_ACCESS_VIOLATION_READ;
      break;
    default: break;
  }
  char name[160];
  if (cpl == 3)
    snprintf(name, sizeof(name), "crash-%s-%#llx", std::string(ExceptionCodeToStr(code)).c_str(),
             (unsigned long long)rip);
  else if (vector == WTFGPU_VEC_PF)  // KiPageFault -> KeBugCheckEx(PAGE_FAULT_IN_NONPAGED_AREA, cr2, access, rip, 0)
    snprintf(name, sizeof(name), "crash-0x50-0x%llx-0x%x-0x%llx-0x0-0x0", (unsigned long long)addr,
             (error & ErrorInstructionFetch) ? 0x10u : (error & ErrorWrite) ? 2u : 0u, (unsigned long long)rip);
  else  // KMODE_EXCEPTION_NOT_HANDLED(NTSTATUS, rip, 0, 0)
    snprintf(name, sizeof(name), "crash-0x1e-0x%x-0x%llx-0x0-0x0-0x0",
             vector == WTFGPU_VEC_DE ? 0xc0000094u : vector == WTFGPU_VEC_UD ? 0xc000001du : 0xc0000005u,
             (unsigned long long)rip);
  return Crash_t(name);
}

// human.cc:38-72
static std::string bytes_to_human(uint64_t B) {
  const char *Unit = "b";
  double V = double(B);
  const double K = 1024, M = K * K, G = M * K;
  if (V >= G) Unit = "gb", V /= G;
  else if (V >= M) Unit = "mb", V /= M;
  else if (V >= K) Unit = "kb", V /= K;
  char b[64];
  snprintf(b, sizeof(b), "%.1f%s", V, Unit);
  return b;
}
static std::string number_to_human(uint64_t N) {
  const char *Unit = "";
  double V = double(N);
  if (V > 1e6) Unit = "m", V /= 1e6;
  else if (V > 1e3) Unit = "k", V /= 1e3;
  char b[64];
  snprintf(b, sizeof(b), "%.1f%s", V, Unit);
  return b;
}

void PrintTestcaseRunStats(const LaneResult &L, size_t AggregateCoverage) {
  printf("--------------------------------------------------\n");
  printf("Run stats:\n");
  printf("Instructions executed: %s (%s unique)\n", number_to_human(L.icount).c_str(),
         number_to_human(AggregateCoverage).c_str());
  printf("          Dirty pages: %s\n", bytes_to_human((uint64_t)L.dirty * Page::Size).c_str());
  printf("      Memory accesses: %s\n", bytes_to_human(L.bytes).c_str());
  printf("       Edges executed: %s (%s unique)\n", number_to_human(L.edges).c_str(),
         number_to_human(L.edges_new).c_str());
}

bool ParseRunnerArgs(int argc, char **argv, RunnerOptions &O) {
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto next = [&](const char *what) -> const char * {
      if (i + 1 >= argc) {
        fprintf(stderr, "%s needs a value\n", what);
        exit(2);
      }
      return argv[++i];
    };
    if (a == "run" || a == "fuzz" || a == "master") O.mode = a;
    else if (a == "--name") O.name = next("--name");
    else if (a == "--target") O.target = next("--target");
    else if (a == "--input") O.input = next("--input");
    else if (a == "--results") O.results = next("--results");
    else if (a == "--limit") O.limit = strtoull(next("--limit"), nullptr, 0);
    else if (a == "--lanes") O.lanes = (uint32_t)strtoul(next("--lanes"), nullptr, 0);
    else if (a == "--overlay-pages") O.overlay_pages = (uint32_t)strtoul(next("--overlay-pages"), nullptr, 0);
    else if (a == "--runs") O.runs = strtoull(next("--runs"), nullptr, 0);
    else if (a == "--seconds") O.seconds = atof(next("--seconds"));
    else if (a == "--seed") O.seed = strtoull(next("--seed"), nullptr, 0);
    else if (a == "--max_len") O.max_len = strtoull(next("--max_len"), nullptr, 0);
    else if (a == "--device") O.device = atoi(next("--device"));
    else if (a == "--full-coverage") O.full_coverage = true;
    else if (a == "--edges") O.edges = true;
    else if (a == "--trace-path") O.trace_path = next("--trace-path");
    else if (a == "--trace-type") O.trace_type = next("--trace-type");
    else if (a == "--trace-cap") O.trace_cap = (uint32_t)strtoul(next("--trace-cap"), nullptr, 0);
    else if (a == "--tenet-cap") O.tenet_cap = strtoull(next("--tenet-cap"), nullptr, 0) & ~7ull;
    else if (a == "--quiet") O.quiet = true;
    else if (a == "--serial-mutation") O.serial_mutation = true;
    else if (a == "--slice-steps") O.slice = strtoull(next("--slice-steps"), nullptr, 0);
    else if (a == "--regroup-steps") O.regroup = strtoull(next("--regroup-steps"), nullptr, 0);
    else if (a == "--stream-run") O.stream_run = true;
    else if (a == "--serial") O.serial = true;
    else if (a == "--module-so") O.module_so = next("--module-so");
    else if (a == "--rank") O.rank = atoi(next("--rank"));
    else if (a == "--world") O.world = atoi(next("--world"));
    else if (a == "--exchange") O.exchange = next("--exchange");
    else if (a == "--nccl-id-file") O.nccl_id_file = next("--nccl-id-file");
    else if (a == "--rccl-force") O.rccl_force = true;
    else if (a == "--address") O.address = next("--address");
    else if (a == "--nodes") O.nodes = atoi(next("--nodes"));
    else if (a == "--batched") O.batched = true;
    else if (a == "--sample") O.sample = next("--sample");
    else if (a == "--sample-every") O.sample_every = strtoull(next("--sample-every"), nullptr, 0);
    else {
      fprintf(stderr, "unknown argument %s\n", a.c_str());
      return false;
    }
  }
  if (const char *e = getenv("WTF_RCCL_FORCE")) O.rccl_force = O.rccl_force || atoi(e) != 0;
  if (O.world < 1 || O.rank < 0 || O.rank >= O.world) {
    fprintf(stderr, "--rank must be in [0, --world)\n");
    return false;
  }
  if (O.mode == "master" && (O.address.empty() || O.nodes < 1)) {
    fprintf(stderr, "master needs --address and --nodes >= 1\n");
    return false;
  }
  if (O.name.empty() || O.target.empty()) {
    fprintf(stderr, "usage: [run|fuzz|master] --name <target> --target <dir> [--input p] [--results f] [--limit n]\n"
                    "       [--lanes n] [--overlay-pages k] [--runs n] [--seconds s] [--seed s] [--full-coverage]\n"
                    "       [--serial-mutation] [--slice-steps s] [--regroup-steps r] [--rank r --world n [--exchange host:port | --nccl-id-file f]]\n"
                    "       [--address tcp://ip:port|unix://path [--batched] [--nodes k]] [--edges]\n"
                    "       [--trace-path dir [--trace-type rip|cov|tenet] [--trace-cap n] [--tenet-cap bytes]] [--module-so m.so] [--serial]\n");
    return false;
  }
  return true;
}

// wtf.cc:300-420 (state loading + sanitisation + symbol store), backend-independent
bool LoadTarget(const RunnerOptions &O, Options_t &Opts, CpuState_t &State) {
  const fs::path T(O.target);
  Opts.TargetName = O.name;
  Opts.StatePath = T / "state";
  Opts.DumpPath = Opts.StatePath / "mem.dmp";
  Opts.CpuStatePath = Opts.StatePath / "regs.json";
  Opts.SymbolFilePath = Opts.StatePath / "symbol-store.json";
  Opts.Limit = O.limit;
  Opts.Edges = O.edges;
  Opts.GpuDevice = O.device;
  Opts.GpuLanes = O.lanes;
  Opts.GpuOverlayPages = O.overlay_pages;
  if (O.full_coverage) Opts.GpuCoverageSet = 8192;
  Opts.Fuzz.Seed = (uint32_t)O.seed;
  if (!LoadCpuStateFromJSON(State, Opts.CpuStatePath)) {
    printf("Failed to load the CPU state from %s\n", Opts.CpuStatePath.string().c_str());
    return false;
  }
  if (!SanitizeCpuState(State)) return false;
  Opts.CpuState = State;
  if (!g_Dbg.Init(Opts.DumpPath, Opts.SymbolFilePath)) return false;
  return true;
}

int RunnerMain(const RunnerOptions &O, Executor_t &Exec, const Options_t &Opts, const CpuState_t &State,
               CoverageExchange_t *X) {
  // --module-so: one private copy of an unchanged module per lane
  // (module_instances.h); lane l runs copy l
  std::unique_ptr<ModuleInstances> Inst;
  Target_t *Target = nullptr;
  std::unique_ptr<Target_t> Copy0;  // a copy: Target_t's own constructor would register it
  if (!O.module_so.empty()) {
    Inst = std::make_unique<ModuleInstances>();
    if (!Inst->Load(O.module_so, O.name, Exec.Lanes())) return 1;
    Copy0 = std::make_unique<Target_t>(Inst->TargetOf(0));
    Target = Copy0.get();
  } else {
    Target = Targets_t::Instance().Get(O.name);
  }
  if (!Target) {
    printf("Target %s not found\n", O.name.c_str());
    Targets_t::Instance().DisplayRegisteredTargets();
    return 1;
  }
  g_Backend = Exec.AsBackend();
  if (Inst ? !Inst->InitAll(Opts, State) : !Target->Init(Opts, State)) {
    printf("Failed to initialize the target\n");
    return 1;
  }
  const uint32_t N = Exec.Lanes();
  ModuleSlots Slots;
  Slots.Capture(N);
  Slots.AttachInstances(Inst.get());
  Exec.SetFullCoverage(O.full_coverage);

  if (O.mode == "run") {
    auto Inputs = list_inputs(O.input.empty() ? fs::path(O.target) / "inputs" : fs::path(O.input));
    // --runs R: each input R times in a row (subcommands.cc:85-88); the run
    // stats are printed for a single input run once (:48)
    const uint64_t Runs = O.runs ? O.runs : 1;
    const bool Stats = Inputs.size() == 1 && Runs == 1 && !O.quiet;
    LaneResult Last;
    // traces (subcommands.cc:52-74): <trace-path>/<input name>.trace; an input
    // whose trace exists is skipped
    const bool Trace = !O.trace_path.empty();
    // cov traces: the reference logs a rip absent from its aggregate coverage
    // (bochscpu_backend.cc:501-516), which the Restore after a traced run
    // empties (:778-789): a traced run's rips unique within it, plus, under
    // --runs, the rips the previous input's untraced repetitions added
    std::unordered_set<uint64_t> TraceSeen;
    if (Trace) {
      if (O.trace_type != "rip" && O.trace_type != "cov" && O.trace_type != "tenet") {
        printf("--trace-type %s is not supported by this backend (rip, cov, tenet)\n", O.trace_type.c_str());
        return 1;
      }
      if (O.trace_type == "tenet") {
        // the device holds lanes x cap bytes: the default is clamped to 32 GiB in all
        const uint64_t Cap = O.tenet_cap ? O.tenet_cap : std::min<uint64_t>(1ull << 24, (32ull << 30) / N) & ~7ull;
        if (!Exec.EnableTenet(Cap)) {
          printf("EnableTenet failed (%u lanes x %llu bytes)\n", N, (unsigned long long)Cap);
          return 1;
        }
      } else if (!Exec.EnableTrace(O.trace_cap)) {
        printf("EnableTrace failed\n");
        return 1;
      }
      fs::create_directories(O.trace_path);
      std::vector<fs::path> Keep;
      for (const fs::path &In : Inputs) {
        if (fs::exists(fs::path(O.trace_path) / (In.filename().string() + ".trace")))
          printf("Skipping %s as it already exists.\n", In.string().c_str());
        else Keep.push_back(In);
      }
      Inputs = Keep;
    }
    // the repetition of each input (0 = its first run: the only one traced,
    // since the reference's Restore closes the trace file after it)
    std::vector<uint64_t> RepOf(Inputs.size(), 0);
    if (Runs > 1) {
      std::vector<fs::path> Rep;
      Rep.reserve(Inputs.size() * Runs);
      RepOf.clear();
      for (const fs::path &In : Inputs)
        for (uint64_t k = 0; k < Runs; k++) {
          Rep.push_back(In);
          RepOf.push_back(k);
        }
      Inputs.swap(Rep);
    }
    auto write_trace = [&](const fs::path &In, uint32_t Lane, uint64_t Rep) -> bool {
      if (Rep) {  // an untraced repetition: its rips join the aggregate the next cov trace starts from
        if (O.trace_type != "cov") return true;
        std::vector<uint64_t> Rips;
        bool Truncated = false;
        if (!Exec.LaneTrace(Lane, Rips, Truncated)) return false;
        TraceSeen.insert(Rips.begin(), Rips.end());
        return true;
      }
      if (O.trace_type == "tenet") {
        std::vector<uint8_t> Bytes;
        bool Truncated = false;
        if (!Exec.LaneTenet(Lane, Bytes, Truncated)) return false;
        FILE *F = fopen((fs::path(O.trace_path) / (In.filename().string() + ".trace")).c_str(), "w");
        if (!F) return false;
        FormatTenet(Bytes.data(), Bytes.size(), F);
        fclose(F);
        if (Truncated) printf("tenet trace of %s truncated at %zu bytes (--tenet-cap)\n", In.string().c_str(), Bytes.size());
        return true;
      }
      std::vector<uint64_t> Rips;
      bool Truncated = false;
      if (!Exec.LaneTrace(Lane, Rips, Truncated)) return false;
      FILE *F = fopen((fs::path(O.trace_path) / (In.filename().string() + ".trace")).c_str(), "w");
      if (!F) return false;
      for (uint64_t R : Rips)
        if (O.trace_type == "rip" || TraceSeen.insert(R).second) fprintf(F, "%#llx\n", (unsigned long long)R);
      TraceSeen.clear();
      fclose(F);
      if (Truncated) printf("trace of %s truncated at %zu rips (--trace-cap)\n", In.string().c_str(), Rips.size());
      return true;
    };
    FILE *Out = O.results.empty() ? stdout : fopen(O.results.c_str(), "w");
    if (!Out) return 1;
    const auto t0 = Clock::now();
    uint64_t Retired = 0;
    auto print = [&](const fs::path &In, const LaneResult &L) {
      std::vector<uint64_t> Cov = L.new_coverage;
      std::sort(Cov.begin(), Cov.end());
      fprintf(Out, "{\"input\":\"%s\",\"result\":\"%s\",\"crash\":\"%s\",\"error\":%d,\"exit\":%u,\"icount\":%llu,",
              json_escape(In.filename().string()).c_str(), TestcaseResultName(L.result).c_str(),
              json_escape(crash_name(L.result)).c_str(), (int)L.error, L.exit_status, (unsigned long long)L.icount);
      fprintf(Out, "\"gprs\":[");
      for (int g = 0; g < 18; g++) fprintf(Out, "%s%llu", g ? "," : "", (unsigned long long)L.gprs[g]);
      fprintf(Out, "],\"coverage\":[");
      for (size_t c = 0; c < Cov.size(); c++) fprintf(Out, "%s%llu", c ? "," : "", (unsigned long long)Cov[c]);
      fprintf(Out, "],\"bytes\":%llu,\"dirty\":%u,\"edges\":%llu,\"edges_new\":%llu,\"handler_fault\":%d}\n",
              (unsigned long long)L.bytes, L.dirty, (unsigned long long)L.edges, (unsigned long long)L.edges_new,
              (int)L.handler_fault);
      Last = L;
    };
    if (O.serial && !Trace) {
      // RunTestcaseAndRestore (client.cc:88-180) restated over the Backend_t
      // interface: InsertTestcase -> Run -> a timeout's new coverage revoked
      // (RevokeLastNewCoverage, :122-125) -> Target.Restore -> Backend.Restore.
      // The module's globals are used as they are (one testcase at a time).
      Backend_t *B = Exec.AsBackend();
      static const Registers_t Order[18] = {
          Registers_t::Rax, Registers_t::Rcx, Registers_t::Rdx, Registers_t::Rbx, Registers_t::Rsp, Registers_t::Rbp,
          Registers_t::Rsi, Registers_t::Rdi, Registers_t::R8,  Registers_t::R9,  Registers_t::R10, Registers_t::R11,
          Registers_t::R12, Registers_t::R13, Registers_t::R14, Registers_t::R15, Registers_t::Rip, Registers_t::Rflags};
      for (const fs::path &In : Inputs) {
        g_Backend = B;
        const std::vector<uint8_t> Buf = ReadFile(In);
        LaneResult L;
        bool Inserted = false;
        try {
          Inserted = Target->InsertTestcase(Buf.data(), Buf.size());
        } catch (const HandlerFault_t &) {  // U43: an engine error for this testcase
          L.error = true;
          L.handler_fault = true;
        }
        if (!Inserted) {
          L.result = L.error ? Crash_t() : Crash_t("insert-testcase-failed");
        } else {
          const std::optional<TestcaseResult_t> Res = B->Run(Buf.data(), Buf.size());
          if (!Res) {  // client.cc:112-115: a backend failure ends the client
            printf("Run failed\n");
            return 1;
          }
          L.result = *Res;
          // printed as the batch path prints it: what the testcase found, even
          // when a timeout then revokes it from the aggregate
          for (const Gva_t &G : B->LastNewCoverage()) L.new_coverage.push_back(G.U64());
          if (std::holds_alternative<Timedout_t>(*Res)) B->RevokeLastNewCoverage();
          L.icount = Exec.LastIcount();
          L.error = Exec.LastError();
          L.handler_fault = Exec.LastHandlerFault();
          Exec.LastRunStats(L);
        }
        for (int g = 0; g < 18; g++) L.gprs[g] = B->GetReg(Order[g]);
        L.rip = L.gprs[16];
        if (!Target->Restore() || !B->Restore(State)) {
          printf("Restore failed\n");
          return 1;
        }
        Retired += L.icount;
        print(In, L);
      }
    }
    if (O.stream_run && Exec.CanStream() && !Trace) {
      // streaming replay: lanes refilled as testcases finish, results printed
      // in input order (parity with the batched replay, tests/test_gpu_tlv.py)
      std::vector<std::vector<uint8_t>> Bufs(Inputs.size());
      std::vector<LaneResult> Res(Inputs.size());
      std::vector<uint8_t> Got(Inputs.size(), 0);
      size_t next = 0, got = 0;
      while (got < Inputs.size()) {
        std::vector<StreamTestcase_t> In;
        for (uint32_t f = Exec.FreeLanes(); f && next < Inputs.size(); f--, next++) {
          Bufs[next] = ReadFile(Inputs[next]);
          In.push_back(StreamTestcase_t{Bufs[next].data(), Bufs[next].size(), next});
        }
        std::vector<StreamResult_t> R;
        size_t Taken = 0;
        if (!Exec.StreamStep(*Target, In, O.slice ? O.slice : 4096, R, &Slots, &Taken)) {
          printf("StreamStep failed\n");
          return 1;
        }
        next -= In.size() - Taken;  // offered again next step
        for (StreamResult_t &F : R) {
          Res[F.tag] = std::move(*F.r);
          Got[F.tag] = 1;
          got++;
        }
      }
      for (size_t i = 0; i < Inputs.size(); i++) {
        Retired += Res[i].icount;
        print(Inputs[i], Res[i]);
      }
    }
    for (size_t b = (O.stream_run && Exec.CanStream() && !Trace) || (O.serial && !Trace) ? Inputs.size() : 0;
         b < Inputs.size(); b += N) {
      const size_t n = std::min<size_t>(N, Inputs.size() - b);
      std::vector<std::vector<uint8_t>> Bufs(n);
      std::vector<std::pair<const uint8_t *, size_t>> Tc(n);
      for (size_t i = 0; i < n; i++) {
        Bufs[i] = ReadFile(Inputs[b + i]);
        Tc[i] = {Bufs[i].data(), Bufs[i].size()};
      }
      if (O.full_coverage) Exec.ResetCoverage();
      std::vector<LaneResult> R;
      if (!Exec.RunBatch(*Target, Tc, R, &Slots)) {
        printf("RunBatch failed\n");
        return 1;
      }
      for (size_t i = 0; i < n; i++) {
        Retired += R[i].icount;
        print(Inputs[b + i], R[i]);
        if (Trace && !write_trace(Inputs[b + i], (uint32_t)i, RepOf[b + i])) {
          printf("trace of %s failed\n", Inputs[b + i].string().c_str());
          return 1;
        }
      }
    }
    if (Out != stdout) fclose(Out);
    if (Stats) PrintTestcaseRunStats(Last, Exec.CoverageSize());
    if (!O.quiet)
      fprintf(stderr, "run: %zu testcases, %llu instructions, %.3f s\n", Inputs.size(), (unsigned long long)Retired,
              secs_since(t0));
    return 0;
  }

  // ---- fuzz against a remote master (wire.h): the client loop
  if (!O.address.empty()) return NodeMain(O, Exec, *Target, Slots);

  // ---- fuzz: in-process master + batched node
  if (X && X->Exchanging() && O.full_coverage) {
    // parity mode resets the map every batch: a merge in flight reads a copy
    // taken when it started, but the shards' maps would mean nothing
    printf("--full-coverage is a single-node parity mode (not with --world > 1)\n");
    return 1;
  }
  FuzzSession F(O, Exec, *Target, Slots, X);
  if (!F.Start()) {
    printf("Nothing to run: empty corpus and no inputs\n");
    return 1;
  }
  const bool Shards = X && X->Exchanging();
  for (;;) {
    // shards stop together, on the consensus of the last merge absorbed
    // (every shard absorbs the same one at the same step)
    if (Shards ? F.AllDone() : F.Done()) break;
    if (!F.Step()) {
      printf("RunBatch failed\n");
      return 1;
    }
  }
  if (Shards && !F.FinishMerge()) return 1;
  F.FlushFiles();
  printf("%s\n", F.SummaryJson().c_str());
  return 0;
}

// ------------------------------------------------------------------ FileWriter
FileWriter::FileWriter() : Th_([this] { Loop(); }) {}

FileWriter::~FileWriter() {
  {
    std::lock_guard<std::mutex> g(Mu_);
    Stop_ = true;
  }
  Cv_.notify_all();
  Th_.join();
}

void FileWriter::Save(std::filesystem::path Path, const uint8_t *Data, size_t Size) {
  {
    std::lock_guard<std::mutex> g(Mu_);
    Q_.emplace_back(std::move(Path), std::vector<uint8_t>(Data, Data + Size));
  }
  Cv_.notify_one();
}

void FileWriter::Flush() {
  std::unique_lock<std::mutex> g(Mu_);
  Idle_.wait(g, [this] { return Q_.empty() && !Busy_; });
}

void FileWriter::Loop() {
  std::unique_lock<std::mutex> g(Mu_);
  for (;;) {
    Cv_.wait(g, [this] { return Stop_ || !Q_.empty(); });
    if (Q_.empty()) return;  // stopping with nothing left
    auto F = std::move(Q_.front());
    Q_.pop_front();
    Busy_ = true;
    g.unlock();
    SaveFile(F.first, F.second.data(), F.second.size());
    g.lock();
    Busy_ = false;
    if (Q_.empty()) Idle_.notify_all();
  }
}

// ------------------------------------------------------------------ FuzzSession
FuzzSession::FuzzSession(const RunnerOptions &O, Executor_t &Exec, Target_t &Target, ModuleSlots &Slots,
                         CoverageExchange_t *X)
    : O_(O), Exec_(Exec), Target_(Target), Slots_(Slots), X_(X),
      Rng_(O.seed + (X ? (uint64_t)X->Rank() : 0)), T_(O.target), Corpus_(T_ / "outputs", Rng_) {}

FuzzSession::~FuzzSession() {
  if (Next_.valid()) Next_.wait();
  Writer_.Flush();
  if (Sample_) fclose(Sample_);
}

void FuzzSession::WriteSample(const uint8_t *Tc, size_t Size, const LaneResult &L) {
  static const char *hex = "0123456789abcdef";
  std::string H(2 * Size, '0');
  for (size_t i = 0; i < Size; i++) {
    H[2 * i] = hex[Tc[i] >> 4];
    H[2 * i + 1] = hex[Tc[i] & 15];
  }
  std::vector<uint64_t> Cov = L.new_coverage;
  std::sort(Cov.begin(), Cov.end());
  fprintf(Sample_, "{\"tc\":\"%s\",\"result\":\"%s\",\"crash\":\"%s\",\"error\":%d,\"icount\":%llu,\"gprs\":[",
          H.c_str(), TestcaseResultName(L.result).c_str(), json_escape(crash_name(L.result)).c_str(), (int)L.error,
          (unsigned long long)L.icount);
  for (int g = 0; g < 18; g++) fprintf(Sample_, "%s%llu", g ? "," : "", (unsigned long long)L.gprs[g]);
  fprintf(Sample_, "],\"coverage\":[");
  for (size_t c = 0; c < Cov.size(); c++) fprintf(Sample_, "%s%llu", c ? "," : "", (unsigned long long)Cov[c]);
  fprintf(Sample_, "]}\n");
}

bool FuzzSession::Start() {
  Exec_.SetWantRegisters(!O_.sample.empty());
  if (!O_.sample.empty()) {
    Sample_ = fopen(O_.sample.c_str(), "w");
    if (!Sample_) return false;
  }
  fs::create_directories(T_ / "outputs");
  fs::create_directories(T_ / "crashes");
  if (Target_.CreateMutator) Mutator_ = Target_.CreateMutator(Rng_, O_.max_len);
  if (!Mutator_) {
    printf("Target %s has no mutator\n", O_.name.c_str());
    return false;
  }
  // the master sends the corpus first (server.h:756-790), then mutations
  for (const auto &P : list_inputs(T_ / "inputs")) {
    const auto B = ReadFile(P);
    Pending_.emplace_back(B.begin(), B.end());
  }
  t0_ = Clock::now();
  stream_ = O_.slice && Exec_.CanStream();
  // inserts prepared where the testcases are made (not for per-lane module
  // copies: each lane calls its own copy's InsertTestcase)
  if (stream_ && Exec_.TakesPrepared() && !Slots_.Instances() && !getenv("WTF_NO_PREPARED_INSERT"))
    Prepare_ = Target_.PrepareInsert;
  if (stream_) {
    Adopt(MakeBatch(Budget(Exec_.Lanes())));
    return !Ready_.empty();
  }
  Batch_ = MakeBatch(Budget(Exec_.Lanes()));
  return !Batch_.empty();
}

void FuzzSession::Adopt(TcBatch &&B) {
  for (std::unique_ptr<TcArena> &A : B) {
    if (!A || A->Count() == 0) continue;
    A->Live = A->Count();
    for (size_t i = 0; i < A->Count(); i++) Ready_.push_back(TcRef{A.get(), (uint32_t)i});
    TcArena *K = A.get();
    Arenas_.emplace(K, std::move(A));
  }
}

// at most n more testcases within the --runs budget
uint64_t FuzzSession::Budget(uint64_t n) const {
  if (!O_.runs) return n;
  const uint64_t made = S_.execs + (stream_ ? InFlight_ + Ready_.size() : 0);
  return made >= O_.runs ? 0 : std::min<uint64_t>(n, O_.runs - made);
}

bool FuzzSession::Done() const {
  if (!stream_) return Batch_.empty();
  if (O_.seconds > 0 && secs_since(t0_) >= O_.seconds) return true;  // in-flight testcases are dropped
  return Ready_.empty() && InFlight_ == 0 && !Next_.valid() &&
         (Budget(1) == 0 || !More(S_.execs) || Corpus_.Size() == 0);
}

bool FuzzSession::More(uint64_t done) const {
  return (O_.runs == 0 || done < O_.runs) && (O_.seconds <= 0 || secs_since(t0_) < O_.seconds);
}

double FuzzSession::WallSeconds() const { return secs_since(t0_); }

// The next n testcases: the corpus inputs first, then mutations of corpus picks.
TcBatch FuzzSession::MakeBatch(uint64_t n) {
  TcBatch Batch;
  size_t Made = 0;
  auto Tail = [&]() -> TcArena & {
    if (Batch.empty()) Batch.push_back(NewArena());
    return *Batch.back();
  };
  while (Made < n && !Pending_.empty()) {
    Tail().Add(Pending_.back().data(), Pending_.back().size());
    Pending_.pop_back();
    Made++;
  }
  // large batches: mutate in fixed chunks on the host threads; chunk c has
  // its own generator, seeded from Rng in chunk order, its own mutator and
  // a read-only view of the corpus (deterministic for a seed whatever the
  // thread count; the corpus does not change while the batch is built)
  const size_t Need = n - Made;
  if (Corpus_.Size() && Need >= kParMutateMin && !O_.serial_mutation) {
    const size_t Chunks = (Need + kMutateChunk - 1) / kMutateChunk;
    std::vector<uint64_t> Seeds(Chunks);
    for (uint64_t &S : Seeds) S = Rng_();
    std::vector<std::unique_ptr<TcArena>> Out(Chunks);
    std::atomic<size_t> NextChunk{0};
    std::atomic<uint64_t> CpuNs{0};
    auto Work = [&]() {
      const uint64_t c0 = ThreadCpuNs();
      for (size_t c; (c = NextChunk.fetch_add(1)) < Chunks;) {
        std::mt19937_64 R(Seeds[c]);
        Corpus_t View(Corpus_, R);
        std::unique_ptr<Mutator_t> M = Target_.CreateMutator(R, O_.max_len);
        // the master mutator's cross-over partner (the last new-coverage
        // testcase) is every chunk mutator's too
        if (HaveNewCov_) M->OnNewCoverage(Testcase_t((const uint8_t *)LastNewCov_.data(), LastNewCov_.size()));
        auto A = NewArena();
        const size_t End = std::min(Need, (c + 1) * kMutateChunk);
        A->Off.reserve(End - c * kMutateChunk + 1);
        std::vector<uint8_t> Scratch;
        for (size_t i = c * kMutateChunk; i < End; i++) {
          const std::string S = M->GetNewTestcase(View);
          A->Add(S.data(), std::min<size_t>(S.size(), O_.max_len));
          if (Prepare_) A->Prepare(Prepare_, Scratch);
        }
        Out[c] = std::move(A);
      }
      CpuNs += ThreadCpuNs() - c0;
    };
    std::vector<std::thread> Pool;
    // (WTF_MUTATE_THREADS: the threads mutating, for A/Bs; the chunks make the
    // batch the same whatever the count)
    static const unsigned MutThreads = [] {
      const char *e = getenv("WTF_MUTATE_THREADS");
      return e && atoi(e) > 0 ? (unsigned)atoi(e) : host_threads();
    }();
    for (unsigned t = 1; t < MutThreads; t++) Pool.emplace_back(Work);
    Work();
    for (std::thread &Th : Pool) Th.join();
    MutateCpuNs_ += CpuNs.load();
    for (std::unique_ptr<TcArena> &A : Out) Batch.push_back(std::move(A));
    Made += Need;
    Batch.push_back(NewArena());  // the serial tail below
  }
  while (Made < n) {
    if (Corpus_.Size() == 0 && Made == 0) break;
    if (Corpus_.Size()) {
      const std::string S = Mutator_->GetNewTestcase(Corpus_);
      Tail().Add(S.data(), std::min<size_t>(S.size(), O_.max_len));
    } else {  // no corpus yet: repeat one of the batch's testcases so far
      size_t k = Rng_() % Made;
      const TcArena *F = nullptr;
      for (const std::unique_ptr<TcArena> &A : Batch) {
        if (k < A->Count()) {
          F = A.get();
          break;
        }
        k -= A->Count();
      }
      const std::vector<uint8_t> Copy(F->Ptr(k), F->Ptr(k) + F->Len(k));
      Tail().Add(Copy.data(), Copy.size());
    }
    Made++;
  }
  Batch.erase(std::remove_if(Batch.begin(), Batch.end(), [](const std::unique_ptr<TcArena> &A) { return A->Count() == 0; }),
              Batch.end());
  return Batch;
}

// One batch: the executor runs it while the next batch is mutated on a host
// thread (a node's master and client overlap the same way; the next batch is
// built from the corpus as it stood before this batch's results); then the
// master's bookkeeping in lane order (server.h:816-886) and, across shards,
// the coverage-map merge.
bool FuzzSession::Step() {
  // Done() is read once per step: a shard that is done keeps joining the other
  // shards' merges, and one that is not always reaches its own merge below
  // (two reads could disagree under --seconds and skip a collective)
  const bool done = Done();
  if (X_ && X_->Exchanging() && done) return MergeCoverage(true);
  if (stream_) {
    const auto tc = Clock::now();
    const bool ok = StreamStep(done);
    S_.call_ms += secs_since(tc) * 1e3;
    return ok;
  }
  BatchRefs_.clear();
  for (const std::unique_ptr<TcArena> &A : Batch_)
    for (size_t i = 0; i < A->Count(); i++) BatchRefs_.push_back(TcRef{A.get(), (uint32_t)i});
  if (BatchRefs_.empty()) return true;
  std::vector<std::pair<const uint8_t *, size_t>> Tc(BatchRefs_.size());
  for (size_t i = 0; i < BatchRefs_.size(); i++) Tc[i] = {BatchRefs_[i].data(), BatchRefs_[i].size()};
  std::vector<LaneResult> R;
  const auto tb = Clock::now();
  const uint64_t after = S_.execs + BatchRefs_.size();
  if (More(after) && Corpus_.Size()) {
    const uint64_t n = O_.runs ? std::min<uint64_t>(Exec_.Lanes(), O_.runs - after) : Exec_.Lanes();
    Next_ = std::async(std::launch::async, &FuzzSession::MakeBatch, this, n);
  }
  if (!Exec_.RunBatch(Target_, Tc, R, &Slots_)) return false;
  S_.run_s += secs_since(tb);
  S_.batches++;
  TcBatch NextBatch;
  if (Next_.valid()) NextBatch = Next_.get();  // before the corpus / mutator change below
  for (size_t i = 0; i < BatchRefs_.size(); i++) Account(BatchRefs_[i].data(), BatchRefs_[i].size(), R[i]);
  if (X_ && X_->Exchanging() && !MergeCoverage(false)) return false;
  if (!NextBatch.empty() || !More(S_.execs))
    Batch_ = std::move(NextBatch);
  else
    Batch_ = MakeBatch(Budget(Exec_.Lanes()));
  return true;
}

// Streaming step (continuous batching): the free lanes get testcases from the
// ready queue, every occupied lane runs one slice, the finished testcases are
// accounted. The producer mutates the next testcases meanwhile, from the
// corpus as it stood before this step's results.
bool FuzzSession::StreamStep(bool Done) {
  if (Done) return true;
  const auto t_step = Clock::now();
  std::vector<StreamTestcase_t> In;
  const bool open = More(S_.execs);
  if (open) {
    const uint32_t free = Exec_.FreeLanes();
    if (Ready_.size() < free && !Next_.valid() && Corpus_.Size()) {  // nothing in the pipe: make them now
      const auto tm = Clock::now();
      Adopt(MakeBatch(Budget(free - Ready_.size())));
      S_.make_ms += secs_since(tm) * 1e3;
    }
    // the next `take` ready testcases, each in a free slot (its tag): taken in
    // bulk, the slots and the executor's descriptors filled on all host threads
    const size_t take = std::min<size_t>(free, Ready_.size());
    while (FreeSlot_.size() < take) {
      FreeSlot_.push_back(Slot_.size());
      Slot_.emplace_back();
    }
    const size_t base = FreeSlot_.size() - take;
    std::vector<TcRef> Refs(Ready_.begin(), Ready_.begin() + (std::ptrdiff_t)take);
    Ready_.erase(Ready_.begin(), Ready_.begin() + (std::ptrdiff_t)take);
    In.resize(take);
    HostPool::Get().For(take, 1024, [&](size_t i) {
      const uint64_t tag = FreeSlot_[base + i];
      const TcRef R = Refs[i];
      Slot_[tag] = R;
      StreamTestcase_t T{R.data(), R.size(), tag};
      if (R.A->Prep.size() == R.A->Count()) {
        T.prep = R.prep();
        T.prep_data = R.prep_data();
        T.prep_size = R.prep_size();
      }
      In[i] = T;
    }, take >= 4096);
    FreeSlot_.resize(base);
    InFlight_ += take;
    const uint64_t want = Budget(Exec_.Lanes() > Ready_.size() ? Exec_.Lanes() - Ready_.size() : 0);
    if (want && Corpus_.Size() && !Next_.valid())
      Next_ = std::async(std::launch::async, &FuzzSession::MakeBatch, this, want);
  }
  std::vector<StreamResult_t> Out;
  const auto tb = Clock::now();
  S_.fill_ms += std::chrono::duration<double, std::milli>(tb - t_step).count();
  size_t Taken = 0;
  const bool ok = Exec_.StreamStep(Target_, In, O_.slice, Out, &Slots_, &Taken);
  S_.run_s += secs_since(tb);
  // testcases the executor did not take go back to the front of the queue
  for (size_t i = In.size(); i-- > Taken;) {
    Ready_.push_front(Slot_[In[i].tag]);
    Slot_[In[i].tag] = TcRef{};
    FreeSlot_.push_back(In[i].tag);
    InFlight_--;
  }
  const auto tw = Clock::now();
  if (Next_.valid()) Adopt(Next_.get());  // before the corpus / mutator change below
  const auto ta = Clock::now();
  S_.produce_wait_ms += std::chrono::duration<double, std::milli>(ta - tw).count();
  if (!ok) return false;
  S_.batches++;
  for (const StreamResult_t &F : Out)
    if (F.tag >= Slot_.size()) return false;
  AccountStep(Out);
  S_.account_ms += secs_since(ta) * 1e3;
  if (X_ && X_->Exchanging() && !MergeCoverage(false)) return false;
  S_.step_ms += secs_since(t_step) * 1e3;
  return true;
}

std::unique_ptr<TcArena> FuzzSession::NewArena() {
  {
    std::lock_guard<std::mutex> g(ArenaPoolMu_);
    if (!ArenaPool_.empty()) {
      std::unique_ptr<TcArena> A = std::move(ArenaPool_.back());
      ArenaPool_.pop_back();
      return A;
    }
  }
  return std::make_unique<TcArena>();
}

void FuzzSession::ReleaseArena(TcArena *A) {
  auto it = Arenas_.find(A);
  if (it == Arenas_.end()) return;
  std::unique_ptr<TcArena> Own = std::move(it->second);
  Arenas_.erase(it);
  Own->Data.clear();
  Own->Off.assign(1, 0);
  Own->Live = 0;
  Own->Prep.clear();
  Own->PrepData.clear();
  Own->PrepOff.assign(1, 0);
  std::lock_guard<std::mutex> g(ArenaPoolMu_);
  if (ArenaPool_.size() < 512) ArenaPool_.push_back(std::move(Own));
}

// The master's bookkeeping of one step's results, in their order (Account for
// each): the counts every result adds are summed on all host threads; only the
// results whose bookkeeping depends on the order (engine errors kept as files,
// crash names not seen yet, new coverage) go through Account one by one. The
// results' slots are freed and their arenas released in bulk.
void FuzzSession::AccountStep(std::vector<StreamResult_t> &Out) {
  const size_t n = Out.size();
  enum : uint8_t { K_SERIAL = 1, K_TIMEOUT = 2, K_CR3 = 4, K_CRASH = 8 };
  std::vector<uint8_t> Kind(n, 0);
  std::vector<TcArena *> Ar(n);
  struct Sum {
    uint64_t retired = 0, timeouts = 0, cr3 = 0, crashes = 0;
  };
  const unsigned T = HostPool::Get().Threads();
  std::vector<Sum> Part(T + 1);
  const bool every = Sample_ != nullptr;  // samples follow the accounting order: all of it serial
  HostPool::Get().For(n, 1024, [&](size_t i) {
    const LaneResult &L = *Out[i].r;
    const TcRef R = Slot_[Out[i].tag];
    Ar[i] = R.A;
    uint8_t k = 0;
    if (every || L.error) {
      k = K_SERIAL;
    } else {
      if (std::holds_alternative<Timedout_t>(L.result)) k |= K_TIMEOUT;
      if (std::holds_alternative<Cr3Change_t>(L.result)) k |= K_CR3;
      if (const Crash_t *C = std::get_if<Crash_t>(&L.result)) {
        k |= K_CRASH;
        if (!C->CrashName.empty() && !CrashNames_.count(C->CrashName)) k = K_SERIAL;  // a new name
      }
      if (!L.new_coverage.empty() && !std::holds_alternative<Timedout_t>(L.result)) k = K_SERIAL;
    }
    Kind[i] = k;
    if (k != K_SERIAL) {
      Sum &s = Part[HostPool::ThreadIndex()];
      s.retired += L.icount;
      s.timeouts += (k & K_TIMEOUT) != 0;
      s.cr3 += (k & K_CR3) != 0;
      s.crashes += (k & K_CRASH) != 0;
    }
  }, n >= 4096);
  // the order-dependent results, in order (counts included: Account adds them)
  uint64_t bulk = 0;
  for (size_t i = 0; i < n; i++) {
    if (Kind[i] != K_SERIAL) {
      bulk++;
      continue;
    }
    const TcRef R = Slot_[Out[i].tag];
    Account(R.data(), R.size(), *Out[i].r, false);
  }
  S_.execs += bulk;
  for (const Sum &s : Part) {
    S_.retired += s.retired;
    S_.timeouts += s.timeouts;
    S_.cr3 += s.cr3;
    S_.crashes += s.crashes;
  }
  // slots back, arenas whose testcases are all accounted released (runs of one arena)
  const size_t fs = FreeSlot_.size();
  FreeSlot_.resize(fs + n);
  HostPool::Get().For(n, 4096, [&](size_t i) {
    Slot_[Out[i].tag] = TcRef{};
    FreeSlot_[fs + i] = Out[i].tag;
  }, n >= 8192);
  InFlight_ -= n;
  for (size_t i = 0; i < n;) {
    size_t j = i + 1;
    while (j < n && Ar[j] == Ar[i]) j++;
    TcArena *A = Ar[i];
    A->Live -= j - i;
    if (A->Live == 0) ReleaseArena(A);  // every testcase of the arena accounted
    i = j;
  }
}

// The master's bookkeeping of one result (server.h:816-886).
void FuzzSession::Account(const uint8_t *Tc, size_t Size, const LaneResult &L, bool KnownCrash) {
  if (Sample_ && S_.execs % std::max<uint64_t>(1, O_.sample_every) == 0) WriteSample(Tc, Size, L);
  S_.execs++;
  S_.retired += L.icount;
  if (L.error) {  // the engine could not finish it: neither a crash nor coverage
    // the first ones are kept under errors/ for triage (engine gaps, not target bugs)
    if (S_.errors < 256) {
      std::error_code ec;
      fs::create_directories(T_ / "errors", ec);
      SaveFile(T_ / "errors" / ("engine-error-" + std::to_string(S_.errors)), Tc, Size);
    }
    S_.errors++;
    S_.error_retired += L.icount;
    return;
  }
  if (std::holds_alternative<Timedout_t>(L.result)) S_.timeouts++;
  if (std::holds_alternative<Cr3Change_t>(L.result)) S_.cr3++;
  if (const Crash_t *C = std::get_if<Crash_t>(&L.result)) {
    S_.crashes++;
    if (!KnownCrash && !C->CrashName.empty()) {
      const auto tc = Clock::now();
      if (CrashNames_.insert(C->CrashName).second) Writer_.Save(T_ / "crashes" / C->CrashName, Tc, Size);
      S_.crashsave_ms += secs_since(tc) * 1e3;
    }
  }
  // a timed-out testcase reports no coverage (the client revokes it,
  // client.cc:122-133); any other result with new coverage, crashes
  // included, joins the corpus after arming the mutator's cross-over
  // (server.h:816-853)
  if (!L.new_coverage.empty() && !std::holds_alternative<Timedout_t>(L.result)) {
    // admitted only if the master's aggregate grows: nodes attribute against
    // their own aggregates, which lack what other nodes found
    const auto tn = Clock::now();
    const size_t Before = Coverage_.size();
    Coverage_.insert(L.new_coverage.begin(), L.new_coverage.end());
    if (Coverage_.size() != Before) {
      Testcase_t Tcase(Tc, Size);
      Mutator_->OnNewCoverage(Tcase);
      LastNewCov_.assign((const char *)Tc, Size);
      HaveNewCov_ = true;
      Corpus_.SaveTestcase(L.result, std::move(Tcase));
    }
    S_.newcov_ms += secs_since(tn) * 1e3;
  }
}

// every shard's coverage map, MAX-reduced over the shards; the
// rips other shards found join this shard's aggregate (so its lanes stop
// reporting them as new). Testcases stay with the shard that found them.
// Deferred by one step (CoverageExchange_t::MergeBegin / MergeEnd): the merge
// a step starts runs while the next step's kernels do, and is absorbed at the
// start of the following merge. Every shard starts one merge per step.
bool FuzzSession::MergeCoverage(bool Done) {
  const auto t = Clock::now();
  if (!AbsorbMerge()) return false;
  uint8_t *Map = nullptr;
  uint64_t Bytes = 0;
  bool Device = false;
  if (!Exec_.CoverageMap(&Map, &Bytes, &Device)) return false;
  // the values outside the map (SURVEY 8(e)'s overflow list): this shard's new ones
  std::vector<uint64_t> Mine;
  Exec_.TakeNewExtra(Mine);
  if (!X_->MergeBegin(Map, Bytes, Device, Mine, Done)) return false;
  MergePending_ = true;
  S_.merge_ms += secs_since(t) * 1e3;
  return true;
}

bool FuzzSession::AbsorbMerge() {
  if (!MergePending_) return true;
  MergePending_ = false;
  const uint8_t *Merged = nullptr;
  uint64_t Bytes = 0;
  std::vector<uint64_t> All;
  bool Every = false;
  if (!X_->MergeEnd(&Merged, &Bytes, All, &Every)) return false;
  uint8_t *Map = nullptr;
  uint64_t MapBytes = 0;
  bool Device = false;
  if (!Exec_.CoverageMap(&Map, &MapBytes, &Device)) return false;
  if (Bytes && Bytes == MapBytes) S_.merged_rips += Exec_.MergeCoverageMap(Merged, Bytes, Device);
  S_.merged_rips += Exec_.AbsorbExtra(All);
  S_.merges++;
  S_.merged_map_bytes += Bytes;
  AllDone_ = Every;
  return true;
}

bool FuzzSession::FinishMerge() {
  const auto t = Clock::now();
  const bool ok = AbsorbMerge();
  S_.merge_ms += secs_since(t) * 1e3;
  return ok;
}

// ---- CoverageExchange_t's default deferred merge: the synchronous collectives
bool CoverageExchange_t::MergeBegin(const uint8_t *Map, uint64_t Bytes, bool Device,
                                    const std::vector<uint64_t> &Extras, bool Done) {
  if (Device) return false;  // device maps: an exchange with its own MergeBegin (RCCL)
  merged_.assign(Map, Map + Bytes);
  merged_device_ = false;
  if (Bytes && !AllReduceMax(merged_.data(), Bytes, false)) return false;
  std::vector<uint64_t> Block(1 + blocks_.Cap()), Blocks;
  Block.resize(blocks_.Pack(Extras, Done, Block.data()));
  if (!AllGatherV(Block, Blocks)) return false;
  return MergeBlocks::Unpack(Blocks.data(), Blocks.size(), (uint64_t)World(), 0, kMergeCap, merged_extra_,
                             &merged_done_);
}

bool CoverageExchange_t::MergeEnd(const uint8_t **Merged, uint64_t *Bytes, std::vector<uint64_t> &AllExtras,
                                  bool *AllDone) {
  *Merged = merged_.data();
  *Bytes = merged_.size();
  AllExtras.swap(merged_extra_);
  merged_extra_.clear();
  *AllDone = merged_done_;
  return true;
}

// user + system CPU time of the process so far (all threads): with wall_s,
// how busy the host cores were
static double ProcessCpuSeconds() {
  struct rusage u {};
  getrusage(RUSAGE_SELF, &u);
  return (double)u.ru_utime.tv_sec + u.ru_utime.tv_usec * 1e-6 + (double)u.ru_stime.tv_sec + u.ru_stime.tv_usec * 1e-6;
}

std::string FuzzSession::SummaryJson() const {
  const double Wall = WallSeconds();
  char b[2048];
  snprintf(b, sizeof(b),
           "{\"mode\":\"fuzz\",\"target\":\"%s\",\"lanes\":%u,\"rank\":%d,\"world\":%d,\"batches\":%llu,"
           "\"execs\":%llu,\"retired\":%llu,\"wall_s\":%.6f,\"run_s\":%.6f,\"execs_per_s\":%.3f,"
           "\"instr_per_s\":%.3f,\"coverage\":%zu,\"corpus\":%zu,\"crashes\":%llu,\"unique_crashes\":%zu,"
           "\"timeouts\":%llu,\"cr3\":%llu,\"errors\":%llu,\"error_retired\":%llu,\"merged_rips\":%llu,"
           "\"merges\":%llu,\"merged_map_bytes\":%llu,"
           "\"merge_ms\":%.3f,\"produce_wait_ms\":%.3f,\"account_ms\":%.3f,\"make_ms\":%.3f,\"step_ms\":%.3f,\"fill_ms\":%.3f,"
           "\"newcov_ms\":%.3f,\"crashsave_ms\":%.3f,\"call_ms\":%.3f,\"cpu_s\":%.3f,\"mutate_cpu_ms\":%.3f,"
           "\"backend\":",
           O_.name.c_str(), Exec_.Lanes(), X_ ? X_->Rank() : 0, X_ ? X_->World() : 1,
           (unsigned long long)S_.batches, (unsigned long long)S_.execs, (unsigned long long)S_.retired, Wall,
           S_.run_s, S_.run_s > 0 ? S_.execs / S_.run_s : 0.0, S_.run_s > 0 ? S_.retired / S_.run_s : 0.0,
           Exec_.CoverageSize(), Corpus_.Size(), (unsigned long long)S_.crashes, CrashNames_.size(),
           (unsigned long long)S_.timeouts, (unsigned long long)S_.cr3, (unsigned long long)S_.errors,
           (unsigned long long)S_.error_retired, (unsigned long long)S_.merged_rips,
           (unsigned long long)S_.merges, (unsigned long long)S_.merged_map_bytes, S_.merge_ms, S_.produce_wait_ms,
           S_.account_ms, S_.make_ms, S_.step_ms, S_.fill_ms, S_.newcov_ms, S_.crashsave_ms, S_.call_ms, ProcessCpuSeconds(),
           MutateCpuNs_.load() * 1e-6);
  return std::string(b) + Exec_.StatsJson() + "}";
}

}  // namespace wtfgpu_host
