// Host-logic checker driver (TEST INFRASTRUCTURE ONLY, never linked into the
// product). One source, built twice by oracle/Makefile:
//   * oracle/_ref/ref_hostcheck: against the reference's own host sources where
//     they lie under /root/reference/src (utils.cc, mutator.cc, FuzzerMutate.cpp,
//     fuzzer_tlv_server.cc, ...; target `ref`);
//   * oracle/hostcheck: against this repository's restatements (libwtfhost.a,
//     -DWTF_AMD_HOST).
// tests/test_host_parity.py compares the two outputs, and both against the
// fixtures tests/golden/gen_host_fixtures.py recorded from the reference build.
// Subcommands:
//
//   cpustate <regs.json>
//       LoadCpuStateFromJSON + SanitizeCpuState (src/wtf/utils.cc:57-258):
//       "OK <0|1>" then one "<field> <hex>" line per CpuState_t field.
//   mutate <libfuzzer|tlv_server> <seed> <maxlen> <count> <newcov_every> <file>...
//       std::mt19937_64 Rng(seed) (server.h:339), Corpus_t over the files in
//       order (corpus.h:56-87, no outputs dir), Mutator = the target's
//       CreateMutator (fuzzer_tlv_server.cc:204-365) or LibfuzzerMutator_t
//       (mutator.cc:8-54, targets.h:25); `count` GetNewTestcase calls, each
//       printed as "T <hex>"; every `newcov_every`-th output (1-based, 0 =
//       never) is fed back through OnNewCoverage (server.h:816-853), which
//       arms libFuzzer's CrossOver.
//   mutate-grow <...same...>  as mutate, and every `newcov_every`-th output
//       also joins the corpus (this repository only: the tlv mutator's
//       parsed-testcase cache over a growing corpus)
//   merge-blocks <cap> <world> <step>...
//       (this repository: merge_block.h) each step is one token per rank,
//       "<n><d|->" joined by ',': rank r queues n new overflow values
//       (r << 32 | running index) and says done with 'd'. Every rank packs
//       its block, the blocks are read back in rank order as the collective
//       delivers them (fixed stride, as RCCL does), and each step prints
//       "S <all done 0|1> <values...>" (hex)
//   blake3 <hexbytes>
//       Blake3HexDigest (utils.cc) of the bytes.
// This repository's build only (the reference exposes neither as a function
// it can link without bochscpu):
//   xof <hexbytes> <outlen>   BLAKE3 extended output (pinned by the official
//                             test vectors, src/libs/BLAKE3/test_vectors)
//   rdrand <seed> <n>         n values of the Rdrand chain from seed
//                             (BochscpuBackend_t::Rdrand, bochscpu_backend.cc:874-885)
//   kdmp <dump> [gva...]      wtf_amd/host/kdmp.cc in oracle/ref_kdmp_dump.cc's
//                             output format (TYPE / CR3 / RIP / PAGE / VT lines),
//                             for comparison with oracle/_ref/kdmp_ref
//   tlv-feed <file>           each testcase of <file> (u32 length + bytes, repeated)
//                             deserialized as fuzzer_tlv_server's InsertTestcase
//                             does (fuzzer_tlv_server.cc:36-40, 67-75; this
//                             repository: TlvServer::TestcaseFeed) and printed as
//                             its packet chunks "F <hex>" (u32 Size, u32 Command,
//                             u16 Id, u16 BodySize, Body), or "F -" when it does
//                             not deserialize (the reference throws)
// Both builds (the reference through yas and socket.h's serializers, this
// repository through wtf_amd/host/wire.cc):
//   wire-testcase <hex>       the master's Testcase message (server.h:720-737)
//   wire-result <hex> <idx> <crashname|-> [rip...]
//                             the client's Result message (client.cc:187-200):
//                             testcase, coverage set, TestcaseResult_t
//   wire-decode <hex>         a Result message decoded: TC / RES / COV lines
//                             (COV sorted)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <memory>
#include <random>
#include <string>
#include <vector>

#ifdef WTF_AMD_HOST
#include "../wtf_amd/host/blake3_lite.h"
#include "../wtf_amd/host/merge_block.h"
#include "../wtf_amd/host/kdmp.h"
#include "../wtf_amd/host/wire.h"
#include "../wtf_amd/host/wtf_api.h"
#else
#include "socket.h"
#include "backend.h"
#include "corpus.h"
#include "mutator.h"
#include "targets.h"
#include "utils.h"
#endif

static std::vector<uint8_t> read_all(const char *path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

static void hexline(const char *tag, const std::string &s) {
  printf("%s ", tag);
  for (unsigned char c : s) printf("%02x", c);
  printf("\n");
}

static int cmd_cpustate(const char *path) {
  CpuState_t S{};
  if (!LoadCpuStateFromJSON(S, path)) {
    printf("LOAD_FAIL\n");
    return 1;
  }
  const bool ok = SanitizeCpuState(S);
  printf("OK %d\n", ok ? 1 : 0);
#define P(name, v) printf(name " %llx\n", (unsigned long long)(v))
  P("rax", S.Rax); P("rbx", S.Rbx); P("rcx", S.Rcx); P("rdx", S.Rdx);
  P("rsi", S.Rsi); P("rdi", S.Rdi); P("rip", S.Rip); P("rsp", S.Rsp);
  P("rbp", S.Rbp); P("r8", S.R8); P("r9", S.R9); P("r10", S.R10);
  P("r11", S.R11); P("r12", S.R12); P("r13", S.R13); P("r14", S.R14);
  P("r15", S.R15); P("rflags", S.Rflags); P("tsc", S.Tsc);
  P("apic_base", S.ApicBase); P("sysenter_cs", S.SysenterCs);
  P("sysenter_esp", S.SysenterEsp); P("sysenter_eip", S.SysenterEip);
  P("pat", S.Pat); P("efer", S.Efer.Flags); P("star", S.Star);
  P("lstar", S.Lstar); P("cstar", S.Cstar); P("sfmask", S.Sfmask);
  P("kernel_gs_base", S.KernelGsBase); P("tsc_aux", S.TscAux);
  P("fpcw", S.Fpcw); P("fpsw", S.Fpsw); P("fptw", S.Fptw); P("fpop", S.Fpop);
  P("cr0", S.Cr0.Flags); P("cr2", S.Cr2); P("cr3", S.Cr3); P("cr4", S.Cr4.Flags);
  P("cr8", S.Cr8); P("xcr0", S.Xcr0); P("dr0", S.Dr0); P("dr1", S.Dr1);
  P("dr2", S.Dr2); P("dr3", S.Dr3); P("dr6", S.Dr6); P("dr7", S.Dr7);
  P("mxcsr", S.Mxcsr); P("mxcsr_mask", S.MxcsrMask);
  P("gdtr.base", S.Gdtr.Base); P("gdtr.limit", S.Gdtr.Limit);
  P("idtr.base", S.Idtr.Base); P("idtr.limit", S.Idtr.Limit);
  const Seg_t *segs[] = {&S.Es, &S.Cs, &S.Ss, &S.Ds, &S.Fs, &S.Gs, &S.Tr, &S.Ldtr};
  const char *names[] = {"es", "cs", "ss", "ds", "fs", "gs", "tr", "ldtr"};
  for (int i = 0; i < 8; i++)
    printf("%s %x %x %llx %x %x\n", names[i], (unsigned)segs[i]->Present, (unsigned)segs[i]->Selector,
           (unsigned long long)segs[i]->Base, (unsigned)segs[i]->Limit, (unsigned)segs[i]->Attr);
  for (int i = 0; i < 8; i++) printf("fpst%d %llx\n", i, (unsigned long long)S.Fpst[i]);
#undef P
  return 0;
}

#ifdef WTF_AMD_HOST
namespace TlvServer {
bool TestcaseFeedBytes(const uint8_t *Buffer, const size_t BufferSize, std::vector<uint8_t> &Feed);
}  // namespace TlvServer
#else
namespace TlvServer {  // the reference's types (fuzzer_tlv_server.cc:23-34), same layout
struct Packet_t {
  uint32_t Command;
  uint16_t Id;
  uint16_t BodySize;
  std::vector<uint8_t> Body;
};
struct Packets_t {
  std::vector<Packet_t> Packets;
};
Packets_t Deserialize(const uint8_t *Buffer, const size_t BufferSize);
}  // namespace TlvServer
#endif

static int cmd_tlv_feed(const char *path) {
  const auto all = read_all(path);
  for (size_t o = 0; o + 4 <= all.size();) {
    uint32_t n;
    memcpy(&n, &all[o], 4);
    if (o + 4 + n > all.size()) return 1;
    const uint8_t *tc = all.data() + o + 4;
    o += 4 + n;
    std::vector<uint8_t> Feed;
    bool ok = true;
#ifdef WTF_AMD_HOST
    ok = TlvServer::TestcaseFeedBytes(tc, n, Feed);
#else
    try {
      const TlvServer::Packets_t P = TlvServer::Deserialize(tc, n);
      for (const TlvServer::Packet_t &Pk : P.Packets) {
        const uint32_t Size = uint32_t(8 + Pk.Body.size());
        const size_t At = Feed.size();
        Feed.resize(At + 4 + Size);
        uint8_t *Q = Feed.data() + At;
        memcpy(Q, &Size, 4);
        memcpy(Q + 4, &Pk.Command, 4);
        memcpy(Q + 8, &Pk.Id, 2);
        memcpy(Q + 10, &Pk.BodySize, 2);
        if (!Pk.Body.empty()) memcpy(Q + 12, Pk.Body.data(), Pk.Body.size());
      }
    } catch (const std::exception &) {
      ok = false;
    }
#endif
    if (!ok) {
      printf("F -\n");
      continue;
    }
    printf("F ");
    for (uint8_t c : Feed) printf("%02x", c);
    printf("\n");
  }
  return 0;
}

static int cmd_mutate(int argc, char **argv, bool grow = false) {
  if (argc < 7) return 2;
  const std::string name = argv[2];
  std::mt19937_64 Rng(strtoull(argv[3], nullptr, 0));
  const size_t maxlen = strtoull(argv[4], nullptr, 0);
  const size_t count = strtoull(argv[5], nullptr, 0);
  const size_t every = strtoull(argv[6], nullptr, 0);
  Corpus_t Corpus("", Rng);
  for (int i = 7; i < argc; i++) {
    const auto b = read_all(argv[i]);
    Corpus.SaveTestcase(Ok_t(), Testcase_t(b.data(), b.size()));
  }
  std::unique_ptr<Mutator_t> M;
  if (name == "libfuzzer") {
    M = LibfuzzerMutator_t::Create(Rng, maxlen);
  } else {
    Target_t *T = Targets_t::Instance().Get(name);
    if (!T) return 3;
    M = T->CreateMutator(Rng, maxlen);
  }
  for (size_t i = 1; i <= count; i++) {
    std::string s = M->GetNewTestcase(Corpus);
    hexline("T", s);
    if (every && i % every == 0) {
      M->OnNewCoverage(Testcase_t((const uint8_t *)s.data(), s.size()));
      if (grow) Corpus.SaveTestcase(Ok_t(), Testcase_t((const uint8_t *)s.data(), s.size()));
    }
  }
  return 0;
}

#ifdef WTF_AMD_HOST
// tlv-prep <seed> <count>: the tlv mutator over a corpus that grows every 64th
// output; each output's PrepareInsert feed (the mutator's own, handed over
// without a parse) against TestcaseFeedBytes (the JSON parsed back), and a
// truncated copy (parsed). Prints "P <testcases> <mismatches>".
static int cmd_tlv_prep(int argc, char **argv) {
  if (argc != 4) return 2;
  std::mt19937_64 Rng(strtoull(argv[2], nullptr, 0));
  const size_t count = strtoull(argv[3], nullptr, 0);
  Corpus_t Corpus("", Rng);
  const std::string seed = "{\"Packets\":[{\"Body\":[65,66,67],\"BodySize\":3,\"Command\":0,\"Id\":0}]}";
  Corpus.SaveTestcase(Ok_t(), Testcase_t((const uint8_t *)seed.data(), seed.size()));
  Target_t *T = Targets_t::Instance().Get("tlv_server");
  if (!T || !T->PrepareInsert) return 3;
  auto M = T->CreateMutator(Rng, 4096);
  size_t bad = 0;
  std::vector<uint8_t> A, B;
  for (size_t i = 1; i <= count; i++) {
    const std::string s = M->GetNewTestcase(Corpus);
    const auto *d = (const uint8_t *)s.data();
    const bool pa = T->PrepareInsert(d, s.size(), A) == PreparedInsert_t::Feed;
    const bool pb = TlvServer::TestcaseFeedBytes(d, s.size(), B);
    if (pa != pb || (pa && A != B)) bad++;
    const size_t cut = s.size() / 2;  // not the mutator's bytes: parsed (and refused)
    const bool qa = T->PrepareInsert(d, cut, A) == PreparedInsert_t::Feed;
    const bool qb = TlvServer::TestcaseFeedBytes(d, cut, B);
    if (qa != qb || (qa && A != B)) bad++;
    if (i % 64 == 0) Corpus.SaveTestcase(Ok_t(), Testcase_t(d, s.size()));
  }
  printf("P %zu %zu\n", count, bad);
  return bad ? 1 : 0;
}

static int cmd_merge_blocks(int argc, char **argv) {
  if (argc < 4) return 2;
  const uint64_t cap = strtoull(argv[2], nullptr, 0), world = strtoull(argv[3], nullptr, 0);
  std::vector<wtfgpu_host::MergeBlocks> ranks;
  for (uint64_t r = 0; r < world; r++) ranks.emplace_back(cap);
  std::vector<uint64_t> next(world, 0);
  for (int a = 4; a < argc; a++) {
    std::vector<uint64_t> blocks(world * (1 + cap), 0);
    const char *p = argv[a];
    for (uint64_t r = 0; r < world; r++) {
      char *e = nullptr;
      const uint64_t n = strtoull(p, &e, 10);
      const bool done = *e == 'd';
      p = e + 1;
      if (*p == ',') p++;
      std::vector<uint64_t> mine;
      for (uint64_t i = 0; i < n; i++) mine.push_back(r << 32 | next[r]++);
      ranks[r].Pack(mine, done, &blocks[r * (1 + cap)]);
    }
    std::vector<uint64_t> all;
    bool every = false;
    if (!wtfgpu_host::MergeBlocks::Unpack(blocks.data(), blocks.size(), world, 1 + cap, cap, all, &every)) {
      printf("BAD\n");
      return 1;
    }
    printf("S %d", every ? 1 : 0);
    for (uint64_t v : all) printf(" %llx", (unsigned long long)v);
    printf("\n");
  }
  return 0;
}

#endif

static std::vector<uint8_t> unhex(const char *p) {
  std::vector<uint8_t> b;
  for (; p[0] && p[1]; p += 2) b.push_back((uint8_t)strtoul(std::string(p, 2).c_str(), nullptr, 16));
  return b;
}

static TestcaseResult_t result_of(int idx, const char *name) {
  switch (idx) {
    case 0: return Ok_t();
    case 1: return Timedout_t();
    case 2: return Cr3Change_t();
    default: return Crash_t(std::string(name) == "-" ? "" : name);
  }
}

static std::string bytes_hex(const std::string &s) {
  std::string o;
  char b[3];
  for (unsigned char c : s) {
    snprintf(b, sizeof(b), "%02x", c);
    o += b;
  }
  return o;
}

static int cmd_wire(int argc, char **argv) {
  const std::string cmd = argv[1];
  const auto tc = unhex(argv[2]);
  const std::string T(tc.begin(), tc.end());
  if (cmd == "wire-testcase") {
#ifdef WTF_AMD_HOST
    printf("%s\n", bytes_hex(wtfgpu_host::wire::EncodeTestcase(tc.data(), tc.size())).c_str());
#else
    yas::mem_ostream Os;
    yas::binary_oarchive<decltype(Os), YasFlags> Oa(Os);
    Oa &T;
    const auto &Buf = Os.get_intrusive_buffer();
    printf("%s\n", bytes_hex(std::string(Buf.data, Buf.size)).c_str());
#endif
    return 0;
  }
  if (cmd == "wire-result" && argc >= 5) {
    const TestcaseResult_t R = result_of(atoi(argv[3]), argv[4]);
    std::vector<uint64_t> Cov;
    for (int i = 5; i < argc; i++) Cov.push_back(strtoull(argv[i], nullptr, 0));
#ifdef WTF_AMD_HOST
    printf("%s\n", bytes_hex(wtfgpu_host::wire::EncodeResult(tc.data(), tc.size(), Cov, R)).c_str());
#else
    tsl::robin_set<Gva_t> Set;
    for (uint64_t g : Cov) Set.emplace(Gva_t(g));
    yas::mem_ostream Os;
    yas::binary_oarchive<decltype(Os), YasFlags> Oa(Os);
    Oa &T &Set &R;
    const auto &Buf = Os.get_intrusive_buffer();
    printf("%s\n", bytes_hex(std::string(Buf.data, Buf.size)).c_str());
#endif
    return 0;
  }
  if (cmd == "wire-decode") {
    std::string Tc;
    std::vector<uint64_t> Cov;
    TestcaseResult_t R;
#ifdef WTF_AMD_HOST
    if (!wtfgpu_host::wire::DecodeResult(T, Tc, Cov, R)) return 1;
#else
    tsl::robin_set<Gva_t> Set;
    yas::mem_istream Is(tc.data(), tc.size());
    yas::binary_iarchive<decltype(Is), YasFlags> Ia(Is);
    Ia &Tc &Set &R;
    for (const Gva_t &g : Set) Cov.push_back(g.U64());
#endif
    std::sort(Cov.begin(), Cov.end());
    printf("TC %s\nRES %zu %s\nCOV", bytes_hex(Tc).c_str(), R.index(),
           std::holds_alternative<Crash_t>(R) ? std::get<Crash_t>(R).CrashName.c_str() : "");
    for (uint64_t g : Cov) printf(" %llx", (unsigned long long)g);
    printf("\n");
    return 0;
  }
  return 2;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const std::string cmd = argv[1];
  if (cmd.rfind("wire-", 0) == 0 && argc >= 3) return cmd_wire(argc, argv);
  if (cmd == "tlv-feed" && argc == 3) return cmd_tlv_feed(argv[2]);
#ifdef WTF_AMD_HOST
  if (cmd == "tlv-prep") return cmd_tlv_prep(argc, argv);
#endif
#ifdef WTF_AMD_HOST
  if (cmd == "xof" && argc == 4) {
    const auto b = unhex(argv[2]);
    std::vector<uint8_t> o(strtoull(argv[3], nullptr, 0));
    wtfgpu_host::blake3_hash(b.data(), b.size(), o.data(), o.size());
    for (uint8_t c : o) printf("%02x", c);
    printf("\n");
    return 0;
  }
  if (cmd == "kdmp" && argc >= 3) {
    wtfgpu_host::KernelDump D;
    if (!D.Parse(argv[2])) {
      printf("PARSE_FAIL\n");
      return 1;
    }
    auto fnv = [](const uint8_t *p) {
      uint64_t h = 1469598103934665603ULL;
      for (size_t i = 0; i < 4096; i++) h = (h ^ p[i]) * 1099511628211ULL;
      return h;
    };
    printf("TYPE %u\nCR3 %llx\nRIP %llx\n", D.DumpType(), (unsigned long long)D.DirectoryTableBase(),
           (unsigned long long)D.ContextRip());
    for (const auto &[gpfn, page] : D.Pages())
      printf("PAGE %llx %llx\n", (unsigned long long)(gpfn << 12), (unsigned long long)fnv(page));
    for (int i = 3; i < argc; i++) {
      const uint64_t gva = strtoull(argv[i], nullptr, 0);
      const auto gpa = D.VirtTranslate(gva);
      if (gpa) printf("VT %llx %llx\n", (unsigned long long)gva, (unsigned long long)*gpa);
      else printf("VT %llx -1\n", (unsigned long long)gva);
    }
    return 0;
  }
  if (cmd == "rdrand" && argc == 4) {
    uint64_t seed = strtoull(argv[2], nullptr, 0);
    for (uint64_t i = 0, n = strtoull(argv[3], nullptr, 0); i < n; i++)
      printf("%016llx\n", (unsigned long long)wtfgpu_host::wtf_rdrand(seed));
    return 0;
  }
#endif
  if (cmd == "cpustate" && argc == 3) return cmd_cpustate(argv[2]);
  if (cmd == "mutate") return cmd_mutate(argc, argv);
  if (cmd == "mutate-grow") return cmd_mutate(argc, argv, true);
#ifdef WTF_AMD_HOST
  if (cmd == "merge-blocks") return cmd_merge_blocks(argc, argv);
#endif
  if (cmd == "blake3" && argc == 3) {
    const auto b = unhex(argv[2]);
    printf("%s\n", Blake3HexDigest(b.data(), b.size()).c_str());
    return 0;
  }
  return 2;
}
