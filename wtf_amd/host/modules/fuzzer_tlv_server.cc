// fuzzer_tlv_server.cc — the tlv_server fuzzer module (src/wtf/fuzzer_tlv_server.cc),
// written against this repository's wtf interface. Behaviour follows the
// reference module:
//  * a testcase is a JSON list of packets {Command, Id, BodySize, Body}
//    (:27-40); InsertTestcase queues them (:67-75);
//  * ProcessPacket breakpoint (:83-166): no packet left -> Stop(Ok); else the
//    next packet is written so that it ends at the end of the packet page
//    (rcx + 0x1000 - size, the guard page catches over-reads), rdx = size;
//    a packet of 0x1000 bytes or more ends the testcase;
//  * return-address breakpoint (:171-179): registers back to the snapshot's
//    so the receive loop calls ProcessPacket again;
//  * printf breakpoint (:184-189): skipped (return 0);
//  * the three handlers are also declared as data (BreakpointAction_t; the
//    packets as Feed chunks at insert): the gpu backend applies them on the
//    device, other backends run the handlers;
//  * user-mode crash detection (:191-194);
//  * the custom mutator (:204-365): Generate 1..10 packets one time in five,
//    otherwise insert / copy-field / delete on a corpus testcase.
// The only changes for batched execution are on GlobalState: it is declared
// thread_local and named with WTF_LANE_STATE_TLS (module_slots.h), and it holds
// only the per-testcase packet queue (the snapshot registers moved out: they
// are read-only after Init). The packet queue is per testcase, so per lane,
// and lanes are serviced on several host threads at once. A backend that
// takes the packets as a Feed (SetFeed true) leaves the queue empty.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../json_lite.h"
#include "../wtf_api.h"
#include "crash_detection_umode.h"

namespace TlvServer {

struct Packet_t {
  uint32_t Command = 0;
  uint16_t Id = 0;
  uint16_t BodySize = 0;
  std::vector<uint8_t> Body;
};

// Fast path of Deserialize for the canonical form the mutator writes (the
// nlohmann dump() of Packets_t: no whitespace, unsigned integers, each packet
// key once): parsed in place, no document tree. Anything else -> false, and
// the general parser below decides. Both give the same packets.
namespace {
struct Cursor {
  const char *p, *e;
  bool lit(const char *s) {
    const size_t n = strlen(s);
    if ((size_t)(e - p) < n || memcmp(p, s, n)) return false;
    p += n;
    return true;
  }
  bool num(uint64_t &v) {
    const char *s = p;
    v = 0;
    while (p < e && *p >= '0' && *p <= '9' && p - s < 19) v = v * 10 + uint64_t(*p++ - '0');
    return p > s && (p == e || *p < '0' || *p > '9') && !(*s == '0' && p - s > 1);
  }
};
}  // namespace

bool FastDeserialize(const uint8_t *Buffer, const size_t BufferSize, std::vector<Packet_t> &Out) {
  Cursor C{(const char *)Buffer, (const char *)Buffer + BufferSize};
  if (!C.lit("{\"Packets\":[")) return false;
  if (C.lit("]}")) return C.p == C.e;
  for (;;) {
    Packet_t P;
    unsigned seen = 0;
    if (!C.lit("{")) return false;
    for (;;) {
      uint64_t v;
      if (C.lit("\"Body\":[")) {
        if (seen & 1) return false;
        seen |= 1;
        if (!C.lit("]")) {
          for (;;) {
            if (!C.num(v)) return false;
            P.Body.push_back((uint8_t)v);
            if (C.lit("]")) break;
            if (!C.lit(",")) return false;
          }
        }
      } else if (C.lit("\"BodySize\":")) {
        if ((seen & 2) || !C.num(v)) return false;
        seen |= 2, P.BodySize = (uint16_t)v;
      } else if (C.lit("\"Command\":")) {
        if ((seen & 4) || !C.num(v)) return false;
        seen |= 4, P.Command = (uint32_t)v;
      } else if (C.lit("\"Id\":")) {
        if ((seen & 8) || !C.num(v)) return false;
        seen |= 8, P.Id = (uint16_t)v;
      } else {
        return false;
      }
      if (C.lit("}")) break;
      if (!C.lit(",")) return false;
    }
    if (seen != 15) return false;
    Out.push_back(std::move(P));
    if (C.lit("]}")) return C.p == C.e;
    if (!C.lit(",")) return false;
  }
}

// JSON testcase -> packets (nlohmann get<>: integers are cast to the field type)
bool Deserialize(const uint8_t *Buffer, const size_t BufferSize, std::vector<Packet_t> &Out) {
  Out.clear();
  if (FastDeserialize(Buffer, BufferSize, Out)) return true;
  Out.clear();
  try {
    const jsonl::Value Root = jsonl::parse(Buffer, BufferSize);
    for (const jsonl::Value &P : Root.at("Packets").array()) {
      Packet_t Pk;
      Pk.Command = (uint32_t)P.at("Command").num_u64();
      Pk.Id = (uint16_t)P.at("Id").num_u64();
      Pk.BodySize = (uint16_t)P.at("BodySize").num_u64();
      for (const jsonl::Value &B : P.at("Body").array()) Pk.Body.push_back((uint8_t)B.num_u64());
      Out.push_back(std::move(Pk));
    }
  } catch (const std::exception &) {
    return false;
  }
  return true;
}

// packets -> JSON as nlohmann's dump() writes it (sorted keys, no spaces).
// Written into one preallocated buffer with a digit table (the mutator calls
// it for every testcase: the node's hottest host loop), same bytes as
// appending std::to_string of each field.
namespace {
struct Digits {
  char s[256][4];
  uint8_t n[256];
  Digits() {
    for (int v = 0; v < 256; v++) n[v] = (uint8_t)snprintf(s[v], sizeof(s[v]), "%d", v);
  }
};
const Digits kDigits;
inline char *PutU64(char *o, uint64_t v) {
  char t[20];
  int n = 0;
  do {
    t[n++] = char('0' + v % 10);
    v /= 10;
  } while (v);
  while (n) *o++ = t[--n];
  return o;
}
inline char *PutLit(char *o, const char *s, size_t n) {
  memcpy(o, s, n);
  return o + n;
}
}  // namespace

std::string Serialize(const std::vector<Packet_t> &Packets) {
  size_t Cap = 16;
  for (const Packet_t &P : Packets) Cap += 72 + 4 * P.Body.size();
  std::string S(Cap, '\0');
  char *o = S.data();
  o = PutLit(o, "{\"Packets\":[", 12);
  for (size_t i = 0; i < Packets.size(); i++) {
    const Packet_t &P = Packets[i];
    if (i) *o++ = ',';
    o = PutLit(o, "{\"Body\":[", 9);
    for (size_t j = 0; j < P.Body.size(); j++) {
      if (j) *o++ = ',';
      const uint8_t b = P.Body[j];
      memcpy(o, kDigits.s[b], 4);  // the table entry is 4 bytes; only n of them count
      o += kDigits.n[b];
    }
    o = PutLit(o, "],\"BodySize\":", 13);
    o = PutU64(o, P.BodySize);
    o = PutLit(o, ",\"Command\":", 11);
    o = PutU64(o, P.Command);
    o = PutLit(o, ",\"Id\":", 6);
    o = PutU64(o, P.Id);
    *o++ = '}';
  }
  o = PutLit(o, "]}", 2);
  S.resize((size_t)(o - S.data()));
  return S;
}

// The snapshot's registers (Init): read-only once set, so kept out of the
// per-testcase state (the reference keeps both in one GlobalState,
// fuzzer_tlv_server.cc:42-65).
CpuState_t Context;
void RestoreGprs(Backend_t *B) {
  const CpuState_t &C = Context;
  B->Rsp(C.Rsp), B->Rip(C.Rip), B->Rax(C.Rax), B->Rbx(C.Rbx), B->Rcx(C.Rcx), B->Rdx(C.Rdx);
  B->Rsi(C.Rsi), B->Rdi(C.Rdi), B->R8(C.R8), B->R9(C.R9), B->R10(C.R10), B->R11(C.R11);
  B->R12(C.R12), B->R13(C.R13), B->R14(C.R14), B->R15(C.R15);
}

// The packet queue (the reference's std::deque, :42-65) as a vector and a head
// index: ModuleSlots swaps it in and out around every call for a lane, and a
// vector moves without allocating (a deque's move constructor allocates).
struct PacketQueue {
  std::vector<Packet_t> Items;
  size_t Head = 0;
  bool empty() const { return Head == Items.size(); }
  const Packet_t &front() const { return Items[Head]; }
  void pop_front() {
    if (++Head == Items.size()) clear();
  }
  void clear() {
    Items.clear();
    Head = 0;
  }
  void emplace_back(Packet_t &&P) { Items.emplace_back(std::move(P)); }
};

thread_local struct {
  PacketQueue Packets;
} GlobalState;
WTF_LANE_STATE_TLS(GlobalState);

// FastDeserialize's grammar, written straight into the Feed layout
// InsertTestcase hands the backend (per packet: u32 Size, u32 Command, u16 Id,
// u16 BodySize, Body): no Packet_t vectors. Same acceptance and the same bytes
// as FastDeserialize + the loop in InsertTestcase; false -> that path decides.
// `Out` must hold BufferSize bytes (a packet takes at least as many JSON
// characters as Feed bytes).
namespace {
inline bool Lit(const char *&p, const char *e, const char *s, size_t n) {
  if ((size_t)(e - p) < n || memcmp(p, s, n)) return false;
  p += n;
  return true;
}
// JSON forbids leading zeros ("007"): such a number goes to the general parser
inline bool Num(const char *&p, const char *e, uint64_t &v) {
  const char *s = p;
  v = 0;
  while (p < e && (unsigned)(*p - '0') < 10 && p - s < 19) v = v * 10 + uint64_t(*p++ - '0');
  return p > s && (p == e || (unsigned)(*p - '0') >= 10) && !(*s == '0' && p - s > 1);
}
}  // namespace

bool FastFeed(const uint8_t *Buffer, const size_t BufferSize, uint8_t *Out, size_t &OutSize) {
  const char *p = (const char *)Buffer, *e = p + BufferSize;
  uint8_t *o = Out;
  if (!Lit(p, e, "{\"Packets\":[", 12)) return false;
  if (Lit(p, e, "]}", 2)) {
    OutSize = 0;
    return p == e;
  }
  for (;;) {
    if (!Lit(p, e, "{", 1)) return false;
    uint8_t *h = o;  // header, filled once the packet is closed
    uint8_t *be = o + 12;
    uint32_t Command = 0;
    uint16_t Id = 0, BodySize = 0;
    unsigned seen = 0;
    for (;;) {
      uint64_t v;
      if (Lit(p, e, "\"Body\":[", 8)) {
        if (seen & 1) return false;
        seen |= 1;
        if (!Lit(p, e, "]", 1)) {
          for (;;) {
            // 1-3 digits and a separator (the usual byte): no general number loop
            if (e - p >= 4 && (unsigned)(p[0] - '0') < 10) {
              const unsigned d0 = (unsigned)(p[0] - '0'), d1 = (unsigned)(p[1] - '0');
              unsigned n = 1, x = d0;
              if (d1 < 10) {
                if (d0 == 0) return false;
                const unsigned d2 = (unsigned)(p[2] - '0');
                x = x * 10 + d1, n = 2;
                if (d2 < 10) x = x * 10 + d2, n = 3;
              }
              if ((unsigned)(p[n] - '0') >= 10) {
                p += n;
                v = x;
              } else if (!Num(p, e, v)) {
                return false;
              }
            } else if (!Num(p, e, v)) {
              return false;
            }
            *be++ = (uint8_t)v;
            if (p < e && *p == ',') {
              p++;
              continue;
            }
            if (p < e && *p == ']') {
              p++;
              break;
            }
            return false;
          }
        }
      } else if (Lit(p, e, "\"BodySize\":", 11)) {
        if ((seen & 2) || !Num(p, e, v)) return false;
        seen |= 2, BodySize = (uint16_t)v;
      } else if (Lit(p, e, "\"Command\":", 10)) {
        if ((seen & 4) || !Num(p, e, v)) return false;
        seen |= 4, Command = (uint32_t)v;
      } else if (Lit(p, e, "\"Id\":", 5)) {
        if ((seen & 8) || !Num(p, e, v)) return false;
        seen |= 8, Id = (uint16_t)v;
      } else {
        return false;
      }
      if (Lit(p, e, "}", 1)) break;
      if (!Lit(p, e, ",", 1)) return false;
    }
    if (seen != 15) return false;
    const uint32_t Size = uint32_t(8 + (be - (o + 12)));
    memcpy(h, &Size, 4);
    memcpy(h + 4, &Command, 4);
    memcpy(h + 8, &Id, 2);
    memcpy(h + 10, &BodySize, 2);
    o = be;
    if (Lit(p, e, "]}", 2)) {
      OutSize = (size_t)(o - Out);
      return p == e;
    }
    if (!Lit(p, e, ",", 1)) return false;
  }
}

// The Feed of a testcase (the packets InsertTestcase queues, as the chunks
// OnProcessPacket writes: u32 Size, u32 Command, u16 Id, u16 BodySize, Body),
// canonical JSON parsed straight into it; `Packets` is filled only when the
// general parser ran. false: the testcase does not deserialize.
bool TestcaseFeed(const uint8_t *Buffer, const size_t BufferSize, std::vector<uint8_t> &Feed,
                  std::vector<Packet_t> &Packets) {
  Packets.clear();
  Feed.resize(BufferSize + 16);
  size_t FeedSize = 0;
  if (FastFeed(Buffer, BufferSize, Feed.data(), FeedSize)) {
    Feed.resize(FeedSize);
    return true;
  }
  Feed.clear();
  if (!Deserialize(Buffer, BufferSize, Packets)) return false;
  for (const Packet_t &P : Packets) {
    const uint32_t Size = uint32_t(sizeof(P.Command) + sizeof(P.Id) + sizeof(P.BodySize) + P.Body.size());
    const size_t At = Feed.size();
    Feed.resize(At + 4 + Size);
    uint8_t *Q = Feed.data() + At;
    memcpy(Q, &Size, 4);
    memcpy(Q + 4, &P.Command, 4);
    memcpy(Q + 8, &P.Id, 2);
    memcpy(Q + 10, &P.BodySize, 2);
    if (!P.Body.empty()) memcpy(Q + 12, P.Body.data(), P.Body.size());
  }
  return true;
}

// TestcaseFeed without the packets (oracle/hostcheck.cc tlv-feed)
bool TestcaseFeedBytes(const uint8_t *Buffer, const size_t BufferSize, std::vector<uint8_t> &Feed) {
  std::vector<Packet_t> Packets;
  return TestcaseFeed(Buffer, BufferSize, Feed, Packets);
}

bool InsertTestcase(const uint8_t *Buffer, const size_t BufferSize) {
  GlobalState.Packets.clear();
  thread_local std::vector<uint8_t> Feed;
  std::vector<Packet_t> Packets;
  if (!TestcaseFeed(Buffer, BufferSize, Feed, Packets)) return false;
  // a backend that serves ProcessPacket from the feed never runs the handler
  // for this testcase: the queue stays empty
  if (g_Backend->SetFeed(Feed.data(), Feed.size())) return true;
  if (Packets.empty() && !Deserialize(Buffer, BufferSize, Packets)) return false;  // the fast path kept none
  for (Packet_t &P : Packets) GlobalState.Packets.emplace_back(std::move(P));
  return true;
}

// InsertTestcase ahead of time (PrepareInsert_t): on a backend that takes the
// feed, InsertTestcase is SetFeed(TestcaseFeed(testcase)) and nothing else (the
// queue it clears is empty after a lane reset)
// The mutator's last testcase on this thread and its feed, written while it
// built the JSON from packets it already held (CustomMutator_t below): a
// PrepareInsert of the same bytes takes that feed instead of parsing the JSON
// back (the parse was half of the node's per-testcase mutation time). Any
// other testcase (a truncated one, a corpus input) is parsed.
namespace {
thread_local struct {
  std::string Json;
  std::vector<uint8_t> Feed;
} LastMutation;
}  // namespace

PreparedInsert_t PrepareInsert(const uint8_t *Buffer, const size_t BufferSize, std::vector<uint8_t> &Out) {
  const auto &M = LastMutation;
  if (BufferSize == M.Json.size() && BufferSize && !memcmp(Buffer, M.Json.data(), BufferSize)) {
    Out.assign(M.Feed.begin(), M.Feed.end());
    return PreparedInsert_t::Feed;
  }
  std::vector<Packet_t> Packets;
  if (!TestcaseFeed(Buffer, BufferSize, Out, Packets)) return PreparedInsert_t::Failed;
  return PreparedInsert_t::Feed;
}

namespace {
// one packet's feed chunk (TestcaseFeed's layout): u32 Size, u32 Command, u16 Id,
// u16 BodySize, Body; Body == nullptr: Len zero bytes
inline void PutChunk(std::vector<uint8_t> &F, uint32_t Command, uint16_t Id, uint16_t BodySize, const uint8_t *Body,
                     uint32_t Len) {
  const size_t At = F.size();
  F.resize(At + 12 + Len);
  uint8_t *Q = F.data() + At;
  const uint32_t Size = 8 + Len;
  memcpy(Q, &Size, 4);
  memcpy(Q + 4, &Command, 4);
  memcpy(Q + 8, &Id, 2);
  memcpy(Q + 10, &BodySize, 2);
  if (Body) memcpy(Q + 12, Body, Len);
  else memset(Q + 12, 0, Len);
}
}  // namespace

void OnProcessPacket(Backend_t *Backend) {
  if (GlobalState.Packets.empty()) return g_Backend->Stop(Ok_t());
  const Packet_t &P = GlobalState.Packets.front();
  const size_t PacketSize = sizeof(P.Command) + sizeof(P.Id) + sizeof(P.BodySize) + P.Body.size();
  if (PacketSize >= 0x1000) {
    GlobalState.Packets.pop_front();
    Backend->Stop(Ok_t());
    printf("This testcase is too big to fit, bailing\n");
    return;
  }
  Backend->Rdx(PacketSize);
  uint64_t Address = Backend->Rcx() + (0x1000 - PacketSize);  // ends at the guard page
  Backend->Rcx(Address);
  if (!Backend->VirtWriteStructDirty(Gva_t(Address), &P.Command)) std::abort();
  Address += sizeof(P.Command);
  if (!Backend->VirtWriteStructDirty(Gva_t(Address), &P.Id)) std::abort();
  Address += sizeof(P.Id);
  if (!Backend->VirtWriteStructDirty(Gva_t(Address), &P.BodySize)) std::abort();
  Address += sizeof(P.BodySize);
  if (!Backend->VirtWriteDirty(Gva_t(Address), P.Body.data(), P.Body.size())) std::abort();
  GlobalState.Packets.pop_front();
}

bool Init(const Options_t &, const CpuState_t &State) {
  Context = State;
  const Gva_t ReturnAddress = Gva_t(g_Backend->VirtRead8(Gva_t(g_Backend->Rsp())));
  if (!g_Backend->SetBreakpoint("tlv_server!ProcessPacket", OnProcessPacket,
                                BreakpointAction_t::Feed(Registers_t::Rcx, Registers_t::Rdx, 0x1000)))
    return false;
  // both handlers below only move registers: their BreakpointAction_t lets the
  // gpu backend apply them on the device (no host round trip per packet)
  if (!g_Backend->SetBreakpoint(
          ReturnAddress, [](Backend_t *) { RestoreGprs(g_Backend); },
          BreakpointAction_t::SetGprs(State))) {
    printf("Failed to SetBreakpoint on the return address.\n");
    return false;
  }
  if (!g_Backend->SetBreakpoint("tlv_server!printf", [](Backend_t *Backend) {
        const std::string Format = Backend->VirtReadString(Backend->GetArgGva(0));
        (void)Format;
        Backend->SimulateReturnFromFunction(0);
      },
      BreakpointAction_t::SimulateReturn(0).AfterReadingString(Registers_t::Rcx))) {
    printf("Failed to SetBreakpoint on printf\n");
    return false;
  }
  if (!SetupUsermodeCrashDetectionHooks()) {
    printf("Failed to SetupUsermodeCrashDetectionHooks\n");
    return false;
  }
  return true;
}

bool Restore() { return true; }

// A corpus testcase as the mutator uses it, parsed once: Deserialize's
// packets, kept as each packet's header fields and its body's JSON text
// ("[65,66]", as Serialize writes it). The mutator then edits packet
// references and writes the result from those texts: no JSON parse, no
// per-packet vectors and no digit loop per mutation (the parse and the
// rewrite were ~1.6 us of the node's ~2.3 us of host work per testcase).
struct ParsedTestcase {
  std::string Bytes;  // the testcase itself: a cache hit compares them
  struct Head {
    uint32_t Command;
    uint16_t Id, BodySize;
  };
  std::vector<Head> Heads;
  std::vector<uint32_t> BodyOff{0};  // body text of packet i: Text[BodyOff[i], BodyOff[i + 1])
  std::string Text;
  std::vector<uint32_t> BinOff{0};  // body bytes of packet i: Bin[BinOff[i], BinOff[i + 1])
  std::string Bin;
};

ParsedTestcase ParseTestcase(const uint8_t *Data, const size_t DataLen) {
  ParsedTestcase P;
  P.Bytes.assign((const char *)Data, DataLen);
  std::vector<Packet_t> Packets;
  Deserialize(Data, DataLen, Packets);
  for (const Packet_t &Pk : Packets) {
    P.Heads.push_back({Pk.Command, Pk.Id, Pk.BodySize});
    P.Text += '[';
    for (size_t j = 0; j < Pk.Body.size(); j++) {
      if (j) P.Text += ',';
      P.Text.append(kDigits.s[Pk.Body[j]], kDigits.n[Pk.Body[j]]);
    }
    P.Text += ']';
    P.BodyOff.push_back((uint32_t)P.Text.size());
    P.Bin.append((const char *)Pk.Body.data(), Pk.Body.size());
    P.BinOff.push_back((uint32_t)P.Bin.size());
  }
  return P;
}

class CustomMutator_t : public Mutator_t {
  std::mt19937_64 &Rng_;
  // corpus testcases parsed so far (the corpus only grows, and its buffers
  // stay where they are; the bytes are compared on every hit all the same)
  std::unordered_map<const uint8_t *, std::unique_ptr<ParsedTestcase>> Parsed_;
  // a packet of the mutated testcase: header fields and whose body it has
  struct Ref {
    uint32_t Command;
    uint16_t Id, BodySize;
    uint32_t Body;
  };
  std::vector<Ref> Refs_;
  // WTF_TLV_MUTATOR_PLAIN=1: every mutation parses and rewrites the testcase
  // as the reference does (tests compare the two streams)
  const bool Plain_ = getenv("WTF_TLV_MUTATOR_PLAIN") != nullptr;

  uint32_t GetUint32(const uint32_t A, const uint32_t B) { return std::uniform_int_distribution<uint32_t>(A, B)(Rng_); }

  // Packets_t with N packets of zero bodies, as Serialize writes it
  std::string Generate() {
    struct G {
      uint32_t Command, Len;
      uint16_t BodySize;
    } Gs[10];
    const uint32_t N = GetUint32(1, 10);
    size_t Cap = 16;
    for (uint32_t Idx = 0; Idx < N; Idx++) {
      G &g = Gs[Idx];
      g.Command = GetUint32(0, 10);
      g.Len = GetUint32(0, 100);
      g.BodySize = (uint16_t)g.Len;
      if (GetUint32(1, 3) == 1) g.BodySize ^= (uint16_t)(1u << GetUint32(0, 15));
      Cap += 72 + 2 * g.Len;
    }
    std::string S(Cap, '\0');
    char *o = S.data();
    o = PutLit(o, "{\"Packets\":[", 12);
    for (uint32_t Idx = 0; Idx < N; Idx++) {
      const G &g = Gs[Idx];
      if (Idx) *o++ = ',';
      o = PutLit(o, "{\"Body\":[", 9);
      if (g.Len) *o++ = '0';
      for (uint32_t j = 1; j < g.Len; j++) {
        o[0] = ',', o[1] = '0';
        o += 2;
      }
      o = PutLit(o, "],\"BodySize\":", 13);
      o = PutU64(o, g.BodySize);
      o = PutLit(o, ",\"Command\":", 11);
      o = PutU64(o, g.Command);
      o = PutLit(o, ",\"Id\":", 6);
      o = PutU64(o, Idx);
      *o++ = '}';
    }
    o = PutLit(o, "]}", 2);
    S.resize((size_t)(o - S.data()));
    std::vector<uint8_t> &F = LastMutation.Feed;
    F.clear();
    for (uint32_t Idx = 0; Idx < N; Idx++) PutChunk(F, Gs[Idx].Command, (uint16_t)Idx, Gs[Idx].BodySize, nullptr, Gs[Idx].Len);
    LastMutation.Json = S;
    return S;
  }

  const ParsedTestcase &Parsed(const Testcase_t &T) {
    std::unique_ptr<ParsedTestcase> &P = Parsed_[T.Buffer_.get()];
    if (!P || P->Bytes.size() != T.BufferSize_ || memcmp(P->Bytes.data(), T.Buffer_.get(), T.BufferSize_))
      P = std::make_unique<ParsedTestcase>(ParseTestcase(T.Buffer_.get(), T.BufferSize_));
    return *P;
  }

  // Mutate below on references to the parsed packets, then written out
  std::string MutateParsed(const ParsedTestcase &P) {
    std::vector<Ref> &R = Refs_;
    R.clear();
    for (uint32_t i = 0; i < P.Heads.size(); i++) R.push_back({P.Heads[i].Command, P.Heads[i].Id, P.Heads[i].BodySize, i});
    switch (GetUint32(0, 2)) {
      case 0:
        if (R.size() <= 10 && !R.empty()) {
          const uint32_t From = GetUint32(0, (uint32_t)R.size() - 1);
          const uint32_t To = GetUint32(0, (uint32_t)R.size());
          const Ref Copy = R[From];
          R.insert(R.begin() + To, Copy);
        }
        break;
      case 1: {
        if (R.empty()) break;
        const uint32_t Src = GetUint32(0, (uint32_t)R.size() - 1);
        const uint32_t Dst = GetUint32(0, (uint32_t)R.size() - 1);
        switch (GetUint32(0, 3)) {
          case 0: R[Dst].Id = R[Src].Id; break;
          case 1: R[Dst].Command = R[Src].Command; break;
          case 2: R[Dst].BodySize = R[Src].BodySize; break;
          case 3: R[Dst].Body = R[Src].Body; break;
        }
        break;
      }
      case 2:
        if (!R.empty()) R.erase(R.begin() + GetUint32(0, (uint32_t)R.size() - 1));
        break;
    }
    size_t Cap = 16;
    for (const Ref &r : R) Cap += 72 + (P.BodyOff[r.Body + 1] - P.BodyOff[r.Body]);
    std::string S(Cap, '\0');
    char *o = S.data();
    o = PutLit(o, "{\"Packets\":[", 12);
    for (size_t i = 0; i < R.size(); i++) {
      const Ref &r = R[i];
      if (i) *o++ = ',';
      o = PutLit(o, "{\"Body\":", 8);
      o = PutLit(o, P.Text.data() + P.BodyOff[r.Body], P.BodyOff[r.Body + 1] - P.BodyOff[r.Body]);
      o = PutLit(o, ",\"BodySize\":", 12);
      o = PutU64(o, r.BodySize);
      o = PutLit(o, ",\"Command\":", 11);
      o = PutU64(o, r.Command);
      o = PutLit(o, ",\"Id\":", 6);
      o = PutU64(o, r.Id);
      *o++ = '}';
    }
    o = PutLit(o, "]}", 2);
    S.resize((size_t)(o - S.data()));
    std::vector<uint8_t> &F = LastMutation.Feed;
    F.clear();
    for (const Ref &r : R)
      PutChunk(F, r.Command, r.Id, r.BodySize, (const uint8_t *)P.Bin.data() + P.BinOff[r.Body],
               P.BinOff[r.Body + 1] - P.BinOff[r.Body]);
    LastMutation.Json = S;
    return S;
  }

  std::string GenerateFromPackets() {
    std::vector<Packet_t> Packets;
    const uint32_t N = GetUint32(1, 10);
    for (uint32_t Idx = 0; Idx < N; Idx++) {
      Packet_t P;
      P.Id = (uint16_t)Idx;
      P.Command = GetUint32(0, 10);
      P.Body.resize(GetUint32(0, 100));
      P.BodySize = (uint16_t)P.Body.size();
      if (GetUint32(1, 3) == 1) P.BodySize ^= (uint16_t)(1u << GetUint32(0, 15));
      Packets.push_back(std::move(P));
    }
    return Serialize(Packets);
  }

  // the reference's Mutate (fuzzer_tlv_server.cc:263-297) on the testcase's own packets
  std::string Mutate(const uint8_t *Data, const size_t DataLen) {
    std::vector<Packet_t> Packets;
    Deserialize(Data, DataLen, Packets);
    switch (GetUint32(0, 2)) {
      case 0:  // insert a copy of a packet somewhere (at most 11 packets)
        if (Packets.size() <= 10 && !Packets.empty()) {
          const uint32_t From = GetUint32(0, (uint32_t)Packets.size() - 1);
          const uint32_t To = GetUint32(0, (uint32_t)Packets.size());
          const Packet_t Copy = Packets[From];
          Packets.insert(Packets.begin() + To, Copy);
        }
        break;
      case 1: {  // copy one field between packets
        if (Packets.empty()) break;
        const uint32_t Src = GetUint32(0, (uint32_t)Packets.size() - 1);
        const uint32_t Dst = GetUint32(0, (uint32_t)Packets.size() - 1);
        switch (GetUint32(0, 3)) {
          case 0: Packets[Dst].Id = Packets[Src].Id; break;
          case 1: Packets[Dst].Command = Packets[Src].Command; break;
          case 2: Packets[Dst].BodySize = Packets[Src].BodySize; break;
          case 3: Packets[Dst].Body = Packets[Src].Body; break;
        }
        break;
      }
      case 2:  // delete a packet
        if (!Packets.empty()) Packets.erase(Packets.begin() + GetUint32(0, (uint32_t)Packets.size() - 1));
        break;
    }
    return Serialize(Packets);
  }

 public:
  CustomMutator_t(std::mt19937_64 &Rng, const size_t) : Rng_(Rng) {}
  static std::unique_ptr<Mutator_t> Create(std::mt19937_64 &Rng, const size_t MaxSize) {
    return std::make_unique<CustomMutator_t>(Rng, MaxSize);
  }
  std::string GetNewTestcase(const Corpus_t &Corpus) override {
    if (GetUint32(1, 5) == 5) return Plain_ ? GenerateFromPackets() : Generate();
    const Testcase_t *T = Corpus.PickTestcase();
    if (!T) {
      printf("The corpus is empty, exiting\n");
      std::abort();
    }
    if (Plain_) return Mutate(T->Buffer_.get(), T->BufferSize_);
    return MutateParsed(Parsed(*T));
  }
};

Target_t TlvServer("tlv_server", Init, InsertTestcase, Restore, CustomMutator_t::Create, PrepareInsert);

}  // namespace TlvServer
