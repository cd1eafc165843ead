// wire.h — the master <-> node protocol.
//
// Framing and encoding are the reference's: every message is a u32 length
// followed by a yas archive in binary, no-header mode (socket.h:124,
// socket.cc:310-358): integers little-endian at full width, a string or set
// as a u64 count then its elements, a TestcaseResult_t variant as a u8 index
// (Ok, Timedout, Cr3Change, Crash) then the alternative (Crash_t: its name).
//
// Reference messages (one testcase per round trip; server.h:720-766,
// client.cc:187-258), so a reference master can drive this node and a
// reference client can serve this master:
//   master -> node   Testcase     : string
//   node   -> master Result       : string testcase, set<u64> coverage, result
// Batched messages (new: N testcases per round trip, one per lane):
//   node   -> master Hello        : string "wtfgpu-batch", u64 lanes
//   master -> node   Batch        : u64 N, N x string
//   node   -> master BatchResult  : u64 N, N x (set<u64> coverage, result,
//                                   u64 retired, u8 engine error)
// A BatchResult lists the results in the Batch's order (the testcases are not
// echoed: the master still holds them).
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "wtf_api.h"

namespace wtfgpu_host::wire {

// yas binary archive writer / reader (the subset the messages use)
struct Writer {
  std::string B;
  void U8(uint8_t V) { B.push_back((char)V); }
  void U64(uint64_t V) { B.append((const char *)&V, 8); }
  void Str(const void *P, size_t N) {
    U64(N);
    B.append((const char *)P, N);
  }
  void Set(const std::vector<uint64_t> &S) {
    U64(S.size());
    for (uint64_t V : S) U64(V);
  }
  void Result(const TestcaseResult_t &R);
};
struct Reader {
  const uint8_t *P, *E;
  bool Ok = true;
  Reader(const void *Data, size_t N) : P((const uint8_t *)Data), E((const uint8_t *)Data + N) {}
  bool Need(size_t N) {
    if ((size_t)(E - P) < N) Ok = false;
    return Ok;
  }
  uint8_t U8() {
    if (!Need(1)) return 0;
    return *P++;
  }
  uint64_t U64() {
    if (!Need(8)) return 0;
    uint64_t V;
    memcpy(&V, P, 8);
    P += 8;
    return V;
  }
  std::string Str() {
    const uint64_t N = U64();
    if (!Need(N)) return {};
    std::string S((const char *)P, N);
    P += N;
    return S;
  }
  std::vector<uint64_t> Set() {
    const uint64_t N = U64();
    std::vector<uint64_t> S;
    if (!Need(N * 8)) return S;
    S.resize(N);
    if (N) memcpy(S.data(), P, N * 8);
    P += N * 8;
    return S;
  }
  TestcaseResult_t Result();
  bool Done() const { return Ok && P == E; }
};

// ---- messages
std::string EncodeTestcase(const uint8_t *Data, size_t Size);
bool DecodeTestcase(const std::string &Msg, std::string &Testcase);
std::string EncodeResult(const uint8_t *Testcase, size_t Size, const std::vector<uint64_t> &Coverage,
                         const TestcaseResult_t &Result);
bool DecodeResult(const std::string &Msg, std::string &Testcase, std::vector<uint64_t> &Coverage,
                  TestcaseResult_t &Result);
constexpr const char *kHello = "wtfgpu-batch";
std::string EncodeHello(uint64_t Lanes);
bool DecodeHello(const std::string &Msg, uint64_t &Lanes);
std::string EncodeBatch(const std::vector<std::pair<const uint8_t *, size_t>> &Testcases);
bool DecodeBatch(const std::string &Msg, std::vector<std::string> &Testcases);
struct WireResult {
  std::vector<uint64_t> Coverage;
  TestcaseResult_t Result;
  uint64_t Retired = 0;
  bool Error = false;
};
std::string EncodeBatchResult(const std::vector<WireResult> &Results);
bool DecodeBatchResult(const std::string &Msg, std::vector<WireResult> &Results);

// ---- sockets (socket.cc): "tcp://ip:port[/]" or "unix://path"
int Listen(const std::string &Address);
int Accept(int ListenFd);
int Dial(const std::string &Address);
bool SendFrame(int Fd, const std::string &Msg);
// false on a closed connection or an error
// A frame longer than MaxBytes is refused (the peer is dropped), so a bad or
// hostile length cannot force a huge allocation.
constexpr uint64_t kMaxFrameBytes = 256ull << 20;
bool ReceiveFrame(int Fd, std::string &Msg, uint64_t MaxBytes = kMaxFrameBytes);
void Close(int Fd);

}  // namespace wtfgpu_host::wire
