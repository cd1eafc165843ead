// wire.cc — see wire.h.
#include "wire.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

namespace wtfgpu_host::wire {

void Writer::Result(const TestcaseResult_t &R) {
  U8((uint8_t)R.index());  // yas std::variant: u8 index, then the alternative (socket.h:84-89)
  if (const Crash_t *C = std::get_if<Crash_t>(&R)) Str(C->CrashName.data(), C->CrashName.size());
}

TestcaseResult_t Reader::Result() {
  switch (U8()) {
    case 0: return Ok_t();
    case 1: return Timedout_t();
    case 2: return Cr3Change_t();
    case 3: return Crash_t(Str());
    default: Ok = false; return Ok_t();
  }
}

std::string EncodeTestcase(const uint8_t *Data, size_t Size) {
  Writer W;
  W.Str(Data, Size);
  return std::move(W.B);
}

bool DecodeTestcase(const std::string &Msg, std::string &Testcase) {
  Reader R(Msg.data(), Msg.size());
  Testcase = R.Str();
  return R.Done();
}

std::string EncodeResult(const uint8_t *Testcase, size_t Size, const std::vector<uint64_t> &Coverage,
                         const TestcaseResult_t &Result) {
  Writer W;
  W.Str(Testcase, Size);
  W.Set(Coverage);
  W.Result(Result);
  return std::move(W.B);
}

bool DecodeResult(const std::string &Msg, std::string &Testcase, std::vector<uint64_t> &Coverage,
                  TestcaseResult_t &Result) {
  Reader R(Msg.data(), Msg.size());
  Testcase = R.Str();
  Coverage = R.Set();
  Result = R.Result();
  return R.Done();
}

std::string EncodeHello(uint64_t Lanes) {
  Writer W;
  W.Str(kHello, strlen(kHello));
  W.U64(Lanes);
  return std::move(W.B);
}

bool DecodeHello(const std::string &Msg, uint64_t &Lanes) {
  Reader R(Msg.data(), Msg.size());
  const std::string H = R.Str();
  Lanes = R.U64();
  return R.Done() && H == kHello && Lanes > 0;
}

std::string EncodeBatch(const std::vector<std::pair<const uint8_t *, size_t>> &Testcases) {
  Writer W;
  size_t Total = 8;
  for (const auto &T : Testcases) Total += 8 + T.second;
  W.B.reserve(Total);
  W.U64(Testcases.size());
  for (const auto &T : Testcases) W.Str(T.first, T.second);
  return std::move(W.B);
}

bool DecodeBatch(const std::string &Msg, std::vector<std::string> &Testcases) {
  Reader R(Msg.data(), Msg.size());
  const uint64_t N = R.U64();
  if (!R.Ok || N > Msg.size() / 8) return false;
  Testcases.resize(N);
  for (uint64_t i = 0; i < N && R.Ok; i++) Testcases[i] = R.Str();
  return R.Done();
}

std::string EncodeBatchResult(const std::vector<WireResult> &Results) {
  Writer W;
  W.U64(Results.size());
  for (const WireResult &X : Results) {
    W.Set(X.Coverage);
    W.Result(X.Result);
    W.U64(X.Retired);
    W.U8(X.Error ? 1 : 0);
  }
  return std::move(W.B);
}

bool DecodeBatchResult(const std::string &Msg, std::vector<WireResult> &Results) {
  Reader R(Msg.data(), Msg.size());
  const uint64_t N = R.U64();
  if (!R.Ok || N > Msg.size() / 8) return false;
  Results.resize(N);
  for (uint64_t i = 0; i < N && R.Ok; i++) {
    Results[i].Coverage = R.Set();
    Results[i].Result = R.Result();
    Results[i].Retired = R.U64();
    Results[i].Error = R.U8() != 0;
  }
  return R.Done();
}

// ------------------------------------------------------------------ sockets
namespace {

struct Addr {
  bool Tcp = true;
  sockaddr_in In{};
  sockaddr_un Un{};
  const sockaddr *Ptr() const { return Tcp ? (const sockaddr *)&In : (const sockaddr *)&Un; }
  socklen_t Len() const { return Tcp ? sizeof(In) : sizeof(Un); }
};

// SockAddrFromString (socket.cc:76-160)
bool parse(const std::string &Address, Addr &A) {
  const size_t P = Address.find("://");
  if (P == std::string::npos) {
    printf("The address %s is malformed.\n", Address.c_str());
    return false;
  }
  const std::string Proto = Address.substr(0, P);
  std::string Rest = Address.substr(P + 3);
  if (!Rest.empty() && Rest.back() == '/') Rest.pop_back();
  if (Proto == "tcp") {
    const size_t C = Rest.rfind(':');
    if (C == std::string::npos) return false;
    A.Tcp = true;
    A.In.sin_family = AF_INET;
    A.In.sin_port = htons((uint16_t)atoi(Rest.c_str() + C + 1));
    return inet_pton(AF_INET, Rest.substr(0, C).c_str(), &A.In.sin_addr) == 1;
  }
  if (Proto == "unix") {
    A.Tcp = false;
    A.Un.sun_family = AF_UNIX;
    if (Rest.size() >= sizeof(A.Un.sun_path)) return false;
    memcpy(A.Un.sun_path, Rest.c_str(), Rest.size() + 1);
    return true;
  }
  printf("Protocol %s is not supported.\n", Proto.c_str());
  return false;
}

bool all(int Fd, const void *P, size_t N, bool Send) {
  char *B = (char *)P;
  while (N) {
    const ssize_t R = Send ? send(Fd, B, N, MSG_NOSIGNAL) : recv(Fd, B, N, 0);
    if (R <= 0) return false;
    B += R;
    N -= (size_t)R;
  }
  return true;
}

}  // namespace

int Listen(const std::string &Address) {
  Addr A;
  if (!parse(Address, A)) return -1;
  const int Fd = socket(A.Tcp ? AF_INET : AF_UNIX, SOCK_STREAM, 0);
  if (Fd < 0) return -1;
  const int One = 1;
  if (A.Tcp) setsockopt(Fd, SOL_SOCKET, SO_REUSEADDR, &One, sizeof(One));
  else unlink(A.Un.sun_path);
  if (bind(Fd, A.Ptr(), A.Len()) != 0 || listen(Fd, 64) != 0) {
    close(Fd);
    return -1;
  }
  return Fd;
}

int Accept(int ListenFd) {
  const int Fd = accept(ListenFd, nullptr, nullptr);
  if (Fd >= 0) {
    const int One = 1;
    setsockopt(Fd, IPPROTO_TCP, TCP_NODELAY, &One, sizeof(One));  // harmless on unix sockets
  }
  return Fd;
}

int Dial(const std::string &Address) {
  Addr A;
  if (!parse(Address, A)) return -1;
  const int Fd = socket(A.Tcp ? AF_INET : AF_UNIX, SOCK_STREAM, 0);
  if (Fd < 0) return -1;
  if (A.Tcp) {
    const int One = 1;
    setsockopt(Fd, IPPROTO_TCP, TCP_NODELAY, &One, sizeof(One));  // socket.cc:292-300
  }
  if (connect(Fd, A.Ptr(), A.Len()) != 0) {
    close(Fd);
    return -1;
  }
  return Fd;
}

bool SendFrame(int Fd, const std::string &Msg) {
  if (Msg.size() > 0xffffffffull) return false;
  const uint32_t N = (uint32_t)Msg.size();
  return all(Fd, &N, 4, true) && all(Fd, Msg.data(), Msg.size(), true);
}

bool ReceiveFrame(int Fd, std::string &Msg, uint64_t MaxBytes) {
  uint32_t N = 0;
  if (!all(Fd, &N, 4, false)) return false;
  if (N > MaxBytes) return false;  // as the reference's Receive rejects frames beyond its buffer (socket.cc:335-340)
  Msg.resize(N);
  return all(Fd, Msg.data(), N, false);
}

void Close(int Fd) {
  if (Fd >= 0) close(Fd);
}

}  // namespace wtfgpu_host::wire
