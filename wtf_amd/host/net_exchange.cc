// net_exchange.cc — CoverageExchange_t over TCP for shards without a GPU
// collective (the oracle twin, CPU tests): rank 0 listens on host:port, the
// other ranks connect; an all-reduce is a gather to rank 0, a byte-wise MAX
// and a broadcast back. The GPU node uses RCCL instead (rccl_exchange.cc).
// Framing follows the reference's socket protocol (u32 little-endian length,
// socket.cc:310-358), one frame per map.
#include "net_exchange.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

namespace wtfgpu_host {

namespace {
bool send_all(int fd, const void *p, size_t n) {
  const uint8_t *b = (const uint8_t *)p;
  while (n) {
    const ssize_t w = send(fd, b, n, MSG_NOSIGNAL);
    if (w <= 0) return false;
    b += w;
    n -= (size_t)w;
  }
  return true;
}
bool recv_all(int fd, void *p, size_t n) {
  uint8_t *b = (uint8_t *)p;
  while (n) {
    const ssize_t r = recv(fd, b, n, 0);
    if (r <= 0) return false;
    b += r;
    n -= (size_t)r;
  }
  return true;
}
bool send_frame(int fd, const uint8_t *p, uint64_t n) {
  const uint32_t len = (uint32_t)n;
  return n <= 0xffffffffull && send_all(fd, &len, 4) && send_all(fd, p, n);
}
bool recv_frame(int fd, std::vector<uint8_t> &out) {
  uint32_t len = 0;
  if (!recv_all(fd, &len, 4)) return false;
  out.resize(len);
  return recv_all(fd, out.data(), len);
}
void nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}
}  // namespace

TcpExchange_t::~TcpExchange_t() {
  for (int fd : peers_)
    if (fd >= 0) close(fd);
  if (listen_ >= 0) close(listen_);
}

bool TcpExchange_t::Connect(const std::string &Host, uint16_t Port, double TimeoutS) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(Port);
  if (inet_pton(AF_INET, Host.c_str(), &a.sin_addr) != 1) return false;
  if (world_ <= 1) return true;
  if (rank_ == 0) {
    listen_ = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(listen_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (bind(listen_, (sockaddr *)&a, sizeof(a)) || listen(listen_, world_)) {
      perror("TcpExchange_t: bind/listen");
      return false;
    }
    peers_.assign(world_, -1);
    for (int i = 1; i < world_; i++) {
      const int fd = accept(listen_, nullptr, nullptr);
      int32_t r = -1;
      if (fd < 0 || !recv_all(fd, &r, 4) || r <= 0 || r >= world_ || peers_[r] >= 0) return false;
      nodelay(fd);
      peers_[r] = fd;
    }
    return true;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (connect(fd, (sockaddr *)&a, sizeof(a)) == 0) {
      nodelay(fd);
      const int32_t r = rank_;
      if (!send_all(fd, &r, 4)) return false;
      peers_.assign(1, fd);
      return true;
    }
    close(fd);
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > TimeoutS) return false;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

bool TcpExchange_t::AllReduceMax(uint8_t *Map, uint64_t Bytes, bool Device) {
  if (Device) return false;  // host maps only
  if (world_ <= 1) return true;
  std::vector<uint8_t> buf;
  if (rank_ != 0) {
    return send_frame(peers_[0], Map, Bytes) && recv_frame(peers_[0], buf) && buf.size() == Bytes &&
           (memcpy(Map, buf.data(), Bytes), true);
  }
  for (int r = 1; r < world_; r++) {  // rank order: the result does not depend on arrival order
    if (!recv_frame(peers_[r], buf) || buf.size() != Bytes) return false;
    for (uint64_t i = 0; i < Bytes; i++) Map[i] = std::max(Map[i], buf[i]);
  }
  for (int r = 1; r < world_; r++)
    if (!send_frame(peers_[r], Map, Bytes)) return false;
  return true;
}

bool TcpExchange_t::AllDone(bool Mine, bool *All) {
  uint8_t notdone = Mine ? 0 : 1;
  if (!AllReduceMax(&notdone, 1, false)) return false;
  *All = notdone == 0;
  return true;
}

// rank 0 concatenates every rank's list in rank order and sends it back
bool TcpExchange_t::AllGatherV(const std::vector<uint64_t> &Mine, std::vector<uint64_t> &All) {
  All = Mine;
  if (world_ <= 1) return true;
  std::vector<uint8_t> buf;
  if (rank_ != 0) {
    if (!send_frame(peers_[0], (const uint8_t *)Mine.data(), Mine.size() * 8) || !recv_frame(peers_[0], buf) ||
        buf.size() % 8)
      return false;
    All.resize(buf.size() / 8);
    if (!buf.empty()) memcpy(All.data(), buf.data(), buf.size());
    return true;
  }
  for (int r = 1; r < world_; r++) {
    if (!recv_frame(peers_[r], buf) || buf.size() % 8) return false;
    const size_t at = All.size();
    All.resize(at + buf.size() / 8);
    if (!buf.empty()) memcpy(All.data() + at, buf.data(), buf.size());
  }
  for (int r = 1; r < world_; r++)
    if (!send_frame(peers_[r], (const uint8_t *)All.data(), All.size() * 8)) return false;
  return true;
}

}  // namespace wtfgpu_host
