// unimpl_hist.h — which opcodes ended testcases as UNIMPLEMENTED engine errors
// (wtfgpu_exit_t.opcode: the instruction's first four bytes). Keyed by the
// opcode after the legacy / REX prefixes: one-byte opcodes 0x00-0xff, 0f xx as
// 0x100 + xx (c4 / c5 VEX and the 0f 38 / 0f 3a maps keep their first byte).
// Diagnostic only (the bench line and the twin report it).
#pragma once
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>
#include <algorithm>

struct UnimplHist {
  std::atomic<uint64_t> n[512] = {};
  // the first kRaw exits' four opcode bytes as they were (diagnostic)
  static constexpr uint32_t kRaw = 96;
  std::atomic<uint32_t> nraw{0};
  uint32_t raw[kRaw] = {};
  static uint32_t key(uint32_t opbytes) {
    for (int i = 0; i < 4; i++) {
      const uint32_t b = (opbytes >> (8 * i)) & 0xff;
      const bool pfx = b == 0x66 || b == 0x67 || b == 0xf0 || b == 0xf2 || b == 0xf3 || b == 0x26 || b == 0x2e ||
                       b == 0x36 || b == 0x3e || b == 0x64 || b == 0x65 || (b & 0xf0) == 0x40;
      if (pfx) continue;
      if (b == 0x0f && i < 3) {
        const uint32_t c = (opbytes >> (8 * (i + 1))) & 0xff;
        return 0x100 + c;
      }
      return b;
    }
    return 0x1ff;
  }
  void add(uint32_t opbytes) {
    n[key(opbytes)].fetch_add(1, std::memory_order_relaxed);
    const uint32_t i = nraw.fetch_add(1, std::memory_order_relaxed);
    if (i < kRaw) raw[i] = opbytes;
  }
  // ["c4e27d18",...]: the sampled exits' bytes in memory order
  std::string raw_json() const {
    std::string s = "[";
    char buf[16];
    const uint32_t m = std::min<uint32_t>(nraw.load(), kRaw);
    for (uint32_t i = 0; i < m; i++) {
      snprintf(buf, sizeof(buf), "%s\"%02x%02x%02x%02x\"", i ? "," : "", raw[i] & 0xff, (raw[i] >> 8) & 0xff,
               (raw[i] >> 16) & 0xff, raw[i] >> 24);
      s += buf;
    }
    return s + "]";
  }
  // {"d9":12,"0f58":3,...}: the `top` most frequent keys
  std::string json(size_t top = 16) const {
    std::vector<std::pair<uint64_t, uint32_t>> v;
    for (uint32_t k = 0; k < 512; k++)
      if (const uint64_t c = n[k].load()) v.emplace_back(c, k);
    std::sort(v.begin(), v.end(), [](auto &a, auto &b) { return a.first > b.first || (a.first == b.first && a.second < b.second); });
    std::string s = "{";
    char buf[48];
    for (size_t i = 0; i < v.size() && i < top; i++) {
      snprintf(buf, sizeof(buf), "%s\"%s%02x\":%llu", i ? "," : "", v[i].second >= 0x100 ? "0f" : "",
               v[i].second & 0xff, (unsigned long long)v[i].first);
      s += buf;
    }
    return s + "}";
  }
};
