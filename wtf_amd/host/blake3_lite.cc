// blake3_lite.cc — see blake3_lite.h.
#include "blake3_lite.h"

#include <array>
#include <cstring>
#include <vector>

namespace wtfgpu_host {

namespace {
constexpr uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                             0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
constexpr int kPerm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum : uint32_t { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };
constexpr size_t kBlock = 64, kChunk = 1024;

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

inline void g(uint32_t *s, int a, int b, int c, int d, uint32_t x, uint32_t y) {
  s[a] = s[a] + s[b] + x;
  s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + y;
  s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr(s[b] ^ s[c], 7);
}

// Full 16-word compression output.
void compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter, uint32_t blen, uint32_t flags,
              uint32_t out[16]) {
  uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    kIV[0], kIV[1], kIV[2], kIV[3], (uint32_t)counter, (uint32_t)(counter >> 32), blen, flags};
  uint32_t m[16];
  memcpy(m, block, sizeof(m));
  for (int r = 0; r < 7; r++) {
    g(s, 0, 4, 8, 12, m[0], m[1]);
    g(s, 1, 5, 9, 13, m[2], m[3]);
    g(s, 2, 6, 10, 14, m[4], m[5]);
    g(s, 3, 7, 11, 15, m[6], m[7]);
    g(s, 0, 5, 10, 15, m[8], m[9]);
    g(s, 1, 6, 11, 12, m[10], m[11]);
    g(s, 2, 7, 8, 13, m[12], m[13]);
    g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      uint32_t t[16];
      for (int i = 0; i < 16; i++) t[i] = m[kPerm[i]];
      memcpy(m, t, sizeof(m));
    }
  }
  for (int i = 0; i < 8; i++) {
    out[i] = s[i] ^ s[i + 8];
    out[i + 8] = s[i + 8] ^ cv[i];
  }
}

void load_block(const uint8_t *p, size_t n, uint32_t w[16]) {
  uint8_t b[kBlock] = {0};
  if (n) memcpy(b, p, n);  // an empty input may come with a null pointer
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)b[4 * i] | (uint32_t)b[4 * i + 1] << 8 | (uint32_t)b[4 * i + 2] << 16 |
           (uint32_t)b[4 * i + 3] << 24;
}

// The node whose output is extended at the root.
struct Node {
  uint32_t cv[8];
  uint32_t block[16];
  uint64_t counter;
  uint32_t blen, flags;
};

// Runs a chunk up to (not including) its last block; returns that last block as a node.
Node chunk_node(const uint8_t *p, size_t n, uint64_t chunk_index) {
  uint32_t cv[8];
  memcpy(cv, kIV, sizeof(cv));
  size_t nblocks = n == 0 ? 1 : (n + kBlock - 1) / kBlock;
  for (size_t b = 0; b + 1 < nblocks; b++) {
    uint32_t w[16], out[16];
    load_block(p + b * kBlock, kBlock, w);
    compress(cv, w, chunk_index, kBlock, b == 0 ? CHUNK_START : 0, out);
    memcpy(cv, out, sizeof(cv));
  }
  Node nd;
  memcpy(nd.cv, cv, sizeof(cv));
  const size_t last = (nblocks - 1) * kBlock;
  nd.blen = (uint32_t)(n - last);
  load_block(p + last, nd.blen, nd.block);
  nd.counter = chunk_index;
  nd.flags = CHUNK_END | (nblocks == 1 ? CHUNK_START : 0);
  return nd;
}

void node_cv(const Node &nd, uint32_t cv[8]) {
  uint32_t out[16];
  compress(nd.cv, nd.block, nd.counter, nd.blen, nd.flags, out);
  memcpy(cv, out, 8 * sizeof(uint32_t));
}

Node parent_node(const uint32_t l[8], const uint32_t r[8]) {
  Node nd;
  memcpy(nd.cv, kIV, sizeof(nd.cv));
  memcpy(nd.block, l, 32);
  memcpy(nd.block + 8, r, 32);
  nd.counter = 0;
  nd.blen = kBlock;
  nd.flags = PARENT;
  return nd;
}
}  // namespace

void blake3_hash(const uint8_t *in, size_t len, uint8_t *out, size_t out_len) {
  const uint64_t nchunks = len == 0 ? 1 : (len + kChunk - 1) / kChunk;
  // CV stack merge: after chunk i (not the last) push its CV, then merge while
  // the number of completed chunks has trailing zero bits.
  std::vector<std::array<uint32_t, 8>> stack;
  Node root{};
  for (uint64_t c = 0; c < nchunks; c++) {
    const size_t off = c * kChunk, n = len - off < kChunk ? len - off : kChunk;
    Node nd = chunk_node(in + off, len ? n : 0, c);
    if (c + 1 == nchunks) {
      // fold the stack into the last chunk from the right
      Node cur = nd;
      while (!stack.empty()) {
        uint32_t rcv[8];
        node_cv(cur, rcv);
        cur = parent_node(stack.back().data(), rcv);
        stack.pop_back();
      }
      root = cur;
      break;
    }
    std::array<uint32_t, 8> cv;
    node_cv(nd, cv.data());
    uint64_t total = c + 1;
    while ((total & 1) == 0) {
      Node p = parent_node(stack.back().data(), cv.data());
      stack.pop_back();
      node_cv(p, cv.data());
      total >>= 1;
    }
    stack.push_back(cv);
  }
  // root output, 64 bytes per counter value
  for (uint64_t blk = 0; out_len > 0; blk++) {
    uint32_t w[16];
    compress(root.cv, root.block, blk, root.blen, root.flags | ROOT, w);
    uint8_t bytes[64];
    for (int i = 0; i < 16; i++)
      for (int k = 0; k < 4; k++) bytes[4 * i + k] = (uint8_t)(w[i] >> (8 * k));
    const size_t n = out_len < 64 ? out_len : 64;
    memcpy(out, bytes, n);
    out += n;
    out_len -= n;
  }
}

uint64_t wtf_rdrand(uint64_t &seed) {
  uint8_t in[8], h[16];
  memcpy(in, &seed, 8);
  blake3_hash(in, 8, h, 16);
  uint64_t lo, hi;
  memcpy(&lo, h, 8);
  memcpy(&hi, h + 8, 8);
  seed = lo;
  return hi;
}

}  // namespace wtfgpu_host

extern "C" void wtfhost_blake3(const uint8_t *in, size_t len, uint8_t *out, size_t out_len) {
  wtfgpu_host::blake3_hash(in, len, out, out_len);
}
