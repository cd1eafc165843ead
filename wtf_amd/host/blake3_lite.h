// blake3_lite.h — BLAKE3 in hash mode (the only mode wtf uses), written from the
// BLAKE3 specification: 7-round compression over 16-word blocks, 1 KiB chunks,
// binary Merkle tree with PARENT nodes, ROOT-flag extendable output.
// Used by the gpu backend's Rdrand (bochscpu_backend.cc:874-885, BLAKE3 1.2.0
// vendored at src/libs/BLAKE3); pinned by the reference's official test vectors
// (tests/golden/blake3_vectors.json, from src/libs/BLAKE3/test_vectors).
#pragma once
#include <cstddef>
#include <cstdint>

namespace wtfgpu_host {

// out_len bytes of the BLAKE3 hash of in[0..len)
void blake3_hash(const uint8_t *in, size_t len, uint8_t *out, size_t out_len);

// Rdrand as wtf defines it: h = blake3(le64(seed))[0..16]; seed = h[0..8];
// returns h[8..16].
uint64_t wtf_rdrand(uint64_t &seed);

}  // namespace wtfgpu_host

extern "C" void wtfhost_blake3(const uint8_t *in, size_t len, uint8_t *out, size_t out_len);
