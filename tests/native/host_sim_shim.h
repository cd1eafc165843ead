// host_sim_shim.h — TEST INFRASTRUCTURE ONLY. Lets g++ compile the device
// headers (wtf_amd/csrc/engine_*.h) for the host so one lane of the interpreter
// can be stepped on the CPU next to the oracle when debugging a divergence.
// Never part of the product: libwtfgpu.so is always the hipcc gfx950 build.
#pragma once
#include <cstdint>
#include <cstring>
#define __device__
#define __host__
#define __global__
#define __forceinline__ inline
#define __noinline__
#define __constant__
#define __shared__
struct uint4 { uint32_t x, y, z, w; };
static inline uint32_t __builtin_amdgcn_readfirstlane(uint32_t v) { return v; }
static inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
static inline unsigned long long __umul64hi(unsigned long long a, unsigned long long b) {
  return (unsigned long long)(((unsigned __int128)a * b) >> 64);
}
static inline long long __mul64hi(long long a, long long b) { return (long long)(((__int128)a * b) >> 64); }
