// engine_sse.h — the SSE / SSE2 and AVX / AVX2 data-movement subset
// (conventions U22 / U23).
//
// Legacy encodings: the integer and data-movement instructions compilers emit
// for x86-64 at the SSE2 baseline (128-bit moves, scalar / half moves, movd /
// movq, logic, integer add / sub / saturate / compare / min / max / multiply,
// shifts, shuffles, unpacks, packs, mask extraction, ldmxcsr / stmxcsr,
// fences, movnti) plus pshufb and ptest (0f 38 00 / 17). VEX encodings: the
// same operations with three operands at 128 and 256 bits (AVX / AVX2 integer),
// vzeroupper / vzeroall, vpshufb, vptest, vpbroadcastb/w/d/q — what the
// runtime's vectorised memcpy / memset / strlen paths run. A UOp with op
// O_SSE carries the opcode byte in `sub`, the mandatory-prefix class in `bsz`
// (0 none, 1 66, 2 f3, 3 f2), `imm` the imm8, and in `opreg` the map and the
// VEX fields (vex_*). Encodings outside the subset (MMX, floating point, the
// other SSE3+ / AVX opcodes) decode as O_UNIMPL, as in the oracle.
//
// The XMM registers, the YMM upper halves and MXCSR live in the lane's cold
// state (P.full[lane], wtfgpu_regs_t: read_regs / write_regs / restore carry
// them). As in exec(), nothing is committed before every access has
// succeeded: 16- and 32-byte stores probe both ends for write permission
// first, so a fault or a copy-on-write restart never leaves half an operand
// written. Legacy SSE leaves bits 255:128 of a destination alone; VEX.128
// zeroes them.
#pragma once
#include "engine_exec.h"
#include "engine_fp.h"

namespace wtfgpu_dev {

__host__ __device__ inline bool s4_form(u32 map, u32 c, u32 pp, bool vex);  // engine_sse4.h
__host__ __device__ inline bool x42_form(u32 map, u32 c, u32 pp, bool vex);  // engine_ext.h
__host__ __device__ inline u32 ax_form(u32 map, u32 c, u32 pp, bool vex);    // engine_avx2x.h
__host__ __device__ inline u32 kop_bits(u32 map, u32 c, u32 pp, u32 w);       // engine_avx512.h
struct UOp;
__device__ __noinline__ int x42_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next);

struct X128 {
  u64 lo, hi;
};

__device__ __forceinline__ u64 xel(const X128 &v, u32 i, u32 w) {
  const u32 bit = i * w * 8;
  const u64 q = bit >= 64 ? v.hi : v.lo;
  return (q >> (bit & 63)) & szmask(w);
}
__device__ __forceinline__ void xset(X128 &v, u32 i, u32 w, u64 x) {
  const u32 bit = i * w * 8, s = bit & 63;
  const u64 mk = szmask(w) << s;
  if (bit >= 64) v.hi = (v.hi & ~mk) | ((x << s) & mk);
  else v.lo = (v.lo & ~mk) | ((x << s) & mk);
}
__device__ __forceinline__ i64 xsel(const X128 &v, u32 i, u32 w) { return (i64)sext(xel(v, i, w), w); }
__device__ __forceinline__ u64 sat_u(i64 x, u32 w) {
  const i64 hi = (i64)szmask(w);
  return (u64)(x < 0 ? 0 : x > hi ? hi : x);
}
__device__ __forceinline__ u64 sat_s(i64 x, u32 w) {
  const i64 hi = (i64)(szmask(w) >> 1), lo = -hi - 1;
  return (u64)(x < lo ? lo : x > hi ? hi : x) & szmask(w);
}

// UOp::opreg of an O_SSE op: bit 0 VEX, bit 1 VEX.L, bit 2 VEX.W, bits 4-7
// VEX.vvvv, bits 8-12 the opcode map (1 = 0f, 2 = 0f 38), bit 16 a legacy
// 66 / f2 / f3 / REX prefix before the VEX prefix (#UD).
__device__ __forceinline__ u32 vex_map(u32 x) { return (x >> 8) & 31; }

// Decode-time check: is (opcode, prefix class, modrm) inside the subset?
// Register-only / memory-only / VEX.L / VEX.vvvv violations are #UD at
// execution, not here.
__device__ __forceinline__ bool sse_valid(u32 map, u32 c, u32 pc, u32 is_mem, u32 r3) {
  if (fp_form(map, c, pc, false) || s4_form(map, c, pc, false) || x42_form(map, c, pc, false))
    return true;  // engine_ssefp.h, engine_sse4.h, engine_ext.h
  if (map == 2) return pc == 1 && (c == 0x00 || c == 0x17);
  if (c == 0xc3) return pc == 0;
  if (c == 0xae) return pc == 0 && (is_mem ? (r3 == 2 || r3 == 3) : r3 >= 5);
  if (c >= 0x60 && c <= 0x6d) return pc == 1;
  if (c == 0x6e || c == 0x74 || c == 0x75 || c == 0x76 || c == 0xc4 || c == 0xc5) return pc == 1;
  if (c == 0x6f || c == 0x7f || c == 0x7e) return pc == 1 || pc == 2;
  if (c == 0x70) return pc != 0;
  if (c >= 0x71 && c <= 0x73) {
    if (pc != 1) return false;
    if (is_mem) return true;  // #UD at execution
    return c == 0x73 ? (r3 == 2 || r3 == 3 || r3 == 6 || r3 == 7) : (r3 == 2 || r3 == 4 || r3 == 6);
  }
  if (c == 0x10 || c == 0x11) return true;
  if ((c >= 0x12 && c <= 0x17) || c == 0x28 || c == 0x29 || c == 0x2b || c == 0x50 || c == 0xc6 ||
      (c >= 0x54 && c <= 0x57))
    return pc <= 1;
  if (c >= 0xd0)
    return pc == 1 && c != 0xd0 && c != 0xe6 && c != 0xf0 && c != 0xf7 && c != 0xff;
  return false;
}
// U36: the encodings some x86-64 CPU defines. Those the engine
// executes are what cpuid_leaf enumerates (SSE .. SSE4.2, SSSE3, AVX, AVX2,
// AES, PCLMULQDQ, BMI1 / BMI2, ADX, MOVBE, FMA, F16C); the other defined ones (
// AVX-VNNI, AVX-IFMA, AVX-NE-CONVERT, GFNI, VAES / VPCLMULQDQ's 256-bit forms,
// SHA, CET, MOVDIR*, ENQCMD, Key Locker, EVEX, ...) are UNIMPLEMENTED (U45: a
// guest picks its paths from the capture host's CPUID, so they are an engine
// gap, never a crash). Only an encoding no CPU defines (a VEX map other than
// 0f / 0f 38 / 0f 3a, an opcode / prefix pair no extension assigns) is #UD,
// decided from the opcode byte before any ModRM fetch. pp: 0 none, 1 66,
// 2 f3, 3 f2.
__host__ __device__ inline bool vex_defined(u32 map, u32 op, u32 pp) {
  if (map == 1) {
    switch (op) {
      case 0x10: case 0x11: case 0x12: case 0x51: case 0x58: case 0x59: case 0x5a: case 0x5c: case 0x5d:
      case 0x5e: case 0x5f: case 0xc2: case 0xae:
        return true;
      case 0x13: case 0x14: case 0x15: case 0x17: case 0x28: case 0x29: case 0x2b: case 0x2e: case 0x2f:
      case 0x50: case 0x54: case 0x55: case 0x56: case 0x57: case 0xc6:
        return pp <= 1;
      case 0x16: case 0x5b: return pp <= 2;
      case 0x2a: case 0x2c: case 0x2d: return pp >= 2;
      case 0x52: case 0x53: return pp == 0 || pp == 2;
      case 0x6f: case 0x7e: case 0x7f: return pp == 1 || pp == 2;
      case 0x70: case 0xe6: return pp >= 1;
      case 0x77: return pp == 0;
      case 0x7c: case 0x7d: case 0xd0: return pp == 1 || pp == 3;
      case 0xf0: return pp == 3;
      case 0x41: case 0x42: case 0x44: case 0x45: case 0x46: case 0x47: case 0x4a: case 0x4b:
      case 0x90: case 0x91: case 0x98: case 0x99:  // the opmask instructions (AVX-512)
        return pp <= 1;
      case 0x92: case 0x93: return pp != 2;
      default:
        return pp == 1 && ((op >= 0x60 && op <= 0x6e) || (op >= 0x71 && op <= 0x76) || op == 0xc4 || op == 0xc5 ||
                           (op >= 0xd1 && op <= 0xfe));
    }
  }
  if (map == 2) {
    // BMI1 / BMI2, AVX-VNNI-INT8 (50 51), AVX-NE-CONVERT (72 b0 b1), AVX-VNNI-INT16 (d2 d3)
    if (op == 0xf5 || op == 0xf7 || op == 0x50 || op == 0x51 || op == 0xb0 || op == 0xd2 || op == 0xd3) return true;
    if (pp == 0) return op == 0xf2 || op == 0xf3;
    if (pp == 2) return op == 0x72 || op == 0xb1;
    if (pp == 3) return op == 0xf6;
    return op <= 0x0f || op == 0x13 || (op >= 0x16 && op <= 0x1a) || (op >= 0x1c && op <= 0x1e) ||
           (op >= 0x20 && op <= 0x25) || (op >= 0x28 && op <= 0x41) || (op >= 0x45 && op <= 0x47) ||
           (op >= 0x52 && op <= 0x53) || (op >= 0x58 && op <= 0x5a) || op == 0x78 || op == 0x79 || op == 0x8c ||
           op == 0x8e || (op >= 0x90 && op <= 0x93) || (op >= 0x96 && op <= 0x9f) || (op >= 0xa6 && op <= 0xaf) ||
           op == 0xb1 || (op >= 0xb4 && op <= 0xbf) ||
           op == 0xcf || (op >= 0xdb && op <= 0xdf);
  }
  if (map == 3) {
    if (pp == 3) return op == 0xf0;  // rorx
    if (pp != 1) return false;
    return op <= 0x02 || (op >= 0x04 && op <= 0x06) || (op >= 0x08 && op <= 0x0f) || (op >= 0x14 && op <= 0x19) ||
           op == 0x1d || (op >= 0x20 && op <= 0x22) || (op >= 0x30 && op <= 0x33) || op == 0x38 || op == 0x39 ||
           (op >= 0x40 && op <= 0x42) ||
           op == 0x44 || op == 0x46 || (op >= 0x4a && op <= 0x4c) || (op >= 0x60 && op <= 0x63) || op == 0xce ||
           op == 0xcf || op == 0xdf;
  }
  return false;
}
// the legacy 0f 38 (map 2) / 0f 3a (map 3) opcodes, same rule
__host__ __device__ inline bool legacy_3byte_defined(u32 map, u32 op, u32 pfx) {
  if (map == 2) {
    if (pfx == 0 && ((op >= 0xc8 && op <= 0xcd) || op == 0xf0 || op == 0xf1 || op == 0xf6 || op == 0xf9)) return true;
    if (pfx == 2 && (op == 0xf6 || op == 0xf8 || op == 0xd8 || (op >= 0xdc && op <= 0xdf))) return true;
    if (pfx == 3 && (op == 0xf0 || op == 0xf1 || op == 0xf8)) return true;
    if (pfx == 1 && (op == 0x37 || (op >= 0x80 && op <= 0x82) || op == 0xcf || (op >= 0xdb && op <= 0xdf) ||
                     op == 0xf0 || op == 0xf1 || op == 0xf5 || op == 0xf6 || op == 0xf8))
      return true;
    return ((op <= 0x0b || (op >= 0x1c && op <= 0x1e)) && pfx <= 1) ||
           (pfx == 1 && (op == 0x10 || op == 0x14 || op == 0x15 || op == 0x17 || (op >= 0x20 && op <= 0x25) ||
                         (op >= 0x28 && op <= 0x2b) || (op >= 0x30 && op <= 0x35) || (op >= 0x38 && op <= 0x41)));
  }
  if (pfx == 0 && op == 0xcc) return true;  // sha1rnds4
  return (op == 0x0f && pfx <= 1) ||
         (pfx == 1 && ((op >= 0x08 && op <= 0x0e) || (op >= 0x14 && op <= 0x17) || (op >= 0x20 && op <= 0x22) ||
                       (op >= 0x40 && op <= 0x42) || op == 0x44 || (op >= 0x60 && op <= 0x63) || op == 0xce ||
                       op == 0xcf || op == 0xdf));
}

__device__ __forceinline__ bool vex_valid(u32 map, u32 c, u32 pp, u32 is_mem, u32 r3) {
  if (fp_form(map, c, pp, true) || s4_form(map, c, pp, true) || x42_form(map, c, pp, true) || ax_form(map, c, pp, true))
    return true;  // engine_ssefp.h, engine_sse4.h, engine_ext.h, engine_avx2x.h
  if (kop_bits(map, c, pp, 0) || kop_bits(map, c, pp, 1)) return true;  // engine_avx512.h (W checked there)
  if (map == 2) return pp == 1 && (c == 0x00 || c == 0x17 || c == 0x58 || c == 0x59 || c == 0x78 || c == 0x79);
  if (map != 1) return false;
  if (c == 0x77) return pp == 0;
  if (c == 0xc3 || c == 0xae) return false;  // movnti has no VEX form; vldmxcsr / vstmxcsr are outside the subset
  return sse_valid(1, c, pp, is_mem, r3);
}

// element-wise ops on w-byte elements
enum : u32 { EW_ADD, EW_SUB, EW_ADDUS, EW_SUBUS, EW_ADDS, EW_SUBS, EW_MINU, EW_MAXU, EW_MINS, EW_MAXS, EW_EQ,
             EW_GT, EW_AVG, EW_MULLO, EW_MULHS, EW_MULHU };
__device__ __noinline__ X128 sse_ewise(u32 k, u32 w, X128 a, X128 b) {
  X128 r{0, 0};
  for (u32 i = 0; i < 16 / w; i++) {
    const u64 x = xel(a, i, w), y = xel(b, i, w);
    const i64 sx = xsel(a, i, w), sy = xsel(b, i, w);
    u64 v;
    switch (k) {
      case EW_ADD: v = x + y; break;
      case EW_SUB: v = x - y; break;
      case EW_ADDUS: v = sat_u((i64)(x + y), w); break;
      case EW_SUBUS: v = sat_u((i64)x - (i64)y, w); break;
      case EW_ADDS: v = sat_s(sx + sy, w); break;
      case EW_SUBS: v = sat_s(sx - sy, w); break;
      case EW_MINU: v = x < y ? x : y; break;
      case EW_MAXU: v = x > y ? x : y; break;
      case EW_MINS: v = sx < sy ? x : y; break;
      case EW_MAXS: v = sx > sy ? x : y; break;
      case EW_EQ: v = x == y ? ~0ull : 0; break;
      case EW_GT: v = sx > sy ? ~0ull : 0; break;
      case EW_AVG: v = (x + y + 1) >> 1; break;
      case EW_MULLO: v = (u64)(sx * sy); break;
      case EW_MULHS: v = (u64)((sx * sy) >> 16); break;
      default: v = (x * y) >> 16; break;
    }
    xset(r, i, w, v);
  }
  return r;
}
// interleave the low (hi = 0) or high halves of a and b, w-byte elements
__device__ __forceinline__ X128 sse_unpack(u32 w, u32 hi, X128 a, X128 b) {
  X128 r{0, 0};
  const u32 n = 8 / w;
  for (u32 i = 0; i < n; i++) {
    xset(r, 2 * i, w, xel(a, i + hi * n, w));
    xset(r, 2 * i + 1, w, xel(b, i + hi * n, w));
  }
  return r;
}
// every w-byte element shifted by cnt: kind 0 logical right, 1 arithmetic right, 2 left
__device__ __forceinline__ X128 sse_shift(u32 kind, u32 w, X128 a, u64 cnt) {
  X128 r{0, 0};
  const u64 bits = 8ull * w;
  for (u32 i = 0; i < 16 / w; i++) {
    u64 v;
    if (kind == 1) v = (u64)(xsel(a, i, w) >> (cnt >= bits ? bits - 1 : cnt));
    else if (cnt >= bits) v = 0;
    else v = kind == 0 ? xel(a, i, w) >> cnt : xel(a, i, w) << cnt;
    xset(r, i, w, v);
  }
  return r;
}

__device__ __forceinline__ X128 xmm_get(const Dev &P, const Lane &L, u32 r) {
  const wtfgpu_regs_t &F = P.full[L.lane];
  return X128{F.xmm[r & 15][0], F.xmm[r & 15][1]};
}
__device__ __forceinline__ void xmm_put(const Dev &P, const Lane &L, u32 r, X128 v) {
  wtfgpu_regs_t &F = P.full[L.lane];
  F.xmm[r & 15][0] = v.lo;
  F.xmm[r & 15][1] = v.hi;
}

// The pages of [ea, ea + n) pass the access check before any byte moves; a
// fault is reported at ea or at the page boundary the operand crosses (as the
// oracle's vprobe, and as the 1-8 byte accesses do).
__device__ __forceinline__ bool span_ok(Lane &L, u64 ea, u32 n, int acc) {
  const u64 last = ea + n - 1;
  if (!xlate(L, ea, acc)) return false;
  return ((ea ^ last) >> 12) == 0 || xlate(L, last & ~0xfffull, acc);
}
// n bytes (1, 2, 4, 8 or 16) at ea, zero-extended
__device__ __forceinline__ bool xload(Lane &L, u64 ea, u32 n, X128 &v) {
  v.lo = v.hi = 0;
  if (n <= 8) return vread(L, ea, n, v.lo);
  tn_mute(L.lane);  // Tenet: one 16-byte access
  const bool ok = span_ok(L, ea, n, ACC_R) && vread(L, ea, 8, v.lo) && vread(L, ea + 8, 8, v.hi);
  return tn_unmute(L.lane, ea, n, TN_R, ok);
}
// n bytes of v to ea
__device__ __forceinline__ bool xstore(Lane &L, u64 ea, u32 n, X128 v) {
  if (n <= 8) return vwrite(L, ea, n, v.lo);
  if (!span_ok(L, ea, n, ACC_WPROBE)) return false;
  tn_mute(L.lane);
  const bool ok = vwrite(L, ea, 8, v.lo) && vwrite(L, ea + 8, 8, v.hi);
  return tn_unmute(L.lane, ea, n, TN_W, ok);
}


// ---------------------------------------------------------------- 256-bit state
struct Y256 {
  X128 l, h;
};
__device__ __forceinline__ Y256 ymm_get(const Dev &P, const Lane &L, u32 r) {
  const wtfgpu_regs_t &F = P.full[L.lane];
  return Y256{X128{F.xmm[r & 15][0], F.xmm[r & 15][1]}, X128{F.ymmh[r & 15][0], F.ymmh[r & 15][1]}};
}
// a VEX destination: VEX.128 zeroes bits 255:128, and every VEX write bits
// 511:256 (MAXVL = 512 on an AVX-512 machine, U47)
__device__ __forceinline__ void ymm_put(const Dev &P, const Lane &L, u32 r, Y256 v, u32 l256) {
  wtfgpu_regs_t &F = P.full[L.lane];
  F.xmm[r & 15][0] = v.l.lo;
  F.xmm[r & 15][1] = v.l.hi;
  F.ymmh[r & 15][0] = l256 ? v.h.lo : 0;
  F.ymmh[r & 15][1] = l256 ? v.h.hi : 0;
  for (u32 q = 0; q < 4; q++) F.zmmh[r & 15][q] = 0;
}
__device__ __forceinline__ bool yload(Lane &L, u64 ea, u32 n, Y256 &v) {
  v.h = X128{0, 0};
  if (n <= 16) return xload(L, ea, n, v.l);
  tn_mute(L.lane);  // Tenet: one 32-byte access
  const bool ok = span_ok(L, ea, n, ACC_R) && xload(L, ea, 16, v.l) && xload(L, ea + 16, 16, v.h);
  return tn_unmute(L.lane, ea, n, TN_R, ok);
}
__device__ __forceinline__ bool ystore(Lane &L, u64 ea, u32 n, Y256 v) {
  if (n <= 16) return xstore(L, ea, n, v.l);
  if (!span_ok(L, ea, n, ACC_WPROBE)) return false;
  tn_mute(L.lane);
  const bool ok = vwrite(L, ea, 8, v.l.lo) && vwrite(L, ea + 8, 8, v.l.hi) && vwrite(L, ea + 16, 8, v.h.lo) &&
                  vwrite(L, ea + 24, 8, v.h.hi);
  return tn_unmute(L.lane, ea, n, TN_W, ok);
}

// The 128-bit lane of the two-source integer / logic / shuffle ops shared by
// the legacy and the VEX encodings: a = first source (the destination for
// legacy SSE, VEX.vvvv for VEX), b = second source (r/m), cnt = the shift
// count of the shift-by-register forms (for VEX.256 the count register's low
// quadword, the same for both lanes). map 2 = 0f 38. false = not such an op.
__device__ __noinline__ bool sse_lane(u32 map, u32 c, u32 pc, X128 a, X128 b, u32 imm, u64 cnt, X128 &r) {
  r = X128{0, 0};
  if (map == 2) {
    if (c != 0x00) return false;
    for (u32 i = 0; i < 16; i++) {  // pshufb
      const u32 s = (u32)xel(b, i, 1);
      xset(r, i, 1, (s & 0x80) ? 0 : xel(a, s & 15, 1));
    }
    return true;
  }
  switch (c) {
    case 0x14: case 0x15: r = sse_unpack(pc ? 8 : 4, c == 0x15, a, b); return true;
    case 0x54: case 0xdb: r = X128{a.lo & b.lo, a.hi & b.hi}; return true;
    case 0x55: case 0xdf: r = X128{~a.lo & b.lo, ~a.hi & b.hi}; return true;
    case 0x56: case 0xeb: r = X128{a.lo | b.lo, a.hi | b.hi}; return true;
    case 0x57: case 0xef: r = X128{a.lo ^ b.lo, a.hi ^ b.hi}; return true;
    case 0x60: case 0x61: case 0x62: case 0x6c:
      r = sse_unpack(c == 0x60 ? 1 : c == 0x61 ? 2 : c == 0x62 ? 4 : 8, 0, a, b);
      return true;
    case 0x68: case 0x69: case 0x6a: case 0x6d:
      r = sse_unpack(c == 0x68 ? 1 : c == 0x69 ? 2 : c == 0x6a ? 4 : 8, 1, a, b);
      return true;
    case 0x63: case 0x67: case 0x6b: {  // packsswb, packuswb, packssdw
      const u32 w = c == 0x6b ? 4 : 2, h = 16 / w;
      for (u32 i = 0; i < 2 * h; i++) {
        const i64 x = i < h ? xsel(a, i, w) : xsel(b, i - h, w);
        xset(r, i, w / 2, c == 0x67 ? sat_u(x, 1) : sat_s(x, w / 2));
      }
      return true;
    }
    case 0x64: case 0x65: case 0x66: r = sse_ewise(EW_GT, 1u << (c - 0x64), a, b); return true;
    case 0x74: case 0x75: case 0x76: r = sse_ewise(EW_EQ, 1u << (c - 0x74), a, b); return true;
    case 0x70:  // pshufd / pshufhw / pshuflw (of b)
      r = b;
      if (pc == 1) {
        for (u32 i = 0; i < 4; i++) xset(r, i, 4, xel(b, (imm >> (2 * i)) & 3, 4));
      } else {
        const u32 o = pc == 2 ? 4 : 0;
        for (u32 i = 0; i < 4; i++) xset(r, i + o, 2, xel(b, ((imm >> (2 * i)) & 3) + o, 2));
      }
      return true;
    case 0xc6:  // shufps / shufpd
      if (pc == 0) {
        xset(r, 0, 4, xel(a, imm & 3, 4));
        xset(r, 1, 4, xel(a, (imm >> 2) & 3, 4));
        xset(r, 2, 4, xel(b, (imm >> 4) & 3, 4));
        xset(r, 3, 4, xel(b, (imm >> 6) & 3, 4));
      } else {
        r = X128{(imm & 1) ? a.hi : a.lo, (imm & 2) ? b.hi : b.lo};
      }
      return true;
    case 0xd1: case 0xd2: case 0xd3: r = sse_shift(0, c == 0xd1 ? 2 : c == 0xd2 ? 4 : 8, a, cnt); return true;
    case 0xe1: case 0xe2: r = sse_shift(1, c == 0xe1 ? 2 : 4, a, cnt); return true;
    case 0xf1: case 0xf2: case 0xf3: r = sse_shift(2, c == 0xf1 ? 2 : c == 0xf2 ? 4 : 8, a, cnt); return true;
    case 0xd4: r = X128{a.lo + b.lo, a.hi + b.hi}; return true;
    case 0xfb: r = X128{a.lo - b.lo, a.hi - b.hi}; return true;
    case 0xfc: case 0xfd: case 0xfe: r = sse_ewise(EW_ADD, 1u << (c - 0xfc), a, b); return true;
    case 0xf8: case 0xf9: case 0xfa: r = sse_ewise(EW_SUB, 1u << (c - 0xf8), a, b); return true;
    case 0xd5: r = sse_ewise(EW_MULLO, 2, a, b); return true;
    case 0xe5: r = sse_ewise(EW_MULHS, 2, a, b); return true;
    case 0xe4: r = sse_ewise(EW_MULHU, 2, a, b); return true;
    case 0xd8: case 0xd9: r = sse_ewise(EW_SUBUS, c - 0xd7, a, b); return true;
    case 0xdc: case 0xdd: r = sse_ewise(EW_ADDUS, c - 0xdb, a, b); return true;
    case 0xe8: case 0xe9: r = sse_ewise(EW_SUBS, c - 0xe7, a, b); return true;
    case 0xec: case 0xed: r = sse_ewise(EW_ADDS, c - 0xeb, a, b); return true;
    case 0xda: r = sse_ewise(EW_MINU, 1, a, b); return true;
    case 0xde: r = sse_ewise(EW_MAXU, 1, a, b); return true;
    case 0xea: r = sse_ewise(EW_MINS, 2, a, b); return true;
    case 0xee: r = sse_ewise(EW_MAXS, 2, a, b); return true;
    case 0xe0: r = sse_ewise(EW_AVG, 1, a, b); return true;
    case 0xe3: r = sse_ewise(EW_AVG, 2, a, b); return true;
    case 0xf4:
      r = X128{(a.lo & 0xffffffffull) * (b.lo & 0xffffffffull), (a.hi & 0xffffffffull) * (b.hi & 0xffffffffull)};
      return true;
    case 0xf5:  // pmaddwd
      for (u32 i = 0; i < 4; i++)
        xset(r, i, 4, (u64)(xsel(a, 2 * i, 2) * xsel(b, 2 * i, 2) + xsel(a, 2 * i + 1, 2) * xsel(b, 2 * i + 1, 2)));
      return true;
    case 0xf6: {  // psadbw
      u64 s0 = 0, s1 = 0;
      for (u32 i = 0; i < 8; i++) {
        const u64 x0 = xel(a, i, 1), y0 = xel(b, i, 1), x1 = xel(a, i + 8, 1), y1 = xel(b, i + 8, 1);
        s0 += x0 > y0 ? x0 - y0 : y0 - x0;
        s1 += x1 > y1 ? x1 - y1 : y1 - x1;
      }
      r = X128{s0, s1};
      return true;
    }
    default: return false;
  }
}

// 71 / 72 / 73 by imm8 of one lane: /2 srl, /4 sra, /6 sll, 73 /3 srldq, /7 slldq
__device__ __forceinline__ X128 sse_shift_imm(u32 c, u32 r3, X128 b, u32 imm) {
  if (c == 0x73 && (r3 == 3 || r3 == 7)) {
    X128 r{0, 0};
    for (u32 i = 0; i < 16; i++) {
      const i32 s = r3 == 3 ? (i32)(i + imm) : (i32)i - (i32)imm;
      if (s >= 0 && s < 16) xset(r, i, 1, xel(b, (u32)s, 1));
    }
    return r;
  }
  return sse_shift(r3 == 2 ? 0 : r3 == 4 ? 1 : 2, c == 0x71 ? 2 : c == 0x72 ? 4 : 8, b, imm);
}

// ptest / vptest: ZF = (a & b) == 0, CF = (~a & b) == 0, AF OF PF SF = 0
__device__ __forceinline__ u64 ptest_flags(u64 fl, Y256 a, Y256 b) {
  const bool z = !((a.l.lo & b.l.lo) | (a.l.hi & b.l.hi) | (a.h.lo & b.h.lo) | (a.h.hi & b.h.hi));
  const bool cf = !((~a.l.lo & b.l.lo) | (~a.l.hi & b.l.hi) | (~a.h.lo & b.h.lo) | (~a.h.hi & b.h.hi));
  return (fl & ~F_STATUS) | (z ? F_ZF : 0) | (cf ? F_CF : 0);
}

__device__ __forceinline__ u64 sse_ea(const Dev &P, const Lane &L, const UOp &u, u64 nrip) {
  u64 ea;
  if (u.riprel) {
    ea = nrip + u.disp;
  } else {
    ea = u.disp;
    if (u.base >= 0) ea += R(L, u.base);
    if (u.index >= 0) ea += R(L, u.index) << u.scale;
  }
  if (u.p67) ea &= 0xffffffffull;
  if (u.seg) ea += u.seg == 4 ? P.fs_base[L.lane] : P.gs_base[L.lane];
  return ea;
}

__device__ __noinline__ int vex_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next);

// ---------------------------------------------------------------- MMX (U37)
// The oracle's exec_mmx: mm i is physical x87 register R(i) = fpst[(i - TOS)
// & 7] (fpst holds ST order); a completed MMX instruction rotates fpst to R
// order (TOS = 0) and marks every tag valid, emms every tag empty. #UD if
// CR0.EM, #NM if CR0.TS, #MF if an unmasked x87 flag is set, then the operand's memory faults;
// nothing is committed before every access succeeded (exec protocol).
// UOp::opreg bit 20 marks an MMX form (decode).
constexpr u32 kMmxForm = 1u << 20;
__host__ __device__ inline bool mmx_opcode(u32 c) {
  return (c >= 0x60 && c <= 0x7f && !(c >= 0x78 && c <= 0x7d)) || c == 0xc4 || c == 0xc5 || (c >= 0xd0 && c <= 0xfe);
}
// the SSSE3 forms on mm registers (no prefix): 0f 38 00-0b / 1c-1e, 0f 3a 0f palignr
__host__ __device__ inline bool ssse3_mm(u32 map, u32 c) {
  return map == 2 ? (c <= 0x0b || (c >= 0x1c && c <= 0x1e)) : (map == 3 && c == 0x0f);
}
__device__ __forceinline__ u64 mmx_get(const wtfgpu_regs_t &F, u32 i) { return F.fpst[(i - ((F.fpsw >> 11) & 7)) & 7]; }
__device__ __forceinline__ void mmx_commit(wtfgpu_regs_t &F) {
  const u32 tos = (F.fpsw >> 11) & 7;
  if (tos) {
    u64 t[8];
    u16 e[8];
    for (u32 j = 0; j < 8; j++) t[j] = F.fpst[(j - tos) & 7], e[j] = F.fpse[(j - tos) & 7];
    for (u32 j = 0; j < 8; j++) F.fpst[j] = t[j], F.fpse[j] = e[j];
  }
  F.fpsw = (u16)(F.fpsw & ~0x3800);
  F.fptw = 0;
}
// an MMX register write: the significand, sign and exponent all ones (after mmx_commit: ST = R order)
__device__ __forceinline__ void mmx_put(wtfgpu_regs_t &F, u32 i, u64 v) {
  F.fpst[i] = v;
  F.fpse[i] = 0xffff;
}

}  // namespace wtfgpu_dev
#include "engine_ssefp.h"  // SSE / AVX floating point: fp_exec
#include "engine_sse4.h"  // SSSE3 / SSE4.1 integer, AVX2 lane-crossing: s4_exec
#include "engine_avx2x.h"  // FMA3, F16C, AVX2 gathers: ax_exec
#include "engine_avx512.h"  // the EVEX subset and the opmask instructions: evex_exec, kop_exec
namespace wtfgpu_dev {

__device__ __noinline__ int mmx_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 c = u.sub, pc = u.bsz, r3 = u.reg & 7, mr = u.reg & 7, mrm = u.rm & 7;
  const bool mem = u.is_mem;
  const u32 imm = (u32)u.imm & 0xff;
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  wtfgpu_regs_t &F = P.full[L.lane];
  const u32 map = vex_map(u.opreg);  // 1, or 2 / 3 for the SSSE3 forms (ssse3_mm)
  bool ud = map == 1 && pc == 0 && (c == 0xd0 || c == 0xd6 || c == 0xe6 || c == 0xf0 || c == 0x6c || c == 0x6d);
  if (map == 1 && c == 0xf7) ud = ud || mem;  // maskmovq: register operands only
  if (map == 1 && c >= 0x71 && c <= 0x73)
    ud = ud || mem || !(c == 0x73 ? (r3 == 2 || r3 == 6) : (r3 == 2 || r3 == 4 || r3 == 6));
  ud = ud || ((c == 0xc5 || c == 0xd7 || (c == 0xd6 && pc)) && mem) || (c == 0xe7 && !mem) || (L.cr0 & 4);
  if (ud) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  if (L.cr0 & 8) {
    set_fault(L, 7, 0, 0);  // #NM
    return X_FAULT;
  }
  if (F.fpsw & ~F.fpcw & 0x3f) {
    set_fault(L, 16, 0, 0);  // #MF: a pending unmasked x87 exception
    return X_FAULT;
  }
  if (map == 1 && c == 0x77) {  // emms
    F.fptw = 0xffff;
    return X_OK;
  }
  if (map >= 2) {  // SSSE3 on mm registers: the 128-bit lane ops on the low quadwords (U41)
    const u64 av = mmx_get(F, mr);
    u64 bv;
    if (mem) {
      if (!vread(L, ea, 8, bv)) return X_FAULT;
    } else {
      bv = mmx_get(F, mrm);
    }
    u64 res = 0;
    if (map == 3) {  // palignr: (a:b) >> 8 * imm, the low quadword
      res = imm >= 16 ? 0 : imm >= 8 ? (imm == 8 ? av : av >> (8 * (imm - 8))) : imm == 0 ? bv
                                                   : (bv >> (8 * imm)) | (av << (64 - 8 * imm));
    } else if (c == 0x00) {  // pshufb: index bits 2:0, bit 7 zeroes
      for (u32 i = 0; i < 8; i++) {
        const u32 k = (u32)(bv >> (8 * i)) & 0xff;
        if (!(k & 0x80)) res |= ((av >> (8 * (k & 7))) & 0xff) << (8 * i);
      }
    } else if ((c >= 0x01 && c <= 0x03) || (c >= 0x05 && c <= 0x07)) {  // horizontal: pairs of a, then of b
      res = s4_lane2(c, X128{av, bv}, X128{0, 0}).lo;
    } else {
      res = s4_lane2(c, X128{av, 0}, X128{bv, 0}).lo;
    }
    mmx_commit(F);
    mmx_put(F, mr, res);
    return X_OK;
  }
  if (c == 0xf7) {  // maskmovq mm1, mm2: the bytes of mm1 whose mm2 byte has bit 7 set, to [rdi]
    const u64 av = mmx_get(F, mr), sel = mmx_get(F, mrm);
    u64 di = R(L, 7);
    if (u.p67) di &= 0xffffffffull;
    if (u.seg) di += u.seg == 4 ? P.fs_base[L.lane] : P.gs_base[L.lane];
    for (u32 i = 0; i < 8; i++)  // every written byte's page checked first
      if (((sel >> (8 * i + 7)) & 1) && !span_ok(L, di + i, 1, ACC_WPROBE)) return X_FAULT;
    tn_mute(L.lane);
    bool ok = true;
    for (u32 i = 0; ok && i < 8; i++)
      if ((sel >> (8 * i + 7)) & 1) ok = vwrite(L, di + i, 1, (av >> (8 * i)) & 0xff);
    if (!tn_unmute(L.lane, di, 8, TN_W, ok)) return X_FAULT;
    mmx_commit(F);
    return X_OK;
  }
  if (c == 0xd6) {  // f3: movq2dq xmm, mm; f2: movdq2q mm, xmm
    if (pc == 2) {
      const u64 v = mmx_get(F, mrm);
      mmx_commit(F);
      xmm_put(P, L, u.reg, X128{v, 0});
    } else {
      const u64 v = xmm_get(P, L, u.rm).lo;
      mmx_commit(F);
      mmx_put(F, mr, v);
    }
    return X_OK;
  }
  const u64 av = mmx_get(F, mr);
  u64 bv = 0;
  const bool rm_src = !(c == 0x7e || c == 0x7f || c == 0xe7 || c == 0x6e || c == 0xc4);
  if (rm_src) {
    if (mem) {
      if (!vread(L, ea, 8, bv)) return X_FAULT;
    } else {
      bv = mmx_get(F, mrm);
    }
  }
  const X128 a{av, 0}, b{bv, 0};
  X128 r{0, 0};
  u64 res = 0;
  bool to_gpr = false;
  switch (c) {
    case 0x6e: {  // movd / movq mm, r/m
      const u32 n = (u.rex & 8) ? 8 : 4;
      u64 v = 0;
      if (mem) {
        if (!vread(L, ea, n, v)) return X_FAULT;
      } else {
        v = R(L, u.rm) & szmask(n);
      }
      res = v;
      break;
    }
    case 0x7e: {  // movd / movq r/m, mm
      const u32 n = (u.rex & 8) ? 8 : 4;
      const u64 v = av & szmask(n);
      if (mem && !vwrite(L, ea, n, v)) return X_FAULT;
      mmx_commit(F);
      if (!mem) RS(L, u.rm, v);
      return X_OK;
    }
    case 0x6f: res = bv; break;
    case 0x7f: case 0xe7:  // movq mm/m64, mm; movntq m64, mm
      if (mem && !vwrite(L, ea, 8, av)) return X_FAULT;
      mmx_commit(F);
      if (!mem) mmx_put(F, mrm, av);
      return X_OK;
    case 0x68: case 0x69: case 0x6a:  // punpckh*: the high halves
      r = sse_unpack(1u << (c - 0x68), 0, X128{av >> 32, 0}, X128{bv >> 32, 0});
      res = r.lo;
      break;
    case 0x63: case 0x67: case 0x6b: {  // packs: a's elements, then b's
      const u32 w = c == 0x6b ? 4 : 2, h = 8 / w;
      for (u32 i = 0; i < 2 * h; i++) {
        const i64 x = i < h ? xsel(a, i, w) : xsel(b, i - h, w);
        xset(r, i, w / 2, c == 0x67 ? sat_u(x, 1) : sat_s(x, w / 2));
      }
      res = r.lo;
      break;
    }
    case 0x70:  // pshufw
      for (u32 i = 0; i < 4; i++) res |= ((bv >> (16 * ((imm >> (2 * i)) & 3))) & 0xffff) << (16 * i);
      break;
    case 0x71: case 0x72: case 0x73:  // by imm8, of mm (r/m)
      r = sse_shift_imm(c, r3, b, imm);
      mmx_commit(F);
      mmx_put(F, mrm, r.lo);
      return X_OK;
    case 0xc4: {  // pinsrw mm, r32/m16, imm8
      u64 v = 0;
      if (mem) {
        if (!vread(L, ea, 2, v)) return X_FAULT;
      } else {
        v = R(L, u.rm);
      }
      const u32 k = imm & 3;
      res = (av & ~(0xffffull << (16 * k))) | ((v & 0xffff) << (16 * k));
      break;
    }
    case 0xc5: to_gpr = true; res = (bv >> (16 * (imm & 3))) & 0xffff; break;  // pextrw
    case 0xd7:  // pmovmskb r32, mm
      to_gpr = true;
      for (u32 i = 0; i < 8; i++) res |= ((bv >> (8 * i + 7)) & 1) << i;
      break;
    case 0xf4: res = (av & 0xffffffffull) * (bv & 0xffffffffull); break;  // pmuludq
    case 0xf5:  // pmaddwd
      for (u32 i = 0; i < 2; i++)
        xset(r, i, 4, (u64)(xsel(a, 2 * i, 2) * xsel(b, 2 * i, 2) + xsel(a, 2 * i + 1, 2) * xsel(b, 2 * i + 1, 2)));
      res = r.lo;
      break;
    case 0xf6:  // psadbw
      for (u32 i = 0; i < 8; i++) {
        const u64 x = (av >> (8 * i)) & 0xff, y = (bv >> (8 * i)) & 0xff;
        res += x > y ? x - y : y - x;
      }
      break;
    default:  // the rest: the 128-bit lane op on the low quadwords (counts: the source quadword)
      if (!sse_lane(1, c, 0, a, b, imm, bv, r)) return X_UNIMPL;
      res = r.lo;
      break;
  }
  mmx_commit(F);
  if (to_gpr) RS(L, u.reg, res);
  else mmx_put(F, mr, res);
  return X_OK;
}

// One attempt at an SSE instruction (exec() protocol: X_FAULT with L.miss set
// asks for a translation service and a rerun).
__device__ __noinline__ int sse_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  if (u.opreg & 1) return vex_exec(P, L, u, nrip, next);
  if (u.opreg & kMmxForm) return mmx_exec(P, L, u, nrip, next);
  next = nrip;
  const u32 c = u.sub, pc = u.bsz, r3 = u.reg & 7, map = vex_map(u.opreg);
  const bool mem = u.is_mem;
  const u32 imm = (u32)u.imm & 0xff;
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  if (map == 1 && c == 0xc3) {  // movnti m32/64, r
    if (!mem) {
      set_fault(L, WTFGPU_VEC_UD, 0, 0);
      return X_FAULT;
    }
    const u32 sz = (u.rex & 8) ? 8 : 4;
    return vwrite(L, ea, sz, R(L, u.reg) & szmask(sz)) ? X_OK : X_FAULT;
  }
  if (map == 1 && c == 0xae && !mem) return X_OK;  // lfence / mfence / sfence
  const bool reg_only = map == 1 && ((c >= 0x71 && c <= 0x73) || c == 0x50 || c == 0xd7 || c == 0xc5);
  const bool mem_only = map == 1 && (c == 0x13 || c == 0x17 || c == 0x2b || c == 0xe7 || c == 0xae ||
                                     ((c == 0x12 || c == 0x16) && pc == 1));
  if ((reg_only && mem) || (mem_only && !mem)) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  const u64 cr4 = P.sys[L.lane].cr4;
  if ((L.cr0 & 4) || !(cr4 & 0x200)) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  if (L.cr0 & 8) {
    set_fault(L, 7, 0, 0);  // #NM
    return X_FAULT;
  }
  if (fp_form(map, c, pc, false)) return fp_exec(P, L, u, nrip, next);
  if (s4_form(map, c, pc, false)) return s4_exec(P, L, u, nrip, next);
  if (x42_form(map, c, pc, false)) return x42_exec(P, L, u, nrip, next);
  // the r/m operand: 16 bytes aligned unless an unaligned move / narrower form
  u32 n = 16;
  bool align = true;
  if (map == 1) {
    switch (c) {
      case 0x10:
      case 0x11: n = pc <= 1 ? 16 : pc == 2 ? 4 : 8; align = false; break;
      case 0x12: case 0x13: case 0x16: case 0x17: case 0xd6: n = 8; align = false; break;
      case 0x6e: case 0x7e: n = (pc == 2 || (u.rex & 8)) ? 8 : 4; align = false; break;
      case 0x6f: case 0x7f: align = pc == 1; break;
      case 0xc4: n = 2; align = false; break;
      case 0xae: n = 4; align = false; break;
      default: break;
    }
  }
  if (mem && n == 16 && align && (ea & 15)) {
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return X_FAULT;
  }
  const bool store = map == 1 && (c == 0x11 || c == 0x13 || c == 0x17 || c == 0x29 || c == 0x2b || c == 0x7f ||
                                  c == 0xe7 || c == 0xd6 || (c == 0x7e && pc == 1) || (c == 0xae && r3 == 3));
  X128 a = xmm_get(P, L, u.reg), b{0, 0}, r{0, 0};
  if (!store) {
    if (mem) {
      if (!xload(L, ea, n, b)) return X_FAULT;
    } else if (map == 1 && (c == 0x6e || c == 0xc4)) {
      b.lo = R(L, u.rm);
    } else {
      b = xmm_get(P, L, u.rm);
    }
  }
  if (map == 2 && c == 0x17) {  // ptest
    L.rflags = ptest_flags(L.rflags, Y256{a, X128{0, 0}}, Y256{b, X128{0, 0}});
    return X_OK;
  }
  // ---- compute: r goes to xmm[reg] unless a case returns itself
  switch (map == 1 ? c : 0x100) {
    case 0x10:
      if (pc <= 1 || mem) r = b;
      else if (pc == 2) r = X128{(a.lo & ~0xffffffffull) | (b.lo & 0xffffffffull), a.hi};
      else r = X128{b.lo, a.hi};
      break;
    case 0x11: case 0x29: case 0x2b: case 0x7f: case 0xe7: {  // stores / register moves to rm
      if (mem) return xstore(L, ea, n, a) ? X_OK : X_FAULT;
      X128 d = xmm_get(P, L, u.rm);
      if (c == 0x11 && pc == 2) d.lo = (d.lo & ~0xffffffffull) | (a.lo & 0xffffffffull);
      else if (c == 0x11 && pc == 3) d.lo = a.lo;
      else d = a;
      xmm_put(P, L, u.rm, d);
      return X_OK;
    }
    case 0x12: r = X128{mem ? b.lo : b.hi, a.hi}; break;  // movlps / movlpd; movhlps
    case 0x16: r = X128{a.lo, b.lo}; break;               // movhps / movhpd; movlhps
    case 0x13: return xstore(L, ea, 8, a) ? X_OK : X_FAULT;
    case 0x17: return xstore(L, ea, 8, X128{a.hi, 0}) ? X_OK : X_FAULT;
    case 0x28: case 0x6f: r = b; break;
    case 0x50: {  // movmskps / movmskpd
      const u32 w = pc ? 8 : 4;
      u64 v = 0;
      for (u32 i = 0; i < 16 / w; i++) v |= (xel(b, i, w) >> (8 * w - 1)) << i;
      RS(L, u.reg, v);
      return X_OK;
    }
    case 0xd7: {  // pmovmskb
      u64 v = 0;
      for (u32 i = 0; i < 16; i++) v |= ((xel(b, i, 1) >> 7) & 1) << i;
      RS(L, u.reg, v);
      return X_OK;
    }
    case 0x6e: r = X128{b.lo & szmask(n), 0}; break;  // movd / movq xmm, r/m
    case 0x7e:
      if (pc == 2) {  // movq xmm, xmm/m64
        r = X128{b.lo, 0};
        break;
      }
      // movd / movq r/m, xmm
      if (mem) return vwrite(L, ea, n, a.lo & szmask(n)) ? X_OK : X_FAULT;
      RS(L, u.rm, a.lo & szmask(n));
      return X_OK;
    case 0x71: case 0x72: case 0x73:
      xmm_put(P, L, u.rm, sse_shift_imm(c, r3, b, imm));
      return X_OK;
    case 0xc4: r = a; xset(r, imm & 7, 2, b.lo & 0xffff); break;  // pinsrw
    case 0xc5: RS(L, u.reg, xel(b, imm & 7, 2)); return X_OK;     // pextrw
    case 0xd6:  // movq xmm/m64, xmm
      if (mem) return xstore(L, ea, 8, a) ? X_OK : X_FAULT;
      xmm_put(P, L, u.rm, X128{a.lo, 0});
      return X_OK;
    case 0xae: {  // ldmxcsr / stmxcsr
      wtfgpu_regs_t &F = P.full[L.lane];
      if (r3 == 3) return vwrite(L, ea, 4, F.mxcsr) ? X_OK : X_FAULT;
      const u32 mask = F.mxcsr_mask ? F.mxcsr_mask : 0xffbfu;
      if ((u32)b.lo & ~mask) {
        set_fault(L, WTFGPU_VEC_GP, 0, 0);
        return X_FAULT;
      }
      F.mxcsr = (u32)b.lo;
      return X_OK;
    }
    default:
      if (!sse_lane(map, c, pc, a, b, imm, b.lo, r)) return X_UNIMPL;
      break;
  }
  xmm_put(P, L, u.reg, r);
  return X_OK;
}

// One attempt at a VEX instruction (U23). dst = reg, a = VEX.vvvv, b = r/m.
__device__ __noinline__ int vex_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, pp = u.bsz, r3 = u.reg & 7, map = vex_map(x);
  if (x & EVX) return evex_exec(P, L, u, nrip, next);                          // engine_avx512.h
  if (kop_bits(map, c, pp, 0) || kop_bits(map, c, pp, 1)) return kop_exec(P, L, u, nrip, next);  // W checked there
  if (fp_form(map, c, pp, true)) return fp_exec(P, L, u, nrip, next);  // its own VEX checks
  if (s4_form(map, c, pp, true)) return s4_exec(P, L, u, nrip, next);
  if (x42_form(map, c, pp, true)) return x42_exec(P, L, u, nrip, next);  // its own VEX checks
  if (ax_form(map, c, pp, true)) return ax_exec(P, L, u, nrip, next);    // its own VEX checks
  const u32 l256 = (x >> 1) & 1, w = (x >> 2) & 1, vvvv = (x >> 4) & 15;
  const bool mem = u.is_mem;
  const u32 imm = (u32)u.imm & 0xff;
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  // ---- #UD: a legacy prefix before VEX, AVX state off, operand-form rules
  bool ud = (x >> 16) & 1;
  const u64 cr4 = P.sys[L.lane].cr4;
  if (!((cr4 >> 18) & 1) || (P.full[L.lane].xcr0 & 6) != 6) ud = true;
  bool two_op = false, no256 = false, reg_only = false, mem_only = false;
  if (map == 1) {
    two_op = ((c == 0x10 || c == 0x11) && (pp <= 1 || mem)) || c == 0x13 || c == 0x17 || c == 0x28 || c == 0x29 ||
             c == 0x2b || c == 0x50 || c == 0x6e || c == 0x6f || c == 0x70 || c == 0x7e || c == 0x7f || c == 0xc5 ||
             c == 0xd6 || c == 0xd7 || c == 0xe7 || c == 0x77;
    no256 = c == 0x12 || c == 0x13 || c == 0x16 || c == 0x17 || c == 0x6e || c == 0x7e || c == 0xc4 || c == 0xc5 ||
            c == 0xd6;
    reg_only = (c >= 0x71 && c <= 0x73) || c == 0x50 || c == 0xd7 || c == 0xc5;
    mem_only = c == 0x13 || c == 0x17 || c == 0x2b || c == 0xe7 || ((c == 0x12 || c == 0x16) && pp == 1);
  } else {
    two_op = c != 0x00;
  }
  if ((two_op && vvvv != 0) || (no256 && l256) || (reg_only && mem) || (mem_only && !mem)) ud = true;
  if (ud) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  if (L.cr0 & 8) {
    set_fault(L, 7, 0, 0);  // #NM
    return X_FAULT;
  }
  if (map == 1 && c == 0x77) {  // vzeroupper / vzeroall
    wtfgpu_regs_t &F = P.full[L.lane];
    for (u32 i = 0; i < 16; i++) {  // zmm0..15 bits 511:128 (all of them: vzeroall); zmm16..31 kept
      F.ymmh[i][0] = F.ymmh[i][1] = 0;
      for (u32 q = 0; q < 4; q++) F.zmmh[i][q] = 0;
      if (l256) F.xmm[i][0] = F.xmm[i][1] = 0;
    }
    return X_OK;
  }
  // ---- the r/m operand's size; aligned moves need 16 / 32-byte alignment
  const u32 vl = l256 ? 32 : 16;
  u32 n = vl;
  bool align = false;
  if (map == 1) {
    switch (c) {
      case 0x10: case 0x11: n = pp <= 1 ? vl : pp == 2 ? 4 : 8; break;
      case 0x12: case 0x13: case 0x16: case 0x17: case 0xd6: n = 8; break;
      case 0x6e: case 0x7e: n = (pp == 2 || w) ? 8 : 4; break;
      case 0xc4: n = 2; break;
      case 0x28: case 0x29: case 0x2b: case 0xe7: align = true; break;
      case 0x6f: case 0x7f: align = pp == 1; break;
      case 0xd1: case 0xd2: case 0xd3: case 0xe1: case 0xe2: case 0xf1: case 0xf2: case 0xf3: n = 16; break;
      default: break;
    }
  } else if (c == 0x58 || c == 0x59 || c == 0x78 || c == 0x79) {
    n = c == 0x78 ? 1 : c == 0x79 ? 2 : c == 0x58 ? 4 : 8;
  }
  if (mem && align && (ea & (vl - 1))) {
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return X_FAULT;
  }
  const bool store = map == 1 && (c == 0x11 || c == 0x13 || c == 0x17 || c == 0x29 || c == 0x2b || c == 0x7f ||
                                  c == 0xe7 || c == 0xd6 || (c == 0x7e && pp == 1));
  const Y256 s = ymm_get(P, L, u.reg);  // the reg operand (a store's source, vptest's first source)
  const Y256 a = ymm_get(P, L, vvvv);
  Y256 b{X128{0, 0}, X128{0, 0}}, r{X128{0, 0}, X128{0, 0}};
  if (!store) {
    if (mem) {
      if (!yload(L, ea, n, b)) return X_FAULT;
    } else if (map == 1 && (c == 0x6e || c == 0xc4)) {
      b.l.lo = R(L, u.rm);
    } else {
      b = ymm_get(P, L, u.rm);
    }
  }
  u32 dst = u.reg;
  if (map == 2) {
    if (c == 0x17) {  // vptest (VEX.128: the low halves only)
      L.rflags = l256 ? ptest_flags(L.rflags, s, b) : ptest_flags(L.rflags, Y256{s.l, X128{0, 0}}, Y256{b.l, X128{0, 0}});
      return X_OK;
    }
    if (c == 0x00) {  // vpshufb
      sse_lane(2, 0, 1, a.l, b.l, 0, 0, r.l);
      if (l256) sse_lane(2, 0, 1, a.h, b.h, 0, 0, r.h);
    } else {  // vpbroadcastb / w / d / q
      const u32 ew = c == 0x78 ? 1 : c == 0x79 ? 2 : c == 0x58 ? 4 : 8;
      const u64 e = xel(b.l, 0, ew);
      for (u32 i = 0; i < 16 / ew; i++) xset(r.l, i, ew, e);
      r.h = r.l;
    }
    ymm_put(P, L, dst, r, l256);
    return X_OK;
  }
  switch (c) {
    case 0x10:
      if (pp <= 1 || mem) r = b;
      else if (pp == 2) r.l = X128{(a.l.lo & ~0xffffffffull) | (b.l.lo & 0xffffffffull), a.l.hi};
      else r.l = X128{b.l.lo, a.l.hi};
      break;
    case 0x11: case 0x29: case 0x2b: case 0x7f: case 0xe7:  // stores / register moves to rm
      if (mem) return ystore(L, ea, c == 0x11 ? n : vl, s) ? X_OK : X_FAULT;
      if (c == 0x11 && pp == 2) r.l = X128{(a.l.lo & ~0xffffffffull) | (s.l.lo & 0xffffffffull), a.l.hi};
      else if (c == 0x11 && pp == 3) r.l = X128{s.l.lo, a.l.hi};
      else r = s;
      ymm_put(P, L, u.rm, r, c == 0x11 && pp >= 2 ? 0 : l256);
      return X_OK;
    case 0x12: r.l = X128{mem ? b.l.lo : b.l.hi, a.l.hi}; break;  // vmovlps / vmovlpd; vmovhlps
    case 0x16: r.l = X128{a.l.lo, b.l.lo}; break;                 // vmovhps / vmovhpd; vmovlhps
    case 0x13: return xstore(L, ea, 8, s.l) ? X_OK : X_FAULT;
    case 0x17: return xstore(L, ea, 8, X128{s.l.hi, 0}) ? X_OK : X_FAULT;
    case 0x28: case 0x6f: r = b; break;
    case 0x50: {  // vmovmskps / vmovmskpd
      const u32 ew = pp ? 8 : 4;
      u64 v = 0;
      for (u32 i = 0; i < 16 / ew; i++) v |= (xel(b.l, i, ew) >> (8 * ew - 1)) << i;
      if (l256)
        for (u32 i = 0; i < 16 / ew; i++) v |= (xel(b.h, i, ew) >> (8 * ew - 1)) << (i + 16 / ew);
      RS(L, u.reg, v);
      return X_OK;
    }
    case 0xd7: {  // vpmovmskb
      u64 v = 0;
      for (u32 i = 0; i < 16; i++) v |= ((xel(b.l, i, 1) >> 7) & 1) << i;
      if (l256)
        for (u32 i = 0; i < 16; i++) v |= ((xel(b.h, i, 1) >> 7) & 1) << (i + 16);
      RS(L, u.reg, v);
      return X_OK;
    }
    case 0x6e: r.l = X128{b.l.lo & szmask(n), 0}; break;  // vmovd / vmovq xmm, r/m
    case 0x7e:
      if (pp == 2) {  // vmovq xmm, xmm/m64
        r.l = X128{b.l.lo, 0};
        break;
      }
      if (mem) return vwrite(L, ea, n, s.l.lo & szmask(n)) ? X_OK : X_FAULT;
      RS(L, u.rm, s.l.lo & szmask(n));
      return X_OK;
    case 0x70:
      sse_lane(1, 0x70, pp, a.l, b.l, imm, 0, r.l);
      if (l256) sse_lane(1, 0x70, pp, a.h, b.h, imm, 0, r.h);
      break;
    case 0x71: case 0x72: case 0x73:  // the destination is VEX.vvvv
      r.l = sse_shift_imm(c, r3, b.l, imm);
      if (l256) r.h = sse_shift_imm(c, r3, b.h, imm);
      dst = vvvv;
      break;
    case 0xc4: r.l = a.l; xset(r.l, imm & 7, 2, b.l.lo & 0xffff); break;  // vpinsrw
    case 0xc5: RS(L, u.reg, xel(b.l, imm & 7, 2)); return X_OK;           // vpextrw
    case 0xd6:  // vmovq xmm/m64, xmm
      if (mem) return xstore(L, ea, 8, s.l) ? X_OK : X_FAULT;
      ymm_put(P, L, u.rm, Y256{X128{s.l.lo, 0}, X128{0, 0}}, 0);
      return X_OK;
    default: {
      // two-source lane ops: vshufpd's high lane takes imm bits 2-3
      if (!sse_lane(1, c, pp, a.l, b.l, imm, b.l.lo, r.l)) return X_UNIMPL;
      if (l256) sse_lane(1, c, pp, a.h, b.h, c == 0xc6 && pp == 1 ? imm >> 2 : imm, b.l.lo, r.h);
      break;
    }
  }
  ymm_put(P, L, dst, r, l256);
  return X_OK;
}

}  // namespace wtfgpu_dev
