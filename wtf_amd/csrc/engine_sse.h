// engine_sse.h — the SSE / SSE2 subset (convention U22).
//
// The legacy-encoded integer and data-movement instructions compilers emit
// for x86-64 at the SSE2 baseline: 128-bit moves, scalar / half moves,
// movd / movq, logic, integer add / sub / saturate / compare / min / max /
// multiply, shifts, shuffles, unpacks, packs, mask extraction, ldmxcsr /
// stmxcsr, fences, movnti. A UOp with op O_SSE carries the opcode byte in
// `sub` and the mandatory-prefix class in `bsz` (0 none, 1 66, 2 f3, 3 f2);
// `imm` is the imm8. Encodings outside the subset (MMX, floating point, SSE3+)
// decode as O_UNIMPL (sse_valid), so lanes exit UNIMPLEMENTED as in the oracle.
//
// The XMM registers and MXCSR live in the lane's cold state (P.full[lane],
// wtfgpu_regs_t: read_regs / write_regs / restore already carry them). As in
// exec(), nothing is committed before every access has succeeded: 16-byte
// stores probe both ends for write permission first, so a fault or a
// copy-on-write restart never leaves half an operand written.
#pragma once
#include "engine_exec.h"

namespace wtfgpu_dev {

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

// Decode-time check: is (opcode, prefix class, modrm) inside the subset?
// Register-only / memory-only violations are #UD at execution, not here.
__device__ __forceinline__ bool sse_valid(u32 c, u32 pc, u32 is_mem, u32 r3) {
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

// n bytes (4, 8 or 16) at ea, zero-extended
__device__ __forceinline__ bool xload(Lane &L, u64 ea, u32 n, X128 &v) {
  v.lo = v.hi = 0;
  if (n <= 8) return vread(L, ea, n, v.lo);
  return vread(L, ea, 8, v.lo) && vread(L, ea + 8, 8, v.hi);
}
// n bytes of v to ea: both ends pass the write check before anything is written
__device__ __forceinline__ bool xstore(Lane &L, u64 ea, u32 n, X128 v) {
  if (n <= 8) return vwrite(L, ea, n, v.lo);
  if (!xlate(L, ea, ACC_WPROBE) || !xlate(L, ea + 15, ACC_WPROBE)) return false;
  return vwrite(L, ea, 8, v.lo) && vwrite(L, ea + 8, 8, v.hi);
}

// One attempt at an SSE instruction (exec() protocol: X_FAULT with L.miss set
// asks for a translation service and a rerun).
__device__ __noinline__ int sse_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 c = u.sub, pc = u.bsz, r3 = u.reg & 7;
  const bool mem = u.is_mem;
  const u32 imm = (u32)u.imm & 0xff;
  u64 ea = 0;
  if (mem) {
    if (u.riprel) {
      ea = nrip + u.disp;
    } else {
      ea = u.disp;
      if (u.base >= 0) ea += R(L, u.base);
      if (u.index >= 0) ea += R(L, u.index) << u.scale;
    }
    if (u.p67) ea &= 0xffffffffull;
    if (u.seg) ea += u.seg == 4 ? P.fs_base[L.lane] : P.gs_base[L.lane];
  }
  if (c == 0xc3) {  // movnti m32/64, r
    if (!mem) {
      set_fault(L, WTFGPU_VEC_UD, 0, 0);
      return X_FAULT;
    }
    const u32 sz = (u.rex & 8) ? 8 : 4;
    return vwrite(L, ea, sz, R(L, u.reg) & szmask(sz)) ? X_OK : X_FAULT;
  }
  if (c == 0xae && !mem) return X_OK;  // lfence / mfence / sfence
  const bool reg_only = (c >= 0x71 && c <= 0x73) || c == 0x50 || c == 0xd7 || c == 0xc5;
  const bool mem_only = c == 0x13 || c == 0x17 || c == 0x2b || c == 0xe7 || c == 0xae ||
                        ((c == 0x12 || c == 0x16) && pc == 1);
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
  // the r/m operand: 16 bytes aligned unless an unaligned move / narrower form
  u32 n = 16;
  bool align = true;
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
  if (mem && n == 16 && align && (ea & 15)) {
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return X_FAULT;
  }
  const bool store = c == 0x11 || c == 0x13 || c == 0x17 || c == 0x29 || c == 0x2b || c == 0x7f || c == 0xe7 ||
                     c == 0xd6 || (c == 0x7e && pc == 1) || (c == 0xae && r3 == 3);
  X128 a = xmm_get(P, L, u.reg), b{0, 0}, r{0, 0};
  if (!store) {
    if (mem) {
      if (!xload(L, ea, n, b)) return X_FAULT;
    } else if (c == 0x6e || c == 0xc4) {
      b.lo = R(L, u.rm);
    } else {
      b = xmm_get(P, L, u.rm);
    }
  }
  // ---- compute: r goes to xmm[reg] unless a case returns itself
  switch (c) {
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
    case 0x14: case 0x15: r = sse_unpack(pc ? 8 : 4, c == 0x15, a, b); break;
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
    case 0x54: case 0xdb: r = X128{a.lo & b.lo, a.hi & b.hi}; break;
    case 0x55: case 0xdf: r = X128{~a.lo & b.lo, ~a.hi & b.hi}; break;
    case 0x56: case 0xeb: r = X128{a.lo | b.lo, a.hi | b.hi}; break;
    case 0x57: case 0xef: r = X128{a.lo ^ b.lo, a.hi ^ b.hi}; break;
    case 0x60: case 0x61: case 0x62: case 0x6c: r = sse_unpack(c == 0x60 ? 1 : c == 0x61 ? 2 : c == 0x62 ? 4 : 8, 0, a, b); break;
    case 0x68: case 0x69: case 0x6a: case 0x6d: r = sse_unpack(c == 0x68 ? 1 : c == 0x69 ? 2 : c == 0x6a ? 4 : 8, 1, a, b); break;
    case 0x63: case 0x67: case 0x6b: {  // packsswb, packuswb, packssdw
      const u32 w = c == 0x6b ? 4 : 2, h = 16 / w;
      for (u32 i = 0; i < 2 * h; i++) {
        const i64 x = i < h ? xsel(a, i, w) : xsel(b, i - h, w);
        xset(r, i, w / 2, c == 0x67 ? sat_u(x, 1) : sat_s(x, w / 2));
      }
      break;
    }
    case 0x64: case 0x65: case 0x66: r = sse_ewise(EW_GT, 1u << (c - 0x64), a, b); break;
    case 0x74: case 0x75: case 0x76: r = sse_ewise(EW_EQ, 1u << (c - 0x74), a, b); break;
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
    case 0x70:
      r = b;
      if (pc == 1) {
        for (u32 i = 0; i < 4; i++) xset(r, i, 4, xel(b, (imm >> (2 * i)) & 3, 4));
      } else {
        const u32 o = pc == 2 ? 4 : 0;
        for (u32 i = 0; i < 4; i++) xset(r, i + o, 2, xel(b, ((imm >> (2 * i)) & 3) + o, 2));
      }
      break;
    case 0x71: case 0x72: case 0x73: {
      if (c == 0x73 && (r3 == 3 || r3 == 7)) {  // psrldq / pslldq (bytes)
        for (u32 i = 0; i < 16; i++) {
          const i32 s = r3 == 3 ? (i32)(i + imm) : (i32)i - (i32)imm;
          if (s >= 0 && s < 16) xset(r, i, 1, xel(b, (u32)s, 1));
        }
      } else {
        r = sse_shift(r3 == 2 ? 0 : r3 == 4 ? 1 : 2, c == 0x71 ? 2 : c == 0x72 ? 4 : 8, b, imm);
      }
      xmm_put(P, L, u.rm, r);
      return X_OK;
    }
    case 0xc4: r = a; xset(r, imm & 7, 2, b.lo & 0xffff); break;  // pinsrw
    case 0xc5: RS(L, u.reg, xel(b, imm & 7, 2)); return X_OK;     // pextrw
    case 0xc6:
      if (pc == 0) {
        xset(r, 0, 4, xel(a, imm & 3, 4));
        xset(r, 1, 4, xel(a, (imm >> 2) & 3, 4));
        xset(r, 2, 4, xel(b, (imm >> 4) & 3, 4));
        xset(r, 3, 4, xel(b, (imm >> 6) & 3, 4));
      } else {
        r = X128{(imm & 1) ? a.hi : a.lo, (imm & 2) ? b.hi : b.lo};
      }
      break;
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
    case 0xd1: case 0xd2: case 0xd3: r = sse_shift(0, c == 0xd1 ? 2 : c == 0xd2 ? 4 : 8, a, b.lo); break;
    case 0xe1: case 0xe2: r = sse_shift(1, c == 0xe1 ? 2 : 4, a, b.lo); break;
    case 0xf1: case 0xf2: case 0xf3: r = sse_shift(2, c == 0xf1 ? 2 : c == 0xf2 ? 4 : 8, a, b.lo); break;
    case 0xd4: r = X128{a.lo + b.lo, a.hi + b.hi}; break;
    case 0xfb: r = X128{a.lo - b.lo, a.hi - b.hi}; break;
    case 0xfc: case 0xfd: case 0xfe: r = sse_ewise(EW_ADD, 1u << (c - 0xfc), a, b); break;
    case 0xf8: case 0xf9: case 0xfa: r = sse_ewise(EW_SUB, 1u << (c - 0xf8), a, b); break;
    case 0xd5: r = sse_ewise(EW_MULLO, 2, a, b); break;
    case 0xe5: r = sse_ewise(EW_MULHS, 2, a, b); break;
    case 0xe4: r = sse_ewise(EW_MULHU, 2, a, b); break;
    case 0xd8: case 0xd9: r = sse_ewise(EW_SUBUS, c - 0xd7, a, b); break;
    case 0xdc: case 0xdd: r = sse_ewise(EW_ADDUS, c - 0xdb, a, b); break;
    case 0xe8: case 0xe9: r = sse_ewise(EW_SUBS, c - 0xe7, a, b); break;
    case 0xec: case 0xed: r = sse_ewise(EW_ADDS, c - 0xeb, a, b); break;
    case 0xda: r = sse_ewise(EW_MINU, 1, a, b); break;
    case 0xde: r = sse_ewise(EW_MAXU, 1, a, b); break;
    case 0xea: r = sse_ewise(EW_MINS, 2, a, b); break;
    case 0xee: r = sse_ewise(EW_MAXS, 2, a, b); break;
    case 0xe0: r = sse_ewise(EW_AVG, 1, a, b); break;
    case 0xe3: r = sse_ewise(EW_AVG, 2, a, b); break;
    case 0xf4: r = X128{(a.lo & 0xffffffffull) * (b.lo & 0xffffffffull), (a.hi & 0xffffffffull) * (b.hi & 0xffffffffull)}; break;
    case 0xf5:  // pmaddwd
      for (u32 i = 0; i < 4; i++)
        xset(r, i, 4, (u64)(xsel(a, 2 * i, 2) * xsel(b, 2 * i, 2) + xsel(a, 2 * i + 1, 2) * xsel(b, 2 * i + 1, 2)));
      break;
    case 0xf6: {  // psadbw
      u64 s0 = 0, s1 = 0;
      for (u32 i = 0; i < 8; i++) {
        const u64 x0 = xel(a, i, 1), y0 = xel(b, i, 1), x1 = xel(a, i + 8, 1), y1 = xel(b, i + 8, 1);
        s0 += x0 > y0 ? x0 - y0 : y0 - x0;
        s1 += x1 > y1 ? x1 - y1 : y1 - x1;
      }
      r = X128{s0, s1};
      break;
    }
    default: return X_UNIMPL;
  }
  xmm_put(P, L, u.reg, r);
  return X_OK;
}

}  // namespace wtfgpu_dev
