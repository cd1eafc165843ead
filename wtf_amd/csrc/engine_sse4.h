// engine_sse4.h — the SSSE3 / SSE4.1 integer forms (legacy 66 0f 38 / 66 0f
// 3a and their VEX encodings) and the AVX / AVX2 lane-crossing forms
// (permutes, 128-bit inserts / extracts, broadcasts, variable shifts), the
// rest of what cpuid_leaf enumerates (convention U41). Included
// by engine_sse.h; sse_exec / vex_exec hand every form s4_form() accepts to
// s4_exec.
//
// Outside (UNIMPLEMENTED): the SSSE3 MMX-register forms (the gathers are in
// engine_avx2x.h).
#pragma once
#include "engine_fp.h"

namespace wtfgpu_dev {

// r/m operand shapes
enum : u32 { S4_FULL, S4_HALF, S4_QUARTER, S4_EIGHTH, S4_B, S4_W, S4_D, S4_DQ, S4_X128, S4_Q };

struct S4Form {
  u32 ok;       // an executed form
  u32 shape;    // r/m operand size class
  u32 align;    // legacy: the 16-byte memory operand must be aligned
  u32 two;      // VEX: vvvv must be 1111
  u32 l;        // VEX.L: 0 any, 1 128 only, 2 256 only
  u32 store;    // the r/m operand is written (extracts)
  u32 memonly;
};

__host__ __device__ inline S4Form s4_desc(u32 map, u32 c, u32 pp, bool vex, u32 w) {
  S4Form f{1, S4_FULL, 1, 0, 0, 0, 0};
  if (pp != 1) return S4Form{0, 0, 0, 0, 0, 0, 0};
  if (map == 2) {
    switch (c) {
      case 0x01: case 0x02: case 0x03: case 0x04: case 0x05: case 0x06: case 0x07: case 0x08: case 0x09: case 0x0a:
      case 0x0b: case 0x28: case 0x29: case 0x2b: case 0x38: case 0x39: case 0x3a: case 0x3b: case 0x3c: case 0x3d:
      case 0x3e: case 0x3f: case 0x40:
        return f;
      case 0x1c: case 0x1d: case 0x1e: f.two = 1; return f;
      case 0x10: if (vex) f.ok = 0; return f;  // pblendvb (VEX: 0f 3a 4c)
      case 0x20: case 0x23: case 0x25: case 0x30: case 0x33: case 0x35: f.shape = S4_HALF; f.align = 0; f.two = 1; return f;
      case 0x21: case 0x24: case 0x31: case 0x34: f.shape = S4_QUARTER; f.align = 0; f.two = 1; return f;
      case 0x22: case 0x32: f.shape = S4_EIGHTH; f.align = 0; f.two = 1; return f;
      case 0x2a: f.two = 1; f.memonly = 1; return f;  // movntdqa
      case 0x41: f.two = 1; f.l = 1; return f;        // phminposuw
      default: break;
    }
    if (!vex) return S4Form{0, 0, 0, 0, 0, 0, 0};
    f.align = 0;
    switch (c) {
      case 0x0c: case 0x0d: return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;               // vpermilps / pd
      case 0x0e: case 0x0f: f.two = 1; return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;    // vtestps / pd
      case 0x16: case 0x36: f.l = 2; return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;      // vpermps / vpermd
      case 0x18: f.two = 1; f.shape = S4_D; return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;  // vbroadcastss
      case 0x19: f.two = 1; f.shape = S4_Q; f.l = 2; return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;  // vbroadcastsd
      case 0x1a: case 0x5a: f.two = 1; f.shape = S4_X128; f.l = 2; f.memonly = 1;     // vbroadcastf128 / i128
        return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;
      case 0x45: case 0x47: return f;                                                  // vpsrlv / vpsllv d / q
      case 0x2c: case 0x2d: case 0x2e: case 0x2f:                                      // vmaskmovps / pd
        f.memonly = 1;
        return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;
      case 0x8c: case 0x8e: f.memonly = 1; return f;                                   // vpmaskmovd / q
      case 0x46: return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;                           // vpsravd
      default: return S4Form{0, 0, 0, 0, 0, 0, 0};
    }
  }
  if (map != 3) return S4Form{0, 0, 0, 0, 0, 0, 0};
  switch (c) {
    case 0x0e: case 0x0f: case 0x42: return f;  // pblendw, palignr, mpsadbw
    case 0x14: f.shape = S4_B; f.align = 0; f.two = 1; f.l = 1; f.store = 1; return f;  // pextrb
    case 0x15: f.shape = S4_W; f.align = 0; f.two = 1; f.l = 1; f.store = 1; return f;  // pextrw
    case 0x16: f.shape = w ? S4_Q : S4_D; f.align = 0; f.two = 1; f.l = 1; f.store = 1; return f;  // pextrd / q
    case 0x17: f.shape = S4_D; f.align = 0; f.two = 1; f.l = 1; f.store = 1; return f;  // extractps
    case 0x20: f.shape = S4_B; f.align = 0; f.l = 1; return f;                          // pinsrb
    case 0x21: f.shape = S4_D; f.align = 0; f.l = 1; return f;                          // insertps
    case 0x22: f.shape = w ? S4_Q : S4_D; f.align = 0; f.l = 1; return f;               // pinsrd / q
    default: break;
  }
  if (!vex) return S4Form{0, 0, 0, 0, 0, 0, 0};
  f.align = 0;
  switch (c) {
    case 0x00: case 0x01: f.two = 1; f.l = 2; return w ? f : S4Form{0, 0, 0, 0, 0, 0, 0};  // vpermq / vpermpd
    case 0x02: return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;                                 // vpblendd
    case 0x04: case 0x05: f.two = 1; return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;           // vpermilps / pd imm
    case 0x06: case 0x46: f.l = 2; return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;            // vperm2f128 / i128
    case 0x18: case 0x38: f.shape = S4_X128; f.l = 2; return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;  // vinsert*128
    case 0x19: case 0x39:                                                                  // vextract*128
      f.shape = S4_X128; f.two = 1; f.l = 2; f.store = 1;
      return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;
    case 0x4c: return w ? S4Form{0, 0, 0, 0, 0, 0, 0} : f;                                 // vpblendvb
    default: return S4Form{0, 0, 0, 0, 0, 0, 0};
  }
}
// decode-time: an executed form (VEX.W is checked at execution)
__host__ __device__ inline bool s4_form(u32 map, u32 c, u32 pp, bool vex) {
  return s4_desc(map, c, pp, vex, 0).ok || s4_desc(map, c, pp, vex, 1).ok;
}

__device__ __forceinline__ u32 s4_bytes(u32 shape, u32 vl) {
  switch (shape) {
    case S4_HALF: return vl / 2;
    case S4_QUARTER: return vl / 4;
    case S4_EIGHTH: return vl / 8;
    case S4_B: return 1;
    case S4_W: return 2;
    case S4_D: return 4;
    case S4_Q: return 8;
    case S4_X128: return 16;
    default: return vl;
  }
}

// one 128-bit lane of the map-2 two-source ops (a = first source, b = second)
__device__ __noinline__ X128 s4_lane2(u32 c, X128 a, X128 b) {
  X128 r{0, 0};
  switch (c) {
    case 0x01: case 0x02: case 0x03: case 0x05: case 0x06: case 0x07: {  // phadd / phsub w d sw
      const u32 ew = (c & 3) == 2 ? 4 : 2, per = 16 / ew, sub = c >= 5, sat = (c & 3) == 3;
      for (u32 i = 0; i < per; i++) {
        const X128 s = i < per / 2 ? a : b;
        const u32 j = (i % (per / 2)) * 2;
        const i64 x = xsel(s, j, ew), y = xsel(s, j + 1, ew), v = sub ? x - y : x + y;
        xset(r, i, ew, sat ? sat_s(v, ew) : (u64)v);
      }
      return r;
    }
    case 0x04:  // pmaddubsw: unsigned bytes of a times signed bytes of b, pairs, signed saturation
      for (u32 i = 0; i < 8; i++) {
        const i64 v = (i64)xel(a, 2 * i, 1) * xsel(b, 2 * i, 1) + (i64)xel(a, 2 * i + 1, 1) * xsel(b, 2 * i + 1, 1);
        xset(r, i, 2, sat_s(v, 2));
      }
      return r;
    case 0x08: case 0x09: case 0x0a: {  // psignb / w / d
      const u32 ew = 1u << (c - 8);
      for (u32 i = 0; i < 16 / ew; i++) {
        const i64 s = xsel(b, i, ew);
        xset(r, i, ew, s < 0 ? (u64)0 - xel(a, i, ew) : s == 0 ? 0 : xel(a, i, ew));
      }
      return r;
    }
    case 0x0b:  // pmulhrsw
      for (u32 i = 0; i < 8; i++) xset(r, i, 2, (u64)((((xsel(a, i, 2) * xsel(b, i, 2)) >> 14) + 1) >> 1));
      return r;
    case 0x1c: case 0x1d: case 0x1e: {  // pabsb / w / d (of b)
      const u32 ew = 1u << (c - 0x1c);
      for (u32 i = 0; i < 16 / ew; i++) {
        const i64 s = xsel(b, i, ew);
        xset(r, i, ew, (u64)(s < 0 ? -s : s));
      }
      return r;
    }
    case 0x28:  // pmuldq: signed dwords 0 and 2
      r.lo = (u64)((i64)(i32)(u32)b.lo * (i64)(i32)(u32)a.lo);
      r.hi = (u64)((i64)(i32)(u32)b.hi * (i64)(i32)(u32)a.hi);
      return r;
    case 0x29: r.lo = a.lo == b.lo ? ~0ull : 0; r.hi = a.hi == b.hi ? ~0ull : 0; return r;  // pcmpeqq
    case 0x2b:  // packusdw
      for (u32 i = 0; i < 4; i++) xset(r, i, 2, sat_u(xsel(a, i, 4), 2));
      for (u32 i = 0; i < 4; i++) xset(r, i + 4, 2, sat_u(xsel(b, i, 4), 2));
      return r;
    case 0x38: return sse_ewise(EW_MINS, 1, a, b);
    case 0x39: return sse_ewise(EW_MINS, 4, a, b);
    case 0x3a: return sse_ewise(EW_MINU, 2, a, b);
    case 0x3b: return sse_ewise(EW_MINU, 4, a, b);
    case 0x3c: return sse_ewise(EW_MAXS, 1, a, b);
    case 0x3d: return sse_ewise(EW_MAXS, 4, a, b);
    case 0x3e: return sse_ewise(EW_MAXU, 2, a, b);
    case 0x3f: return sse_ewise(EW_MAXU, 4, a, b);
    case 0x40: return sse_ewise(EW_MULLO, 4, a, b);
    default: {  // 0x41 phminposuw (of b)
      u32 best = 0;
      for (u32 i = 1; i < 8; i++)
        if (xel(b, i, 2) < xel(b, best, 2)) best = i;
      r.lo = xel(b, best, 2) | ((u64)best << 16);
      return r;
    }
  }
}

// pmovsx / pmovzx: the source's low elements widened (c: 20-25 sign, 30-35 zero)
__device__ __forceinline__ Y256 s4_pmov(u32 c, const Y256 &b, u32 vl) {
  static const u8 from[6] = {1, 1, 1, 2, 2, 4}, to[6] = {2, 4, 8, 4, 8, 8};
  const u32 k = c & 7, fw = from[k], tw = to[k], sx = c < 0x30;
  Y256 r{X128{0, 0}, X128{0, 0}};
  for (u32 i = 0; i < vl / tw; i++) {
    u64 v = xel(b.l, i, fw);
    if (sx) v = sext(v, fw);
    yset(r, i, tw, v & szmask(tw));
  }
  return r;
}

__device__ __noinline__ int s4_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, pp = u.bsz, map = vex_map(x);
  const bool vex = x & 1, mem = u.is_mem;
  // W: the element size where it picks one (every mode); for (v)pextrq /
  // (v)pinsrq the GPR size, whose VEX.W1 32-bit code ignores (the W0 forms)
  const u32 l256 = vex ? (x >> 1) & 1 : 0, vvvv = vex ? (x >> 4) & 15 : 0;
  const u32 W = (vex ? (x >> 2) & 1 : (u.rex >> 3) & 1) &
                ~(u32)(map == 3 && (c == 0x16 || c == 0x22) && (L.efer & EFER_M32) ? 1 : 0);
  const u32 imm = (u32)u.imm & 0xff;
  const u32 vl = l256 ? 32 : 16;
  const S4Form f = s4_desc(map, c, pp, vex, W);
  // ---- #UD / #NM (the legacy CR checks ran in sse_exec)
  bool ud = !f.ok || (f.memonly && !mem);
  if (vex) {
    const u64 cr4 = P.sys[L.lane].cr4;
    if (((x >> 16) & 1) || !((cr4 >> 18) & 1) || (P.full[L.lane].xcr0 & 6) != 6) ud = true;
    if ((f.two && vvvv != 0) || (f.l == 1 && l256) || (f.l == 2 && !l256)) ud = true;
  }
  if (ud) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  if (vex && (L.cr0 & 8)) {
    set_fault(L, 7, 0, 0);  // #NM
    return X_FAULT;
  }
  const u32 n = s4_bytes(f.shape, vl);
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  if (mem && ((!vex && f.align && n == 16 && (ea & 15)) || (vex && map == 2 && c == 0x2a && (ea & (vl - 1))))) {
    // legacy 16-byte operands are aligned; vmovntdqa too, at its own size
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return X_FAULT;
  }
  const Y256 s = vex ? ymm_get(P, L, u.reg) : Y256{xmm_get(P, L, u.reg), X128{0, 0}};  // reg operand
  const Y256 a = vex ? ymm_get(P, L, vvvv) : s;                                         // first source
  // ---- vmaskmovps / pd, vpmaskmovd / q: only the elements whose mask (vvvv) sign bit is set
  // touch memory, so only they fault; a store checks them all before it writes
  if (map == 2 && ((c >= 0x2c && c <= 0x2f) || c == 0x8c || c == 0x8e)) {
    const u32 ew = (c == 0x2d || c == 0x2f || (c >= 0x8c && W)) ? 8 : 4, ne = vl / ew;
    if (c == 0x2e || c == 0x2f || c == 0x8e) {
      for (u32 i = 0; i < ne; i++)
        if ((yel(a, i, ew) >> (8 * ew - 1)) && !span_w(L, ea + i * ew, ew)) return X_FAULT;
      for (u32 i = 0; i < ne; i++)
        if ((yel(a, i, ew) >> (8 * ew - 1)) && !vwrite(L, ea + i * ew, ew, yel(s, i, ew))) return X_FAULT;
      return X_OK;
    }
    Y256 r{X128{0, 0}, X128{0, 0}};
    for (u32 i = 0; i < ne; i++)
      if (yel(a, i, ew) >> (8 * ew - 1)) {
        u64 v;
        if (!vread(L, ea + i * ew, ew, v)) return X_FAULT;
        yset(r, i, ew, v);
      }
    ymm_put(P, L, u.reg, r, l256);
    return X_OK;
  }
  // ---- extracts: reg -> r/m
  if (f.store) {
    u64 v;
    X128 wide{0, 0};
    switch (c) {
      case 0x14: v = xel(s.l, imm & 15, 1); break;
      case 0x15: v = xel(s.l, imm & 7, 2); break;
      case 0x16: v = W ? xel(s.l, imm & 1, 8) : xel(s.l, imm & 3, 4); break;
      case 0x17: v = xel(s.l, imm & 3, 4); break;
      default: wide = (imm & 1) ? s.h : s.l; v = 0; break;  // vextract*128
    }
    if (mem) {
      if (f.shape == S4_X128) return xstore(L, ea, 16, wide) ? X_OK : X_FAULT;
      return vwrite(L, ea, n, v & szmask(n)) ? X_OK : X_FAULT;
    }
    if (f.shape == S4_X128) {
      ymm_put(P, L, u.rm, Y256{wide, X128{0, 0}}, 0);
      return X_OK;
    }
    RS(L, u.rm, v & szmask(W && c == 0x16 ? 8 : 4));  // a 32-bit destination is zero-extended
    return X_OK;
  }
  // ---- the r/m source
  Y256 b{X128{0, 0}, X128{0, 0}};
  if (mem) {
    if (!yload(L, ea, n, b)) return X_FAULT;
  } else if (map == 3 && (c == 0x20 || c == 0x22)) {
    b.l.lo = R(L, u.rm);
  } else {
    b = vex ? ymm_get(P, L, u.rm) : Y256{xmm_get(P, L, u.rm), X128{0, 0}};
  }
  Y256 r{X128{0, 0}, X128{0, 0}};
  if (map == 2) {
    switch (c) {
      case 0x20: case 0x21: case 0x22: case 0x23: case 0x24: case 0x25:
      case 0x30: case 0x31: case 0x32: case 0x33: case 0x34: case 0x35:
        r = s4_pmov(c, b, vl);
        break;
      case 0x2a: r = b; break;  // movntdqa
      case 0x10: {              // pblendvb (xmm0)
        const X128 m = xmm_get(P, L, 0);
        for (u32 i = 0; i < 16; i++) xset(r.l, i, 1, (xel(m, i, 1) >> 7) ? xel(b.l, i, 1) : xel(a.l, i, 1));
        break;
      }
      case 0x0c: case 0x0d: {  // vpermilps / pd by register: per 128-bit lane
        const u32 ew = c == 0x0c ? 4 : 8;
        for (u32 i = 0; i < vl / ew; i++) {
          const u32 lane0 = (i * ew) & 16, sel = c == 0x0c ? (u32)yel(b, i, 4) & 3 : ((u32)yel(b, i, 8) >> 1) & 1;
          yset(r, i, ew, yel(a, lane0 / ew + sel, ew));
        }
        break;
      }
      case 0x0e: case 0x0f: {  // vtestps / pd: the sign bits only
        const u32 ew = c == 0x0e ? 4 : 8;
        bool z = true, cf = true;
        for (u32 i = 0; i < vl / ew; i++) {
          const u64 x1 = yel(s, i, ew) >> (8 * ew - 1), y1 = yel(b, i, ew) >> (8 * ew - 1);
          if (x1 & y1) z = false;
          if (!x1 && y1) cf = false;
        }
        L.rflags = (L.rflags & ~F_STATUS) | (z ? F_ZF : 0) | (cf ? F_CF : 0);
        return X_OK;
      }
      case 0x16: case 0x36:  // vpermps / vpermd: indices from the first source
        for (u32 i = 0; i < 8; i++) yset(r, i, 4, yel(b, (u32)yel(a, i, 4) & 7, 4));
        break;
      case 0x18: case 0x19: {  // vbroadcastss / sd (memory or the low element of an xmm)
        const u32 ew = c == 0x18 ? 4 : 8;
        for (u32 i = 0; i < vl / ew; i++) yset(r, i, ew, xel(b.l, 0, ew));
        break;
      }
      case 0x1a: case 0x5a: r = Y256{b.l, b.l}; break;  // vbroadcastf128 / i128
      case 0x45: case 0x46: case 0x47: {  // vpsrlv / vpsrav / vpsllv: counts per element
        const u32 ew = (c == 0x46 || !W) ? 4 : 8, bits = 8 * ew;
        for (u32 i = 0; i < vl / ew; i++) {
          const u64 cnt = yel(b, i, ew), v = yel(a, i, ew);
          u64 o;
          if (c == 0x46) o = (u64)((i64)sext(v, ew) >> (cnt >= bits ? bits - 1 : cnt));
          else if (cnt >= bits) o = 0;
          else o = c == 0x45 ? v >> cnt : v << cnt;
          yset(r, i, ew, o & szmask(ew));
        }
        break;
      }
      default:
        r.l = s4_lane2(c, a.l, b.l);
        if (l256) r.h = s4_lane2(c, a.h, b.h);
        break;
    }
  } else {
    switch (c) {
      case 0x0e: case 0x02: {  // pblendw (imm per word, per lane) / vpblendd (imm per dword)
        const u32 ew = c == 0x0e ? 2 : 4;
        for (u32 i = 0; i < vl / ew; i++) yset(r, i, ew, ((imm >> (i & 7)) & 1) ? yel(b, i, ew) : yel(a, i, ew));
        break;
      }
      case 0x42:  // mpsadbw: per lane, 8 sums of 4 absolute byte differences (the upper lane: imm[5:3])
        for (u32 h = 0; h < vl / 16; h++) {
          const X128 al = h ? a.h : a.l, bl = h ? b.h : b.l;
          const u32 im = h ? (imm >> 3) : imm, o1 = ((im >> 2) & 1) * 4, o2 = (im & 3) * 4;
          X128 o{0, 0};
          for (u32 j = 0; j < 8; j++) {
            u32 s = 0;
            for (u32 k = 0; k < 4; k++) {
              const i32 d = (i32)xel(al, o1 + j + k, 1) - (i32)xel(bl, o2 + k, 1);
              s += (u32)(d < 0 ? -d : d);
            }
            xset(o, j, 2, s);
          }
          if (h) r.h = o;
          else r.l = o;
        }
        break;
      case 0x0f:  // palignr: per lane, (a:b) >> 8 * imm
        for (u32 h = 0; h < vl / 16; h++) {
          const X128 al = h ? a.h : a.l, bl = h ? b.h : b.l;
          X128 o{0, 0};
          for (u32 i = 0; i < 16; i++) {
            const u32 k = i + imm;
            xset(o, i, 1, k < 16 ? xel(bl, k, 1) : k < 32 ? xel(al, k - 16, 1) : 0);
          }
          if (h) r.h = o;
          else r.l = o;
        }
        break;
      case 0x20: r.l = a.l; xset(r.l, imm & 15, 1, b.l.lo & 0xff); break;  // pinsrb
      case 0x22:                                                            // pinsrd / q
        r.l = a.l;
        if (W) xset(r.l, imm & 1, 8, b.l.lo);
        else xset(r.l, imm & 3, 4, b.l.lo & 0xffffffffull);
        break;
      case 0x21: {  // insertps: element count_s of b (memory: the dword), to count_d, then the zero mask
        const u64 e = mem ? (b.l.lo & 0xffffffffull) : xel(b.l, (imm >> 6) & 3, 4);
        r.l = a.l;
        xset(r.l, (imm >> 4) & 3, 4, e);
        for (u32 i = 0; i < 4; i++)
          if ((imm >> i) & 1) xset(r.l, i, 4, 0);
        break;
      }
      case 0x00: case 0x01:  // vpermq / vpermpd
        for (u32 i = 0; i < 4; i++) yset(r, i, 8, yel(b, (imm >> (2 * i)) & 3, 8));
        break;
      case 0x04: case 0x05: {  // vpermilps / pd by imm
        const u32 ew = c == 0x04 ? 4 : 8;
        for (u32 i = 0; i < vl / ew; i++) {
          const u32 lane0 = (i * ew) & 16;
          const u32 sel = c == 0x04 ? (imm >> (2 * (i & 3))) & 3 : (imm >> (i & 3)) & 1;
          yset(r, i, ew, yel(b, lane0 / ew + sel, ew));
        }
        break;
      }
      case 0x06: case 0x46:  // vperm2f128 / i128
        for (u32 h = 0; h < 2; h++) {
          const u32 sel = (imm >> (4 * h)) & 15;
          const X128 src = (sel & 8) ? X128{0, 0} : (sel & 3) == 0 ? a.l : (sel & 3) == 1 ? a.h : (sel & 3) == 2 ? b.l : b.h;
          if (h) r.h = src;
          else r.l = src;
        }
        break;
      case 0x18: case 0x38:  // vinsertf128 / i128
        r = a;
        if (imm & 1) r.h = b.l;
        else r.l = b.l;
        break;
      default: {  // 0x4c vpblendvb: the mask register in imm8[7:4]
        const Y256 m = ymm_get(P, L, imm >> 4);
        for (u32 i = 0; i < vl; i++) yset(r, i, 1, (yel(m, i, 1) >> 7) ? yel(b, i, 1) : yel(a, i, 1));
        break;
      }
    }
  }
  if (vex) ymm_put(P, L, u.reg, r, l256);
  else xmm_put(P, L, u.reg, r.l);
  return X_OK;
}

}  // namespace wtfgpu_dev
