// engine_avx2x.h — FMA3, F16C and the AVX2 gathers (convention U46,
// DESIGN.md §5): the forms a guest picks from a capture host's CPUID (ucrt's
// math paths select FMA3 this way; vectorised code gathers). Included by
// engine_sse.h after engine_sse4.h; vex_exec hands every form ax_form()
// accepts to ax_exec. VEX only, mandatory prefix 66.
//
//   FMA3    0f 38 96-9f a6-af b6-bf: vfmaddsub / vfmsubadd (x6 / x7),
//           vfmadd / vfmsub / vfnmadd / vfnmsub packed (x8 xa xc xe) and scalar
//           (x9 xb xd xf); the high nibble is the operand order (9: 132,
//           a: 213, b: 231); VEX.W selects binary64. a * b + c with one
//           rounding (f_fma); NaNs: the first of a, b, c (the multiplicands,
//           then the addend, whatever the encoding's order), quietened, its
//           sign kept by the negated forms; IE for any SNaN or an invalid
//           product / sum, which then raise no DE (the host's order).
//   F16C    0f 38 13 vcvtph2ps (exact; IE for an SNaN; DAZ does not apply to
//           binary16), 0f 3a 1d vcvtps2ph (imm8[2] ? MXCSR.RC : imm8[1:0];
//           DAZ applies, FTZ does not: binary16 denormals are results);
//           VEX.W1 or vvvv != 1111 is #UD. A memory destination is written
//           after the conversion, so an unmasked exception faults first.
//   gathers 0f 38 90-93 vpgatherdd / dq / qd / qq, vgatherdps / dpd / qps /
//           qpd: VSIB (#UD without a SIB byte, for a register operand, or when
//           two of destination, index and mask are one register); element j
//           loads when mask element j's sign is set, in order from element 0,
//           and its mask element is cleared once it is in the destination;
//           a faulting element leaves the earlier elements done (dest written,
//           mask cleared) and the rest untouched, as the SDM describes and a
//           restart completes; at the end the whole mask register is zero.
//           Destination and mask keep the VEX.128 / qd-qps rules: bits above
//           the elements written (above 64 for the two-element qd / qps) are
//           zeroed at completion.
//
// Exceptions of the arithmetic forms as engine_ssefp.h (U40): every element
// is computed with flags, an unmasked IE / DE / ZE sets only those, any other
// unmasked flag sets them all, and the instruction faults (#XM, or #UD without
// CR4.OSXMMEXCPT) with its destination unwritten.
#pragma once
#include "engine_fp.h"

namespace wtfgpu_dev {

// 1 FMA3, 2 F16C, 3 gather; 0 otherwise
__host__ __device__ inline u32 ax_form(u32 map, u32 c, u32 pp, bool vex) {
  if (!vex || pp != 1) return 0;
  if (map == 2) {
    if ((c >= 0x96 && c <= 0x9f) || (c >= 0xa6 && c <= 0xaf) || (c >= 0xb6 && c <= 0xbf)) return 1;
    if (c == 0x13) return 2;
    if (c >= 0x90 && c <= 0x93) return 3;
    return 0;
  }
  return map == 3 && c == 0x1d ? 2 : 0;
}

__device__ __forceinline__ u32 clz128(u128 x) {
  const u64 hi = (u64)(x >> 64);
  return hi ? (u32)__builtin_clzll(hi) : 64 + (u32)__builtin_clzll((u64)x);
}
__device__ __forceinline__ u128 jam_shr128(u128 x, u32 n) {
  if (n == 0) return x;
  if (n >= 127) return (u128)(x != 0);
  return (x >> n) | (u128)((x & ((((u128)1) << n) - 1)) != 0);
}

// a * b + c with one rounding; negp negates the product, negc the addend
// (exact, before the sum). w: 0 binary32, 1 binary64.
__device__ __noinline__ u64 f_fma(FEnv &v, u64 a, u64 b, u64 c, u32 negp, u32 negc, u32 w) {
  const bool na = f_nan(a, w), nb = f_nan(b, w), nc = f_nan(c, w);
  if (na || nb || nc) {
    if (f_snan(a, w) || f_snan(b, w) || f_snan(c, w)) v.fl |= FE_I;
    return f_quiet(na ? a : nb ? b : c, w);
  }
  a = f_daz(v, a, w);
  b = f_daz(v, b, w);
  c = f_daz(v, c, w);
  const bool ia = f_inf(a, w), ib = f_inf(b, w), za = f_zero(a, w), zb = f_zero(b, w), ic = f_inf(c, w);
  const u32 sp = f_sign(a, w) ^ f_sign(b, w) ^ negp, sc = f_sign(c, w) ^ negc;
  // invalid: 0 * inf, or an infinite product meeting the opposite infinity
  if ((ia && zb) || (ib && za) || ((ia || ib) && ic && sp != sc)) {
    v.fl |= FE_I;
    return f_indef(w);
  }
  if (f_den(a, w) || f_den(b, w) || f_den(c, w)) v.fl |= FE_D;
  if (ia || ib) return f_infv(sp, w);
  if (ic) return f_infv(sc, w);
  const u64 cs = (c & ~f_signed(1, w)) | f_signed(sc, w);
  if (za || zb) return f_addsub(v, f_signed(sp, w), cs, w);  // a zero product: an addition's rules
  i32 ea, eb;
  u64 ma, mb;
  f_unpack(a, w, ea, ma);
  f_unpack(b, w, eb, mb);
  // the exact product: P / 2^125 * 2^X (P < 2^127)
  const u128 P = ((u128)ma * mb) << 1;
  const i32 X = ea + eb + 2 - 2 * fBias(w);
  u128 S;
  u32 s;
  i32 Xr;
  if (f_zero(c, w)) {  // a nonzero product plus a zero: the product, rounded once
    S = P;
    s = sp;
    Xr = X;
  } else {
    i32 ec;
    u64 mc;
    f_unpack(cs, w, ec, mc);
    const u128 C = (u128)mc << 63;  // C / 2^125 * 2^XC
    const i32 XC = ec + 1 - fBias(w);
    u128 Pa = P, Ca = C;
    if (X >= XC) {
      Ca = jam_shr128(C, (u32)(X - XC));
      Xr = X;
    } else {
      Pa = jam_shr128(P, (u32)(XC - X));
      Xr = XC;
    }
    if (sp == sc) {
      S = Pa + Ca;
      s = sp;
    } else if (Pa >= Ca) {
      S = Pa - Ca;
      s = sp;
    } else {
      S = Ca - Pa;
      s = sc;
    }
    if (S == 0) return f_signed(v.rc == 1, w);  // an exact zero sum: +0, -0 rounding down
  }
  // S / 2^125 * 2^Xr, S's leading one at bit L -> m (leading one at bit 62)
  const u32 L = 127 - clz128(S);
  const u64 m = L >= 62 ? (u64)jam_shr128(S, L - 62) : (u64)S << (62 - L);
  return f_round(v, s, (i32)L - 126 + Xr + fBias(w), m, w);
}

// binary16 -> binary32 (exact); IE for an SNaN; DAZ does not apply
__device__ __forceinline__ u64 f_from_half(FEnv &v, u64 h) {
  const u32 s = (u32)(h >> 15) & 1, ex = (u32)(h >> 10) & 31;
  const u64 fr = h & 0x3ff;
  if (ex == 31) {
    if (fr && !(fr & 0x200)) v.fl |= FE_I;
    return ((u64)s << 31) | 0x7f800000ull | (fr ? ((fr | 0x200) << 13) : 0);
  }
  if (ex == 0 && fr == 0) return (u64)s << 31;
  i32 e;
  u64 m;
  f_unpack(h, 2, e, m);
  FEnv exact = v;  // no rounding happens: a binary16 value fits binary32
  return f_round(exact, s, e - fBias(2) + fBias(0), m, 0);
}

// binary32 -> binary16 under rc; DAZ applies, FTZ does not
__device__ __noinline__ u64 f_to_half(FEnv &v, u64 x, u32 rc) {
  const u32 s = f_sign(x, 0);
  if (f_nan(x, 0)) {
    if (f_snan(x, 0)) v.fl |= FE_I;
    return ((u64)s << 15) | 0x7e00 | (f_frac(x, 0) >> 13);
  }
  x = f_daz(v, x, 0);
  if (f_den(x, 0)) v.fl |= FE_D;
  if (f_inf(x, 0)) return ((u64)s << 15) | 0x7c00;
  if (f_zero(x, 0)) return (u64)s << 15;
  i32 e;
  u64 m;
  f_unpack(x, 0, e, m);
  FEnv h = v;
  h.rc = rc;
  h.ftz = 0;
  const u64 r = f_round(h, s, e - fBias(0) + fBias(2), m, 2);
  v.fl |= h.fl;
  return r;
}

// one element's address of a gather: base + disp + sext(index) << scale
__device__ __forceinline__ u64 vsib_ea(const Dev &P, const Lane &L, const UOp &u, u64 idx) {
  u64 ea = u.disp + (u.base >= 0 ? R(L, u.base) : 0) + (idx << u.scale);
  if (u.p67) ea &= 0xffffffffull;
  if (u.seg) ea += u.seg == 4 ? P.fs_base[L.lane] : P.gs_base[L.lane];
  return ea;
}

// (ax_exec checked the #UD rules: a SIB byte, three distinct registers)
__device__ __noinline__ int ax_gather(const Dev &P, Lane &L, const UOp &u, u32 c, u32 l256, u32 W, u32 vvvv) {
  const u32 dst = u.reg & 15, msk = vvvv;
  const u32 ew = W ? 8 : 4, iw = (c & 1) ? 8 : 4;
  // elements: the wider of data and index fills the vector length
  const u32 n = (l256 ? 32 : 16) / (ew > iw ? ew : iw);
  const Y256 ix = ymm_get(P, L, (u32)u.index);
  wtfgpu_regs_t &F = P.full[L.lane];
  for (u32 j = 0; j < n; j++) {
    const Y256 mk = ymm_get(P, L, msk);
    if (!(yel(mk, j, ew) >> (8 * ew - 1))) continue;
    const u64 iv = yel(ix, j, iw), idx = iw == 4 ? (u64)(i64)(i32)(u32)iv : iv;
    u64 val;
    if (!vread(L, vsib_ea(P, L, u, idx), ew, val)) return X_FAULT;  // earlier elements stay done
    Y256 d = ymm_get(P, L, dst), m2 = mk;
    yset(d, j, ew, val);
    yset(m2, j, ew, 0);
    F.xmm[dst][0] = d.l.lo, F.xmm[dst][1] = d.l.hi, F.ymmh[dst][0] = d.h.lo, F.ymmh[dst][1] = d.h.hi;
    F.xmm[msk][0] = m2.l.lo, F.xmm[msk][1] = m2.l.hi, F.ymmh[msk][0] = m2.h.lo, F.ymmh[msk][1] = m2.h.hi;
    for (u32 q = 0; q < 4; q++) F.zmmh[dst][q] = F.zmmh[msk][q] = 0;  // VEX: bits 511:256 (U47)
  }
  // completion: bits above the n elements of the destination zeroed, the mask all zero
  Y256 d = ymm_get(P, L, dst);
  const u32 bytes = n * ew;
  if (bytes <= 8) d.l.hi = 0;
  if (bytes <= 16) d.h = X128{0, 0};
  ymm_put(P, L, dst, d, 1);
  ymm_put(P, L, msk, Y256{X128{0, 0}, X128{0, 0}}, 0);
  return X_OK;
}

__device__ __noinline__ int ax_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, map = vex_map(x);
  const u32 l256 = (x >> 1) & 1, W = (x >> 2) & 1, vvvv = (x >> 4) & 15;
  const u32 kind = ax_form(map, c, u.bsz, true);
  const u64 cr4 = P.sys[L.lane].cr4;
  bool ud = ((x >> 16) & 1) || !((cr4 >> 18) & 1) || (P.full[L.lane].xcr0 & 6) != 6;
  if (kind == 2 && (W || vvvv != 0)) ud = true;
  // gathers: no memory operand or no SIB (the decoder leaves index < 0), or
  // two of destination, index and mask the same register
  if (kind == 3 && (!u.is_mem || u.index < 0 || (u.reg & 15) == vvvv || (u.reg & 15) == (u32)u.index ||
                    vvvv == (u32)u.index))
    ud = true;
  if (ud) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  if (L.cr0 & 8) {
    set_fault(L, 7, 0, 0);  // #NM
    return X_FAULT;
  }
  if (kind == 3) return ax_gather(P, L, u, c, l256, W, vvvv);
  const bool mem = u.is_mem;
  const u32 vl = l256 ? 32 : 16, imm = (u32)u.imm & 0xff;
  wtfgpu_regs_t &F = P.full[L.lane];
  FEnv v = fenv_mx(F.mxcsr);
  Y256 r{X128{0, 0}, X128{0, 0}};
  u32 keep256 = l256;
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  if (kind == 2 && map == 3) {  // vcvtps2ph: reg -> r/m
    const Y256 s = ymm_get(P, L, u.reg);
    const u32 rc = (imm & 4) ? v.rc : imm & 3;
    for (u32 i = 0; i < vl / 4; i++) xset(r.l, i, 2, f_to_half(v, yel(s, i, 4), rc));
    const u32 pre = v.fl & 7;
    if (pre & ~v.masks) {
      F.mxcsr |= pre;
      return xm_fault(L, cr4);
    }
    if (v.fl & ~v.masks & 63) {
      F.mxcsr |= v.fl;
      return xm_fault(L, cr4);
    }
    if (mem) {
      if (!xstore(L, ea, vl / 2, r.l)) return X_FAULT;  // MXCSR's flags only once the store is done
    } else {
      ymm_put(P, L, u.rm, r, 0);
    }
    F.mxcsr |= v.fl;
    return X_OK;
  }
  // ---- the r/m source
  u32 n = vl;
  const u32 ew = W ? 8 : 4;
  const bool scalar = kind == 1 && (c & 1) && (c & 15) >= 9;
  if (kind == 2) n = vl / 2;  // vcvtph2ps: xmm / m64, or m128
  else if (scalar) n = ew;
  Y256 b{X128{0, 0}, X128{0, 0}};
  if (mem) {
    if (!yload(L, ea, n, b)) return X_FAULT;
  } else {
    b = ymm_get(P, L, u.rm);
    if (kind == 2 && !l256) b.l.hi = 0, b.h = X128{0, 0};
  }
  if (kind == 2) {  // vcvtph2ps
    for (u32 i = 0; i < vl / 4; i++) yset(r, i, 4, f_from_half(v, yel(b, i, 2)));
  } else {
    const Y256 d = ymm_get(P, L, u.reg), s2 = ymm_get(P, L, vvvv);
    const u32 ord = c >> 4, f = c & 15;  // 9: 132, a: 213, b: 231
    const Y256 &A = ord == 0x9 ? d : s2;
    const Y256 &B = ord == 0xa ? d : b;
    const Y256 &C = ord == 0x9 ? s2 : ord == 0xa ? b : d;
    const u32 negp = f >= 0xc;  // vfnm*
    const u32 ne = scalar ? 1 : vl / ew;
    if (scalar) {
      r = Y256{d.l, X128{0, 0}};
      keep256 = 0;
    }
    for (u32 i = 0; i < ne; i++) {
      u32 negc;
      if (f == 6) negc = (i & 1) ^ 1;       // vfmaddsub: even elements subtract
      else if (f == 7) negc = i & 1;        // vfmsubadd: odd elements subtract
      else negc = f == 0xa || f == 0xb || f == 0xe || f == 0xf;
      yset(r, i, ew, f_fma(v, yel(A, i, ew), yel(B, i, ew), yel(C, i, ew), negp, negc, W));
    }
  }
  const u32 pre = v.fl & 7;
  if (pre & ~v.masks) {
    F.mxcsr |= pre;
    return xm_fault(L, cr4);
  }
  if (v.fl & ~v.masks & 63) {
    F.mxcsr |= v.fl;
    return xm_fault(L, cr4);
  }
  F.mxcsr |= v.fl;
  ymm_put(P, L, u.reg, r, keep256);
  return X_OK;
}

}  // namespace wtfgpu_dev
