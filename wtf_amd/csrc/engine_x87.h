// engine_x87.h — x87 arithmetic (convention U42): the d8-df
// forms other than the control instructions of engine_sys.h, over the 80-bit
// registers of the lane's cold state (fpst = significand, fpse = sign and
// exponent, both in ST order; TOP in FSW; the full tag word in fptw).
//
// Extended-precision arithmetic in integers: a 128-bit working significand
// (the 64 result bits, the rest a rounding word), one rounding per result at
// FCW.PC's precision (24 / 53 / 64 bits; PC applies to fadd / fsub / fmul /
// fdiv / fsqrt and their integer / popping forms only), FCW.RC, tininess after
// rounding, C1 = rounded up. Exceptions follow SDM vol. 1 8.5: stack overflow /
// underflow (IE + SF, C1), invalid operands (SNaN, unsupported formats: IE),
// QNaN propagation (x87 rule: the larger significand), DE, ZE, OE, UE, PE.
// Masked: the default result. Unmasked IE / DE / ZE: no result, no pop;
// unmasked OE / UE: the result with its exponent wrapped by 24576 (register
// destinations; a memory destination is not written). Any unmasked exception
// sets ES and B; the next waiting x87 instruction then takes #MF first.
// FOP / FIP / FDP are not maintained (U32). The transcendental forms (f2xm1,
// fyl2x, fptan, fpatan, fyl2xp1, fsincos, fsin, fcos) stay UNIMPLEMENTED.
// fbld / fbstp: 18 packed BCD digits and a sign byte (x87 vectors pin them).
#pragma once
#include "engine_fp.h"

namespace wtfgpu_dev {

struct F80 {
  u64 m;   // significand, integer bit J at 63
  u32 se;  // sign << 15 | biased exponent
};

enum : u32 { SW_IE = 1, SW_DE = 2, SW_ZE = 4, SW_OE = 8, SW_UE = 16, SW_PE = 32, SW_SF = 64, SW_ES = 0x80,
             SW_C0 = 0x100, SW_C1 = 0x200, SW_C2 = 0x400, SW_C3 = 0x4000, SW_B = 0x8000 };

struct XEnv {
  u32 rc, masks;  // FCW.RC, FCW bits 5:0 (1 = masked)
  u32 fl;         // flags raised (SW_IE .. SW_PE, SW_SF)
  u32 c1;         // the last rounding went up in magnitude
};

enum : u32 { XC_ZERO, XC_DEN, XC_NORM, XC_INF, XC_QNAN, XC_SNAN, XC_UNSUP };

__device__ __forceinline__ u32 x_sign(F80 a) { return (a.se >> 15) & 1; }
__device__ __forceinline__ i32 x_exp(F80 a) { return (i32)(a.se & 0x7fff); }
__device__ __forceinline__ u32 x_class(F80 a) {
  const i32 e = x_exp(a);
  const bool j = (a.m >> 63) != 0;
  if (e == 0) return a.m == 0 ? XC_ZERO : XC_DEN;  // pseudo-denormals (J = 1) are denormal operands
  if (e == 0x7fff) {
    if (!j) return XC_UNSUP;  // pseudo-infinity / pseudo-NaN
    if ((a.m << 1) == 0) return XC_INF;
    return ((a.m >> 62) & 1) ? XC_QNAN : XC_SNAN;
  }
  return j ? XC_NORM : XC_UNSUP;  // unnormal
}
__device__ __forceinline__ bool x_nan(u32 c) { return c == XC_QNAN || c == XC_SNAN; }
__device__ __forceinline__ F80 x_indef() { return F80{0xc000000000000000ull, 0xffff}; }
__device__ __forceinline__ F80 x_zero(u32 s) { return F80{0, s << 15}; }
__device__ __forceinline__ F80 x_inf(u32 s) { return F80{0x8000000000000000ull, (s << 15) | 0x7fff}; }
__device__ __forceinline__ F80 x_quiet(F80 a) { return F80{a.m | 0x4000000000000000ull, a.se}; }
__device__ __forceinline__ u32 x_tag(F80 a) { return tag_of(a.m, a.se); }

__device__ __forceinline__ u128 jam128(u128 x, u32 n) {
  if (n == 0) return x;
  if (n >= 128) return x != 0;
  return (x >> n) | (u128)((x << (128 - n)) != 0);
}

// finite nonzero a -> biased exponent e and significand with J at 63
__device__ __forceinline__ void x_unpack(F80 a, i32 &e, u64 &m) {
  e = x_exp(a);
  m = a.m;
  if (e == 0) e = 1;  // denormals and pseudo-denormals: 2^(1 - 16383)
  const u32 sh = (u32)__builtin_clzll(m);
  m <<= sh;
  e -= (i32)sh;
}

// (-1)^s * W / 2^127 * 2^(exp - 16383) rounded at prec (24 / 53 / 64) bits;
// W has its leading one at bit 127
__device__ __noinline__ F80 x_round(XEnv &v, u32 s, i32 exp, u128 W, u32 prec) {
  const u32 G = 128 - prec;
  const u128 one = 1, half = one << (G - 1), mask = (one << G) - 1;
  const u32 rc = v.rc;
  const u128 inc = rc == 0 ? half : rc == 3 ? (u128)0 : ((rc == 1) == (s != 0)) ? mask : (u128)0;
  v.c1 = 0;
  bool wrapped = false;
  if (exp <= 0) {
    const bool tiny = exp < 0 || (W + inc) >= W;  // no carry out of bit 127: still below 2^-16382
    if (tiny && !(v.masks & SW_UE) && exp + 24576 <= 0) {  // unmasked, beyond the wrap: a zero
      v.fl |= SW_UE | SW_PE;
      return x_zero(s);
    }
    if (tiny && !(v.masks & SW_UE)) {  // unmasked: the exponent wrapped into range
      exp += 24576;
      v.fl |= SW_UE;
      wrapped = true;
    } else {
      W = jam128(W, (u32)(1 - exp));
      exp = 0;
      const u128 rb = W & mask;
      if (rb) {
        if (tiny) v.fl |= SW_UE;
        v.fl |= SW_PE;
      }
      const u128 base = W & ~mask;
      W += inc;
      if (rc == 0 && rb == half) W &= ~(one << G);
      W &= ~mask;
      v.c1 = W > base;
      if (W >> 127) exp = 1;
      return F80{(u64)(W >> 64), (s << 15) | (u32)exp};
    }
  }
  if (!wrapped && (exp >= 0x7fff || (exp == 0x7ffe && (W + inc) < W))) {
    if (!(v.masks & SW_OE) && exp - 24576 < 0x7fff) {
      exp -= 24576;
      v.fl |= SW_OE;
    } else {
      v.fl |= SW_OE | SW_PE;
      if (inc) {
        v.c1 = 1;
        return x_inf(s);
      }
      return F80{(u64)(~mask >> 64), (s << 15) | 0x7ffe};  // the largest finite at this precision
    }
  }
  const u128 rb = W & mask, base = W & ~mask;
  if (rb) v.fl |= SW_PE;
  u128 R = W + inc;
  bool up;
  if (R < W) {  // carry: the significand became 2^128
    R = one << 127;
    exp++;
    up = true;
  } else {
    if (rc == 0 && rb == half) R &= ~(one << G);
    R &= ~mask;
    up = R != base;
  }
  v.c1 = rb != 0 && up;
  return F80{(u64)(R >> 64), (s << 15) | (u32)exp};
}

// x87 NaN propagation (SDM vol. 1 table 4-7): an SNaN is quietened (IE); a
// QNaN beats an SNaN; of two NaNs of the same kind the larger significand
// (then the smaller sign / exponent word) wins; the default NaN for invalid operations
__device__ __noinline__ F80 x_nan2(XEnv &v, F80 a, u32 ca, F80 b, u32 cb) {
  if (ca == XC_SNAN || cb == XC_SNAN) v.fl |= SW_IE;
  if (!x_nan(cb)) return x_quiet(a);
  if (!x_nan(ca)) return x_quiet(b);
  if (ca != cb) return x_quiet(ca == XC_QNAN ? a : b);
  const u64 ma = a.m & 0x3fffffffffffffffull, mb = b.m & 0x3fffffffffffffffull;
  if (ma != mb) return x_quiet(ma > mb ? a : b);
  return x_quiet(a.se <= b.se ? a : b);
}

enum : u32 { XO_ADD, XO_SUB, XO_MUL, XO_DIV };

// a op b on operands already checked for NaN / unsupported; prec 24 / 53 / 64
__device__ __noinline__ F80 x_arith(XEnv &v, u32 op, F80 a, F80 b, u32 prec) {
  const u32 ca = x_class(a), cb = x_class(b);
  u32 sa = x_sign(a), sb = x_sign(b);
  if (op == XO_SUB) sb ^= 1;
  if (op == XO_ADD || op == XO_SUB) {
    if ((ca == XC_DEN || cb == XC_DEN)) v.fl |= SW_DE;
    if (ca == XC_INF || cb == XC_INF) {
      if (ca == XC_INF && cb == XC_INF && sa != sb) {
        v.fl |= SW_IE;
        return x_indef();
      }
      return x_inf(ca == XC_INF ? sa : sb);
    }
    if (ca == XC_ZERO && cb == XC_ZERO) return x_zero(sa == sb ? sa : (v.rc == 1));
    i32 ea, eb;
    u64 ma, mb;
    if (ca == XC_ZERO) {
      x_unpack(b, eb, mb);
      return x_round(v, sb, eb, (u128)mb << 64, prec);
    }
    if (cb == XC_ZERO) {
      x_unpack(a, ea, ma);
      return x_round(v, sa, ea, (u128)ma << 64, prec);
    }
    x_unpack(a, ea, ma);
    x_unpack(b, eb, mb);
    if (eb > ea || (eb == ea && mb > ma)) {
      const u32 ts = sa;
      sa = sb, sb = ts;
      const i32 te = ea;
      ea = eb, eb = te;
      const u64 tm = ma;
      ma = mb, mb = tm;
    }
    // one guard bit above for the carry: W = m << 63
    const u128 A = (u128)ma << 63, B = jam128((u128)mb << 63, (u32)(ea - eb));
    if (sa == sb) {
      u128 S = A + B;
      i32 e = ea;
      if (S >> 127) e++;
      else S <<= 1;
      return x_round(v, sa, e, S, prec);
    }
    u128 D = A - B;
    if (D == 0) return x_zero(v.rc == 1);
    const u32 hi = (u64)(D >> 64) ? (u32)__builtin_clzll((u64)(D >> 64)) : 64 + (u32)__builtin_clzll((u64)D);
    D <<= hi;
    return x_round(v, sa, ea + 1 - (i32)hi, D, prec);
  }
  const u32 s = sa ^ sb;
  if (op == XO_MUL) {
    if (ca == XC_INF || cb == XC_INF) {
      if (ca == XC_ZERO || cb == XC_ZERO) {
        v.fl |= SW_IE;
        return x_indef();
      }
      if (ca == XC_DEN || cb == XC_DEN) v.fl |= SW_DE;
      return x_inf(s);
    }
    if (ca == XC_DEN || cb == XC_DEN) v.fl |= SW_DE;
    if (ca == XC_ZERO || cb == XC_ZERO) return x_zero(s);
    i32 ea, eb;
    u64 ma, mb;
    x_unpack(a, ea, ma);
    x_unpack(b, eb, mb);
    u128 P = (u128)ma * mb;
    i32 e = ea + eb - 16383 + 1;
    if (!(P >> 127)) {
      P <<= 1;
      e--;
    }
    return x_round(v, s, e, P, prec);
  }
  // XO_DIV
  if ((ca == XC_INF && cb == XC_INF) || (ca == XC_ZERO && cb == XC_ZERO)) {
    v.fl |= SW_IE;
    return x_indef();
  }
  if (ca == XC_INF) {
    if (cb == XC_DEN) v.fl |= SW_DE;
    return x_inf(s);
  }
  if (cb == XC_INF) {
    if (ca == XC_DEN) v.fl |= SW_DE;
    return x_zero(s);
  }
  if (cb == XC_ZERO) {  // a finite nonzero
    v.fl |= SW_ZE;
    return x_inf(s);
  }
  if (ca == XC_DEN || cb == XC_DEN) v.fl |= SW_DE;
  if (ca == XC_ZERO) return x_zero(s);
  i32 ea, eb;
  u64 ma, mb;
  x_unpack(a, ea, ma);
  x_unpack(b, eb, mb);
  // 128 quotient bits of ma / mb, the integer bit first
  u128 r = ma, q = 0;
  for (int i = 0; i < 128; i++) {
    q <<= 1;
    if (r >= mb) {
      r -= mb;
      q |= 1;
    }
    r <<= 1;
  }
  i32 e = ea - eb + 16383;
  if (!(q >> 127)) {
    q <<= 1;
    e--;
  }
  q |= (u128)(r != 0);
  return x_round(v, s, e, q, prec);
}

__device__ __noinline__ F80 x_sqrt(XEnv &v, F80 a, u32 prec) {
  const u32 c = x_class(a);
  if (c == XC_ZERO) return a;
  if (x_sign(a)) {
    v.fl |= SW_IE;
    return x_indef();
  }
  if (c == XC_INF) return a;
  if (c == XC_DEN) v.fl |= SW_DE;
  i32 e;
  u64 m;
  x_unpack(a, e, m);
  i32 E = e - 16383;
  u128 N = (u128)m << 63;
  if (E & 1) {
    N <<= 1;
    E -= 1;
  }
  u64 r = 0;
  for (int i = 63; i >= 0; i--) {
    const u64 t = r | (1ull << i);
    if ((u128)t * t <= N) r = t;
  }
  const u128 rem = N - (u128)r * r;
  const u64 ext = rem > r ? 0x8000000000000001ull : (rem ? 1 : 0);
  return x_round(v, 0, E / 2 + 16383, ((u128)r << 64) | ext, prec);
}

// 32 / 64-bit float -> extended: exact; a NaN keeps its quiet bit (the
// arithmetic or FLD decides IE), den = a denormal source (DE)
__device__ __noinline__ F80 x_from_f(u64 x, u32 w, bool &den) {
  const u32 s = f_sign(x, w);
  const i32 ex = f_exp(x, w);
  const u64 fr = f_frac(x, w);
  const u32 F = fF(w);
  den = ex == 0 && fr != 0;
  if (ex == fEmax(w)) return F80{(1ull << 63) | (fr << (63 - F)), (s << 15) | 0x7fff};
  if (ex == 0 && fr == 0) return x_zero(s);
  if (ex == 0) {
    const u32 sh = (u32)__builtin_clzll(fr);  // fr * 2^(1 - bias - F) = (fr << sh) / 2^63 * 2^(64 - sh - bias - F)
    return F80{fr << sh, (s << 15) | (u32)(64 - (i32)sh - fBias(w) - (i32)F + 16383)};
  }
  return F80{(1ull << 63) | (fr << (63 - F)), (s << 15) | (u32)(ex - fBias(w) + 16383)};
}

// extended -> 32 / 64-bit float, rounded per RC (FST / FSTP m32 / m64)
__device__ __noinline__ u64 x_to_f(XEnv &v, F80 a, u32 w) {
  const u32 c = x_class(a), s = x_sign(a);
  if (c == XC_UNSUP) {
    v.fl |= SW_IE;
    return f_indef(w);
  }
  if (x_nan(c)) {
    if (c == XC_SNAN) v.fl |= SW_IE;
    return f_infv(s, w) | (1ull << (fF(w) - 1)) | ((a.m << 2) >> (64 - (fF(w) - 1)));
  }
  if (c == XC_INF) return f_infv(s, w);
  if (c == XC_ZERO) return f_signed(s, w);
  i32 e;
  u64 m;
  x_unpack(a, e, m);
  // engine_fp.h's rounding: m / 2^62 * 2^(e' + 1 - bias), 62 - F guard bits + sticky
  FEnv f{v.rc, 0, 0, (v.masks & SW_UE ? FE_U : 0) | (v.masks & SW_OE ? FE_O : 0) | FE_I | FE_D | FE_Z | FE_P, 0};
  const u64 m62 = (m >> 1) | (m & 1);
  const u64 r = f_round(f, s, e - 16383 + fBias(w) - 1, m62, w);
  // an unmasked OE / UE stores nothing and raises no PE
  if ((f.fl & FE_O && !(v.masks & SW_OE)) || (f.fl & FE_U && !(v.masks & SW_UE))) f.fl &= ~FE_P;
  v.fl |= (f.fl & FE_O ? SW_OE : 0) | (f.fl & FE_U ? SW_UE : 0) | (f.fl & FE_P ? SW_PE : 0);
  // C1: rounded up in magnitude
  v.c1 = 0;
  if (f.fl & FE_P) {
    i32 er;
    u64 mr;
    const u64 mag = f_mag(r, w);
    if (f_inf(r, w)) v.c1 = 1;
    else if (mag) {
      f_unpack(r, w, er, mr);  // compare |r| with |a|
      const i32 ea = e - 16383, eb = er + 1 - fBias(w);
      const u64 ma = m >> 1, mb = mr;
      v.c1 = eb > ea || (eb == ea && mb > ma);
    }
  }
  return r;
}

// integer -> extended (exact)
__device__ __forceinline__ F80 x_from_int(i64 x) {
  if (!x) return x_zero(0);
  const u32 s = x < 0;
  const u64 mag = s ? (u64)0 - (u64)x : (u64)x;
  const u32 sh = (u32)__builtin_clzll(mag);
  return F80{mag << sh, (s << 15) | (u32)(16383 + 63 - (i32)sh)};
}

// |a| (finite nonzero, e / m unpacked) split at the binary point: the integer
// part q (E < 64) and where the fraction lies: 0 none, 1 below half, 2 half, 3 above
__device__ __forceinline__ u64 x_intpart(i32 e, u64 m, u32 &frac) {
  const i32 E = e - 16383;  // |a| = m / 2^63 * 2^E, E < 64
  if (E >= 63) {
    frac = 0;
    return m << (E - 63);
  }
  const u32 sh = (u32)(63 - E);
  if (sh > 64) {
    frac = 1;
    return 0;
  }
  if (sh == 64) {
    frac = m == (1ull << 63) ? 2 : 3;
    return 0;
  }
  const u64 rem = m & ((1ull << sh) - 1), half = 1ull << (sh - 1);
  frac = rem == 0 ? 0 : rem < half ? 1 : rem == half ? 2 : 3;
  return m >> sh;
}
__device__ __forceinline__ bool x_round_up(u32 rc, u32 s, u64 q, u32 frac) {
  if (!frac) return false;
  if (rc == 0) return frac == 3 || (frac == 2 && (q & 1));
  if (rc == 1) return s != 0;
  if (rc == 2) return s == 0;
  return false;
}

// extended -> signed integer of isz bytes, rounded by rc; false: invalid (IE)
__device__ __noinline__ bool x_to_int(XEnv &v, F80 a, u32 isz, u32 rc, u64 &out) {
  const u32 c = x_class(a), s = x_sign(a);
  v.c1 = 0;
  if (c == XC_UNSUP || x_nan(c) || c == XC_INF) {
    v.fl |= SW_IE;
    return false;
  }
  if (c == XC_ZERO) {
    out = 0;
    return true;
  }
  i32 e;
  u64 m;
  x_unpack(a, e, m);
  if (e - 16383 >= 64) {
    v.fl |= SW_IE;
    return false;
  }
  u32 frac;
  const u64 q = x_intpart(e, m, frac);
  const bool up = x_round_up(rc, s, q, frac);
  const u64 q2 = q + up;
  const u64 lim = (isz == 8 ? (1ull << 63) : isz == 4 ? (1ull << 31) : (1ull << 15)) - (s ? 0 : 1);
  if ((up && q2 == 0) || q2 > lim) {
    v.fl |= SW_IE;
    return false;
  }
  if (frac) {
    v.fl |= SW_PE;
    v.c1 = up;
  }
  out = (s ? (u64)0 - q2 : q2) & szmask(isz);
  return true;
}

// FRNDINT: to an integral value per RC (no PC)
__device__ __noinline__ F80 x_rndint(XEnv &v, F80 a) {
  const u32 c = x_class(a), s = x_sign(a);
  v.c1 = 0;
  if (c == XC_ZERO || c == XC_INF) return a;
  if (c == XC_DEN) v.fl |= SW_DE;
  i32 e;
  u64 m;
  x_unpack(a, e, m);
  if (e - 16383 >= 63) return F80{m, (s << 15) | (u32)e};
  u32 frac;
  const u64 q = x_intpart(e, m, frac);
  if (!frac) return F80{m, (s << 15) | (u32)e};
  const bool up = x_round_up(v.rc, s, q, frac);
  v.fl |= SW_PE;
  v.c1 = up;
  const u64 q2 = q + up;  // q < 2^63: no carry out
  if (!q2) return x_zero(s);
  const F80 r = x_from_int((i64)q2);
  return F80{r.m, (s << 15) | (r.se & 0x7fff)};
}

// FSCALE: a * 2^trunc(b) (b finite non-NaN; the specials are handled by the caller)
__device__ __noinline__ F80 x_scale(XEnv &v, F80 a, F80 b) {
  const u32 ca = x_class(a);
  if (ca == XC_DEN || x_class(b) == XC_DEN) v.fl |= SW_DE;
  if (ca == XC_ZERO || ca == XC_INF) return a;
  // trunc(b) as an integer, clamped (anything beyond +-2^16 over- / underflows anyway)
  i64 n = 0;
  const u32 cb = x_class(b);
  if (cb == XC_NORM) {
    i32 eb;
    u64 mb;
    x_unpack(b, eb, mb);
    const i32 E = eb - 16383;
    if (E >= 20) n = 1 << 20;
    else if (E >= 0) n = (i64)(mb >> (63 - E));
    if (x_sign(b)) n = -n;
  }
  i32 e;
  u64 m;
  x_unpack(a, e, m);
  return x_round(v, x_sign(a), e + (i32)n, (u128)m << 64, 64);
}


// ---------------------------------------------------------------- the register stack
// fpst / fpse hold ST order; the tag word is physical (R(p), p = TOP + i)
__device__ __forceinline__ u32 x_top(const wtfgpu_regs_t &F) { return (F.fpsw >> 11) & 7u; }
__device__ __forceinline__ bool st_empty(const wtfgpu_regs_t &F, u32 i) {
  return ((F.fptw >> (2 * ((x_top(F) + i) & 7))) & 3) == 3;
}
__device__ __forceinline__ F80 st_rd(const wtfgpu_regs_t &F, u32 i) { return F80{F.fpst[i & 7], F.fpse[i & 7]}; }
__device__ __forceinline__ void st_settag(wtfgpu_regs_t &F, u32 i, u32 t) {
  const u32 p = 2 * ((x_top(F) + i) & 7);
  F.fptw = (u16)((F.fptw & ~(3u << p)) | (t << p));
}
__device__ __forceinline__ void st_wr(wtfgpu_regs_t &F, u32 i, F80 v) {
  F.fpst[i & 7] = v.m;
  F.fpse[i & 7] = (u16)v.se;
  st_settag(F, i, 0);  // non-empty; x87_retag computes the class
}
__device__ __forceinline__ void st_settop(wtfgpu_regs_t &F, u32 top) { F.fpsw = (u16)((F.fpsw & ~0x3800u) | ((top & 7) << 11)); }
// push: TOP - 1, ST(i) <- ST(i - 1), the new ST(0) is the old ST(7)'s register
__device__ __noinline__ void st_push(wtfgpu_regs_t &F) {
  const u64 m7 = F.fpst[7];
  const u16 e7 = F.fpse[7];
  for (int j = 7; j > 0; j--) F.fpst[j] = F.fpst[j - 1], F.fpse[j] = F.fpse[j - 1];
  F.fpst[0] = m7;
  F.fpse[0] = e7;
  st_settop(F, x_top(F) - 1);
}
// pop: ST(0)'s register empty, TOP + 1, ST(i) <- ST(i + 1)
__device__ __noinline__ void st_pop(wtfgpu_regs_t &F) {
  st_settag(F, 0, 3);
  const u64 m0 = F.fpst[0];
  const u16 e0 = F.fpse[0];
  for (int j = 0; j < 7; j++) F.fpst[j] = F.fpst[j + 1], F.fpse[j] = F.fpse[j + 1];
  F.fpst[7] = m0;
  F.fpse[7] = e0;
  st_settop(F, x_top(F) + 1);
}
// every non-empty register's tag from its contents (what FSTENV reports)
__device__ __noinline__ void x87_retag(wtfgpu_regs_t &F) {
  const u32 top = x_top(F);
  u32 w = F.fptw;
  for (u32 p = 0; p < 8; p++)
    if (((w >> (2 * p)) & 3) != 3) {
      const u32 i = (p - top) & 7;
      w = (w & ~(3u << (2 * p))) | (tag_of(F.fpst[i], F.fpse[i]) << (2 * p));
    }
  F.fptw = (u16)w;
}

// ---------------------------------------------------------------- comparisons
// 0 greater, 1 less, 2 equal, 3 unordered; quiet: only SNaN / unsupported raise IE
__device__ __noinline__ u32 x_compare(XEnv &v, F80 a, F80 b, bool quiet) {
  const u32 ca = x_class(a), cb = x_class(b);
  if (ca == XC_UNSUP || cb == XC_UNSUP || ca == XC_SNAN || cb == XC_SNAN || (!quiet && (x_nan(ca) || x_nan(cb)))) {
    v.fl |= SW_IE;
    return 3;
  }
  if (x_nan(ca) || x_nan(cb)) return 3;
  if (ca == XC_DEN || cb == XC_DEN) v.fl |= SW_DE;
  const u32 sa = x_sign(a), sb = x_sign(b);
  if (ca == XC_ZERO && cb == XC_ZERO) return 2;
  // total order on (sign, magnitude)
  int mag;  // |a| vs |b|
  if (ca == XC_ZERO) mag = -1;
  else if (cb == XC_ZERO) mag = 1;
  else if (ca == XC_INF || cb == XC_INF) mag = (ca == XC_INF) - (cb == XC_INF);
  else {
    i32 ea, eb;
    u64 ma, mb;
    x_unpack(a, ea, ma);
    x_unpack(b, eb, mb);
    mag = ea != eb ? (ea > eb ? 1 : -1) : ma != mb ? (ma > mb ? 1 : -1) : 0;
  }
  if (ca == XC_ZERO) return sb ? 0 : 1;  // 0 vs nonzero b
  if (cb == XC_ZERO) return sa ? 1 : 0;
  if (sa != sb) return sa ? 1 : 0;
  if (mag == 0) return 2;
  return ((mag > 0) != (sa != 0)) ? 0 : 1;
}

// a op b with the x87 operand rules: unsupported formats and SNaNs (IE), NaN
// propagation, then x_arith; bden: an operand came from a denormal m32 / m64 (DE)
__device__ __noinline__ F80 x_binop(XEnv &v, u32 op, F80 a, F80 b, u32 prec, bool bden) {
  const u32 ca = x_class(a), cb = x_class(b);
  if (ca == XC_UNSUP || cb == XC_UNSUP) {
    v.fl |= SW_IE;
    return x_indef();
  }
  if (x_nan(ca) || x_nan(cb)) return x_nan2(v, a, ca, b, cb);
  if (bden && !(op == XO_DIV && cb == XC_ZERO)) v.fl |= SW_DE;  // x / 0 reports ZE alone
  return x_arith(v, op, a, b, prec);
}

// ---------------------------------------------------------------- constants
// FLD1 ... FLDZ (d9 e8-ee): the 64-bit value rounded toward zero, + 1 ulp when
// the mode rounds it up (read from the host for the four RC values)
__device__ __forceinline__ F80 x_const(u32 k, u32 rc) {
  u64 m = 0;
  u32 se = 0, near_up = 0;
  switch (k) {
    case 0: m = 0x8000000000000000ull, se = 0x3fff; break;                 // 1
    case 1: m = 0xd49a784bcd1b8afeull, se = 0x4000; break;                 // log2(10)
    case 2: m = 0xb8aa3b295c17f0bbull, se = 0x3fff, near_up = 1; break;    // log2(e)
    case 3: m = 0xc90fdaa22168c234ull, se = 0x4000, near_up = 1; break;    // pi
    case 4: m = 0x9a209a84fbcff798ull, se = 0x3ffd, near_up = 1; break;    // log10(2)
    case 5: m = 0xb17217f7d1cf79abull, se = 0x3ffe, near_up = 1; break;    // ln(2)
    default: return x_zero(0);
  }
  if (k != 0 && (rc == 2 || (rc == 0 && near_up))) m++;
  return F80{m, se};
}

// ---------------------------------------------------------------- FSCALE / FXTRACT
__device__ __noinline__ F80 x_fscale(XEnv &v, F80 a, F80 b) {
  const u32 ca = x_class(a), cb = x_class(b);
  if (ca == XC_UNSUP || cb == XC_UNSUP) {
    v.fl |= SW_IE;
    return x_indef();
  }
  if (x_nan(ca) || x_nan(cb)) return x_nan2(v, a, ca, b, cb);
  if (cb == XC_INF) {
    if (ca == XC_DEN) v.fl |= SW_DE;
    if (x_sign(b)) {  // * 2^-inf
      if (ca == XC_INF) {
        v.fl |= SW_IE;
        return x_indef();
      }
      return x_zero(x_sign(a));
    }
    if (ca == XC_ZERO) {
      v.fl |= SW_IE;
      return x_indef();
    }
    return x_inf(x_sign(a));
  }
  return x_scale(v, a, b);
}

// ---------------------------------------------------------------- FPREM / FPREM1
// ST0 - q * ST1, exact; q truncated (fprem) or to nearest even (fprem1). With
// an exponent difference D >= 64 the reduction is partial: q's top N bits,
// q * 2^(D - N) with N = 32 + D mod 32 (the host's choice; C2 = 1). cc: raw
// C3 (2) C2 (4) C0 (1) with C0 = q bit 2, C3 = q bit 1, C1 = q bit 0;
// kPremC2Only: C2 = 0, C0 / C3 kept.
constexpr u32 kPremC2Only = 0x100;
__device__ __noinline__ F80 x_fprem(XEnv &v, F80 a, F80 b, bool near, u32 &cc) {
  const u32 ca = x_class(a), cb = x_class(b);
  cc = kPremC2Only;
  v.c1 = 0;
  if (ca == XC_UNSUP || cb == XC_UNSUP) {
    v.fl |= SW_IE;
    return x_indef();
  }
  if (x_nan(ca) || x_nan(cb)) return x_nan2(v, a, ca, b, cb);
  if (ca == XC_INF || cb == XC_ZERO) {  // IE alone, beside a denormal too
    v.fl |= SW_IE;
    return x_indef();
  }
  if (ca == XC_DEN || cb == XC_DEN) v.fl |= SW_DE;
  cc = 0;
  if (ca == XC_ZERO) return a;
  i32 ea, eb;
  u64 ma, mb;
  x_unpack(a, ea, ma);
  u32 s = x_sign(a);
  // q = 0: a itself (a pseudo-denormal comes back with exponent 1)
  const F80 a1 = (x_exp(a) == 0 && (a.m >> 63)) ? F80{a.m, a.se | 1} : a;
  if (cb == XC_INF) return a1;
  x_unpack(b, eb, mb);
  const i32 D = ea - eb;
  if (D < -1 || (D == -1 && !near)) return x_round(v, s, ea, (u128)ma << 64, 64);  // tiny: UE rules
  const bool partial = D >= 64;
  const i32 steps = partial ? 32 + (D & 31) : D;  // quotient bits below the top one
  // long division of ma by mb at the scale of mb * 2^(D - steps)
  u128 r = ma;
  u64 q = 0;
  if (D >= 0) {
    for (i32 i = steps; i >= 0; i--) {
      q <<= 1;
      if (r >= mb) {
        r -= mb;
        q |= 1;
      }
      if (i) r <<= 1;
    }
  }
  // r < mb: the remainder is r * 2^(eb + D - steps - 63) (D >= 0), or a itself (D = -1)
  i32 re = D >= 0 ? eb + D - steps : ea;
  if (near && !partial) {
    // compare 2r with mb at the same scale (D = -1: r = ma at 2^(ea), mb at 2^(ea + 1))
    const u128 twice = D >= 0 ? r << 1 : r;
    if (twice > mb || (twice == mb && (q & 1))) {
      q++;
      r = (D >= 0 ? (u128)mb : (u128)mb << 1) - (D >= 0 ? r : r);
      if (D < 0) re = ea;  // |b| - |a| at a's scale: (2 mb - ma) * 2^(ea - 63)
      s ^= 1;
    }
  }
  if (partial) cc = 4;
  else {
    cc = ((q >> 2) & 1) | (((q >> 1) & 1) << 1);
    v.c1 = q & 1;
  }
  if (r == 0) return x_zero(x_sign(a) ^ 0);
  // normalise r (< 2^65) to bit 127 and round (exact; only a tiny result can raise UE)
  const u32 lz = (u64)(r >> 64) ? (u32)__builtin_clzll((u64)(r >> 64)) : 64 + (u32)__builtin_clzll((u64)r);
  const u128 W = r << lz;
  XEnv w = v;
  const F80 res = x_round(w, s, re + 127 - (i32)lz - 63 + 0, W, 64);
  v.fl = w.fl;
  return res;
}

// ---------------------------------------------------------------- memory operands
enum : u32 { XM_NONE, XM_F32, XM_F64, XM_F80, XM_I16, XM_I32, XM_I64, XM_BCD };
__device__ __forceinline__ u32 xm_bytes(u32 k) {
  return k == XM_F32 || k == XM_I32 ? 4 : k == XM_F64 || k == XM_I64 ? 8 : (k == XM_F80 || k == XM_BCD) ? 10
         : k == XM_I16 ? 2 : 0;
}
// packed BCD (fbld): digit i in nibble i of bytes 0-8, the sign in byte 9's bit
// 7; a nibble above 9 counts with its binary value, as the hardware reads it
__device__ __forceinline__ F80 x_from_bcd(u64 lo, u64 hi) {
  u64 v = 0, p = 1;
  for (u32 i = 0; i < 18; i++, p *= 10) v += (i < 16 ? (lo >> (4 * i)) & 15 : (hi >> (4 * (i - 16))) & 15) * p;
  const u32 s = (u32)(hi >> 15) & 1;
  if (!v) return F80{0, s << 15};
  const F80 r = x_from_int((i64)v);
  return F80{r.m, r.se | (s << 15)};
}
// fbstp: |q| <= 10^18 - 1 as 18 digits, sign s; the BCD indefinite otherwise
__device__ __forceinline__ void x_to_bcd(u64 q, u32 s, u64 &lo, u64 &hi) {
  lo = 0;
  hi = (u64)s << 15;
  for (u32 i = 0; i < 18; i++, q /= 10) {
    const u64 d = q % 10;
    if (i < 16) lo |= d << (4 * i);
    else hi |= d << (4 * (i - 16));
  }
}
// a memory source as an extended value (den: denormal m32 / m64)
__device__ __forceinline__ F80 xm_value(u32 k, u64 lo, u64 hi, bool &den) {
  den = false;
  switch (k) {
    case XM_F32: return x_from_f(lo & 0xffffffffull, 0, den);
    case XM_F64: return x_from_f(lo, 1, den);
    case XM_F80: return F80{lo, (u32)hi & 0xffff};
    case XM_I16: return x_from_int((i64)(int16_t)lo);
    case XM_I32: return x_from_int((i64)(int32_t)lo);
    case XM_BCD: return x_from_bcd(lo, hi);
    default: return x_from_int((i64)lo);
  }
}
__device__ __forceinline__ bool xm_read(Lane &L, u64 va, u32 k, u64 &lo, u64 &hi) {
  hi = 0;
  if (k == XM_F80 || k == XM_BCD) return vread(L, va, 8, lo) && vread(L, va + 8, 2, hi);
  return vread(L, va, xm_bytes(k), lo);
}
__device__ __forceinline__ bool xm_write(Lane &L, u64 va, u32 k, u64 lo, u64 hi) {
  if (k == XM_F80 || k == XM_BCD) return span_w(L, va, 10) && vwrite(L, va, 8, lo) && vwrite(L, va + 8, 2, hi);
  return vwrite(L, va, xm_bytes(k), lo);
}

// ---------------------------------------------------------------- one instruction
// x87_arith (exec protocol: X_FAULT with L.miss set asks for a translation and
// a rerun, so nothing is committed before the memory access succeeded)
enum : u32 { XA_ADD, XA_MUL, XA_COM, XA_COMP, XA_SUB, XA_SUBR, XA_DIV, XA_DIVR };

__device__ __noinline__ int x87_arith(const Dev &P, Lane &L, const UOp &u, u64 va) {
  wtfgpu_regs_t &F = P.full[L.lane];
  const u32 op = u.sub & 0xff, r3 = u.reg & 7, mem = u.is_mem, ri = u.rm & 7;
  const u32 modrm = 0xc0 | (r3 << 3) | ri;
  u32 mk = XM_NONE;
  bool store = false;
  if (mem) {
    switch (op) {
      case 0xd8: mk = XM_F32; break;
      case 0xdc: mk = XM_F64; break;
      case 0xda: mk = XM_I32; break;
      case 0xde: mk = XM_I16; break;
      case 0xd9:
        if (r3 == 1) return fault_x(L, WTFGPU_VEC_UD, 0);
        mk = XM_F32;
        store = r3 != 0;
        break;
      case 0xdb:
        if (r3 == 4 || r3 == 6) return fault_x(L, WTFGPU_VEC_UD, 0);
        mk = r3 >= 5 ? XM_F80 : XM_I32;
        store = r3 != 0 && r3 != 5;
        break;
      case 0xdd:
        if (r3 == 5) return fault_x(L, WTFGPU_VEC_UD, 0);
        mk = r3 == 1 ? XM_I64 : XM_F64;
        store = r3 != 0;
        break;
      default:  // df
        mk = r3 == 4 || r3 == 6 ? XM_BCD : r3 == 5 || r3 == 7 ? XM_I64 : XM_I16;
        store = r3 != 0 && r3 != 4 && r3 != 5;
        break;
    }
  } else {
    bool ud = false;
    switch (op) {
      case 0xd9:
        if (modrm >= 0xf0 && !(modrm == 0xf4 || modrm == 0xf5 || modrm == 0xf6 || modrm == 0xf7 || modrm == 0xf8 ||
                               modrm == 0xfa || modrm == 0xfc || modrm == 0xfd))
          return X_UNIMPL;  // transcendental
        ud = (modrm >= 0xd1 && modrm <= 0xd7) || modrm == 0xe2 || modrm == 0xe3 || modrm == 0xe6 || modrm == 0xe7 ||
             modrm == 0xef;
        break;
      case 0xda: ud = modrm >= 0xe0 && modrm != 0xe9; break;
      case 0xdb: ud = (modrm >= 0xe5 && modrm <= 0xe7) || modrm >= 0xf8; break;
      case 0xdd: ud = modrm >= 0xf0; break;
      case 0xde: ud = modrm >= 0xd8 && modrm <= 0xdf && modrm != 0xd9; break;
      case 0xdf: ud = (modrm >= 0xe1 && modrm <= 0xe7) || modrm >= 0xf8; break;
      default: break;
    }
    if (ud) return fault_x(L, WTFGPU_VEC_UD, 0);
  }
  if (L.cr0 & 0xc) return fault_x(L, VEC_NM, 0);
  if (op == 0xdb && !mem && (modrm == 0xe0 || modrm == 0xe1 || modrm == 0xe4)) return X_OK;  // fneni fndisi fnsetpm
  if (x87_pending(F)) return fault_x(L, VEC_MF, 0);

  XEnv v{(F.fpcw >> 10) & 3u, F.fpcw & 0x3fu, 0, 0};
  const u32 pcf = (F.fpcw >> 8) & 3, prec = pcf == 0 ? 24 : pcf == 2 ? 53 : 64;
  u64 mlo = 0, mhi = 0;
  if (mem && !store && !xm_read(L, va, mk, mlo, mhi)) return X_FAULT;
  u32 c1mode = 0;  // 0: C1 := v.c1; 1: C1 unchanged
  u32 cc = 0xffffffffu;  // C3 C2 C0 when set (compare forms)
  const u32 masks = v.masks;
  // stack underflow / overflow raise IE + SF; C1 = 1 on overflow
  bool suppress = false;  // an unmasked pre-computation exception: no result, no pop
  auto underflow = [&]() {
    v.fl |= SW_IE | SW_SF;
    v.c1 = 0;
    if (!(masks & SW_IE)) suppress = true;
  };
  auto overflow = [&]() {
    v.fl |= SW_IE | SW_SF;
    v.c1 = 1;
    if (!(masks & SW_IE)) suppress = true;
  };
  // an unmasked pre-computation exception: the result's own flags are not raised
  auto pre_unmasked = [&]() {
    if (!(v.fl & ~masks & (SW_IE | SW_DE | SW_ZE))) return false;
    v.fl &= SW_IE | SW_DE | SW_ZE | SW_SF;
    if (!(v.fl & SW_SF)) v.c1 = 0;
    return true;
  };

  if (store) {
    // fst / fstp / fist / fistp / fisttp / fstp m80 (d9 /2 /3, db /1 /2 /3 /7, dd /1 /2 /3, df /1 /2 /3 /7)
    const bool pop = r3 != 2;
    u64 lo = 0, hi = 0;
    bool write = true;
    if (st_empty(F, 0)) {
      underflow();
      write = !suppress;
      switch (mk) {
        case XM_F32: lo = f_indef(0); break;
        case XM_F64: lo = f_indef(1); break;
        case XM_F80: case XM_BCD: lo = 0xc000000000000000ull, hi = 0xffff; break;
        case XM_I16: lo = 0x8000; break;
        case XM_I32: lo = 0x80000000ull; break;
        default: lo = 0x8000000000000000ull; break;
      }
    } else {
      const F80 a = st_rd(F, 0);
      if (mk == XM_F80) {
        lo = a.m, hi = a.se;
      } else if (mk == XM_F32 || mk == XM_F64) {
        lo = x_to_f(v, a, mk == XM_F64);
        write = !(v.fl & ~masks & (SW_IE | SW_OE | SW_UE));
      } else if (mk == XM_BCD) {  // fbstp: rounded by RC, at most 18 digits
        u64 q = 0;
        bool ok = x_to_int(v, a, 8, v.rc, q);
        const u32 sgn = x_sign(a);
        if (ok) {
          const u64 mag = sgn ? (u64)0 - q : q;
          if (mag > 999999999999999999ull) {
            v.fl = (v.fl & ~(SW_PE)) | SW_IE;
            v.c1 = 0;
            ok = false;
          } else {
            x_to_bcd(mag, sgn, lo, hi);
          }
        }
        if (!ok) {
          lo = 0xc000000000000000ull, hi = 0xffff;
          write = (masks & SW_IE) != 0;
        }
      } else {
        const u32 isz = mk == XM_I16 ? 2 : mk == XM_I32 ? 4 : 8;
        const u32 rc = r3 == 1 ? 3u : v.rc;  // fisttp truncates
        if (!x_to_int(v, a, isz, rc, lo)) {
          lo = isz == 2 ? 0x8000 : isz == 4 ? 0x80000000ull : 0x8000000000000000ull;
          write = (masks & SW_IE) != 0;
        }
      }
    }
    if (write && !xm_write(L, va, mk, lo, hi)) return X_FAULT;
    if (write && pop) st_pop(F);
    suppress = !write;
  } else if (mem && (op == 0xd9 || op == 0xdd || op == 0xdb || op == 0xdf)) {
    // fld m32 / m64 / m80, fild m16 / m32 / m64
    bool den;
    F80 x = xm_value(mk, mlo, mhi, den);
    if (!st_empty(F, 7)) {  // a stack overflow hides the source's own exceptions
      overflow();
      x = x_indef();
    } else {
      if (mk == XM_F32 || mk == XM_F64) {
        if (x_class(x) == XC_SNAN) {
          v.fl |= SW_IE;
          x = x_quiet(x);
        }
        if (den) v.fl |= SW_DE;  // loads anyway
      }
      if (v.fl & ~masks & SW_IE) suppress = true;
    }
    if (!suppress) {
      st_push(F);
      st_wr(F, 0, x);
    }
  } else if (op == 0xd8 || op == 0xdc || op == 0xde || (op == 0xda && mem)) {
    // arithmetic and compares: mem (ST0 op m), d8 reg (ST0 op ST(i)), dc / de reg (ST(i) op ST0)
    const bool rev_dst = !mem && (op == 0xdc || op == 0xde);
    const u32 k = (op == 0xde && !mem && modrm == 0xd9) ? XA_COMP : r3;
    const bool cmp = k == XA_COM || k == XA_COMP;
    const u32 di = (rev_dst && !cmp) ? ri : 0;  // destination
    const u32 si = mem ? 8 : (rev_dst && !cmp) ? 0 : ri;  // the other operand (8: memory)
    bool bden = false;
    const bool empty = st_empty(F, di) || (si < 8 && st_empty(F, si));
    F80 d = st_rd(F, di), sv = si < 8 ? st_rd(F, si) : xm_value(mk, mlo, mhi, bden);
    u32 npop = (op == 0xde && !mem) ? 1 : 0;
    if (k == XA_COMP) npop = (op == 0xde && !mem && modrm == 0xd9) ? 2 : 1;
    if (cmp) {
      if (empty) {
        underflow();
        cc = 3;
      } else {
        cc = x_compare(v, d, sv, false);
        if (bden && !(v.fl & SW_IE)) v.fl |= SW_DE;
        if (pre_unmasked()) suppress = true;
      }
      v.c1 = 0;
      if (!suppress)
        for (u32 i = 0; i < npop; i++) st_pop(F);
    } else {
      F80 r;
      if (empty) {
        underflow();
        r = x_indef();
      } else {
        // rev_dst swaps the sense: dc / de e0 = fsubr ST(i), ST0 (ST0 - ST(i)) ...
        const bool swap = ((k == XA_SUBR || k == XA_DIVR) != rev_dst);
        const u32 aop = k == XA_ADD ? XO_ADD : k == XA_MUL ? XO_MUL : (k == XA_SUB || k == XA_SUBR) ? XO_SUB : XO_DIV;
        r = swap ? x_binop(v, aop, sv, d, prec, bden) : x_binop(v, aop, d, sv, prec, bden);
        if (pre_unmasked()) suppress = true;
      }
      if (!suppress) {
        st_wr(F, di, r);
        if (npop) st_pop(F);
      }
    }
  } else {
    // the register forms of d9 db dd df (and da's fcmov / fucompp)
    const u32 g = modrm & 0xf8;
    if (op == 0xd9 && g == 0xc0) {  // fld ST(i)
      F80 x = st_rd(F, ri);
      if (st_empty(F, ri)) {
        underflow();
        x = x_indef();
      } else if (!st_empty(F, 7)) {
        overflow();
        x = x_indef();
      }
      if (!suppress) {
        st_push(F);
        st_wr(F, 0, x);
      }
    } else if ((op == 0xd9 && g == 0xc8) || (op == 0xdd && g == 0xc8) || (op == 0xdf && g == 0xc8)) {  // fxch
      F80 a = st_rd(F, 0), b = st_rd(F, ri);
      const bool ea = st_empty(F, 0), eb = st_empty(F, ri);
      if (ea || eb) {
        underflow();
        if (ea) a = x_indef();
        if (eb) b = x_indef();
      }
      v.c1 = 0;
      if (!suppress) {
        st_wr(F, 0, b);
        st_wr(F, ri, a);
      }
    } else if ((op == 0xdd && (g == 0xd0 || g == 0xd8)) || (op == 0xd9 && g == 0xd8) || (op == 0xdf && (g == 0xd0 || g == 0xd8))) {
      // fst / fstp ST(i) (and the d9 d8 / df d0 / df d8 aliases of fstp)
      F80 x = st_rd(F, 0);
      if (st_empty(F, 0) && op == 0xd9) {  // FSTP1: no underflow, nothing stored
        v.c1 = 0;
        st_pop(F);
      } else {
        if (st_empty(F, 0)) {
          underflow();
          x = x_indef();
        }
        if (!suppress) {
          st_wr(F, ri, x);
          if (!(op == 0xdd && g == 0xd0)) st_pop(F);
        }
      }
    } else if ((op == 0xdd && (g == 0xe0 || g == 0xe8)) || (op == 0xda && modrm == 0xe9)) {  // fucom / fucomp / fucompp
      const u32 i = op == 0xda ? 1 : ri;
      if (st_empty(F, 0) || st_empty(F, i)) {
        underflow();
        cc = 3;
      } else {
        cc = x_compare(v, st_rd(F, 0), st_rd(F, i), true);
        if (pre_unmasked()) suppress = true;
      }
      v.c1 = 0;
      if (!suppress) {
        if (op == 0xda || g == 0xe8) st_pop(F);
        if (op == 0xda) st_pop(F);
      }
    } else if ((op == 0xdb || op == 0xdf) && (g == 0xe8 || g == 0xf0)) {  // fucomi / fcomi (p)
      u32 r = 3;
      if (st_empty(F, 0) || st_empty(F, ri)) underflow();
      else {
        r = x_compare(v, st_rd(F, 0), st_rd(F, ri), g == 0xe8);
        if (pre_unmasked()) suppress = true;
      }
      c1mode = (v.fl & SW_SF) ? 0 : 1;
      const u64 zpc = r == 3 ? 0x45ull : r == 2 ? 0x40ull : r == 1 ? 0x01ull : 0;
      L.rflags = (L.rflags & ~F_STATUS) | zpc;  // written even when an unmasked exception holds the pop
      if (!suppress && op == 0xdf) st_pop(F);
    } else if (op == 0xda || (op == 0xdb && g <= 0xd8)) {  // fcmovcc
      const u64 fl = L.rflags;
      const u32 cf = fl & 1, zf = (fl >> 6) & 1, pf = (fl >> 2) & 1;
      const u32 t = (modrm >> 3) & 3;
      bool c = t == 0 ? cf : t == 1 ? zf : t == 2 ? (cf | zf) : pf;
      if (op == 0xdb) c = !c;
      if (st_empty(F, 0) || st_empty(F, ri)) {
        underflow();
        if (!suppress) st_wr(F, 0, x_indef());
      } else if (c) {
        st_wr(F, 0, st_rd(F, ri));
      }
      c1mode = (v.fl & SW_SF) ? 0 : 1;
    } else if (op == 0xdd && g == 0xc0) {  // ffree
      st_settag(F, ri, 3);
    } else if (op == 0xdf && g == 0xc0) {  // ffreep
      st_settag(F, ri, 3);
      st_pop(F);
    } else if (op == 0xd9 && modrm == 0xd0) {  // fnop
      c1mode = 1;
    } else if (op == 0xd9 && modrm == 0xf6) {  // fdecstp
      st_settop(F, x_top(F) - 1);
      u64 m7 = F.fpst[7];
      u16 e7 = F.fpse[7];
      for (int j = 7; j > 0; j--) F.fpst[j] = F.fpst[j - 1], F.fpse[j] = F.fpse[j - 1];
      F.fpst[0] = m7, F.fpse[0] = e7;
    } else if (op == 0xd9 && modrm == 0xf7) {  // fincstp
      st_settop(F, x_top(F) + 1);
      const u64 m0 = F.fpst[0];
      const u16 e0 = F.fpse[0];
      for (int j = 0; j < 7; j++) F.fpst[j] = F.fpst[j + 1], F.fpse[j] = F.fpse[j + 1];
      F.fpst[7] = m0, F.fpse[7] = e0;
    } else if (op == 0xd9 && modrm >= 0xe8 && modrm <= 0xee) {  // fld1 ... fldz
      F80 x = x_const(modrm - 0xe8, v.rc);
      if (!st_empty(F, 7)) {
        overflow();
        x = x_indef();
      }
      if (!suppress) {
        st_push(F);
        st_wr(F, 0, x);
      }
    } else if (op == 0xd9 && modrm == 0xe5) {  // fxam
      const F80 a = st_rd(F, 0);
      const u32 c = x_class(a);
      u32 k;
      if (st_empty(F, 0)) k = 5;
      else if (c == XC_UNSUP) k = 0;
      else if (x_nan(c)) k = 1;
      else if (c == XC_NORM) k = 2;
      else if (c == XC_INF) k = 3;
      else if (c == XC_ZERO) k = 4;
      else k = 6;  // denormal
      // k = C3 C2 C0
      cc = 0x80000000u | ((k & 4) ? 2 : 0) | ((k & 2) ? 4 : 0) | (k & 1);  // raw C3 (2) C2 (4) C0 (1)
      v.c1 = x_sign(a);
    } else {
      // the one-operand ST0 forms: fchs fabs ftst fxtract fsqrt frndint fscale
      if (st_empty(F, 0) || ((modrm == 0xfd || modrm == 0xf5 || modrm == 0xf8) && st_empty(F, 1))) {
        underflow();
        if (modrm == 0xf5 || modrm == 0xf8) cc = 0x40000000u;  // fprem: C2 = 0
        if (modrm == 0xe4) cc = 3;
        else if (!suppress) {
          st_wr(F, 0, x_indef());
          if (modrm == 0xf4) {  // fxtract: the underflow hides an overflow
            st_push(F);
            st_wr(F, 0, x_indef());
          }
        }
        if (modrm == 0xe4) v.c1 = 0;
      } else {
        const F80 a = st_rd(F, 0);
        switch (modrm) {
          case 0xe0: st_wr(F, 0, F80{a.m, a.se ^ 0x8000}); break;  // fchs
          case 0xe1: st_wr(F, 0, F80{a.m, a.se & 0x7fff}); break;  // fabs
          case 0xe4:                                                 // ftst
            cc = x_compare(v, a, x_zero(0), false);
            pre_unmasked();
            v.c1 = 0;
            break;
          case 0xfa: {  // fsqrt
            const u32 c = x_class(a);
            F80 r;
            if (c == XC_UNSUP) {
              v.fl |= SW_IE;
              r = x_indef();
            } else if (x_nan(c)) {
              r = x_nan2(v, a, c, a, c);
            } else {
              r = x_sqrt(v, a, prec);
            }
            if (!pre_unmasked()) st_wr(F, 0, r);
            break;
          }
          case 0xfc: {  // frndint
            const u32 c = x_class(a);
            F80 r;
            if (c == XC_UNSUP) {
              v.fl |= SW_IE;
              r = x_indef();
            } else if (x_nan(c)) {
              r = x_nan2(v, a, c, a, c);
            } else {
              r = x_rndint(v, a);
            }
            if (!pre_unmasked()) st_wr(F, 0, r);
            break;
          }
          case 0xfd: {  // fscale
            const F80 r = x_fscale(v, a, st_rd(F, 1));
            if (!pre_unmasked()) st_wr(F, 0, r);
            break;
          }
          case 0xf5: case 0xf8: {  // fprem1, fprem
            u32 qb;
            const F80 r = x_fprem(v, a, st_rd(F, 1), modrm == 0xf5, qb);
            cc = (qb & kPremC2Only) ? 0x40000000u : 0x80000000u | qb;
            if (!pre_unmasked()) st_wr(F, 0, r);
            else cc = 0x40000000u;  // no result: C2 = 0, C0 / C3 kept
            break;
          }
          default: {  // fxtract (f4)
            const u32 c = x_class(a);
            F80 sig, ex;
            if (!st_empty(F, 7)) {  // a stack overflow hides the operand's exceptions
              overflow();
              sig = ex = x_indef();
            } else if (c == XC_UNSUP) {
              v.fl |= SW_IE;
              sig = ex = x_indef();
            } else if (x_nan(c)) {
              sig = ex = x_nan2(v, a, c, a, c);
            } else if (c == XC_ZERO) {
              v.fl |= SW_ZE;
              sig = a;
              ex = x_inf(1);
            } else if (c == XC_INF) {
              sig = a;
              ex = x_inf(0);
            } else {
              if (c == XC_DEN) v.fl |= SW_DE;
              i32 e;
              u64 m;
              x_unpack(a, e, m);
              sig = F80{m, (x_sign(a) << 15) | 0x3fff};
              ex = x_from_int((i64)(e - 16383));
            }
            if (!suppress && !pre_unmasked()) {
              st_wr(F, 0, ex);
              st_push(F);
              st_wr(F, 0, sig);
            }
            break;
          }
        }
      }
    }
  }
  // status word: sticky flags, C1, condition codes, ES / B
  u32 sw = F.fpsw | (v.fl & 0x7fu);
  if (c1mode == 0) sw = (sw & ~SW_C1) | (v.c1 ? SW_C1 : 0);
  if (cc == 0x40000000u) {
    sw &= ~SW_C2;
  } else if (cc != 0xffffffffu) {
    if (cc & 0x80000000u) {
      sw = (sw & ~(SW_C0 | SW_C2 | SW_C3)) | ((cc & 1) ? SW_C0 : 0) | ((cc & 4) ? SW_C2 : 0) | ((cc & 2) ? SW_C3 : 0);
    } else {
      const u32 bits = cc == 3 ? (SW_C0 | SW_C2 | SW_C3) : cc == 2 ? SW_C3 : cc == 1 ? SW_C0 : 0;
      sw = (sw & ~(SW_C0 | SW_C2 | SW_C3)) | bits;
    }
  }
  F.fpsw = (u16)fsw_norm(sw, F.fpcw);
  x87_retag(F);
  return X_OK;
}

}  // namespace wtfgpu_dev
