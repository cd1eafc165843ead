// engine_fp.h — IEEE-754 binary32 / binary64 arithmetic under the x86 SSE
// rules, in integer arithmetic (conventions U39 / U40): MXCSR
// rounding control, DAZ and FTZ, the six exception flags (IE DE ZE OE UE PE in
// MXCSR bit order), x86 NaN propagation (the first source's NaN, quietened,
// else the second's; the default NaN is the negative "real indefinite") and
// the integer indefinite of out-of-range conversions. The GPU's own floating
// point has no per-lane rounding mode or flags, so none of it is used here.
//
// Numbers are unpacked to a sign, an exponent e and a 63-bit significand m
// with its leading one at bit 62: x = m / 2^62 * 2^(e + 1 - bias), i.e. e is
// the biased exponent minus one (the packing adds m's leading one into the
// exponent field). Rounding keeps 62 - F guard bits plus a sticky bit, so
// every operation rounds once, as the hardware does. Tininess is detected
// after rounding; FTZ flushes a tiny result (underflow masked) to a zero of
// its sign with UE and PE. Unmasked OE / UE report the flags the hardware
// sets for an exponent-unbounded result (the instruction then faults and its
// destination is not written, so the returned value is unused).
//
// Rare-path code: the entries are noinline so none of it enters k_run's fast loop.
#pragma once
#include "engine_exec.h"

namespace wtfgpu_dev {

typedef unsigned __int128 u128;

// the SSE / AVX floating-point forms engine_ssefp.h executes: map 1 = 0f,
// 2 = 0f 38, 3 = 0f 3a; pp 0 none, 1 66, 2 f3, 3 f2
__host__ __device__ inline bool fp_form(u32 map, u32 c, u32 pp, bool vex) {
  if (map == 1) {
    switch (c) {
      case 0x51: case 0x58: case 0x59: case 0x5c: case 0x5d: case 0x5e: case 0x5f: case 0xc2: case 0x5a:
        return true;
      case 0x5b: return pp <= 2;
      case 0x52: case 0x53: return pp == 0 || pp == 2;  // rsqrt / rcp ps, ss
      case 0x2e: case 0x2f: return pp <= 1;
      case 0x2a: case 0x2c: case 0x2d: return pp >= 2 || !vex;  // pp 0 / 1: the MMX-operand conversions
      case 0xe6: return pp >= 1;
      case 0x7c: case 0x7d: case 0xd0: return pp == 1 || pp == 3;
      case 0x12: return pp >= 2;
      case 0x16: return pp == 2;
      case 0xf0: return pp == 3;
      default: return false;
    }
  }
  if (pp != 1) return false;
  if (map == 2) return !vex && (c == 0x14 || c == 0x15);
  if (map == 3) return (c >= 0x08 && c <= 0x0d) || c == 0x40 || c == 0x41 || (vex && (c == 0x4a || c == 0x4b));
  return false;
}


enum : u32 { FE_I = 1, FE_D = 2, FE_Z = 4, FE_O = 8, FE_U = 16, FE_P = 32 };

struct FEnv {
  u32 rc;     // rounding: 0 nearest even, 1 down, 2 up, 3 toward zero
  u32 daz, ftz;
  u32 masks;  // FE_* bits, 1 = masked
  u32 fl;     // flags raised so far
};
__device__ __forceinline__ FEnv fenv_mx(u32 mx) {
  return FEnv{(mx >> 13) & 3, (mx >> 6) & 1, (mx >> 15) & 1, (mx >> 7) & 63, 0};
}

// w: 0 binary32 (value in the low 32 bits), 1 binary64, 2 binary16 (F16C)
__device__ __forceinline__ u32 fF(u32 w) { return w == 1 ? 52 : w == 2 ? 10 : 23; }
__device__ __forceinline__ i32 fEmax(u32 w) { return w == 1 ? 0x7ff : w == 2 ? 0x1f : 0xff; }
__device__ __forceinline__ i32 fBias(u32 w) { return w == 1 ? 1023 : w == 2 ? 15 : 127; }
__device__ __forceinline__ u32 fSb(u32 w) { return w == 1 ? 63 : w == 2 ? 15 : 31; }
__device__ __forceinline__ u32 f_sign(u64 x, u32 w) { return (u32)(x >> fSb(w)) & 1; }
__device__ __forceinline__ i32 f_exp(u64 x, u32 w) { return (i32)((x >> fF(w)) & (u64)fEmax(w)); }
__device__ __forceinline__ u64 f_frac(u64 x, u32 w) { return x & ((1ull << fF(w)) - 1); }
__device__ __forceinline__ u64 f_mag(u64 x, u32 w) { return x & ((1ull << fSb(w)) - 1); }
__device__ __forceinline__ bool f_nan(u64 x, u32 w) { return f_exp(x, w) == fEmax(w) && f_frac(x, w); }
__device__ __forceinline__ bool f_snan(u64 x, u32 w) { return f_nan(x, w) && !((x >> (fF(w) - 1)) & 1); }
__device__ __forceinline__ bool f_inf(u64 x, u32 w) { return f_exp(x, w) == fEmax(w) && !f_frac(x, w); }
__device__ __forceinline__ bool f_zero(u64 x, u32 w) { return f_mag(x, w) == 0; }
__device__ __forceinline__ bool f_den(u64 x, u32 w) { return f_exp(x, w) == 0 && f_frac(x, w); }
__device__ __forceinline__ u64 f_quiet(u64 x, u32 w) { return x | (1ull << (fF(w) - 1)); }
__device__ __forceinline__ u64 f_indef(u32 w) { return w == 1 ? 0xfff8000000000000ull : w == 2 ? 0xfe00ull : 0xffc00000ull; }
__device__ __forceinline__ u64 f_signed(u32 s, u32 w) { return (u64)s << fSb(w); }
__device__ __forceinline__ u64 f_infv(u32 s, u32 w) { return f_signed(s, w) | ((u64)fEmax(w) << fF(w)); }
// DAZ reads a denormal source as a zero of its sign
__device__ __forceinline__ u64 f_daz(const FEnv &v, u64 x, u32 w) {
  return (v.daz && f_den(x, w)) ? f_signed(f_sign(x, w), w) : x;
}
__device__ __forceinline__ u64 jam_shr(u64 x, u32 n) {
  if (n == 0) return x;
  return n >= 63 ? (u64)(x != 0) : (x >> n) | (u64)((x & ((1ull << n) - 1)) != 0);
}

// finite nonzero x -> (e, m), m's leading one at bit 62
__device__ __forceinline__ void f_unpack(u64 x, u32 w, i32 &e, u64 &m) {
  const u32 F = fF(w);
  const i32 ex = f_exp(x, w);
  const u64 fr = f_frac(x, w);
  if (ex) {
    e = ex - 1;
    m = ((1ull << F) | fr) << (62 - F);
  } else {
    const u32 sh = (u32)__builtin_clzll(fr) - 1;
    m = fr << sh;
    e = (i32)(62 - F) - (i32)sh;
  }
}

// (-1)^s * m / 2^62 * 2^(e + 1 - bias) rounded to format w (m != 0, m < 2^63)
__device__ __noinline__ u64 f_round(FEnv &v, u32 s, i32 e, u64 m, u32 w) {
  const u32 G = 62 - fF(w);
  const u64 half = 1ull << (G - 1), mask = (1ull << G) - 1;
  const u64 inc = v.rc == 0 ? half : v.rc == 3 ? 0 : ((v.rc == 1) == (s != 0)) ? mask : 0;
  const i32 emax = fEmax(w);
  if (e < 0) {
    const bool tiny = e < -1 || m + inc < (1ull << 63);
    if (tiny && !(v.masks & FE_U)) {  // unmasked underflow: the instruction faults
      v.fl |= FE_U | ((m & mask) ? FE_P : 0);
      return 0;
    }
    if (tiny && v.ftz) {
      v.fl |= FE_U | FE_P;
      return f_signed(s, w);
    }
    m = jam_shr(m, (u32)-e);
    e = 0;
    if (tiny && (m & mask)) v.fl |= FE_U;
  } else if (e > emax - 2 || (e == emax - 2 && m + inc >= (1ull << 63))) {
    if (!(v.masks & FE_O)) {  // unmasked overflow: the instruction faults
      v.fl |= FE_O | ((m & mask) ? FE_P : 0);
      return 0;
    }
    v.fl |= FE_O | FE_P;
    return inc ? f_infv(s, w) : f_infv(s, w) - 1;  // the largest finite when rounding toward it
  }
  const u64 rb = m & mask;
  if (rb) v.fl |= FE_P;
  u64 q = (m + inc) >> G;
  if (v.rc == 0 && rb == half) q &= ~1ull;
  if (!q) e = 0;
  return f_signed(s, w) + ((u64)e << fF(w)) + q;
}

// a value already in range and exact at format w's precision (no flags)
__device__ __forceinline__ u64 f_norm_round(FEnv &v, u32 s, i32 e, u64 m, u32 w) {
  const u32 sh = (u32)__builtin_clzll(m) - 1;
  return f_round(v, s, e - (i32)sh, m << sh, w);
}

// x86 NaN rule for two sources: IE for an SNaN; the first source's NaN
// (quietened) if it is one, else the second's
__device__ __forceinline__ bool f_nan2(FEnv &v, u64 a, u64 b, u32 w, u64 &r) {
  const bool na = f_nan(a, w), nb = f_nan(b, w);
  if (!na && !nb) return false;
  if (f_snan(a, w) || f_snan(b, w)) v.fl |= FE_I;
  r = f_quiet(na ? a : b, w);
  return true;
}

// |a| + / - |b| on finite values (DAZ applied, not both zero)
__device__ __noinline__ u64 f_addsub(FEnv &v, u64 a, u64 b, u32 w) {
  u32 sa = f_sign(a, w), sb = f_sign(b, w);
  if (f_zero(a, w) && f_zero(b, w)) return sa == sb ? a : f_signed(v.rc == 1, w);
  i32 ea = 0, eb = 0;
  u64 ma = 0, mb = 0;
  if (!f_zero(a, w)) f_unpack(a, w, ea, ma);
  if (!f_zero(b, w)) f_unpack(b, w, eb, mb);
  if (!ma) return f_round(v, sb, eb, mb, w);
  if (!mb) return f_round(v, sa, ea, ma, w);
  if (eb > ea || (eb == ea && mb > ma)) {  // a = the larger magnitude
    const u32 ts = sa;
    sa = sb, sb = ts;
    const i32 te = ea;
    ea = eb, eb = te;
    const u64 tm = ma;
    ma = mb, mb = tm;
  }
  const u64 mbs = jam_shr(mb, (u32)(ea - eb));
  if (sa == sb) {
    u64 m = ma + mbs;
    if (m >> 63) {
      m = jam_shr(m, 1);
      ea++;
    }
    return f_round(v, sa, ea, m, w);
  }
  const u64 m = ma - mbs;
  if (!m) return f_signed(v.rc == 1, w);
  return f_norm_round(v, sa, ea, m, w);
}

__device__ __noinline__ u64 f_mul(FEnv &v, u64 a, u64 b, u32 w) {
  const u32 s = f_sign(a, w) ^ f_sign(b, w);
  if (f_inf(a, w) || f_inf(b, w)) {
    if (f_zero(a, w) || f_zero(b, w)) {
      v.fl |= FE_I;
      return f_indef(w);
    }
    return f_infv(s, w);
  }
  if (f_zero(a, w) || f_zero(b, w)) return f_signed(s, w);
  i32 ea, eb;
  u64 ma, mb;
  f_unpack(a, w, ea, ma);
  f_unpack(b, w, eb, mb);
  const u128 p = (u128)ma * mb;  // [2^124, 2^126)
  i32 e = ea + eb + 1 - fBias(w);
  u32 sh = 62;
  if (p >> 125) {
    sh = 63;
    e++;
  }
  const u64 m = (u64)(p >> sh) | (u64)((p & ((((u128)1) << sh) - 1)) != 0);
  return f_round(v, s, e, m, w);
}

__device__ __noinline__ u64 f_div(FEnv &v, u64 a, u64 b, u32 w) {
  const u32 s = f_sign(a, w) ^ f_sign(b, w);
  const bool ia = f_inf(a, w), ib = f_inf(b, w), za = f_zero(a, w), zb = f_zero(b, w);
  if ((ia && ib) || (za && zb)) {
    v.fl |= FE_I;
    return f_indef(w);
  }
  if (ia) return f_infv(s, w);
  if (ib || za) return f_signed(s, w);
  if (zb) {
    v.fl |= FE_Z;
    return f_infv(s, w);
  }
  i32 ea, eb;
  u64 ma, mb;
  f_unpack(a, w, ea, ma);
  f_unpack(b, w, eb, mb);
  // 64 quotient bits of ma / mb: q = floor(ma / mb * 2^63), remainder -> sticky
  u64 r = ma, q = 0;
  for (int i = 0; i < 64; i++) {
    q <<= 1;
    if (r >= mb) {
      r -= mb;
      q |= 1;
    }
    r <<= 1;
  }
  i32 e = ea - eb + fBias(w) - 2;
  u64 m = q | (u64)(r != 0);
  if (q >> 63) {
    m = jam_shr(m, 1);
    e++;
  }
  return f_round(v, s, e, m, w);
}

// sqrt of a finite or infinite non-NaN value (DAZ applied)
__device__ __noinline__ u64 f_sqrt(FEnv &v, u64 a, u32 w) {
  if (f_zero(a, w)) return a;
  if (f_sign(a, w)) {
    v.fl |= FE_I;
    return f_indef(w);
  }
  if (f_inf(a, w)) return a;
  i32 e;
  u64 m;
  f_unpack(a, w, e, m);
  i32 E = e + 1 - fBias(w);  // unbiased
  u128 n = (u128)m << 62;   // sqrt(n) has its leading one at bit 62
  if (E & 1) {
    n <<= 1;
    E -= 1;
  }
  u64 r = 0;
  for (int i = 62; i >= 0; i--) {
    const u64 t = r | (1ull << i);
    if ((u128)t * t <= n) r = t;
  }
  const u64 sm = r | (u64)((u128)r * r != n);
  return f_round(v, 0, E / 2 + fBias(w) - 1, sm, w);
}

// ordered comparisons of non-NaN values
__device__ __forceinline__ bool f_eq(u64 a, u64 b, u32 w) { return a == b || (f_zero(a, w) && f_zero(b, w)); }
__device__ __forceinline__ bool f_lt(u64 a, u64 b, u32 w) {
  if (f_zero(a, w) && f_zero(b, w)) return false;
  const u32 sa = f_sign(a, w), sb = f_sign(b, w);
  if (sa != sb) return sa != 0;
  return sa ? f_mag(a, w) > f_mag(b, w) : f_mag(a, w) < f_mag(b, w);
}

enum : u32 { FOP_ADD, FOP_SUB, FOP_MUL, FOP_DIV, FOP_MIN, FOP_MAX, FOP_SQRT };

}  // namespace wtfgpu_dev
#include "engine_rcp_tab.h"  // the host CPU's RCPPS / RSQRTPS tables (scripts/gen_rcp_tables.c)
namespace wtfgpu_dev {
// RCPPS / RSQRTPS of one binary32 (U40): a table of the result at the
// reference exponent, rescaled; no flags, MXCSR ignored. rcp: +-0 and
// denormals -> +-inf, +-inf -> +-0, a tiny result -> +-0. rsqrt: a negative
// nonzero -> the default NaN, +-0 and denormals -> +-inf, +inf -> +0. NaNs
// quietened. (Matches the host on every exponent and sign: tests/golden fp vectors.)
__device__ __forceinline__ u32 f_rcp32(u32 x) {
  const u32 s = x & 0x80000000u, e = (x >> 23) & 0xff, m = x & 0x7fffff;
  if (e == 0xff) return m ? (x | 0x400000u) : s;
  if (e == 0) return s | 0x7f800000u;
  const u32 t = kRcpTab[m >> 12];
  const i32 re = (i32)((t >> 23) & 0xff) + 127 - (i32)e;
  if (re <= 0) return s;
  return s | ((u32)re << 23) | (t & 0x7fffff);
}
__device__ __forceinline__ u32 f_rsq32(u32 x) {
  const u32 s = x & 0x80000000u, e = (x >> 23) & 0xff, m = x & 0x7fffff;
  if (e == 0xff) return m ? (x | 0x400000u) : (s ? 0xffc00000u : 0u);
  if (e == 0) return s | 0x7f800000u;
  if (s) return 0xffc00000u;
  const u32 t = kRsqTab[(((e & 1) ^ 1) << 10) | (m >> 13)];
  const i32 k = ((i32)e - 127 - ((e & 1) ? 0 : 1)) / 2;  // x = y * 4^k, y in [1, 4)
  return ((u32)((i32)((t >> 23) & 0xff) - k) << 23) | (t & 0x7fffff);
}

// one element of an SSE arithmetic op: a = the first source (the
// destination of a legacy form), b = the second; sqrt reads b only
__device__ __noinline__ u64 f_arith(FEnv &v, u32 op, u64 a, u64 b, u32 w) {
  u64 r;
  if (op == FOP_MIN || op == FOP_MAX) {
    // the second source unless a is strictly less (min) / greater (max);
    // a NaN in either (IE, quiet or not) or two zeros also give the second
    a = f_daz(v, a, w);
    b = f_daz(v, b, w);  // the second source comes back DAZ-read, NaN case included
    if (f_nan(a, w) || f_nan(b, w)) {
      v.fl |= FE_I;
      return b;
    }
    if (f_den(a, w) || f_den(b, w)) v.fl |= FE_D;
    const bool pick_a = op == FOP_MIN ? f_lt(a, b, w) : f_lt(b, a, w);
    return pick_a ? a : b;
  }
  if (op == FOP_SQRT) {
    if (f_nan(b, w)) {
      if (f_snan(b, w)) v.fl |= FE_I;
      return f_quiet(b, w);
    }
    b = f_daz(v, b, w);
    // an invalid operand (negative, nonzero) outranks the denormal one
    if (f_den(b, w) && !f_sign(b, w)) v.fl |= FE_D;
    return f_sqrt(v, b, w);
  }
  if (f_nan2(v, a, b, w, r)) return r;
  a = f_daz(v, a, w);
  b = f_daz(v, b, w);
  // DE, unless a higher-priority exception (divide by zero) is raised
  if ((f_den(a, w) || f_den(b, w)) && !(op == FOP_DIV && f_zero(b, w))) v.fl |= FE_D;
  switch (op) {
    case FOP_ADD:
    case FOP_SUB: {
      if (op == FOP_SUB) b ^= f_signed(1, w);
      const bool ia = f_inf(a, w), ib = f_inf(b, w);
      if (ia || ib) {
        if (ia && ib && f_sign(a, w) != f_sign(b, w)) {
          v.fl |= FE_I;
          return f_indef(w);
        }
        return ia ? a : b;
      }
      return f_addsub(v, a, b, w);
    }
    case FOP_MUL: return f_mul(v, a, b, w);
    default: return f_div(v, a, b, w);
  }
}

// CMPPS / CMPSS predicate imm (0-31): all ones or zero. Signalling predicates
// raise IE for a QNaN, every predicate for an SNaN.
__device__ __noinline__ bool f_cmp(FEnv &v, u64 a, u64 b, u32 w, u32 pred) {
  const bool un = f_nan(a, w) || f_nan(b, w);
  const bool sig = (((pred & 3) == 1) || ((pred & 3) == 2)) != (((pred >> 4) & 1) != 0);
  if (f_snan(a, w) || f_snan(b, w) || (un && sig)) v.fl |= FE_I;
  bool eq = false, lt = false;
  if (!un) {
    a = f_daz(v, a, w);
    b = f_daz(v, b, w);
    if (f_den(a, w) || f_den(b, w)) v.fl |= FE_D;
    eq = f_eq(a, b, w);
    lt = f_lt(a, b, w);
  }
  switch (pred & 15) {
    case 0: return !un && eq;
    case 1: return !un && lt;
    case 2: return !un && (lt || eq);
    case 3: return un;
    case 4: return un || !eq;
    case 5: return un || !lt;
    case 6: return un || !(lt || eq);
    case 7: return !un;
    case 8: return un || eq;
    case 9: return un || lt;
    case 10: return un || lt || eq;
    case 11: return false;
    case 12: return !un && !eq;
    case 13: return !un && !lt;
    case 14: return !un && !(lt || eq);
    default: return true;
  }
}

// COMISS / UCOMISS: ZF PF CF = 111 unordered, 001 less, 100 equal, 000
// greater; OF SF AF cleared. comis (signalling) raises IE for any NaN.
__device__ __noinline__ u64 f_comi(FEnv &v, u64 a, u64 b, u32 w, bool signalling, u64 rflags) {
  rflags &= ~F_STATUS;
  if (f_nan(a, w) || f_nan(b, w)) {
    if (signalling || f_snan(a, w) || f_snan(b, w)) v.fl |= FE_I;
    return rflags | F_ZF | F_PF | F_CF;
  }
  a = f_daz(v, a, w);
  b = f_daz(v, b, w);
  if (f_den(a, w) || f_den(b, w)) v.fl |= FE_D;
  if (f_eq(a, b, w)) return rflags | F_ZF;
  return f_lt(a, b, w) ? rflags | F_CF : rflags;
}

// float -> signed integer of isz bytes (4 / 8); rc 3 for the truncating forms.
// NaN, infinity or out of range: IE and the integer indefinite (no PE).
__device__ __noinline__ u64 f_to_int(FEnv &v, u64 x, u32 w, u32 isz, u32 rc) {
  x = f_daz(v, x, w);
  const u64 indef = isz == 8 ? 0x8000000000000000ull : 0x80000000ull;
  if (f_nan(x, w) || f_inf(x, w)) {
    v.fl |= FE_I;
    return indef;
  }
  if (f_zero(x, w)) return 0;
  const u32 s = f_sign(x, w);
  i32 e;
  u64 m;
  f_unpack(x, w, e, m);
  const i32 E = e + 1 - fBias(w);  // |x| = m / 2^62 * 2^E
  if (E > 63) {
    v.fl |= FE_I;
    return indef;
  }
  u64 q, rem, half;
  bool inexact;
  if (E >= 62) {  // integral: m << (E - 62) (E = 63 only fits as -2^63)
    if (E == 63 && !(s && m == (1ull << 62))) {
      v.fl |= FE_I;
      return indef;
    }
    q = E == 63 ? (1ull << 63) : m;
    rem = 0;
    half = 0;
    inexact = false;
  } else {
    const u32 sh = (u32)(62 - E);  // >= 1
    if (sh >= 64) {
      q = 0;
      rem = m;  // < half of one (m / 2^sh < 1/2)
      half = ~0ull;
    } else {
      q = m >> sh;
      rem = m & ((1ull << sh) - 1);
      half = 1ull << (sh - 1);
    }
    inexact = rem != 0;
  }
  bool up = false;
  if (inexact) {
    if (rc == 0) up = rem > half || (rem == half && (q & 1));
    else if (rc == 1) up = s;
    else if (rc == 2) up = !s;
  }
  q += up;
  const u64 lim = (isz == 8 ? (1ull << 63) : (1ull << 31)) - (s ? 0 : 1);
  if (q > lim) {
    v.fl |= FE_I;
    return indef;
  }
  if (inexact) v.fl |= FE_P;
  return (s ? (u64)0 - q : q) & szmask(isz);
}

// signed integer -> float of format w
__device__ __noinline__ u64 f_from_int(FEnv &v, i64 x, u32 w) {
  if (x == 0) return 0;
  const u32 s = x < 0;
  const u64 mag = s ? (u64)0 - (u64)x : (u64)x;
  u64 m;
  i32 E;
  if (mag >> 63) {
    m = jam_shr(mag, 1);
    E = 63;
  } else {
    const u32 sh = (u32)__builtin_clzll(mag) - 1;
    m = mag << sh;
    E = 62 - (i32)sh;
  }
  return f_round(v, s, E + fBias(w) - 1, m, w);
}

// format conversion (cvtss2sd / cvtsd2ss and the packed forms)
__device__ __noinline__ u64 f_convert(FEnv &v, u64 x, u32 from, u32 to) {
  const u32 s = f_sign(x, from);
  if (f_nan(x, from)) {
    if (f_snan(x, from)) v.fl |= FE_I;
    const u64 fr = f_frac(x, from) | (1ull << (fF(from) - 1));
    const u64 f2 = to > from ? fr << (fF(to) - fF(from)) : fr >> (fF(from) - fF(to));
    return f_infv(s, to) | f2;
  }
  x = f_daz(v, x, from);
  if (f_den(x, from)) v.fl |= FE_D;
  if (f_inf(x, from)) return f_infv(s, to);
  if (f_zero(x, from)) return f_signed(s, to);
  i32 e;
  u64 m;
  f_unpack(x, from, e, m);
  return f_round(v, s, e - fBias(from) + fBias(to), m, to);
}

// ROUNDSS / ROUNDPS: to an integral value in format w with rounding rc;
// nopre suppresses PE (imm8 bit 3). IE only for an SNaN.
__device__ __noinline__ u64 f_round_int(FEnv &v, u64 x, u32 w, u32 rc, bool nopre) {
  if (f_nan(x, w)) {
    if (f_snan(x, w)) v.fl |= FE_I;
    return f_quiet(x, w);
  }
  x = f_daz(v, x, w);
  if (f_inf(x, w) || f_zero(x, w)) return x;
  const u32 F = fF(w), s = f_sign(x, w);
  const i32 E = f_exp(x, w) - fBias(w);  // denormals: E < 0
  if (E >= (i32)F) return x;
  u64 r;
  bool inexact, up = false;
  if (E < 0) {  // |x| < 1: zero or one
    const bool gt_half = E == -1 && f_frac(x, w) != 0, is_half = E == -1 && f_frac(x, w) == 0;
    inexact = true;
    if (rc == 0) up = gt_half;
    else if (rc == 1) up = s;
    else if (rc == 2) up = !s;
    (void)is_half;
    r = f_signed(s, w) | (up ? (u64)fBias(w) << F : 0);
  } else {
    const u64 unit = 1ull << (F - (u32)E), rem = x & (unit - 1), q = x & ~(unit - 1);
    inexact = rem != 0;
    if (inexact) {
      const u64 half = unit >> 1;
      if (rc == 0) up = rem > half || (rem == half && (q & unit));
      else if (rc == 1) up = s;
      else if (rc == 2) up = !s;
    }
    r = up ? q + unit : q;
  }
  if (inexact && !nopre) v.fl |= FE_P;
  return r;
}

}  // namespace wtfgpu_dev
