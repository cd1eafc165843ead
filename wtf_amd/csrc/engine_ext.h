// engine_ext.h — the instruction-set extensions cpuid_leaf enumerates beyond
// SSE4.1 / AVX2 (convention U45):
//   * general-purpose forms (UOp op O_GEXT, gext_exec): BMI1 (andn, bextr,
//     blsi / blsmsk / blsr), BMI2 (bzhi, pdep, pext, mulx, rorx, sarx / shlx /
//     shrx), ADX (adcx, adox), MOVBE, CRC32 (f2 0f 38 f0 / f1);
//   * SIMD forms (an O_SSE op, x42_exec): SSE4.2 (pcmpgtq, pcmpestri /
//     pcmpestrm / pcmpistri / pcmpistrm), AES (aesenc / enclast / dec /
//     declast / imc / keygenassist) and PCLMULQDQ, legacy and VEX.128 (and
//     VEX.256 vpcmpgtq).
// Everything is integer arithmetic; the oracle computes the same forms
// (oracle/x86_oracle_ext.inc) and both are pinned by native vectors
// (tests/golden/ext_vectors.json.gz). Flags the SDM leaves undefined are
// cleared (U45). VAES / VPCLMULQDQ (their VEX.256 forms) are defined but not
// enumerated: UNIMPLEMENTED, never #UD.
#pragma once
#include "engine_sse.h"

namespace wtfgpu_dev {

// ---------------------------------------------------------------- general-purpose forms
enum : u32 {
  GX_NONE = 0, GX_ANDN, GX_BLS, GX_BZHI, GX_BEXTR, GX_SHLX, GX_SARX, GX_SHRX, GX_PDEP, GX_PEXT, GX_MULX,
  GX_RORX, GX_ADCX, GX_ADOX, GX_MOVBE, GX_CRC32
};
// pp: 0 none, 1 66, 2 f3, 3 f2 (the legacy class: f3 / f2 win over 66)
__host__ __device__ inline u32 gx_form(u32 map, u32 c, u32 pp, bool vex) {
  if (vex) {
    if (map == 3) return (c == 0xf0 && pp == 3) ? GX_RORX : GX_NONE;
    if (map != 2) return GX_NONE;
    switch (c) {
      case 0xf2: return pp == 0 ? GX_ANDN : GX_NONE;
      case 0xf3: return pp == 0 ? GX_BLS : GX_NONE;
      case 0xf5: return pp == 0 ? GX_BZHI : pp == 2 ? GX_PEXT : pp == 3 ? GX_PDEP : GX_NONE;
      case 0xf6: return pp == 3 ? GX_MULX : GX_NONE;
      case 0xf7: return pp == 0 ? GX_BEXTR : pp == 1 ? GX_SHLX : pp == 2 ? GX_SARX : GX_SHRX;
      default: return GX_NONE;
    }
  }
  if (map != 2) return GX_NONE;
  if (c == 0xf0 || c == 0xf1) return pp == 3 ? GX_CRC32 : pp <= 1 ? GX_MOVBE : GX_NONE;
  if (c == 0xf6) return pp == 1 ? GX_ADCX : pp == 2 ? GX_ADOX : GX_NONE;
  return GX_NONE;
}

__device__ __forceinline__ u64 gx_szf(u64 res, u32 sz) {
  return ((res & szmask(sz)) == 0 ? F_ZF : 0) | (msb(res, sz) ? F_SF : 0);
}
// CRC-32C (Castagnoli, reflected polynomial 0x82f63b78), n bytes of v, no
// pre / post inversion (the instruction's)
__device__ __forceinline__ u32 crc32c(u32 crc, u64 v, u32 n) {
  for (u32 i = 0; i < 8 * n; i++) {
    crc ^= (u32)(v >> i) & 1;
    crc = (crc >> 1) ^ ((crc & 1) ? 0x82f63b78u : 0u);
  }
  return crc;
}
__device__ __forceinline__ u64 pdep64(u64 src, u64 mask) {
  u64 r = 0;
  for (u64 bb = 1; mask; bb += bb) {
    if (src & bb) r |= mask & (0 - mask);
    mask &= mask - 1;
  }
  return r;
}
__device__ __forceinline__ u64 pext64(u64 src, u64 mask) {
  u64 r = 0;
  for (u64 bb = 1; mask; bb += bb) {
    if (src & mask & (0 - mask)) r |= bb;
    mask &= mask - 1;
  }
  return r;
}

// One attempt at a general-purpose extension form. UOp: sub = opcode, bsz =
// prefix class, opreg = VEX fields / map (as O_SSE), asz = the legacy operand
// size (REX.W 8, 66 2, else 4).
__device__ __noinline__ int gext_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, pp = u.bsz, map = vex_map(x);
  const bool vex = x & 1, mem = u.is_mem;
  const u32 f = gx_form(map, c, pp, vex);
  const u32 vvvv = (x >> 4) & 15;
  // adcx's 66 is its mandatory prefix, not an operand-size override
  // (VEX.W1 is a 64-bit operand in 64-bit mode only: 32-bit code runs it at 32 bits)
  const u32 sz = vex ? (((x >> 2) & 1) && !(L.efer & EFER_M32) ? 8 : 4) : f == GX_ADCX ? (((u.rex >> 3) & 1) ? 8 : 4) : u.asz;
  // #UD: a legacy prefix before VEX, VEX.L = 1 (no CR4.OSXSAVE / XCR0 gate on
  // the VEX-encoded general-purpose forms); the register form of movbe;
  // group 17 beyond /1 /2 /3
  const u32 r3 = u.reg & 7;
  if (f == GX_NONE || (vex && (((x >> 16) & 1) || ((x >> 1) & 1))) || (f == GX_MOVBE && !mem) ||
      (f == GX_BLS && (r3 < 1 || r3 > 3))) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  const u64 m = szmask(sz);
  if (f == GX_MOVBE && c == 0xf1) {  // movbe m, r: the only store
    const u64 v = R(L, u.reg);
    u64 s = 0;
    for (u32 i = 0; i < sz; i++) s |= ((v >> (8 * i)) & 0xff) << (8 * (sz - 1 - i));
    return vwrite(L, ea, sz, s) ? X_OK : X_FAULT;
  }
  // the r/m source (crc32 f0: a byte)
  const u32 ssz = (f == GX_CRC32 && c == 0xf0) ? 1 : sz;
  u64 b = 0;
  if (mem) {
    if (!vread(L, ea, ssz, b)) return X_FAULT;
  } else {
    b = getr(L, u.rex, u.rm, ssz);
  }
  b &= szmask(ssz);
  const u64 v = R(L, vvvv) & m;
  const u32 bits = 8 * sz;
  u64 fl = L.rflags, res = 0;
  switch (f) {
    case GX_ANDN:
      res = ~v & b & m;
      fl = (fl & ~F_STATUS) | gx_szf(res, sz);
      break;
    case GX_BLS: {  // the destination is vvvv
      res = r3 == 1 ? (b & (b - 1)) : r3 == 2 ? (b ^ (b - 1)) : (b & (0 - b));
      res &= m;
      const bool cfv = r3 == 3 ? b != 0 : b == 0;
      fl = (fl & ~F_STATUS) | (r3 == 2 ? (msb(res, sz) ? F_SF : 0) : gx_szf(res, sz)) | (cfv ? F_CF : 0);
      RS(L, vvvv, res);
      L.rflags = fl;
      return X_OK;
    }
    case GX_BZHI: {
      const u32 n = (u32)(v & 0xff);
      res = n < bits ? b & ((1ull << n) - 1) : b;
      fl = (fl & ~F_STATUS) | gx_szf(res, sz) | (n > bits - 1 ? F_CF : 0);
      break;
    }
    case GX_BEXTR: {
      const u32 st = (u32)(v & 0xff), ln = (u32)((v >> 8) & 0xff);
      res = st >= bits ? 0 : (b >> st);
      if (ln < 64) res &= (1ull << ln) - 1;
      res &= m;
      fl = (fl & ~F_STATUS) | (res == 0 ? F_ZF : 0);
      break;
    }
    case GX_SHLX: res = (b << (v & (bits - 1))) & m; break;
    case GX_SHRX: res = b >> (v & (bits - 1)); break;
    case GX_SARX: res = (u64)((i64)sext(b, sz) >> (v & (bits - 1))) & m; break;
    case GX_PDEP: res = pdep64(v, b) & m; break;
    case GX_PEXT: res = pext64(v, b) & m; break;
    case GX_RORX: {
      const u32 k = (u32)u.imm & (bits - 1);
      res = k ? ((b >> k) | (b << (bits - k))) & m : b;
      break;
    }
    case GX_MULX: {  // reg := high, vvvv := low (the high half wins when they are one register)
      const u64 d = R(L, 2) & m;
      u64 lo, hi;
      if (sz == 8) {
        lo = d * b;
        hi = __umul64hi(d, b);
      } else {
        const u64 p = d * b;
        lo = p & 0xffffffffull;
        hi = p >> 32;
      }
      RS(L, vvvv, lo);
      RS(L, u.reg, hi);
      return X_OK;
    }
    case GX_ADCX:
    case GX_ADOX: {
      const u64 cf = f == GX_ADCX ? (fl & F_CF) : ((fl >> 11) & 1);
      const u64 a = R(L, u.reg) & m;
      res = (a + b + cf) & m;
      const bool carry = sz == 8 ? (res < a || (cf && res == a)) : ((a + b + cf) >> bits) != 0;
      const u64 bit = f == GX_ADCX ? F_CF : F_OF;
      fl = (fl & ~bit) | (carry ? bit : 0);
      break;
    }
    case GX_MOVBE: {  // movbe r, m (16-bit: the register's upper bits stay)
      u64 s = 0;
      for (u32 i = 0; i < sz; i++) s |= ((b >> (8 * i)) & 0xff) << (8 * (sz - 1 - i));
      setr(L, u.rex, u.reg, sz, s);
      return X_OK;
    }
    default: {  // GX_CRC32: the destination is r32, or r64 with REX.W (zero-extended)
      const u32 crc = crc32c((u32)R(L, u.reg), b, ssz);
      RS(L, u.reg, (u64)crc);
      return X_OK;
    }
  }
  setr(L, u.rex, u.reg, sz, res);
  L.rflags = fl;
  return X_OK;
}

// ---------------------------------------------------------------- SIMD forms
// 66 0f 38 37 db-df, 66 0f 3a 44 60-63 df; VEX the same (pp = 66); SHA:
// 0f 38 c8-cd, 0f 3a cc (no prefix, no VEX form)
__host__ __device__ inline bool x42_form(u32 map, u32 c, u32 pp, bool vex) {
  if (pp == 0 && !vex) return (map == 2 && c >= 0xc8 && c <= 0xcd) || (map == 3 && c == 0xcc);
  if (pp != 1) return false;
  if (map == 2) return c == 0x37 || (c >= 0xdb && c <= 0xdf);
  if (map == 3) return c == 0x44 || (c >= 0x60 && c <= 0x63) || c == 0xdf;
  return false;
}

__constant__ u8 kAesSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82, 0xc9,
    0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f,
    0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07,
    0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3,
    0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58,
    0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3,
    0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f,
    0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73, 0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88,
    0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac,
    0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a,
    0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70,
    0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11,
    0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42,
    0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

// GF(2^8) arithmetic modulo x^8 + x^4 + x^3 + x + 1 (MixColumns, and the
// inverse S-box as inverse affine map + field inverse: no second table)
__device__ __forceinline__ u32 gf_mul(u32 a, u32 b) {
  u32 r = 0;
  for (int i = 0; i < 8; i++) {
    if (b & 1) r ^= a;
    const u32 hi = a & 0x80;
    a = (a << 1) & 0xff;
    if (hi) a ^= 0x1b;
    b >>= 1;
  }
  return r;
}
// x^254 = x^-1 in GF(2^8) (0 -> 0)
__device__ __forceinline__ u32 gf_inv(u32 x) {
  u32 r = 1, p = x;
  for (u32 e = 254; e; e >>= 1) {
    if (e & 1) r = gf_mul(r, p);
    p = gf_mul(p, p);
  }
  return x ? r : 0;
}
__device__ __forceinline__ u32 rotl8(u32 x, u32 k) { return ((x << k) | (x >> (8 - k))) & 0xff; }
// InvSubBytes: the inverse affine map, then the field inverse
__device__ __forceinline__ u32 aes_inv_sbox(u32 y) {
  const u32 x = rotl8(y, 1) ^ rotl8(y, 3) ^ rotl8(y, 6) ^ 0x05;
  return gf_inv(x);
}

__device__ __forceinline__ u32 xb(const X128 &v, u32 i) { return (u32)xel(v, i, 1); }

// state byte i = row i % 4, column i / 4
__device__ __noinline__ X128 aes_round(X128 s, X128 k, u32 kind) {
  // kind: 0 enc, 1 enclast, 2 dec, 3 declast, 4 imc (InvMixColumns only)
  u8 t[16];
  for (u32 i = 0; i < 16; i++) {
    const u32 r = i & 3, col = i >> 2;
    if (kind == 4) t[i] = (u8)xb(s, i);
    else if (kind < 2) t[i] = kAesSbox[xb(s, r + 4 * ((col + r) & 3))];  // ShiftRows, SubBytes
    else t[i] = (u8)aes_inv_sbox(xb(s, r + 4 * ((col - r) & 3)));       // InvShiftRows, InvSubBytes
  }
  X128 o{0, 0};
  for (u32 col = 0; col < 4; col++) {
    const u32 a0 = t[4 * col], a1 = t[4 * col + 1], a2 = t[4 * col + 2], a3 = t[4 * col + 3];
    u32 b0 = a0, b1 = a1, b2 = a2, b3 = a3;
    if (kind == 0) {  // MixColumns
      b0 = gf_mul(a0, 2) ^ gf_mul(a1, 3) ^ a2 ^ a3;
      b1 = a0 ^ gf_mul(a1, 2) ^ gf_mul(a2, 3) ^ a3;
      b2 = a0 ^ a1 ^ gf_mul(a2, 2) ^ gf_mul(a3, 3);
      b3 = gf_mul(a0, 3) ^ a1 ^ a2 ^ gf_mul(a3, 2);
    } else if (kind == 2 || kind == 4) {  // InvMixColumns
      b0 = gf_mul(a0, 14) ^ gf_mul(a1, 11) ^ gf_mul(a2, 13) ^ gf_mul(a3, 9);
      b1 = gf_mul(a0, 9) ^ gf_mul(a1, 14) ^ gf_mul(a2, 11) ^ gf_mul(a3, 13);
      b2 = gf_mul(a0, 13) ^ gf_mul(a1, 9) ^ gf_mul(a2, 14) ^ gf_mul(a3, 11);
      b3 = gf_mul(a0, 11) ^ gf_mul(a1, 13) ^ gf_mul(a2, 9) ^ gf_mul(a3, 14);
    }
    xset(o, 4 * col, 1, b0);
    xset(o, 4 * col + 1, 1, b1);
    xset(o, 4 * col + 2, 1, b2);
    xset(o, 4 * col + 3, 1, b3);
  }
  if (kind != 4) {
    o.lo ^= k.lo;
    o.hi ^= k.hi;
  }
  return o;
}
__device__ __forceinline__ u32 aes_subword(u32 w) {
  u32 r = 0;
  for (u32 i = 0; i < 4; i++) r |= (u32)kAesSbox[(w >> (8 * i)) & 0xff] << (8 * i);
  return r;
}
// aeskeygenassist: [SubWord(X1), RotWord(SubWord(X1)) ^ rcon, SubWord(X3), RotWord(SubWord(X3)) ^ rcon]
__device__ __forceinline__ X128 aes_keygen(X128 s, u32 rcon) {
  const u32 x1 = aes_subword((u32)(s.lo >> 32)), x3 = aes_subword((u32)(s.hi >> 32));
  const u32 r1 = ((x1 >> 8) | (x1 << 24)) ^ rcon, r3 = ((x3 >> 8) | (x3 << 24)) ^ rcon;
  return X128{(u64)x1 | ((u64)r1 << 32), (u64)x3 | ((u64)r3 << 32)};
}
// carry-less 64 x 64 -> 128
__device__ __forceinline__ X128 clmul64(u64 a, u64 b) {
  X128 r{0, 0};
  for (u32 i = 0; i < 64; i++)
    if ((b >> i) & 1) {
      r.lo ^= a << i;
      if (i) r.hi ^= a >> (64 - i);
    }
  return r;
}

// pcmpXstrX (SDM "Packed Compare String"): IntRes2 and the flags. a = the
// register operand (xmm1), b = r/m; la / lb the valid element counts.
__device__ __noinline__ u32 pcmpstr(X128 a, X128 b, u32 imm, u32 la, u32 lb, u64 &fl) {
  const u32 w = (imm & 1) ? 2 : 1, n = 16 / w, sgn = (imm >> 1) & 1, agg = (imm >> 2) & 3;
  auto el = [&](const X128 &v, u32 i) -> i64 { return sgn ? xsel(v, i, w) : (i64)xel(v, i, w); };
  u32 r1 = 0;
  for (u32 j = 0; j < n; j++) {
    bool bit;
    if (agg == 0) {  // equal any: b[j] is one of a's valid elements
      bit = false;
      if (j < lb)
        for (u32 i = 0; i < la; i++) bit = bit || el(a, i) == el(b, j);
    } else if (agg == 1) {  // ranges: a[2k] <= b[j] <= a[2k + 1] for a valid pair
      bit = false;
      if (j < lb)
        for (u32 i = 0; i + 1 < n; i += 2) {
          const bool ge = i < la && el(b, j) >= el(a, i), le = i + 1 < la && el(b, j) <= el(a, i + 1);
          bit = bit || (ge && le);
        }
    } else if (agg == 2) {  // equal each: both invalid is a match, one invalid is not
      bit = (j >= la && j >= lb) ? true : (j < la && j < lb) ? el(a, j) == el(b, j) : false;
    } else {  // equal ordered: a (up to its length) occurs in b at j
      bit = true;
      for (u32 i = 0; i + j < n; i++) {
        const bool m = i >= la ? true : (i + j >= lb ? false : el(a, i) == el(b, i + j));
        bit = bit && m;
      }
    }
    r1 |= (bit ? 1u : 0u) << j;
  }
  const u32 full = (1u << n) - 1, pol = (imm >> 4) & 3;
  u32 r2 = r1;
  if (pol == 1) r2 = ~r1 & full;
  else if (pol == 3) r2 = r1 ^ ((1u << lb) - 1);
  fl = (fl & ~F_STATUS) | (r2 ? F_CF : 0) | (lb < n ? F_ZF : 0) | (la < n ? F_SF : 0) | ((r2 & 1) ? F_OF : 0);
  return r2;
}
// the valid length of an implicit-length operand: up to its first zero element
__device__ __forceinline__ u32 str_len(X128 v, u32 w) {
  for (u32 i = 0; i < 16 / w; i++)
    if (xel(v, i, w) == 0) return i;
  return 16 / w;
}
// an explicit length: |rax| / |rdx| (REX.W / VEX.W: 64-bit, else 32-bit), at most the element count
__device__ __forceinline__ u32 str_elen(u64 r, u32 wide, u32 n) {
  const i64 s = wide ? (i64)r : (i64)(i32)(u32)r;
  const u64 m = s < 0 ? (u64)0 - (u64)s : (u64)s;
  return m > n ? n : (u32)m;
}

// SHA-1 / SHA-256 message and round helpers (SDM vol. 2 SHA1RNDS4 ..
// SHA256MSG2); dwords d[0] = bits 31:0 .. d[3] = bits 127:96
__device__ __forceinline__ u32 rol32(u32 x, u32 k) { return (x << k) | (x >> (32 - k)); }
__device__ __forceinline__ u32 ror32(u32 x, u32 k) { return (x >> k) | (x << (32 - k)); }
__device__ __forceinline__ void x4(const X128 &v, u32 *d) {
  d[0] = (u32)v.lo, d[1] = (u32)(v.lo >> 32), d[2] = (u32)v.hi, d[3] = (u32)(v.hi >> 32);
}
__device__ __forceinline__ X128 x4set(u32 d0, u32 d1, u32 d2, u32 d3) {
  return X128{(u64)d0 | ((u64)d1 << 32), (u64)d2 | ((u64)d3 << 32)};
}
// c: 0f 38 c8 sha1nexte, c9 sha1msg1, ca sha1msg2, cb sha256rnds2 (wk = xmm0),
// cc sha256msg1, cd sha256msg2; 0f 3a cc sha1rnds4 (imm: f / K)
__device__ __noinline__ X128 sha_op(u32 map, u32 c, X128 a, X128 b, X128 wk, u32 imm) {
  u32 s[4], t[4], w[4];
  x4(a, s);
  x4(b, t);
  if (map == 3) {  // sha1rnds4: A B C D from src1, W0+E W1 W2 W3 from src2
    const u32 K[4] = {0x5A827999u, 0x6ED9EBA1u, 0x8F1BBCDCu, 0xCA62C1D6u};
    const u32 f = imm & 3;
    u32 A = s[3], B = s[2], C = s[1], D = s[0], E = 0;
    const u32 W[4] = {t[3], t[2], t[1], t[0]};
    for (u32 i = 0; i < 4; i++) {
      const u32 fv = f == 0 ? ((B & C) ^ (~B & D)) : f == 2 ? ((B & C) ^ (B & D) ^ (C & D)) : (B ^ C ^ D);
      const u32 nA = fv + rol32(A, 5) + W[i] + E + K[f];
      E = D, D = C, C = rol32(B, 30), B = A, A = nA;
    }
    return x4set(D, C, B, A);
  }
  switch (c) {
    case 0xc8:  // sha1nexte
      return x4set(t[0], t[1], t[2], t[3] + rol32(s[3], 30));
    case 0xc9:  // sha1msg1
      return x4set(t[2] ^ s[0], t[3] ^ s[1], s[0] ^ s[2], s[1] ^ s[3]);
    case 0xca: {  // sha1msg2
      const u32 w16 = rol32(s[3] ^ t[2], 1), w17 = rol32(s[2] ^ t[1], 1), w18 = rol32(s[1] ^ t[0], 1);
      const u32 w19 = rol32(s[0] ^ w16, 1);
      return x4set(w19, w18, w17, w16);
    }
    case 0xcb: {  // sha256rnds2: A B E F from src2, C D G H from src1, WK0 / WK1 from xmm0
      x4(wk, w);
      u32 A = t[3], B = t[2], C = s[3], D = s[2], E = t[1], F = t[0], G = s[1], H = s[0];
      for (u32 i = 0; i < 2; i++) {
        const u32 ch = (E & F) ^ (~E & G), maj = (A & B) ^ (A & C) ^ (B & C);
        const u32 s0 = ror32(A, 2) ^ ror32(A, 13) ^ ror32(A, 22), s1 = ror32(E, 6) ^ ror32(E, 11) ^ ror32(E, 25);
        const u32 t1 = ch + s1 + w[i] + H;
        H = G, G = F, F = E, E = t1 + D, D = C, C = B, B = A, A = t1 + maj + s0;
      }
      return x4set(F, E, B, A);
    }
    case 0xcc: {  // sha256msg1
      auto sg0 = [](u32 x) { return ror32(x, 7) ^ ror32(x, 18) ^ (x >> 3); };
      return x4set(s[0] + sg0(s[1]), s[1] + sg0(s[2]), s[2] + sg0(s[3]), s[3] + sg0(t[0]));
    }
    default: {  // 0xcd sha256msg2
      auto sg1 = [](u32 x) { return ror32(x, 17) ^ ror32(x, 19) ^ (x >> 10); };
      const u32 w16 = s[0] + sg1(t[2]), w17 = s[1] + sg1(t[3]), w18 = s[2] + sg1(w16), w19 = s[3] + sg1(w17);
      return x4set(w16, w17, w18, w19);
    }
  }
}

// One attempt at a SIMD extension form (legacy: the CR0 / CR4 checks ran in sse_exec).
__device__ __noinline__ int x42_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, map = vex_map(x);
  const bool vex = x & 1, mem = u.is_mem;
  // W: the explicit-length forms' rax / rdx (64-bit mode only, as u.rex)
  const u32 l256 = vex ? (x >> 1) & 1 : 0, W = (u.rex >> 3) & 1, vvvv = vex ? (x >> 4) & 15 : 0;
  const u32 imm = (u32)u.imm & 0xff;
  const bool str = map == 3 && c >= 0x60 && c <= 0x63;
  const bool sha = (map == 2 && c >= 0xc8 && c <= 0xcd) || (map == 3 && c == 0xcc);
  const bool two = (map == 2 && c == 0xdb) || (map == 3 && c == 0xdf) || str || sha;
  if (vex) {
    // VAES / VPCLMULQDQ (VEX.256): defined, not enumerated, not executed
    if (l256 && ((map == 2 && c >= 0xdc) || (map == 3 && c == 0x44))) return X_UNIMPL;
    const u64 cr4 = P.sys[L.lane].cr4;
    bool ud = ((x >> 16) & 1) || !((cr4 >> 18) & 1) || (P.full[L.lane].xcr0 & 6) != 6;
    if ((two && vvvv != 0) || (l256 && !(map == 2 && c == 0x37))) ud = true;
    if (ud) {
      set_fault(L, WTFGPU_VEC_UD, 0, 0);
      return X_FAULT;
    }
    if (L.cr0 & 8) {
      set_fault(L, 7, 0, 0);  // #NM
      return X_FAULT;
    }
  }
  const u32 vl = l256 ? 32 : 16;
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  if (mem && !vex && !str && (ea & 15)) {  // legacy 16-byte operands are aligned; the string forms are not
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return X_FAULT;
  }
  Y256 b{X128{0, 0}, X128{0, 0}};
  if (mem) {
    if (!yload(L, ea, vl, b)) return X_FAULT;
  } else {
    b = vex ? ymm_get(P, L, u.rm) : Y256{xmm_get(P, L, u.rm), X128{0, 0}};
  }
  const Y256 s = vex ? ymm_get(P, L, u.reg) : Y256{xmm_get(P, L, u.reg), X128{0, 0}};
  const Y256 a = vex && !two ? ymm_get(P, L, vvvv) : s;  // the first source
  if (str) {
    const u32 w = (imm & 1) ? 2 : 1, n = 16 / w;
    const bool expl = c <= 0x61;
    const u32 la = expl ? str_elen(R(L, 0), W, n) : str_len(a.l, w);
    const u32 lb = expl ? str_elen(R(L, 2), W, n) : str_len(b.l, w);
    u64 fl = L.rflags;
    const u32 r2 = pcmpstr(a.l, b.l, imm, la, lb, fl);
    if (c & 1) {  // index -> ecx: the least or (imm bit 6) most significant set bit, n if none
      u32 idx = n;
      if (r2) idx = (imm & 0x40) ? 31 - (u32)__builtin_clz(r2) : (u32)__builtin_ctz(r2);
      RS(L, 1, idx);
    } else {  // mask -> xmm0: the bits, or (imm bit 6) each element all ones / zeros
      X128 m{0, 0};
      if (imm & 0x40) {
        for (u32 i = 0; i < n; i++) xset(m, i, w, ((r2 >> i) & 1) ? szmask(w) : 0);
      } else {
        m.lo = r2;
      }
      if (vex) ymm_put(P, L, 0, Y256{m, X128{0, 0}}, 0);
      else xmm_put(P, L, 0, m);
    }
    L.rflags = fl;
    return X_OK;
  }
  Y256 r{X128{0, 0}, X128{0, 0}};
  if (sha) {
    r.l = sha_op(map, c, a.l, b.l, c == 0xcb ? xmm_get(P, L, 0) : X128{0, 0}, imm);
  } else if (map == 2 && c == 0x37) {  // pcmpgtq
    for (u32 i = 0; i < vl / 8; i++) yset(r, i, 8, (i64)yel(a, i, 8) > (i64)yel(b, i, 8) ? ~0ull : 0);
  } else if (map == 2) {  // aesimc (db), aesenc / enclast / dec / declast (dc-df): state a, round key b
    r.l = c == 0xdb ? aes_round(b.l, X128{0, 0}, 4) : aes_round(a.l, b.l, c - 0xdc);
  } else if (c == 0x44) {  // pclmulqdq
    r.l = clmul64((imm & 1) ? a.l.hi : a.l.lo, (imm & 0x10) ? b.l.hi : b.l.lo);
  } else {  // 0xdf aeskeygenassist
    r.l = aes_keygen(b.l, imm);
  }
  if (vex) ymm_put(P, L, u.reg, r, l256);
  else xmm_put(P, L, u.reg, r.l);
  return X_OK;
}

}  // namespace wtfgpu_dev
