// engine_avx512.h — the AVX-512 subset: EVEX-encoded moves,
// logic, add / sub, unsigned min / max, compares and tests into opmask
// registers, vpternlog and broadcasts at 128 / 256 / 512 bits with merging or
// zeroing masks, and the VEX-encoded opmask instructions (kmov, kortest,
// ktest, kadd, kunpck, the k logic and shifts) — what vectorised memcpy / memset / strlen /
// memchr / strcmp paths built for AVX-512 run. Every other EVEX encoding is
// UNIMPLEMENTED (U36). The state (zmm0-31, k0-7) lives in the lane's cold
// state (wtfgpu_regs_t: xmm / ymmh / zmmh for zmm0-15, zmm_hi for 16-31, k).
//
// Memory: an element whose mask bit is 0 is neither read nor written, so it
// cannot fault (memory fault suppression); every page is checked before
// anything is written; the aligned forms need VL alignment unless every
// element is masked off. A load's fault is reported at the first selected
// byte that faults; a masked store's at its lowest selected element's first
// byte or else its highest one's last byte (what native execution reports). Faults are raised in the order #UD, #NM, #GP
// (alignment), then the memory access, as the VEX forms do (U23).
#pragma once

namespace wtfgpu_dev {

// UOp::opreg of an EVEX op: O_SSE's VEX fields (bit 0 set, bit 2 W, bits 4-7
// vvvv[3:0], bits 8-12 the map, bit 16 a prefix before it) plus bit 17 EVEX,
// bits 18-19 L'L, bit 20 z, bit 21 b, bits 22-24 aaa, bit 25 V' (vvvv[4]).
// UOp::reg and UOp::rm carry the 5-bit register numbers (R' and X included).
constexpr u32 EVX = 1u << 17;
__host__ __device__ inline u32 evex_ll(u32 x) { return (x >> 18) & 3; }
__host__ __device__ inline u32 evex_vvvv(u32 x) { return ((x >> 4) & 15) | (((x >> 26) & 1) << 4); }

enum : u32 {
  EZ_NONE = 0, EZ_MOV, EZ_LOGIC, EZ_ADD, EZ_SUB, EZ_MINU, EZ_MAXU, EZ_CMPEQ, EZ_CMPGT, EZ_CMP, EZ_TESTM,
  EZ_TERN, EZ_BCAST, EZ_BCASTR
};
struct EForm {
  u32 kind, es, sub;  // sub: logic op (0 and 1 andn 2 or 3 xor), cmp signedness (1 signed), testm negation
  bool store, aligned, bcastok, kdest;
  bool nt = false;    // the non-temporal moves: memory operand only, no masking (aaa != 0: #UD)
};

// The subset, by (map, opcode, pp, W). pp: 0 none, 1 66, 2 f3, 3 f2.
__host__ __device__ inline EForm evex_form(u32 map, u32 c, u32 pp, u32 w) {
  EForm f{EZ_NONE, 0, 0, false, false, false, false};
  if (map == 1) {
    if ((c == 0x10 || c == 0x11 || c == 0x28 || c == 0x29) && pp <= 1 && w == pp)  // vmovups/upd, vmovaps/apd
      return EForm{EZ_MOV, pp ? 8u : 4u, 0, (c & 1) != 0, c >= 0x28, false, false};
    if ((c == 0x2b && pp <= 1 && w == pp) || (c == 0xe7 && pp == 1 && !w))  // vmovntps / pd, vmovntdq
      return EForm{EZ_MOV, c == 0x2b && pp ? 8u : 4u, 0, true, true, false, false, true};
    if (c == 0x6f || c == 0x7f) {
      if (pp == 1) return EForm{EZ_MOV, w ? 8u : 4u, 0, c == 0x7f, true, false, false};   // vmovdqa32 / 64
      if (pp == 2) return EForm{EZ_MOV, w ? 8u : 4u, 0, c == 0x7f, false, false, false};  // vmovdqu32 / 64
      if (pp == 3) return EForm{EZ_MOV, w ? 2u : 1u, 0, c == 0x7f, false, false, false};  // vmovdqu8 / 16
      return f;
    }
    if (pp != 1) return f;
    switch (c) {
      case 0xdb: return EForm{EZ_LOGIC, w ? 8u : 4u, 0, false, false, true, false};
      case 0xdf: return EForm{EZ_LOGIC, w ? 8u : 4u, 1, false, false, true, false};
      case 0xeb: return EForm{EZ_LOGIC, w ? 8u : 4u, 2, false, false, true, false};
      case 0xef: return EForm{EZ_LOGIC, w ? 8u : 4u, 3, false, false, true, false};
      case 0xfc: return EForm{EZ_ADD, 1, 0, false, false, false, false};
      case 0xfd: return EForm{EZ_ADD, 2, 0, false, false, false, false};
      case 0xfe: return w ? f : EForm{EZ_ADD, 4, 0, false, false, true, false};
      case 0xd4: return w ? EForm{EZ_ADD, 8, 0, false, false, true, false} : f;
      case 0xf8: return EForm{EZ_SUB, 1, 0, false, false, false, false};
      case 0xf9: return EForm{EZ_SUB, 2, 0, false, false, false, false};
      case 0xfa: return w ? f : EForm{EZ_SUB, 4, 0, false, false, true, false};
      case 0xfb: return w ? EForm{EZ_SUB, 8, 0, false, false, true, false} : f;
      case 0xda: return EForm{EZ_MINU, 1, 0, false, false, false, false};
      case 0xde: return EForm{EZ_MAXU, 1, 0, false, false, false, false};
      case 0x74: return EForm{EZ_CMPEQ, 1, 0, false, false, false, true};
      case 0x75: return EForm{EZ_CMPEQ, 2, 0, false, false, false, true};
      case 0x76: return w ? f : EForm{EZ_CMPEQ, 4, 0, false, false, true, true};
      case 0x64: return EForm{EZ_CMPGT, 1, 0, false, false, false, true};
      case 0x65: return EForm{EZ_CMPGT, 2, 0, false, false, false, true};
      case 0x66: return w ? f : EForm{EZ_CMPGT, 4, 0, false, false, true, true};
      default: return f;
    }
  }
  if (map == 2) {
    if ((c == 0x26 || c == 0x27) && (pp == 1 || pp == 2))  // vptestm / vptestnm b w (26), d q (27)
      return EForm{EZ_TESTM, c == 0x26 ? (w ? 2u : 1u) : (w ? 8u : 4u), pp == 2 ? 1u : 0u, false, false, c == 0x27,
                   true};
    if (pp != 1) return f;
    switch (c) {
      case 0x2a: return w ? f : EForm{EZ_MOV, 4, 0, false, true, false, false, true};  // vmovntdqa
      case 0x29: return w ? EForm{EZ_CMPEQ, 8, 0, false, false, true, true} : f;
      case 0x37: return w ? EForm{EZ_CMPGT, 8, 0, false, false, true, true} : f;
      case 0x3a: return EForm{EZ_MINU, 2, 0, false, false, false, false};
      case 0x3e: return EForm{EZ_MAXU, 2, 0, false, false, false, false};
      case 0x78: return w ? f : EForm{EZ_BCAST, 1, 0, false, false, false, false};
      case 0x79: return w ? f : EForm{EZ_BCAST, 2, 0, false, false, false, false};
      case 0x58: return w ? f : EForm{EZ_BCAST, 4, 0, false, false, false, false};
      case 0x59: return w ? EForm{EZ_BCAST, 8, 0, false, false, false, false} : f;
      case 0x7a: return w ? f : EForm{EZ_BCASTR, 1, 0, false, false, false, false};
      case 0x7b: return w ? f : EForm{EZ_BCASTR, 2, 0, false, false, false, false};
      case 0x7c: return EForm{EZ_BCASTR, w ? 8u : 4u, 0, false, false, false, false};
      default: return f;
    }
  }
  if (map == 3 && pp == 1) {
    if (c == 0x25) return EForm{EZ_TERN, w ? 8u : 4u, 0, false, false, true, false};
    if (c == 0x3e || c == 0x3f) return EForm{EZ_CMP, w ? 2u : 1u, c & 1, false, false, false, true};
    if (c == 0x1e || c == 0x1f) return EForm{EZ_CMP, w ? 8u : 4u, c & 1, false, false, true, true};
  }
  return f;
}

// disp8 * N (SDM 2.7.5): full-vector forms scale by the vector length, a
// broadcast memory operand (EVEX.b, or the broadcast instructions' element)
// by the element size. vl: 16 / 32 / 64.
__host__ __device__ inline u32 evex_disp8_n(const EForm &f, u32 vl, u32 b) {
  if (f.kind == EZ_BCAST || (b && f.bcastok)) return f.es;
  return vl;
}

// The VEX-encoded opmask instructions (0f 41-47 / 90-93 / 98 / 99, 0f 3a
// 30-33): operand bits (8 / 16 / 32 / 64), 0 = not one of them.
__host__ __device__ inline u32 kop_bits(u32 map, u32 c, u32 pp, u32 w) {
  if (map == 3) return (c >= 0x30 && c <= 0x33 && pp == 1) ? ((c & 1) ? (w ? 64u : 32u) : (w ? 16u : 8u)) : 0u;
  if (map != 1) return 0;
  const bool grp = (c >= 0x41 && c <= 0x47 && c != 0x43) || c == 0x4a || c == 0x90 || c == 0x91 || c == 0x98 ||
                   c == 0x99;
  if (grp) return pp == 0 ? (w ? 64u : 16u) : pp == 1 ? (w ? 32u : 8u) : 0u;
  if (c == 0x4b) return pp == 1 ? (w ? 0u : 16u) : pp == 0 ? (w ? 64u : 32u) : 0u;  // kunpckbw / wd / dq: result bits
  if (c == 0x92 || c == 0x93) return pp == 0 ? (w ? 0u : 16u) : pp == 1 ? (w ? 0u : 8u) : pp == 3 ? (w ? 64u : 32u) : 0u;
  return 0;
}

struct Z512 {
  u64 q[8];
};
__device__ __forceinline__ Z512 zmm_get(const Dev &P, const Lane &L, u32 r) {
  const wtfgpu_regs_t &F = P.full[L.lane];
  Z512 v;
  if (r < 16) {
    v.q[0] = F.xmm[r][0], v.q[1] = F.xmm[r][1], v.q[2] = F.ymmh[r][0], v.q[3] = F.ymmh[r][1];
    for (u32 i = 0; i < 4; i++) v.q[4 + i] = F.zmmh[r][i];
  } else {
    for (u32 i = 0; i < 8; i++) v.q[i] = F.zmm_hi[r - 16][i];
  }
  return v;
}
// an EVEX destination: the bits above the vector length zeroed
__device__ __forceinline__ void zmm_put(const Dev &P, const Lane &L, u32 r, Z512 v, u32 vl) {
  wtfgpu_regs_t &F = P.full[L.lane];
  for (u32 i = vl / 8; i < 8; i++) v.q[i] = 0;
  if (r < 16) {
    F.xmm[r][0] = v.q[0], F.xmm[r][1] = v.q[1], F.ymmh[r][0] = v.q[2], F.ymmh[r][1] = v.q[3];
    for (u32 i = 0; i < 4; i++) F.zmmh[r][i] = v.q[4 + i];
  } else {
    for (u32 i = 0; i < 8; i++) F.zmm_hi[r - 16][i] = v.q[i];
  }
}
__device__ __forceinline__ u64 zel(const Z512 &v, u32 i, u32 w) {
  const u32 bit = i * w * 8;
  return (v.q[bit >> 6] >> (bit & 63)) & szmask(w);
}
__device__ __forceinline__ void zset(Z512 &v, u32 i, u32 w, u64 x) {
  const u32 bit = i * w * 8, s = bit & 63;
  const u64 mk = szmask(w) << s;
  v.q[bit >> 6] = (v.q[bit >> 6] & ~mk) | ((x << s) & mk);
}
__device__ __forceinline__ u64 kmask_bits(u32 n) { return n >= 64 ? ~0ull : (1ull << n) - 1; }

// The selected elements of an n-element operand at ea (es bytes each): every
// page checked first (loads: the selected elements' pages), then the moves.
__device__ __forceinline__ bool zspan(Lane &L, u64 ea, u32 es, u32 n, u64 sel, int acc) {
  if (sel == kmask_bits(n)) return span_ok(L, ea, es * n, acc);
  for (u32 i = 0; i < n; i++)
    if (((sel >> i) & 1) && !span_ok(L, ea + (u64)i * es, es, acc)) return false;
  return true;
}
__device__ __forceinline__ bool zload(Lane &L, u64 ea, u32 es, u32 n, u64 sel, Z512 &v) {
  for (u32 i = 0; i < 8; i++) v.q[i] = 0;
  if (!sel) return true;
  tn_mute(L.lane);  // Tenet: one access of the operand
  bool ok = zspan(L, ea, es, n, sel, ACC_R);
  if (ok && sel == kmask_bits(n) && es * n >= 8) {
    for (u32 i = 0; ok && i < es * n / 8; i++) ok = vread(L, ea + 8 * i, 8, v.q[i]);
  } else {
    for (u32 i = 0; ok && i < n; i++) {
      u64 x = 0;
      if ((sel >> i) & 1) ok = vread(L, ea + (u64)i * es, es, x);
      zset(v, i, es, x);
    }
  }
  return tn_unmute(L.lane, ea, es * n, TN_R, ok);
}
// A masked store (aaa != 0) checks two bytes, as the hardware reports them:
// the lowest selected element's first byte, then the highest one's last byte
// (native vectors: a fault on the upper page is reported at that last byte).
__device__ __forceinline__ bool zstore(Lane &L, u64 ea, u32 es, u32 n, u64 sel, bool masked, const Z512 &v) {
  if (!sel) return true;
  if (masked) {
    const u32 lo = __builtin_ctzll(sel), hi = 63 - __builtin_clzll(sel);
    if (!xlate(L, ea + (u64)lo * es, ACC_WPROBE) || !xlate(L, ea + (u64)hi * es + es - 1, ACC_WPROBE)) return false;
  } else if (!zspan(L, ea, es, n, sel, ACC_WPROBE)) {
    return false;
  }
  tn_mute(L.lane);
  bool ok = true;
  if (sel == kmask_bits(n) && es * n >= 8) {
    for (u32 i = 0; ok && i < es * n / 8; i++) ok = vwrite(L, ea + 8 * i, 8, v.q[i]);
  } else {
    for (u32 i = 0; ok && i < n; i++)
      if ((sel >> i) & 1) ok = vwrite(L, ea + (u64)i * es, es, zel(v, i, es));
  }
  return tn_unmute(L.lane, ea, es * n, TN_W, ok);
}

__device__ __forceinline__ int z_ud(Lane &L) {
  set_fault(L, WTFGPU_VEC_UD, 0, 0);
  return X_FAULT;
}

__device__ __noinline__ int evex_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, pp = u.bsz, map = vex_map(x), w = (x >> 2) & 1;
  const u32 ll = evex_ll(x), z = (x >> 21) & 1, b = (x >> 22) & 1, aaa = (x >> 23) & 7, vvvv = evex_vvvv(x);
  const bool mem = u.is_mem;
  const EForm f = evex_form(map, c, pp, w);
  wtfgpu_regs_t &F = P.full[L.lane];
  // ---- #UD: a prefix before EVEX, the AVX-512 state off, encodings the form forbids
  bool ud = ((x >> 16) & 1) || f.kind == EZ_NONE || ll == 3;
  if (!((P.sys[L.lane].cr4 >> 18) & 1) || (F.xcr0 & 0xe6) != 0xe6) ud = true;
  const bool two = f.kind == EZ_MOV || f.kind == EZ_BCAST || f.kind == EZ_BCASTR;
  if (two && vvvv != 0) ud = true;
  if (b && (!mem || !f.bcastok)) ud = true;          // no rounding control in these forms
  if (z && (f.kdest || (f.store && mem) || aaa == 0)) ud = true;  // a k or memory destination merges only; z needs a mask
  if (f.nt && (!mem || aaa != 0)) ud = true;                        // non-temporal moves: memory, no mask
  if (f.kind == EZ_BCASTR && mem) ud = true;
  if (ud) return z_ud(L);
  if (L.cr0 & 8) {
    set_fault(L, 7, 0, 0);  // #NM
    return X_FAULT;
  }
  const u32 vl = 16u << ll, es = f.es, n = vl / es;
  const u64 all = kmask_bits(n), sel = aaa ? (F.k[aaa] & all) : all;
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  if (mem && f.aligned && sel && (ea & (vl - 1))) {  // no #GP when every element is masked off
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return X_FAULT;
  }
  const u32 dst = u.reg & 31;
  // ---- stores
  if (f.kind == EZ_MOV && f.store && mem) {
    const Z512 s = zmm_get(P, L, dst);
    return zstore(L, ea, es, n, sel, aaa != 0, s) ? X_OK : X_FAULT;
  }
  // ---- the r/m source (a broadcast element, the selected elements, or a register)
  Z512 bsrc;
  if (f.kind == EZ_BCASTR) {
    for (u32 i = 0; i < 8; i++) bsrc.q[i] = 0;
    zset(bsrc, 0, es, R(L, u.rm & 15) & szmask(es));
  } else if (mem) {
    const bool one = b || f.kind == EZ_BCAST;
    // the elements the result needs: a k destination's and a merge's
    // masked-off ones are not read (fault suppression)
    if (!zload(L, ea, one ? es : es, one ? 1 : n, one ? (sel ? 1ull : 0ull) : sel, bsrc)) return X_FAULT;
    if (b) {
      const u64 e0 = zel(bsrc, 0, es);
      for (u32 i = 0; i < n; i++) zset(bsrc, i, es, e0);
    }
  } else {
    bsrc = zmm_get(P, L, (f.store ? dst : u.rm) & 31);
  }
  const Z512 a = zmm_get(P, L, vvvv);
  const Z512 old = zmm_get(P, L, (f.store && !mem) ? (u.rm & 31) : dst);
  const u32 imm = (u32)u.imm & 0xff;
  if (f.kdest) {  // compares and tests: a mask of n bits
    u64 k = 0;
    for (u32 i = 0; i < n; i++) {
      const u64 p = zel(a, i, es), q = zel(bsrc, i, es);
      bool t;
      switch (f.kind) {
        case EZ_CMPEQ: t = p == q; break;
        case EZ_CMPGT: t = (i64)sext(p, es) > (i64)sext(q, es); break;
        case EZ_TESTM: t = ((p & q) != 0) != (f.sub != 0); break;
        default: {  // EZ_CMP: imm[2:0] 0 eq 1 lt 2 le 3 false 4 neq 5 nlt 6 nle 7 true
          const bool lt = f.sub ? (i64)sext(p, es) < (i64)sext(q, es) : p < q;
          const bool eq = p == q;
          const u32 pr = imm & 7;
          t = pr == 0 ? eq : pr == 1 ? lt : pr == 2 ? (lt || eq) : pr == 3 ? false : pr == 4 ? !eq
              : pr == 5 ? !lt : pr == 6 ? !(lt || eq) : true;
        }
      }
      k |= (u64)t << i;
    }
    F.k[u.reg & 7] = k & sel;
    return X_OK;
  }
  Z512 r = old;
  for (u32 i = 0; i < n; i++) {
    if (!((sel >> i) & 1)) {
      if (z) zset(r, i, es, 0);
      continue;
    }
    const u64 p = zel(a, i, es), q = zel(bsrc, i, es);
    u64 v;
    switch (f.kind) {
      case EZ_MOV: v = q; break;
      case EZ_LOGIC: v = f.sub == 0 ? (p & q) : f.sub == 1 ? (~p & q) : f.sub == 2 ? (p | q) : (p ^ q); break;
      case EZ_ADD: v = p + q; break;
      case EZ_SUB: v = p - q; break;
      case EZ_MINU: v = p < q ? p : q; break;
      case EZ_MAXU: v = p > q ? p : q; break;
      case EZ_TERN: {  // bit j of the result: imm8[(dst << 2) | (src1 << 1) | src2] of bit j
        const u64 d = zel(old, i, es);
        v = 0;
        for (u32 t = 0; t < 8; t++) {
          if (!((imm >> t) & 1)) continue;
          v |= ((t & 4) ? d : ~d) & ((t & 2) ? p : ~p) & ((t & 1) ? q : ~q);
        }
        break;
      }
      default: v = zel(bsrc, 0, es); break;  // broadcasts
    }
    zset(r, i, es, v & szmask(es));
  }
  zmm_put(P, L, (f.store && !mem) ? (u.rm & 31) : dst, r, vl);
  return X_OK;
}

// The VEX-encoded opmask instructions.
__device__ __noinline__ int kop_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, pp = u.bsz, map = vex_map(x), w = (x >> 2) & 1, l = (x >> 1) & 1;
  const u32 vvvv = (x >> 4) & 15, bits = kop_bits(map, c, pp, w);
  wtfgpu_regs_t &F = P.full[L.lane];
  const bool mem = u.is_mem;
  // VEX.L: 1 for the two-source ops (logic, kadd, kunpck), else 0; vvvv: only they name a register
  const bool two_src = map == 1 && ((c >= 0x41 && c <= 0x47 && c != 0x44) || c == 0x4a || c == 0x4b);
  bool ud = ((x >> 16) & 1) || !bits || l != (two_src ? 1u : 0u) || (!two_src && vvvv != 0);
  if (!((P.sys[L.lane].cr4 >> 18) & 1) || (F.xcr0 & 0xe6) != 0xe6) ud = true;
  if (mem && !(map == 1 && (c == 0x90 || c == 0x91))) ud = true;  // only kmov has memory forms
  if (!mem && map == 1 && c == 0x91) ud = true;
  if (ud) return z_ud(L);
  const u64 mk = kmask_bits(bits);
  const u32 kr = u.reg & 7, km = u.rm & 7;
  if (map == 3) {  // kshiftr / kshiftl
    const u32 cnt = (u32)u.imm & 0xff;
    const u64 s = F.k[km] & mk;
    F.k[kr] = cnt >= bits ? 0 : (((c & 2) ? (s << cnt) : (s >> cnt)) & mk);
    return X_OK;
  }
  switch (c) {
    case 0x90:
      if (mem) {
        u64 v;
        if (!vread(L, sse_ea(P, L, u, nrip), bits / 8, v)) return X_FAULT;
        F.k[kr] = v & mk;
      } else {
        F.k[kr] = F.k[km] & mk;
      }
      return X_OK;
    case 0x91: return vwrite(L, sse_ea(P, L, u, nrip), bits / 8, F.k[kr] & mk) ? X_OK : X_FAULT;
    case 0x92: F.k[kr] = R(L, u.rm & 15) & mk; return X_OK;
    case 0x93: RS(L, u.reg & 15, F.k[km] & mk); return X_OK;  // a 32-bit destination zero-extended
    case 0x98:
    case 0x99: {
      const u64 p = F.k[kr] & mk, q = F.k[km] & mk;
      const bool zf = c == 0x98 ? (p | q) == 0 : (p & q) == 0;
      const bool cf = c == 0x98 ? (p | q) == mk : (~p & q & mk) == 0;
      L.rflags = (L.rflags & ~F_STATUS) | (zf ? F_ZF : 0) | (cf ? F_CF : 0);
      return X_OK;
    }
    case 0x44: F.k[kr] = ~F.k[km] & mk; return X_OK;
    case 0x4b: {  // kunpck: the first source's low half above the second source's low half
      const u32 h = bits / 2;
      const u64 hm = kmask_bits(h);
      F.k[kr] = ((F.k[vvvv & 7] & hm) << h) | (F.k[km] & hm);
      return X_OK;
    }
    default: {
      const u64 p = F.k[vvvv & 7] & mk, q = F.k[km] & mk;
      const u64 v = c == 0x41 ? (p & q) : c == 0x42 ? (~p & q) : c == 0x45 ? (p | q) : c == 0x46 ? ~(p ^ q)
                  : c == 0x4a ? p + q : (p ^ q);  // 4a: kadd
      F.k[kr] = v & mk;
      return X_OK;
    }
  }
}

}  // namespace wtfgpu_dev
