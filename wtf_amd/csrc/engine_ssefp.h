// engine_ssefp.h — the SSE / SSE2 / SSE3 / SSE4.1 floating-point forms and
// their VEX encodings (conventions U39 / U40), on the integer
// arithmetic of engine_fp.h. Included by engine_sse.h after its operand
// helpers; sse_exec / vex_exec hand every form fp_form() accepts to fp_exec.
//
//   arithmetic   0f 51 58 59 5c 5d 5e 5f (ps pd ss sd), cmp 0f c2, comis /
//                ucomis 0f 2f / 2e, SSE3 hadd / hsub / addsub (0f 7c 7d d0)
//   conversions  0f 5a (ps2pd pd2ps ss2sd sd2ss), 0f 5b (dq2ps ps2dq
//                tps2dq), 0f e6 (dq2pd pd2dq tpd2dq), f3 / f2 0f 2a
//                (si2ss / si2sd), f3 / f2 0f 2c / 2d (t)ss2si / (t)sd2si
//   moves        movsldup / movshdup / movddup (0f 12 / 16), lddqu (f2 0f f0),
//                blendps / blendpd (0f 3a 0c / 0d), blendvps / blendvpd
//                (0f 38 14 / 15; VEX 0f 3a 4a / 4b)
//   rounding     roundps / pd / ss / sd (0f 3a 08-0b)
//
// The MMX-operand conversions (cvtpi2ps, cvtps2pi, ... without an f2 / f3
// prefix), dpps / dppd and the approximations rcpps / rsqrtps (vendor-
// specific tables, not IEEE) stay UNIMPLEMENTED. Exceptions: every element is
// computed with flags; an unmasked pre-computation exception (IE DE ZE) sets
// only those flags, any other unmasked exception sets all of them; either way
// the instruction faults with #XM (CR4.OSXMMEXCPT) or #UD and writes nothing
// but MXCSR (SDM vol. 1 11.5.2).
#pragma once
#include "engine_fp.h"

namespace wtfgpu_dev {

__device__ __forceinline__ u64 yel(const Y256 &v, u32 i, u32 ew) {
  const u32 per = 16 / ew;
  return i < per ? xel(v.l, i, ew) : xel(v.h, i - per, ew);
}
__device__ __forceinline__ void yset(Y256 &v, u32 i, u32 ew, u64 x) {
  const u32 per = 16 / ew;
  if (i < per) xset(v.l, i, ew, x);
  else xset(v.h, i - per, ew, x);
}

__device__ __forceinline__ int xm_fault(Lane &L, u64 cr4) {
  set_fault(L, (cr4 >> 10) & 1 ? 19u : (u32)WTFGPU_VEC_UD, 0, 0);  // #XM, or #UD without CR4.OSXMMEXCPT
  return X_FAULT;
}

enum : u32 { FK_ARITH, FK_CMP, FK_COMI, FK_CVTF, FK_CVTI, FK_CVTPD, FK_SI2F, FK_F2SI, FK_HADD, FK_DUP, FK_LDDQU,
             FK_ROUND, FK_BLEND, FK_BLENDV, FK_DP, FK_RCP, FK_MMXCVT };

__device__ __noinline__ int fp_exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 x = u.opreg, c = u.sub, pp = u.bsz, map = vex_map(x);
  const bool vex = x & 1, mem = u.is_mem;
  // W: the integer operand's size (cvtsi2s* / cvt(t)s*2si: 64-bit mode only,
  // as u.rex); VW: VEX.W as encoded (vblendv W1 is #UD in every mode)
  const u32 l256 = vex ? (x >> 1) & 1 : 0, W = (u.rex >> 3) & 1, VW = vex ? (x >> 2) & 1 : 0;
  const u32 vvvv = vex ? (x >> 4) & 15 : 0;
  const u32 imm = (u32)u.imm & 0xff;
  const u64 cr4 = P.sys[L.lane].cr4;
  const u32 vl = l256 ? 32 : 16;
  // ---- the form: kind, element format, r/m operand size, alignment, VEX shape
  u32 k = FK_ARITH, w = 0, n = vl;
  bool scalar = false, two_op = false, align = !vex;
  if (map == 1) {
    switch (c) {
      case 0x2e: case 0x2f: k = FK_COMI; w = pp; scalar = true; two_op = true; break;
      case 0x5a:
        k = FK_CVTF;
        w = pp & 1;
        scalar = pp >= 2;
        two_op = pp <= 1;
        if (pp == 0) n = l256 ? 16 : 8, align = false;
        break;
      case 0x5b: k = FK_CVTI; two_op = true; break;
      case 0x52: case 0x53:  // rsqrt / rcp: ps, ss
        k = FK_RCP;
        scalar = pp == 2;
        two_op = pp == 0;
        break;
      case 0xe6:
        k = FK_CVTPD;
        two_op = true;
        if (pp == 2) n = l256 ? 16 : 8, align = false;
        break;
      case 0x2a: case 0x2c: case 0x2d:
        if (pp <= 1) {  // cvtpi2ps / cvtpi2pd (mm / m64 source), cvt(t)ps2pi / cvt(t)pd2pi (mm destination)
          k = FK_MMXCVT;
          w = pp & 1;
          n = (c != 0x2a && pp == 1) ? 16 : 8;
          break;
        }
        if (c == 0x2a) {
          k = FK_SI2F;
          w = pp & 1;
          scalar = true;
          n = W ? 8 : 4;
        } else {
          k = FK_F2SI;
          w = pp & 1;
          scalar = true;
          two_op = true;
        }
        break;
      case 0x7c: case 0x7d: case 0xd0: k = FK_HADD; w = pp == 1; break;
      case 0x12: case 0x16:
        k = FK_DUP;
        two_op = true;
        if (pp == 3 && !l256) n = 8, align = false;
        break;
      case 0xf0: k = FK_LDDQU; two_op = true; align = false; break;
      case 0xc2: k = FK_CMP; w = pp & 1; scalar = pp >= 2; break;
      default:  // 51 58 59 5c 5d 5e 5f
        w = pp & 1;
        scalar = pp >= 2;
        two_op = c == 0x51 && !scalar;
        break;
    }
  } else if (map == 2) {
    k = FK_BLENDV;
    w = c & 1;
  } else if (c == 0x40 || c == 0x41) {  // dpps / dppd
    k = FK_DP;
    w = c & 1;
  } else if (c <= 0x0b) {
    k = FK_ROUND;
    w = c & 1;
    scalar = c >= 0x0a;
    two_op = !scalar;
  } else {
    k = c == 0x0c || c == 0x0d ? FK_BLEND : FK_BLENDV;
    w = c & 1;
  }
  const u32 ew = w ? 8 : 4;
  if (scalar && k != FK_SI2F) n = (k == FK_CVTF) ? (pp == 2 ? 4 : 8) : ew;
  if (scalar) align = false;
  // ---- #UD / #NM (the legacy checks ran in sse_exec)
  if (vex) {
    bool ud = (x >> 16) & 1;
    if (!((cr4 >> 18) & 1) || (P.full[L.lane].xcr0 & 6) != 6) ud = true;
    if (two_op && vvvv != 0) ud = true;
    if (k == FK_BLENDV && VW) ud = true;
    if (k == FK_DP && w && l256) ud = true;  // vdppd has no 256-bit form
    if (k == FK_LDDQU && !mem) ud = true;
    if (ud) {
      set_fault(L, WTFGPU_VEC_UD, 0, 0);
      return X_FAULT;
    }
    if (L.cr0 & 8) {
      set_fault(L, 7, 0, 0);  // #NM
      return X_FAULT;
    }
  } else if (k == FK_LDDQU && !mem) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  // an MMX register operand: a pending unmasked x87 exception first (#MF), as mmx_exec
  if (k == FK_MMXCVT && (c != 0x2a || !mem) && (P.full[L.lane].fpsw & ~P.full[L.lane].fpcw & 0x3f)) {
    set_fault(L, 16, 0, 0);
    return X_FAULT;
  }
  const u64 ea = mem ? sse_ea(P, L, u, nrip) : 0;
  if (mem && align && n == 16 && (ea & 15)) {
    set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return X_FAULT;
  }
  // ---- operands: a = first source (legacy: the destination; VEX: vvvv), b = r/m
  const Y256 a = vex ? ymm_get(P, L, vvvv) : Y256{xmm_get(P, L, u.reg), X128{0, 0}};
  Y256 b{X128{0, 0}, X128{0, 0}};
  if (mem) {
    if (!yload(L, ea, n, b)) return X_FAULT;
  } else if (k == FK_SI2F) {
    b.l.lo = R(L, u.rm) & szmask(n);
  } else {
    b = vex ? ymm_get(P, L, u.rm) : Y256{xmm_get(P, L, u.rm), X128{0, 0}};
  }
  wtfgpu_regs_t &F = P.full[L.lane];
  FEnv v = fenv_mx(F.mxcsr);
  Y256 r = scalar ? Y256{a.l, X128{0, 0}} : Y256{X128{0, 0}, X128{0, 0}};
  u32 keep256 = l256;  // VEX: whether the result keeps bits 255:128
  const u32 ne = vl / ew;
  u32 gpr_out = 0;
  u64 gval = 0;
  switch (k) {
    case FK_ARITH: {
      const u32 op = c == 0x51 ? FOP_SQRT : c == 0x58 ? FOP_ADD : c == 0x59 ? FOP_MUL : c == 0x5c ? FOP_SUB
                     : c == 0x5d ? FOP_MIN : c == 0x5e ? FOP_DIV : FOP_MAX;
      if (scalar) {
        xset(r.l, 0, ew, f_arith(v, op, xel(a.l, 0, ew), xel(b.l, 0, ew), w));
        keep256 = 0;
      } else {
        const Y256 s1 = (vex || op != FOP_SQRT) ? a : b;
        for (u32 i = 0; i < ne; i++) yset(r, i, ew, f_arith(v, op, yel(s1, i, ew), yel(b, i, ew), w));
      }
      break;
    }
    case FK_CMP: {
      const u32 pred = vex ? imm & 31 : imm & 7;
      if (scalar) {
        xset(r.l, 0, ew, f_cmp(v, xel(a.l, 0, ew), xel(b.l, 0, ew), w, pred) ? szmask(ew) : 0);
        keep256 = 0;
      } else {
        for (u32 i = 0; i < ne; i++) yset(r, i, ew, f_cmp(v, yel(a, i, ew), yel(b, i, ew), w, pred) ? szmask(ew) : 0);
      }
      break;
    }
    case FK_COMI: {
      const X128 s = xmm_get(P, L, u.reg);
      const u64 fl = f_comi(v, xel(s, 0, ew), xel(b.l, 0, ew), w, c == 0x2f, L.rflags);
      const u32 pre = v.fl & 7;
      if (pre & ~v.masks) {
        F.mxcsr |= pre;
        return xm_fault(L, cr4);
      }
      F.mxcsr |= v.fl;
      L.rflags = fl;
      return X_OK;
    }
    case FK_CVTF:
      if (pp == 0) {  // cvtps2pd
        for (u32 i = 0; i < vl / 8; i++) yset(r, i, 8, f_convert(v, yel(b, i, 4), 0, 1));
      } else if (pp == 1) {  // cvtpd2ps: an xmm result
        for (u32 i = 0; i < vl / 8; i++) yset(r, i, 4, f_convert(v, yel(b, i, 8), 1, 0));
        keep256 = 0;
      } else if (pp == 2) {  // cvtss2sd
        xset(r.l, 0, 8, f_convert(v, xel(b.l, 0, 4), 0, 1));
        keep256 = 0;
      } else {  // cvtsd2ss
        xset(r.l, 0, 4, f_convert(v, xel(b.l, 0, 8), 1, 0));
        keep256 = 0;
      }
      break;
    case FK_CVTI:
      for (u32 i = 0; i < vl / 4; i++) {
        const u64 e = yel(b, i, 4);
        yset(r, i, 4, pp == 0 ? f_from_int(v, (i64)(i32)(u32)e, 0) : f_to_int(v, e, 0, 4, pp == 2 ? 3 : v.rc));
      }
      break;
    case FK_CVTPD:
      if (pp == 2) {  // cvtdq2pd
        for (u32 i = 0; i < vl / 8; i++) yset(r, i, 8, f_from_int(v, (i64)(i32)(u32)yel(b, i, 4), 1));
      } else {  // cvttpd2dq / cvtpd2dq: an xmm result
        for (u32 i = 0; i < vl / 8; i++) yset(r, i, 4, f_to_int(v, yel(b, i, 8), 1, 4, pp == 1 ? 3 : v.rc));
        keep256 = 0;
      }
      break;
    case FK_SI2F:
      xset(r.l, 0, ew, f_from_int(v, W ? (i64)b.l.lo : (i64)(i32)(u32)b.l.lo, w));
      keep256 = 0;
      break;
    case FK_F2SI:
      gpr_out = 1;
      gval = f_to_int(v, xel(b.l, 0, ew), w, W ? 8 : 4, c == 0x2c ? 3 : v.rc);
      break;
    case FK_HADD:
      for (u32 h = 0; h < vl / 16; h++) {
        const X128 al = h ? a.h : a.l, bl = h ? b.h : b.l;
        X128 o{0, 0};
        const u32 per = 16 / ew;
        for (u32 i = 0; i < per; i++) {
          u64 e;
          if (c == 0xd0) {  // addsub: even elements subtract
            e = f_arith(v, (i & 1) ? FOP_ADD : FOP_SUB, xel(al, i, ew), xel(bl, i, ew), w);
          } else {  // hadd / hsub: pairs of a, then pairs of b
            const X128 sv = i < per / 2 ? al : bl;
            const u32 j = (i % (per / 2)) * 2;
            e = f_arith(v, c == 0x7c ? FOP_ADD : FOP_SUB, xel(sv, j, ew), xel(sv, j + 1, ew), w);
          }
          xset(o, i, ew, e);
        }
        if (h) r.h = o;
        else r.l = o;
      }
      break;
    case FK_DUP:
      for (u32 h = 0; h < vl / 16; h++) {
        const X128 bl = h ? b.h : b.l;
        X128 o;
        if (pp == 3) {
          o = X128{bl.lo, bl.lo};
        } else {
          const u32 odd = c == 0x16;
          const u64 e0 = xel(bl, odd, 4), e1 = xel(bl, 2 + odd, 4);
          o = X128{e0 | (e0 << 32), e1 | (e1 << 32)};
        }
        if (h) r.h = o;
        else r.l = o;
      }
      break;
    case FK_LDDQU: r = b; break;
    case FK_ROUND: {
      const u32 rc = (imm & 4) ? v.rc : imm & 3;
      if (scalar) {
        xset(r.l, 0, ew, f_round_int(v, xel(b.l, 0, ew), w, rc, imm & 8));
        keep256 = 0;
      } else {
        for (u32 i = 0; i < ne; i++) yset(r, i, ew, f_round_int(v, yel(b, i, ew), w, rc, imm & 8));
      }
      break;
    }
    case FK_BLEND:
      for (u32 i = 0; i < ne; i++) yset(r, i, ew, ((imm >> i) & 1) ? yel(b, i, ew) : yel(a, i, ew));
      break;
    case FK_MMXCVT:
      if (c == 0x2a) {  // two int32 -> the low two floats (the rest of xmm stays) / two doubles
        const u64 src = mem ? b.l.lo : mmx_get(F, u.rm & 7);
        r.l = a.l;
        if (pp) {
          r.l.lo = f_from_int(v, (i64)(i32)(u32)src, 1);
          r.l.hi = f_from_int(v, (i64)(i32)(u32)(src >> 32), 1);
        } else {
          xset(r.l, 0, 4, f_from_int(v, (i64)(i32)(u32)src, 0));
          xset(r.l, 1, 4, f_from_int(v, (i64)(i32)(u32)(src >> 32), 0));
        }
      } else {  // two floats / doubles -> two int32 in mm (2c: truncated)
        const u32 rc = c == 0x2c ? 3u : v.rc, e2 = pp ? 8 : 4;
        const u64 lo = f_to_int(v, xel(b.l, 0, e2), pp, 4, rc), hi = f_to_int(v, xel(b.l, 1, e2), pp, 4, rc);
        gval = (lo & 0xffffffffull) | (hi << 32);
        gpr_out = 2;
      }
      break;
    case FK_RCP:
      if (scalar) {
        xset(r.l, 0, 4, c == 0x53 ? f_rcp32((u32)xel(b.l, 0, 4)) : f_rsq32((u32)xel(b.l, 0, 4)));
        keep256 = 0;
      } else {
        for (u32 i = 0; i < ne; i++) yset(r, i, 4, c == 0x53 ? f_rcp32((u32)yel(b, i, 4)) : f_rsq32((u32)yel(b, i, 4)));
      }
      break;
    case FK_DP: {
      // SDM DPPS / DPPD, as the hardware evaluates the sum: per 128-bit lane,
      // products t_j (imm8[7:4] selects, else +0.0); dpps: for element i
      // s_i = t_(i^1) + t_i, then s_i + s_(i^2); dppd: t_0 + t_1 for both;
      // written where imm8[3:0] selects (+0.0 elsewhere). The operand order
      // only shows in which NaN propagates (the fp vectors pin it). An
      // unmasked exception ends the instruction at the step that raised it,
      // the flags of the steps before it already in MXCSR (native vectors).
      const u32 per = 16 / ew, nl = vl / 16;
      u64 t[8], s1[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      auto trapped = [&]() {
        if (v.fl & ~v.masks & 63) return true;
        F.mxcsr |= v.fl;  // the step completed: its flags stand
        v.fl = 0;
        return false;
      };
      for (u32 j = 0; j < per * nl; j++)
        t[j] = ((imm >> (4 + j % per)) & 1) ? f_arith(v, FOP_MUL, yel(a, j, ew), yel(b, j, ew), w) : 0;
      if (!trapped())
        for (u32 j = 0; j < per * nl; j++)
          s1[j] = per == 4 ? f_arith(v, FOP_ADD, t[j ^ 1], t[j], w) : f_arith(v, FOP_ADD, t[j & ~1u], t[j | 1], w);
      if (!trapped() && per == 4)
        for (u32 j = 0; j < per * nl; j++) t[j] = f_arith(v, FOP_ADD, s1[j], s1[j ^ 2], w);
      else
        for (u32 j = 0; j < per * nl; j++) t[j] = s1[j];
      for (u32 j = 0; j < per * nl; j++) yset(r, j, ew, ((imm >> (j % per)) & 1) ? t[j] : 0);
      break;
    }
    default: {  // FK_BLENDV: the mask is xmm0 (legacy) or the register in imm8[7:4]
      const Y256 m = vex ? ymm_get(P, L, imm >> 4) : Y256{xmm_get(P, L, 0), X128{0, 0}};
      for (u32 i = 0; i < ne; i++) yset(r, i, ew, (yel(m, i, ew) >> (8 * ew - 1)) ? yel(b, i, ew) : yel(a, i, ew));
      break;
    }
  }
  // ---- exceptions (SDM vol. 1 11.5.2), then the results
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
  if (k == FK_MMXCVT && (c != 0x2a || !mem)) mmx_commit(F);  // the x87 -> MMX transition
  if (gpr_out == 2) {
    mmx_put(F, u.reg & 7, gval);
    return X_OK;
  }
  if (gpr_out) {
    RS(L, u.reg, gval);
    return X_OK;
  }
  if (vex) ymm_put(P, L, u.reg, r, keep256);
  else xmm_put(P, L, u.reg, r.l);
  return X_OK;
}

}  // namespace wtfgpu_dev
