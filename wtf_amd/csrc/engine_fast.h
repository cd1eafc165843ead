// engine_fast.h — the hot-path form of a decoded instruction.
//
// decode() (engine_ops.h) produces a general UOp that the generic exec()
// pipeline interprets field by field. That generality is paid on every step
// (operand-location switches, sizes, prefixes), so at uop-cache fill time the
// UOp is also digested into an FOp: a compute op plus a set of pipeline flags
// (which operands are registers / immediates / memory, where the address comes
// from, what is written back), with registers, sizes and the effective-address
// recipe resolved and packed into 8 dwords. fast_exec() is then one short
// pipeline with a single memory-read and a single memory-write site, so the
// call-free fast loop of k_run stays small.
//
// Anything outside the common forms (segment or address-size overrides,
// high-byte registers, string ops, mul/div, system instructions, ...) keeps op
// FO_GENERIC and runs through exec() in the slow step; so does any fast
// attempt that meets something the fast path does not handle (TLB miss, first
// write to a page, write to a page-table page, page-crossing access,
// permission fault): it sets L.miss, commits nothing, and the slow step re-runs
// the instruction with exec(). The fast path only re-states semantics exec()
// already has, with the same helpers (alu2, shift_op, cond, szmask, sext).
#pragma once
#include "engine_ops.h"

namespace wtfgpu_dev {

// compute ops
enum : u32 {
  FO_GENERIC = 0,
  FO_NOP,
  FO_MOV,     // res = b
  FO_ALU,     // res = alu2(sub, a, b); sub 7 (cmp) writes nothing
  FO_LEA,     // res = ea
  FO_INCDEC,  // res = a +/- 1, CF kept
  FO_JCC,     // next = nrip + imm if cond(sub)
  FO_JMP,     // next = nrip + imm, or b (FF_BREG)
  FO_CALL,    // res = nrip (pushed), next = nrip + imm, or b (FF_BREG)
  FO_RET,     // next = b (popped)
  FO_MOVX,    // res = zext/sext(b, szb), sub 1 = sign
  FO_SHIFT,   // res = shift_op(sub, a, imm)
  FO_CMOV,    // res = cond(sub) ? b : a
  FO_SETCC,   // res = cond(sub)
  FO_BT,      // bt / bts / btr / btc (sub 4..7) of register a, bit b: CF, res
  FO_UNARY,   // sub 0: res = ~a (not); sub 1: res = 0 - a, flags (neg)
  // SSE / AVX data movement (engine_sse.h semantics), ra = the xmm / ymm
  // register, sz = operand bytes / 8; sub bit 0: aligned form, bit 1: VEX
  // (VEX.128 zeroes bits 255:128), bit 2 (FO_VMOV): the zeroing xor idiom
  FO_VLD,     // ymm[ra] = mem
  FO_VST,     // mem = ymm[ra]
  FO_VMOV,    // ymm[ra] = ymm[rb] (or 0)
  FO_VZU,     // vzeroupper
};
// pipeline flags
enum : u32 {
  FF_AREG = 1,      // a = R(ra)
  FF_BREG = 2,      // b = R(rb) (else b = imm)
  FF_EA = 4,        // address = effective address
  FF_PUSH = 8,      // address = rsp - 8, rsp -= 8 at commit
  FF_POP = 16,      // address = rsp, rsp += 8 + imm at commit (imm only for ret)
  FF_MR_A = 32,     // memory read into a (read-modify-write when FF_MW)
  FF_MR_B = 64,     // memory read into b
  FF_MW = 128,      // memory write of res at the address
  FF_WRA = 256,     // register write of res into ra
  FF_FLAGS = 512,   // rflags updated by the op
};

constexpr u32 NOREG = 16;
constexpr u32 FR_HB = 32;  // register field flag: the high byte (bits 15:8) of register & 3

struct FOp {
  u32 w0;  // op | sub << 8 | sz << 12 | szb << 16 | len << 20 | scale << 26 | riprel << 28 | seg << 29 (1 fs, 2 gs)
  u32 fl;  // FF_*
  u32 w2;  // ra | rb << 8 | base << 16 | index << 24
  u32 pad;
  u64 disp, imm;
};

__device__ __forceinline__ u32 fo_op(const FOp &f) { return f.w0 & 0xff; }
__device__ __forceinline__ u32 fo_sub(const FOp &f) { return (f.w0 >> 8) & 0xf; }
__device__ __forceinline__ u32 fo_sz(const FOp &f) { return (f.w0 >> 12) & 0xf; }
__device__ __forceinline__ u32 fo_szb(const FOp &f) { return (f.w0 >> 16) & 0xf; }
__device__ __forceinline__ u32 fo_len(const FOp &f) { return (f.w0 >> 20) & 0x3f; }
__device__ __forceinline__ u32 fo_scale(const FOp &f) { return (f.w0 >> 26) & 3; }
__device__ __forceinline__ u32 fo_riprel(const FOp &f) { return (f.w0 >> 28) & 1; }
__device__ __forceinline__ u32 fo_seg(const FOp &f) { return (f.w0 >> 29) & 3; }
__device__ __forceinline__ u32 fo_ra(const FOp &f) { return f.w2 & 0xff; }
__device__ __forceinline__ u32 fo_rb(const FOp &f) { return (f.w2 >> 8) & 0xff; }
__device__ __forceinline__ u32 fo_base(const FOp &f) { return (f.w2 >> 16) & 0xff; }
__device__ __forceinline__ u32 fo_index(const FOp &f) { return (f.w2 >> 24) & 0xff; }

// ---------------------------------------------------------------- digest (fill time, uniform)
__device__ __forceinline__ u32 loc_regno(const UOp &u, u32 loc) {
  switch (loc) {
    case L_GREG: return u.reg;
    case L_RM: return u.is_mem ? NOREG : u.rm;
    case L_RAX: return 0;
    case L_OPREG: return u.opreg;
    default: return NOREG;
  }
}

// The moves memcpy / memset loops run (legacy and VEX movdqu / movdqa /
// movups / movaps loads, stores and register moves, the pxor / xorps zeroing
// idiom, vzeroupper); every other O_SSE form stays generic.
__device__ __forceinline__ void digest_sse(const UOp &u, u32 &op, u32 &sub, u32 &ra, u32 &rb, u32 &sz) {
  const u32 x = u.opreg, c = u.sub, pp = u.bsz;
  const bool vex = x & 1;
  if (vex_map(x) != 1 || (x & 0x30000)) return;  // a bad prefix, EVEX (engine_avx512.h)
  const u32 vvvv = vex ? (x >> 4) & 15 : 0;
  sz = vex && ((x >> 1) & 1) ? 4 : 2;
  sub = vex ? 2 : 0;
  if (vex && c == 0x77) {  // vzeroupper (vzeroall stays generic)
    if (sz == 2) op = FO_VZU;
    return;
  }
  const bool load = ((c == 0x6f) && (pp == 1 || pp == 2)) || ((c == 0x10 || c == 0x28) && pp <= 1);
  const bool store = ((c == 0x7f) && (pp == 1 || pp == 2)) || ((c == 0x11 || c == 0x29) && pp <= 1);
  const bool aligned = c == 0x28 || c == 0x29 || (pp == 1 && (c == 0x6f || c == 0x7f));
  if ((load || store) && vvvv == 0) {
    if (aligned) sub |= 1;
    if (!u.is_mem) op = FO_VMOV, ra = load ? u.reg : u.rm, rb = load ? u.rm : u.reg;
    else op = load ? FO_VLD : FO_VST, ra = u.reg;
    return;
  }
  // pxor / xorps / xorpd x, x (VEX: vvvv == r/m): zero
  if (((c == 0xef && pp == 1) || (c == 0x57 && pp <= 1)) && !u.is_mem && (vex ? vvvv : u.reg) == u.rm)
    op = FO_VMOV, sub |= 4, ra = u.reg, rb = u.rm;
}

__device__ __forceinline__ void digest(const UOp &u, FOp &f) {
  u32 op = FO_GENERIC, fl = 0, sub = u.sub;
  const u32 ra = loc_regno(u, u.asrc), rb = loc_regno(u, u.bsrc);
  const bool amem = u.asrc == L_RM && u.is_mem;
  const bool bmem = u.bsrc == L_RM && u.is_mem;
  const bool areg = ra != NOREG, breg = rb != NOREG, bimm = u.bsrc == L_IMM;
  // high-byte registers (ah/ch/dh/bh) stay on the generic path
  // high-byte registers (ah / ch / dh / bh: an 8-bit register 4..7 without
  // REX) are register (r & 3) with bit FR_HB: read shifted down by 8, written
  // merged into bits 15:8 (ops whose a / b / destination go through the
  // pipeline below; the rest stay generic)
  const bool hba = !u.rex && u.asz == 1 && areg && ra >= 4 && ra < 8;
  const bool hbb = !u.rex && u.bsz == 1 && breg && rb >= 4 && rb < 8;
  const bool hb = (hba || hbb) &&
                  !(u.op == O_ALU || u.op == O_TEST || u.op == O_MOV || u.op == O_MOVZX || u.op == O_MOVSX ||
                    u.op == O_INCDEC || u.op == O_NOT || u.op == O_NEG || u.op == O_SETCC || u.op == O_SHIFT);
  u64 imm = u.imm;
  u32 ra_ = ra, rb_ = rb, sz_ = u.asz;
  if (u.op == O_SSE && u.supported && !u.seg && !u.p67) {
    digest_sse(u, op, sub, ra_, rb_, sz_);
  } else if (u.supported && !u.p67 && !u.rep && !hb) {
    switch (u.op) {
      case O_NOP: op = FO_NOP; break;
      case O_MOV:
        if (areg && breg) op = FO_MOV, fl = FF_BREG | FF_WRA;
        else if (areg && bimm) op = FO_MOV, fl = FF_WRA;
        else if (areg && bmem) op = FO_MOV, fl = FF_EA | FF_MR_B | FF_WRA;
        else if (amem && breg) op = FO_MOV, fl = FF_BREG | FF_EA | FF_MW;
        else if (amem && bimm) op = FO_MOV, fl = FF_EA | FF_MW;
        break;
      case O_ALU: {
        const u32 w = u.sub != 7;  // cmp reads its destination, never writes it
        if (areg && breg) op = FO_ALU, fl = FF_AREG | FF_BREG | (w ? FF_WRA : 0);
        else if (areg && bimm) op = FO_ALU, fl = FF_AREG | (w ? FF_WRA : 0);
        else if (areg && bmem) op = FO_ALU, fl = FF_AREG | FF_EA | FF_MR_B | (w ? FF_WRA : 0);
        else if (amem && breg) op = FO_ALU, fl = FF_BREG | FF_EA | FF_MR_A | (w ? FF_MW : 0);
        else if (amem && bimm) op = FO_ALU, fl = FF_EA | FF_MR_A | (w ? FF_MW : 0);
        if (op) fl |= FF_FLAGS;
        break;
      }
      case O_TEST:
        sub = 4;
        if (areg && breg) op = FO_ALU, fl = FF_AREG | FF_BREG | FF_FLAGS;
        else if (areg && bimm) op = FO_ALU, fl = FF_AREG | FF_FLAGS;
        else if (amem && breg) op = FO_ALU, fl = FF_BREG | FF_EA | FF_MR_A | FF_FLAGS;
        else if (amem && bimm) op = FO_ALU, fl = FF_EA | FF_MR_A | FF_FLAGS;
        break;
      case O_NOT:
      case O_NEG:
        sub = u.op == O_NEG ? 1 : 0;
        if (areg) op = FO_UNARY, fl = FF_AREG | FF_WRA;
        else if (amem) op = FO_UNARY, fl = FF_EA | FF_MR_A | FF_MW;
        if (op && u.op == O_NEG) fl |= FF_FLAGS;
        break;
      case O_LEA:
        if (areg && u.is_mem) op = FO_LEA, fl = FF_EA | FF_WRA;
        break;
      case O_INCDEC:
        if (areg) op = FO_INCDEC, fl = FF_AREG | FF_WRA | FF_FLAGS;
        break;
      case O_JCC: op = FO_JCC; break;
      case O_JMP:  // relative, or a 64-bit register (the memory forms stay generic)
        if (bimm) op = FO_JMP;
        else if (breg && u.bsz == 8) op = FO_JMP, fl = FF_BREG;
        break;
      case O_CALL:
        if (bimm) op = FO_CALL, fl = FF_PUSH | FF_MW;
        else if (breg && u.bsz == 8) op = FO_CALL, fl = FF_BREG | FF_PUSH | FF_MW;
        else if (bmem && u.bsz == 8) op = FO_CALL, fl = FF_EA | FF_MR_B | FF_PUSH | FF_MW;  // call [mem]
        break;
      case O_RET: op = FO_RET, fl = FF_POP | FF_MR_B; break;
      case O_PUSH:
        if (breg && u.asz == 8) op = FO_MOV, fl = FF_BREG | FF_PUSH | FF_MW;
        break;
      case O_POP:
        if (areg && u.asrc == L_OPREG && u.bsz == 8) op = FO_MOV, fl = FF_POP | FF_MR_B | FF_WRA, imm = 0;
        break;
      case O_MOVZX:
      case O_MOVSX:
        sub = u.op == O_MOVSX ? 1 : 0;
        if (areg && breg) op = FO_MOVX, fl = FF_BREG | FF_WRA;
        else if (areg && bmem) op = FO_MOVX, fl = FF_EA | FF_MR_B | FF_WRA;
        break;
      case O_SHIFT:
        if (areg && (bimm || u.bsrc == L_ONE)) {
          op = FO_SHIFT, fl = FF_AREG | FF_WRA | FF_FLAGS;
          if (u.bsrc == L_ONE) imm = 1;
        } else if (areg && u.bsrc == L_CL) {  // the count in cl (shift_op masks it)
          op = FO_SHIFT, fl = FF_AREG | FF_BREG | FF_WRA | FF_FLAGS, rb_ = 1;
        }
        break;
      case O_BT:  // register forms only (a memory bit string reaches past the operand)
        if (areg && (breg || bimm) && u.sub >= 4)
          op = FO_BT, fl = FF_AREG | (breg ? FF_BREG : 0) | (u.sub != 4 ? FF_WRA : 0) | FF_FLAGS;
        break;
      case O_CMOV:
        if (areg && breg) op = FO_CMOV, fl = FF_AREG | FF_BREG | FF_WRA;
        break;
      case O_SETCC:
        if (areg) op = FO_SETCC, fl = FF_WRA;
        break;
      default: break;
    }
    // an fs / gs override only matters to a memory operand's address; any
    // other fast form with one stays generic
    // (lea computes the offset alone: generic too)
    if (u.seg && (!(fl & FF_EA) || op == FO_LEA)) op = FO_GENERIC;
  }
  if (hba) ra_ = (ra - 4) | FR_HB;
  if (hbb) rb_ = (rb - 4) | FR_HB;
  const u32 base = u.base >= 0 ? (u32)u.base : NOREG, index = u.index >= 0 ? (u32)u.index : NOREG;
  const u32 fseg = u.seg == 4 ? 1 : u.seg == 5 ? 2 : 0;
  f.w0 = op | (sub & 0xf) << 8 | (sz_ & 0xf) << 12 | (u.bsz & 0xf) << 16 | (u.len & 0x3f) << 20 |
         (u.scale & 3) << 26 | (u.riprel & 1) << 28 | fseg << 29;
  f.fl = fl;
  f.w2 = (ra_ & 0xff) | (rb_ & 0xff) << 8 | (base & 0xff) << 16 | (index & 0xff) << 24;
  f.pad = 0;
  f.disp = u.disp;
  f.imm = imm;
}

// ---------------------------------------------------------------- execute (per lane)
// Register write without high-byte forms (digest excludes them): setr().
__device__ __forceinline__ void wr(Lane &L, u32 r, u32 sz, u64 v) {
  if (sz == 8) RS(L, r, v);
  else if (sz == 4) RS(L, r, v & 0xffffffffull);
  else if (sz == 2) RS(L, r, (R(L, r) & ~0xffffull) | (v & 0xffff));
  else RS(L, r, (R(L, r) & ~0xffull) | (v & 0xff));
}

// Fast translation: TLB hit with the permission already granted, and for a
// write a private (copy-on-write done) page that is not a page-table page.
// A TLB miss or a first write to a shared page -> L.miss = 2 with the address:
// k_run serves it in registers (fast_fill) and retries. Everything else ->
// L.miss = 1, the slow step takes over.
#ifndef WTFGPU_FAST_NB
#define WTFGPU_FAST_NB 1  // branch-free translation and unconditional loads in the fast path
#endif
#if WTFGPU_FAST_NB
// The same decisions as selects, without per-lane branches (each early return
// was an exec-mask region): the first failure of the attempt sets L.miss.
__device__ __forceinline__ u8 *fxlate(Lane &L, u64 va, u32 sz, int acc) {
  u64 td;
  const bool w = acc == ACC_W;
  const bool cross = (va & 0xfff) + sz > 4096;
  const bool hit = tlb_get(L, va >> 12, td);
  const bool pok = perm_ok(L, td, acc);
  const u64 kind = td & (T_PRIV | T_PT);
  const bool m2 = !cross && (!hit || (pok && w && kind == 0));
  const bool ok = !cross && hit && pok && (!w || kind == T_PRIV);
  const bool first = !ok && L.miss == 0;
  L.miss = first ? (m2 ? 2u : 1u) : L.miss;
  L.miss_va = first && m2 ? va : L.miss_va;
  L.miss_acc = first && m2 ? (u32)acc : L.miss_acc;
  return ok ? (u8 *)(uintptr_t)(td & ~0xfffull) + (va & 0xfff) : nullptr;
}
// sz bytes at p, read as the two aligned words around it, both loads issued
// whatever the alignment (the second stays in p's page: at a page's last word
// it re-reads the first, and is then unused); p may be the safe zero page.
__device__ __forceinline__ u64 load_le2(const u8 *p, u32 sz) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)7;
  const u32 off = (u32)((uintptr_t)p & 7);
  const u64 lo = *(const u64 *)a;
  const u64 hi = *(const u64 *)((a & 0xff8) != 0xff8 ? a + 8 : a);
  const u64 v = off ? (lo >> (8 * off)) | (hi << (64 - 8 * off)) : lo;
  return v & szmask(sz);
}
#else
__device__ __forceinline__ u8 *fxlate(Lane &L, u64 va, u32 sz, int acc) {
  u64 td;
  const bool w = acc == ACC_W;
  if ((va & 0xfff) + sz > 4096) {
    L.miss = 1;
    return nullptr;
  }
  const bool hit = tlb_get(L, va >> 12, td);
  if (!hit || (perm_ok(L, td, acc) && w && (td & (T_PRIV | T_PT)) == 0)) {
    L.miss = 2;
    L.miss_va = va;
    L.miss_acc = (u32)acc;
    return nullptr;
  }
  if (!perm_ok(L, td, acc) || (w && ((td & (T_PRIV | T_PT)) != T_PRIV))) {
    L.miss = 1;
    return nullptr;
  }
  return (u8 *)(uintptr_t)(td & ~0xfffull) + (va & 0xfff);
}
#endif

// 16 / 32 bytes at p (inside one page): aligned words, funnel-shifted when p
// is not 8-byte aligned (the word past the operand is read only then, and it
// lies in the same page).
__device__ __forceinline__ void vload(const u8 *p, u32 k, u64 *v) {
  const u64 *w = (const u64 *)((uintptr_t)p & ~(uintptr_t)7);
  const u32 sh = 8 * (u32)((uintptr_t)p & 7);
  if (!sh) {
    for (u32 i = 0; i < k; i++) v[i] = w[i];
    return;
  }
  u64 prev = w[0];
  for (u32 i = 0; i < k; i++) {
    const u64 nx = w[i + 1];
    v[i] = (prev >> sh) | (nx << (64 - sh));
    prev = nx;
  }
}
// The store side: whole words in the middle, the two partial end words merged
// (the page is the lane's own overlay copy, no other lane writes it).
__device__ __forceinline__ void vstore(u8 *p, u32 k, const u64 *v) {
  u64 *w = (u64 *)((uintptr_t)p & ~(uintptr_t)7);
  const u32 sh = 8 * (u32)((uintptr_t)p & 7);
  if (!sh) {
    for (u32 i = 0; i < k; i++) w[i] = v[i];
    return;
  }
  const u64 keep = (1ull << sh) - 1;
  const u64 first = w[0], last = w[k];
  w[0] = (first & keep) | (v[0] << sh);
  for (u32 i = 1; i < k; i++) w[i] = (v[i - 1] >> (64 - sh)) | (v[i] << sh);
  w[k] = (last & ~keep) | (v[k - 1] >> (64 - sh));
}

// The FO_V* ops. Anything the generic path would check or fault on (SSE / AVX
// state off in cr0 / cr4 / xcr0, a misaligned aligned form, a TLB miss, a first
// write, a page-crossing operand) leaves through L.miss to exec().
__device__ __forceinline__ int fast_vec(wtfgpu_regs_t *full, Lane &L, const FOp &f, u64 nrip) {
  const u32 op = fo_op(f), sub = fo_sub(f), k = fo_sz(f), n = 8 * k;
  if (!((L.simd >> ((sub >> 1) & 1)) & 1)) {
    L.miss = 1;
    return X_FAULT;
  }
  wtfgpu_regs_t &F = full[L.lane];
  if (op == FO_VZU) {
    for (u32 i = 0; i < 16; i++) F.ymmh[i][0] = F.ymmh[i][1] = 0;
    if (L.simd & 4)
      for (u32 i = 0; i < 16; i++) F.zmmh[i][0] = F.zmmh[i][1] = F.zmmh[i][2] = F.zmmh[i][3] = 0;
    return X_OK;
  }
  const u32 ra = fo_ra(f) & 15;
  u64 v[4] = {0, 0, 0, 0};
  if (op == FO_VMOV) {
    const u32 rb = fo_rb(f) & 15;
    if (!(sub & 4)) v[0] = F.xmm[rb][0], v[1] = F.xmm[rb][1];
    if (!(sub & 4) && n == 32) v[2] = F.ymmh[rb][0], v[3] = F.ymmh[rb][1];
  } else {
    u64 addr = f.disp + (fo_riprel(f) ? nrip : 0);
    if (fo_base(f) != NOREG) addr += R(L, fo_base(f));
    if (fo_index(f) != NOREG) addr += R(L, fo_index(f)) << fo_scale(f);
    if ((sub & 1) && (addr & (n - 1))) {
      L.miss = 1;
      return X_FAULT;
    }
    u8 *mp = fxlate(L, addr, n, op == FO_VST ? ACC_W : ACC_R);
    if (!mp) return X_FAULT;
    L.pend += n;
    if (op == FO_VST) {
      v[0] = F.xmm[ra][0], v[1] = F.xmm[ra][1], v[2] = F.ymmh[ra][0], v[3] = F.ymmh[ra][1];
      vstore(mp, k, v);
      return X_OK;
    }
    vload(mp, k, v);
  }
  F.xmm[ra][0] = v[0];
  F.xmm[ra][1] = v[1];
  if (n == 32 || (sub & 2)) {  // VEX.128 zeroes the upper half, legacy SSE keeps it
    F.ymmh[ra][0] = v[2];
    F.ymmh[ra][1] = v[3];
  }
  if ((sub & 2) && (L.simd & 4)) F.zmmh[ra][0] = F.zmmh[ra][1] = F.zmmh[ra][2] = F.zmmh[ra][3] = 0;  // MAXVL 512
  return X_OK;
}

// The Dev arrays the fast path reads, taken once by the caller (k_run keeps
// them in registers rather than reloading them from the kernel argument's
// scratch copy each step).
struct FastMem {
  wtfgpu_regs_t *full;
  const Dev *P;    // the rest (fs / gs bases: segment-override operands only) read when needed
  const u8 *safe;  // the pool's zero page: what a lane whose access missed reads instead
};
__device__ __forceinline__ FastMem fast_mem(const Dev &P) { return FastMem{P.full, &P, P.pool}; }

// One exit and one commit on every path: a failed attempt (ok = false, L.miss
// set) writes the unchanged values back. The guest registers are an array the
// compiler keeps in VGPRs and indexes with s_set_gpr_idx; a register write
// under a uniform branch, or an early return that skips the writes, makes that
// array a phi of copies (~80 v_mov per wave-step). Here rsp and the
// destination are written exactly once each, unconditionally.
// kRegOnly: the caller knows the form touches no memory (no FF_PUSH / FF_POP
// / FF_MR_* / FF_MW, not a vector move): the memory stages compile out and
// the attempt cannot miss.
template <bool kRegOnly = false>
__device__ __forceinline__ int fast_exec(const FastMem &M, Lane &L, const FOp &f, u64 nrip, u64 &next) {
  next = nrip;
  const u32 F = f.fl, op = fo_op(f), sub = fo_sub(f), sz = fo_sz(f);
  const u64 rsp = R(L, 4);
  u64 res = 0, fl = L.rflags, fo;
  bool ok = true;
  if (!kRegOnly && op >= FO_VLD) {
    ok = fast_vec(M.full, L, f, nrip) == X_OK;  // xmm / ymm state only (memory), no GPR
  } else {
    u64 a = (F & FF_AREG) ? R(L, fo_ra(f)) >> ((fo_ra(f) & FR_HB) >> 2) : 0;
    u64 b = (F & FF_BREG) ? R(L, fo_rb(f)) >> ((fo_rb(f) & FR_HB) >> 2) : f.imm;
    u64 addr = 0;
    if (F & FF_EA) {
      addr = f.disp + (fo_riprel(f) ? nrip : 0);
      if (fo_base(f) != NOREG) addr += R(L, fo_base(f));
      if (fo_index(f) != NOREG) addr += R(L, fo_index(f)) << fo_scale(f);
      if (fo_seg(f)) addr += (fo_seg(f) == 1 ? M.P->fs_base : M.P->gs_base)[L.lane];
    } else if (F & FF_PUSH) {
      addr = rsp - 8;
    } else {
      addr = rsp;
    }
    // ---- the memory read
    u8 *mp = nullptr;
    // (a write to the read's own address makes it a read-modify-write; call
    // [mem] reads its target and writes the stack)
    const bool rmw = (F & FF_MW) && (F & (FF_MR_A | FF_MR_B)) && !(F & FF_PUSH);
    if (!kRegOnly && (F & (FF_MR_A | FF_MR_B))) {
      const u32 rsz = (F & (FF_PUSH | FF_POP)) ? 8 : (op == FO_MOVX ? fo_szb(f) : sz);
      mp = fxlate(L, addr, rsz, rmw ? ACC_W : ACC_R);
#if WTFGPU_FAST_NB
      const u64 v = load_le2(mp ? mp : M.safe, rsz);  // a missed lane reads the zero page, unused
      L.pend += mp ? rsz : 0;
      if (F & FF_MR_A) a = mp ? v : a;
      else b = mp ? v : b;
      ok = mp != nullptr;
#else
      if (mp) {
        const u64 v = load_le(mp, rsz);
        L.pend += rsz;
        if (F & FF_MR_A) a = v;
        else b = v;
      } else {
        ok = false;
      }
#endif
    }
    // ---- compute (pure)
    switch (op) {
      case FO_MOV: res = b; break;
      case FO_ALU:
        res = alu2(sub, a, b, sz, fl, fo);
        fl = with_status(fl, fo);
        break;
      case FO_LEA: res = addr; break;
      case FO_INCDEC:
        res = alu2(sub ? 5 : 0, a, 1, sz, fl, fo);
        fl = (fl & ~(F_STATUS & ~F_CF)) | (fo & ~F_CF);
        break;
      case FO_JCC:
        if (cond(fl, sub)) next = nrip + f.imm;
        break;
      case FO_JMP: next = (F & FF_BREG) ? b : nrip + b; break;
      case FO_CALL:  // indirect: the target in a register or read from memory
        res = nrip;
        next = (F & (FF_BREG | FF_MR_B)) ? b : nrip + b;
        break;
      case FO_UNARY:
        if (sub) {
          res = alu2(5, 0, a, sz, fl, fo);
          fl = with_status(fl, fo);
        } else {
          res = ~a;
        }
        break;
      case FO_RET: next = b; break;
      case FO_MOVX: {
        const u32 szb = fo_szb(f);
        b &= szmask(szb);
        res = sub ? sext(b, szb) : b;
        break;
      }
      case FO_SHIFT: res = shift_op(sub, a, (u32)b, sz, fl); break;  // b: the immediate, or rcx
      case FO_BT: {
        const u64 bitoff = b & (8 * sz - 1);
        res = sub == 5 ? (a | (1ull << bitoff)) : sub == 6 ? (a & ~(1ull << bitoff)) : (a ^ (1ull << bitoff));
        fl = (fl & ~F_CF) | ((a >> bitoff) & 1);
        break;
      }
      case FO_CMOV:
        // a false condition still zero-extends a 32-bit destination
        res = cond(fl, sub) ? b : a;
        break;
      case FO_SETCC: res = cond(fl, sub) ? 1 : 0; break;
      default: break;
    }
    // ---- the memory write
    if (!kRegOnly && ok && (F & FF_MW)) {
      const u32 wsz = (F & FF_PUSH) ? 8 : sz;
      if (!rmw) mp = fxlate(L, (F & FF_PUSH) ? rsp - 8 : addr, wsz, ACC_W);
      if (mp) {
        store_le(mp, wsz, res & szmask(wsz));
        L.pend += wsz;
      } else {
        ok = false;
      }
    }
  }
  // ---- commit (rsp first: pop rsp ends with the popped value)
#if WTFGPU_FAST_WB_ALWAYS
  const u64 nrsp = !ok ? rsp : (F & FF_PUSH) ? rsp - 8 : (F & FF_POP) ? rsp + 8 + (op == FO_RET ? f.imm : 0) : rsp;
  RS(L, 4, nrsp);
  const u32 wi = fo_ra(f) & 15, hs = (fo_ra(f) & FR_HB) >> 2;
  const u64 old = R(L, wi), mk = szmask(sz) << hs;
  // wr(): 8 / 4 bytes replace (4 zero-extends), 2 / 1 merge into the old value
  const u64 nv = (ok && (F & FF_WRA)) ? (sz >= 4 ? (res & mk) : ((old & ~mk) | ((res << hs) & mk))) : old;
  RS(L, wi, nv);
#else
  // (written under the op's uniform flags: ops that write no register skip
  // the indexed read-back and write)
  if (F & (FF_PUSH | FF_POP)) RS(L, 4, !ok ? rsp : (F & FF_PUSH) ? rsp - 8 : rsp + 8 + (op == FO_RET ? f.imm : 0));
  if (F & FF_WRA) {
    const u32 wi = fo_ra(f) & 15, hs = (fo_ra(f) & FR_HB) >> 2;  // hs: 8 for a high-byte register
    const u64 old = R(L, wi), mk = szmask(sz) << hs;
    // wr(): 8 / 4 bytes replace (4 zero-extends), 2 / 1 merge into the old value
    RS(L, wi, ok ? (sz >= 4 ? (res & mk) : ((old & ~mk) | ((res << hs) & mk))) : old);
  }
#endif
  if (ok && (F & FF_FLAGS)) L.rflags = fl;
  return ok ? X_OK : X_FAULT;
}
__device__ __forceinline__ int fast_exec(const Dev &P, Lane &L, const FOp &f, u64 nrip, u64 &next) {
  return fast_exec(fast_mem(P), L, f, nrip, next);
}

}  // namespace wtfgpu_dev
