// engine_fast.h — the hot-path form of a decoded instruction.
//
// decode() (engine_ops.h) produces a general UOp that the generic exec()
// pipeline interprets field by field. That generality is paid on every step
// (operand-location switches, sizes, prefixes), so at uop-cache fill time the
// UOp is also digested into an FOp: one `kind` per common operand form, with
// registers, sizes and the effective-address recipe resolved. fast_exec()
// then runs a short body per kind. Anything outside those forms (segment or
// address-size overrides, high-byte registers, string ops, mul/div, system
// instructions, ...) keeps kind FK_GENERIC and goes through exec() unchanged,
// so the fast path only ever re-states semantics exec() already has (the same
// helpers: alu2, shift_op, cond, vread/vwrite).
#pragma once
#include "engine_ops.h"

namespace wtfgpu_dev {

enum : u32 {
  FK_GENERIC = 0,
  FK_NOP,
  FK_MOV_RR,    // ra <- rb
  FK_MOV_RI,    // ra <- imm
  FK_LOAD,      // ra <- [ea]
  FK_STORE,     // [ea] <- rb
  FK_STORE_I,   // [ea] <- imm
  FK_ALU_RR,    // ra <- ra op rb (sub = alu op; 7 = cmp writes nothing)
  FK_ALU_RI,    // ra <- ra op imm
  FK_ALU_RM,    // ra <- ra op [ea]
  FK_ALU_MR,    // [ea] <- [ea] op rb
  FK_ALU_MI,    // [ea] <- [ea] op imm
  FK_TEST_RR,   // flags of ra & rb
  FK_TEST_RI,   // flags of ra & imm
  FK_LEA,       // ra <- ea
  FK_INCDEC_R,  // ra <- ra +/- 1 (sub 0 inc, 1 dec), CF kept
  FK_JCC,       // rip <- nrip + imm if cond(sub)
  FK_JMP,       // rip <- nrip + imm
  FK_CALL,      // push nrip; rip <- nrip + imm
  FK_RET,       // rip <- pop; rsp += imm
  FK_PUSH_R,    // push rb
  FK_POP_R,     // ra <- pop
  FK_MOVX_RR,   // ra <- zext/sext(rb, szb) (sub 1 = sign)
  FK_MOVX_RM,   // ra <- zext/sext([ea], szb)
  FK_SHIFT_RI,  // ra <- shift(sub, ra, imm)
  FK_CMOV_RR,   // ra <- cond(sub) ? rb : ra
  FK_SETCC_R,   // ra.b <- cond(sub)
};

constexpr u32 NOREG = 16;

struct FOp {
  u32 kind, len, sz, szb;
  u32 ra, rb, sub, base;
  u32 index, scale, riprel, pad;
  u64 disp, imm;
};

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

__device__ __forceinline__ void digest(const UOp &u, FOp &f) {
  f.kind = FK_GENERIC;
  f.len = u.len;
  f.sz = u.asz;
  f.szb = u.bsz;
  f.sub = u.sub;
  f.base = u.base >= 0 ? (u32)u.base : NOREG;
  f.index = u.index >= 0 ? (u32)u.index : NOREG;
  f.scale = u.scale;
  f.riprel = u.riprel;
  f.pad = 0;
  f.disp = u.disp;
  f.imm = u.imm;
  f.ra = loc_regno(u, u.asrc);
  f.rb = loc_regno(u, u.bsrc);
  if (!u.supported || u.seg || u.p67 || u.rep) return;
  // high-byte registers (ah/ch/dh/bh) stay on the generic path
  const bool hb = !u.rex && ((u.asz == 1 && ((u.asrc == L_GREG && u.reg >= 4 && u.reg < 8) ||
                                             (u.asrc == L_RM && !u.is_mem && u.rm >= 4 && u.rm < 8) ||
                                             (u.asrc == L_OPREG && u.opreg >= 4 && u.opreg < 8))) ||
                             (u.bsz == 1 && ((u.bsrc == L_GREG && u.reg >= 4 && u.reg < 8) ||
                                             (u.bsrc == L_RM && !u.is_mem && u.rm >= 4 && u.rm < 8))));
  if (hb) return;
  const bool amem = u.asrc == L_RM && u.is_mem;
  const bool bmem = u.bsrc == L_RM && u.is_mem;
  const bool areg = f.ra != NOREG;
  const bool breg = f.rb != NOREG;
  const bool bimm = u.bsrc == L_IMM;
  switch (u.op) {
    case O_NOP: f.kind = FK_NOP; break;
    case O_MOV:
      if (areg && breg) f.kind = FK_MOV_RR;
      else if (areg && bimm) f.kind = FK_MOV_RI;
      else if (areg && bmem) f.kind = FK_LOAD;
      else if (amem && breg) f.kind = FK_STORE;
      else if (amem && bimm) f.kind = FK_STORE_I;
      break;
    case O_ALU:
      if (areg && breg) f.kind = FK_ALU_RR;
      else if (areg && bimm) f.kind = FK_ALU_RI;
      else if (areg && bmem) f.kind = FK_ALU_RM;
      else if (amem && breg) f.kind = FK_ALU_MR;
      else if (amem && bimm) f.kind = FK_ALU_MI;
      break;
    case O_TEST:
      if (areg && breg) f.kind = FK_TEST_RR;
      else if (areg && bimm) f.kind = FK_TEST_RI;
      break;
    case O_LEA:
      if (areg && u.is_mem) f.kind = FK_LEA;
      break;
    case O_INCDEC:
      if (areg) f.kind = FK_INCDEC_R;
      break;
    case O_JCC: f.kind = FK_JCC; break;
    case O_JMP:
      if (bimm) f.kind = FK_JMP;
      break;
    case O_CALL:
      if (bimm) f.kind = FK_CALL;
      break;
    case O_RET: f.kind = FK_RET; break;
    case O_PUSH:
      if (breg && u.asz == 8) f.kind = FK_PUSH_R;
      break;
    case O_POP:
      if (areg && u.asrc == L_OPREG && u.bsz == 8) f.kind = FK_POP_R;
      break;
    case O_MOVZX:
    case O_MOVSX:
      f.sub = u.op == O_MOVSX ? 1 : 0;
      if (areg && breg) f.kind = FK_MOVX_RR;
      else if (areg && bmem) f.kind = FK_MOVX_RM;
      break;
    case O_SHIFT:
      if (areg && (bimm || u.bsrc == L_ONE)) {
        f.kind = FK_SHIFT_RI;
        if (u.bsrc == L_ONE) f.imm = 1;
      }
      break;
    case O_CMOV:
      if (areg && breg) f.kind = FK_CMOV_RR;
      break;
    case O_SETCC:
      if (areg) f.kind = FK_SETCC_R;
      break;
    default: break;
  }
}

// ---------------------------------------------------------------- execute (per lane)
// Register write without high-byte forms (digest excludes them): setr().
__device__ __forceinline__ void wr(Lane &L, u32 r, u32 sz, u64 v) {
  if (sz == 8) RS(L, r, v);
  else if (sz == 4) RS(L, r, v & 0xffffffffull);
  else if (sz == 2) RS(L, r, (R(L, r) & ~0xffffull) | (v & 0xffff));
  else RS(L, r, (R(L, r) & ~0xffull) | (v & 0xff));
}

__device__ __forceinline__ u64 fea(const Lane &L, const FOp &f, u64 nrip) {
  u64 ea = f.disp + (f.riprel ? nrip : 0);
  if (f.base != NOREG) ea += R(L, f.base);
  if (f.index != NOREG) ea += R(L, f.index) << f.scale;
  return ea;
}

// One attempt; same contract as exec(): X_OK with `next`, or X_FAULT with
// L.miss set (retry after service_miss) / L.status set (architectural fault).
// Nothing is committed before every memory access has succeeded.
__device__ __forceinline__ int fast_exec(Lane &L, const FOp &f, u64 nrip, u64 &next) {
  next = nrip;
  const u32 sz = f.sz;
  const u64 mk = szmask(sz);
  u64 fl = L.rflags, fo;
  switch (f.kind) {
    case FK_NOP: return X_OK;
    case FK_MOV_RR: wr(L, f.ra, sz, R(L, f.rb)); return X_OK;
    case FK_MOV_RI: wr(L, f.ra, sz, f.imm); return X_OK;
    case FK_LOAD: {
      u64 v;
      if (!vread(L, fea(L, f, nrip), sz, v)) return X_FAULT;
      wr(L, f.ra, sz, v);
      return X_OK;
    }
    case FK_STORE: return vwrite(L, fea(L, f, nrip), sz, R(L, f.rb) & mk) ? X_OK : X_FAULT;
    case FK_STORE_I: return vwrite(L, fea(L, f, nrip), sz, f.imm & mk) ? X_OK : X_FAULT;
    case FK_ALU_RR:
    case FK_ALU_RI:
    case FK_ALU_RM: {
      u64 b;
      if (f.kind == FK_ALU_RM) {
        if (!vread(L, fea(L, f, nrip), sz, b)) return X_FAULT;
      } else {
        b = f.kind == FK_ALU_RR ? R(L, f.rb) : f.imm;
      }
      const u64 res = alu2(f.sub, R(L, f.ra), b, sz, fl, fo);
      if (f.sub != 7) wr(L, f.ra, sz, res);
      L.rflags = with_status(fl, fo);
      return X_OK;
    }
    case FK_ALU_MR:
    case FK_ALU_MI: {
      const u64 ea = fea(L, f, nrip);
      u64 a;
      if (!vread(L, ea, sz, a, f.sub == 7 ? ACC_R : ACC_W)) return X_FAULT;
      const u64 res = alu2(f.sub, a, f.kind == FK_ALU_MR ? R(L, f.rb) : f.imm, sz, fl, fo);
      if (f.sub != 7 && !vwrite(L, ea, sz, res)) return X_FAULT;
      L.rflags = with_status(fl, fo);
      return X_OK;
    }
    case FK_TEST_RR:
    case FK_TEST_RI:
      alu2(4, R(L, f.ra), f.kind == FK_TEST_RR ? R(L, f.rb) : f.imm, sz, fl, fo);
      L.rflags = with_status(fl, fo);
      return X_OK;
    case FK_LEA: wr(L, f.ra, sz, fea(L, f, nrip)); return X_OK;
    case FK_INCDEC_R: {
      const u64 res = alu2(f.sub ? 5 : 0, R(L, f.ra), 1, sz, fl, fo);
      wr(L, f.ra, sz, res);
      L.rflags = (fl & ~(F_STATUS & ~F_CF)) | (fo & ~F_CF);
      return X_OK;
    }
    case FK_JCC:
      if (cond(fl, f.sub)) next = nrip + f.imm;
      return X_OK;
    case FK_JMP: next = nrip + f.imm; return X_OK;
    case FK_CALL: {
      const u64 rsp = R(L, 4);
      if (!vwrite(L, rsp - 8, 8, nrip)) return X_FAULT;
      RS(L, 4, rsp - 8);
      next = nrip + f.imm;
      return X_OK;
    }
    case FK_RET: {
      const u64 rsp = R(L, 4);
      u64 t;
      if (!vread(L, rsp, 8, t)) return X_FAULT;
      RS(L, 4, rsp + 8 + f.imm);
      next = t;
      return X_OK;
    }
    case FK_PUSH_R: {
      const u64 rsp = R(L, 4);
      if (!vwrite(L, rsp - 8, 8, R(L, f.rb))) return X_FAULT;
      RS(L, 4, rsp - 8);
      return X_OK;
    }
    case FK_POP_R: {
      const u64 rsp = R(L, 4);
      u64 t;
      if (!vread(L, rsp, 8, t)) return X_FAULT;
      RS(L, 4, rsp + 8);  // rsp first: pop rsp loads the popped value (exec() commit order)
      RS(L, f.ra, t);
      return X_OK;
    }
    case FK_MOVX_RR:
    case FK_MOVX_RM: {
      u64 b;
      if (f.kind == FK_MOVX_RM) {
        if (!vread(L, fea(L, f, nrip), f.szb, b)) return X_FAULT;
      } else {
        b = R(L, f.rb);
      }
      b &= szmask(f.szb);
      wr(L, f.ra, sz, f.sub ? sext(b, f.szb) : b);
      return X_OK;
    }
    case FK_SHIFT_RI: {
      const u64 res = shift_op(f.sub, R(L, f.ra), (u32)f.imm, sz, fl);
      wr(L, f.ra, sz, res);
      L.rflags = fl;
      return X_OK;
    }
    case FK_CMOV_RR: {
      const bool t = cond(fl, f.sub);
      if (t) wr(L, f.ra, sz, R(L, f.rb));
      else if (sz == 4) wr(L, f.ra, 4, R(L, f.ra));
      return X_OK;
    }
    case FK_SETCC_R: wr(L, f.ra, 1, cond(fl, f.sub) ? 1 : 0); return X_OK;
    default: return X_UNIMPL;
  }
}

}  // namespace wtfgpu_dev
