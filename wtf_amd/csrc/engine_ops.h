// engine_ops.h — decode into a wave-uniform micro-op and execute it per lane.
//
// Every supported instruction is decoded (once per RIP group, scalar work)
// into a UOp: an operation, an A operand (destination / first source), a B
// operand (second source) and their sizes. exec() is then one fixed pipeline:
//   1. register / immediate operands;
//   2. the single memory read (B, or A for read-modify-write);
//   3. a pure compute switch on the operation;
//   4. the single memory write (A);
//   5. commit: registers, flags, rsp, rip.
// Steps 2 and 4 are the only guest-memory call sites, so the kernel stays
// small, and nothing is committed before every access has succeeded: a TLB
// miss / first write abandons the attempt and the kernel re-runs it after
// service_miss (engine_exec.h); a fault leaves no trace (U11). Rep string
// instructions run their own loop and commit per iteration (x86 semantics).
#pragma once
#include "engine_exec.h"

namespace wtfgpu_dev {

enum { X_OK = 0, X_FAULT = 1, X_UNIMPL = 2, X_INT3 = 3, X_HLT = 4, X_CR3 = 5, X_KEEP = 6 };

// operations
enum : u32 {
  O_ALU = 0,  // sub: 0 add,1 or,2 adc,3 sbb,4 and,5 sub,6 xor,7 cmp
  O_TEST, O_MOV, O_MOVZX, O_MOVSX, O_XCHG, O_XADD, O_CMPXCHG, O_INCDEC, O_NOT, O_NEG,
  O_SHIFT, O_SHXD, O_MULDIV, O_IMUL, O_BT, O_BSF, O_BSR, O_TZCNT, O_LZCNT, O_POPCNT,
  O_CMOV, O_SETCC, O_BSWAP, O_CBW, O_CWD, O_LAHF, O_SAHF, O_FLAGOP, O_NOP, O_JCC, O_JMP,
  O_CALL, O_RET, O_PUSH, O_POP, O_PUSHF, O_POPF, O_LEAVE, O_STRING, O_INT3, O_HLT, O_UD,
  O_LEA, O_SYS, O_SSE, O_UNIMPL,
  O_SYS2,  // engine_sys.h: system / far-transfer / I/O / x87-control (sub = opcode | 0x100 for 0f)
  O_LOOP,  // loopne / loope / loop / jrcxz (sub = opcode & 3)
  O_GEXT   // engine_ext.h: BMI1 / BMI2 / ADX / MOVBE / CRC32 (sub = opcode, fields as O_SSE)
};
// operand locations
enum : u32 {
  L_NONE = 0, L_GREG, L_RM, L_RAX, L_OPREG, L_IMM, L_ONE, L_CL, L_PUSH, L_POP, L_MOFFS,
  L_RBPMEM, L_XLAT
};
// size kinds
enum : u32 { Z_B = 0, Z_V, Z_STK, Z_Q, Z_W, Z_D };

struct UOp {
  u32 len, op, sub, asrc, bsrc, asz, bsz;
  u32 aread, awrite, bwrite;
  u32 reg, rm, opreg, is_mem, riprel, p67, rex, rep, seg;  // p67: bit 0 32-bit addresses, bit 1 32-bit code (U29)
  i32 base, index;
  u32 scale;
  u64 disp, imm;
  u32 supported, opbytes;
};
}  // namespace wtfgpu_dev
#include "engine_sse.h"  // the SSE / SSE2 subset: sse_valid (decode), sse_exec (exec)
namespace wtfgpu_dev {

// ---------------------------------------------------------------- registers
__device__ __forceinline__ u64 getr(const Lane &L, u32 rex, u32 r, u32 sz) {
  if (sz == 1) {
    if (!rex && r >= 4 && r < 8) return (R(L, r - 4) >> 8) & 0xff;
    return R(L, r) & 0xff;
  }
  return R(L, r) & szmask(sz);
}
__device__ __forceinline__ void setr(Lane &L, u32 rex, u32 r, u32 sz, u64 v) {
  if (sz == 1) {
    if (!rex && r >= 4 && r < 8) {
      RS(L, r - 4, (R(L, r - 4) & ~0xff00ull) | ((v & 0xff) << 8));
    } else {
      RS(L, r, (R(L, r) & ~0xffull) | (v & 0xff));
    }
  } else if (sz == 2) {
    RS(L, r, (R(L, r) & ~0xffffull) | (v & 0xffff));
  } else if (sz == 4) {
    RS(L, r, v & 0xffffffffull);
  } else {
    RS(L, r, v);
  }
}
}  // namespace wtfgpu_dev
#include "engine_ext.h"  // the extensions beyond SSE4.1 / AVX2 (U45): gext_exec, x42_exec
namespace wtfgpu_dev {

// fs / gs bases are cold: read from lane memory when an override appears
__device__ __forceinline__ u64 segbase(const Dev &P, const Lane &L, u32 seg) {
  return seg == 4 ? P.fs_base[L.lane] : (seg == 5 ? P.gs_base[L.lane] : 0);
}

// ---------------------------------------------------------------- decode tables
// entry: op(6) | asrc(4)<<6 | bsrc(4)<<10 | asz(3)<<14 | bsz(3)<<17 | aread<<20 |
//        awrite<<21 | bwrite<<22 | modrm<<23 | immk(3)<<24 | group(4)<<27
#define E(op, a, b, az, bz, ar, aw, bw, m, ik, grp)                                                        \
  ((u32)(op) | ((u32)(a) << 6) | ((u32)(b) << 10) | ((u32)(az) << 14) | ((u32)(bz) << 17) |             \
   ((u32)(ar) << 20) | ((u32)(aw) << 21) | ((u32)(bw) << 22) | ((u32)(m) << 23) | ((u32)(ik) << 24) | \
   ((u32)(grp) << 27))
#define UN E(O_UNIMPL, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
// invalid in 64-bit mode (push / pop of es cs ss ds, daa das aaa aas, pusha
// popa, the 82 alias of 80, far call / jmp, aam aad salc): #UD
#define UDE E(O_UD, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0)
enum : u32 { K_NONE = 0, K_B, K_W, K_Z, K_V, K_MOFFS, K_D, K_ENTER /* iw ib */ };
enum : u32 { G_NONE = 0, G_1, G_2, G_3, G_4, G_5, G_8F, G_C6, G_BA, G_ALU };

#define ALU4                                                                             \
  E(O_ALU, L_RM, L_GREG, Z_B, Z_B, 1, 1, 0, 1, K_NONE, G_ALU),                            \
      E(O_ALU, L_RM, L_GREG, Z_V, Z_V, 1, 1, 0, 1, K_NONE, G_ALU),                        \
      E(O_ALU, L_GREG, L_RM, Z_B, Z_B, 1, 1, 0, 1, K_NONE, G_ALU),                        \
      E(O_ALU, L_GREG, L_RM, Z_V, Z_V, 1, 1, 0, 1, K_NONE, G_ALU),                        \
      E(O_ALU, L_RAX, L_IMM, Z_B, Z_B, 1, 1, 0, 0, K_B, G_ALU),                           \
      E(O_ALU, L_RAX, L_IMM, Z_V, Z_V, 1, 1, 0, 0, K_Z, G_ALU), UDE, UDE
#define JCC E(O_JCC, 0, L_IMM, 0, Z_Q, 0, 0, 0, 0, K_B, 0)
#define PUSHR E(O_PUSH, L_PUSH, L_OPREG, Z_STK, Z_STK, 0, 1, 0, 0, K_NONE, 0)
#define POPR E(O_POP, L_OPREG, L_POP, Z_STK, Z_STK, 0, 1, 0, 0, K_NONE, 0)
#define XCHGR E(O_XCHG, L_RAX, L_OPREG, Z_V, Z_V, 1, 1, 1, 0, K_NONE, 0)
#define MOVR8 E(O_MOV, L_OPREG, L_IMM, Z_B, Z_B, 0, 1, 0, 0, K_B, 0)
#define MOVRV E(O_MOV, L_OPREG, L_IMM, Z_V, Z_V, 0, 1, 0, 0, K_V, 0)
#define STR(sz) E(O_STRING, 0, 0, sz, sz, 0, 0, 0, 0, K_NONE, 0)
#define FLG E(O_FLAGOP, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0)
// engine_sys.h instructions: asz = the operand size, bsz = 2 with a 66 prefix
#define S2 E(O_SYS2, 0, 0, Z_V, Z_STK, 0, 0, 0, 0, K_NONE, 0)
#define S2M E(O_SYS2, 0, 0, Z_V, Z_STK, 0, 0, 0, 1, K_NONE, 0)
#define S2B E(O_SYS2, 0, 0, Z_V, Z_STK, 0, 0, 0, 0, K_B, 0)
#define LOOPX E(O_LOOP, 0, L_IMM, 0, Z_Q, 0, 0, 0, 0, K_B, 0)

__constant__ u32 kMap1[256] = {
    /*00*/ ALU4, ALU4, ALU4, ALU4, ALU4, ALU4, ALU4, ALU4,
    /*40*/ UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN,
    /*50*/ PUSHR, PUSHR, PUSHR, PUSHR, PUSHR, PUSHR, PUSHR, PUSHR, POPR, POPR, POPR, POPR, POPR, POPR, POPR, POPR,
    /*60*/ UDE, UDE, UN /* EVEX (U45) */, E(O_MOVSX, L_GREG, L_RM, Z_V, Z_D, 0, 1, 0, 1, K_NONE, 0), UN, UN, UN, UN,
    /*68*/ E(O_PUSH, L_PUSH, L_IMM, Z_STK, Z_STK, 0, 1, 0, 0, K_Z, 0),
    E(O_IMUL, L_GREG, L_RM, Z_V, Z_V, 0, 1, 0, 1, K_Z, 0),
    E(O_PUSH, L_PUSH, L_IMM, Z_STK, Z_STK, 0, 1, 0, 0, K_B, 0),
    E(O_IMUL, L_GREG, L_RM, Z_V, Z_V, 0, 1, 0, 1, K_B, 0), STR(Z_B), STR(Z_V), STR(Z_B), STR(Z_V),
    /*70*/ JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC, JCC,
    /*80*/ E(O_ALU, L_RM, L_IMM, Z_B, Z_B, 1, 1, 0, 1, K_B, G_1), E(O_ALU, L_RM, L_IMM, Z_V, Z_V, 1, 1, 0, 1, K_Z, G_1),
    UDE, E(O_ALU, L_RM, L_IMM, Z_V, Z_V, 1, 1, 0, 1, K_B, G_1),
    E(O_TEST, L_RM, L_GREG, Z_B, Z_B, 1, 0, 0, 1, K_NONE, 0), E(O_TEST, L_RM, L_GREG, Z_V, Z_V, 1, 0, 0, 1, K_NONE, 0),
    E(O_XCHG, L_RM, L_GREG, Z_B, Z_B, 1, 1, 1, 1, K_NONE, 0), E(O_XCHG, L_RM, L_GREG, Z_V, Z_V, 1, 1, 1, 1, K_NONE, 0),
    /*88*/ E(O_MOV, L_RM, L_GREG, Z_B, Z_B, 0, 1, 0, 1, K_NONE, 0), E(O_MOV, L_RM, L_GREG, Z_V, Z_V, 0, 1, 0, 1, K_NONE, 0),
    E(O_MOV, L_GREG, L_RM, Z_B, Z_B, 0, 1, 0, 1, K_NONE, 0), E(O_MOV, L_GREG, L_RM, Z_V, Z_V, 0, 1, 0, 1, K_NONE, 0),
    S2M, E(O_LEA, L_GREG, 0, Z_V, Z_V, 0, 1, 0, 1, K_NONE, 0), S2M,
    E(O_POP, L_RM, L_POP, Z_STK, Z_STK, 0, 1, 0, 1, K_NONE, G_8F),
    /*90*/ XCHGR, XCHGR, XCHGR, XCHGR, XCHGR, XCHGR, XCHGR, XCHGR,
    /*98*/ E(O_CBW, 0, 0, Z_V, Z_V, 0, 0, 0, 0, K_NONE, 0), E(O_CWD, 0, 0, Z_V, Z_V, 0, 0, 0, 0, K_NONE, 0), UDE, S2,
    E(O_PUSHF, L_PUSH, 0, Z_STK, Z_STK, 0, 1, 0, 0, K_NONE, 0), E(O_POPF, 0, L_POP, Z_STK, Z_STK, 0, 0, 0, 0, K_NONE, 0),
    E(O_SAHF, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), E(O_LAHF, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0),
    /*a0*/ E(O_MOV, L_RAX, L_MOFFS, Z_B, Z_B, 0, 1, 0, 0, K_MOFFS, 0), E(O_MOV, L_RAX, L_MOFFS, Z_V, Z_V, 0, 1, 0, 0, K_MOFFS, 0),
    E(O_MOV, L_MOFFS, L_RAX, Z_B, Z_B, 0, 1, 0, 0, K_MOFFS, 0), E(O_MOV, L_MOFFS, L_RAX, Z_V, Z_V, 0, 1, 0, 0, K_MOFFS, 0),
    STR(Z_B), STR(Z_V), STR(Z_B), STR(Z_V),
    /*a8*/ E(O_TEST, L_RAX, L_IMM, Z_B, Z_B, 1, 0, 0, 0, K_B, 0), E(O_TEST, L_RAX, L_IMM, Z_V, Z_V, 1, 0, 0, 0, K_Z, 0),
    STR(Z_B), STR(Z_V), STR(Z_B), STR(Z_V), STR(Z_B), STR(Z_V),
    /*b0*/ MOVR8, MOVR8, MOVR8, MOVR8, MOVR8, MOVR8, MOVR8, MOVR8, MOVRV, MOVRV, MOVRV, MOVRV, MOVRV, MOVRV, MOVRV, MOVRV,
    /*c0*/ E(O_SHIFT, L_RM, L_IMM, Z_B, Z_B, 1, 1, 0, 1, K_B, G_2), E(O_SHIFT, L_RM, L_IMM, Z_V, Z_B, 1, 1, 0, 1, K_B, G_2),
    E(O_RET, 0, L_POP, Z_Q, Z_Q, 0, 0, 0, 0, K_W, 0), E(O_RET, 0, L_POP, Z_Q, Z_Q, 0, 0, 0, 0, K_NONE, 0), UN, UN,
    E(O_MOV, L_RM, L_IMM, Z_B, Z_B, 0, 1, 0, 1, K_B, G_C6), E(O_MOV, L_RM, L_IMM, Z_V, Z_V, 0, 1, 0, 1, K_Z, G_C6),
    /*c8*/ E(O_SYS2, 0, 0, Z_V, Z_STK, 0, 0, 0, 0, K_ENTER, 0), E(O_LEAVE, 0, L_RBPMEM, Z_Q, Z_Q, 0, 0, 0, 0, K_NONE, 0),
    E(O_SYS2, 0, 0, Z_V, Z_STK, 0, 0, 0, 0, K_W, 0), S2,
    E(O_INT3, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), S2B, UDE, E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0),
    /*d0*/ E(O_SHIFT, L_RM, L_ONE, Z_B, Z_B, 1, 1, 0, 1, K_NONE, G_2), E(O_SHIFT, L_RM, L_ONE, Z_V, Z_B, 1, 1, 0, 1, K_NONE, G_2),
    E(O_SHIFT, L_RM, L_CL, Z_B, Z_B, 1, 1, 0, 1, K_NONE, G_2), E(O_SHIFT, L_RM, L_CL, Z_V, Z_B, 1, 1, 0, 1, K_NONE, G_2),
    UDE, UDE, UDE, E(O_MOV, L_RAX, L_XLAT, Z_B, Z_B, 0, 1, 0, 0, K_NONE, 0),
    /*d8*/ S2M, S2M, S2M, S2M, S2M, S2M, S2M, S2M,
    /*e0*/ LOOPX, LOOPX, LOOPX, LOOPX, S2B, S2B, S2B, S2B,
    /*e8*/ E(O_CALL, L_PUSH, L_IMM, Z_Q, Z_Q, 0, 1, 0, 0, K_D, 0), E(O_JMP, 0, L_IMM, Z_Q, Z_Q, 0, 0, 0, 0, K_D, 0), UDE,
    E(O_JMP, 0, L_IMM, Z_Q, Z_Q, 0, 0, 0, 0, K_B, 0), S2, S2, S2, S2,
    /*f0*/ UN, S2, UN, UN, E(O_HLT, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), FLG,
    E(O_TEST, L_RM, L_IMM, Z_B, Z_B, 1, 0, 0, 1, K_NONE, G_3), E(O_TEST, L_RM, L_IMM, Z_V, Z_V, 1, 0, 0, 1, K_NONE, G_3),
    /*f8*/ FLG, FLG, S2, S2, FLG, FLG,
    E(O_INCDEC, L_RM, 0, Z_B, Z_B, 1, 1, 0, 1, K_NONE, G_4), E(O_INCDEC, L_RM, 0, Z_V, Z_V, 1, 1, 0, 1, K_NONE, G_5),
};

#define NOPM E(O_NOP, 0, 0, 0, 0, 0, 0, 0, 1, K_NONE, 0)
#define CMOV E(O_CMOV, L_GREG, L_RM, Z_V, Z_V, 1, 1, 0, 1, K_NONE, 0)
#define JCC32 E(O_JCC, 0, L_IMM, 0, Z_Q, 0, 0, 0, 0, K_D, 0)
#define SETCC E(O_SETCC, L_RM, 0, Z_B, Z_B, 0, 1, 0, 1, K_NONE, 0)
#define BSWAP E(O_BSWAP, L_OPREG, 0, Z_V, Z_V, 1, 1, 0, 0, K_NONE, 0)
#define BTRW E(O_BT, L_RM, L_GREG, Z_V, Z_V, 1, 1, 0, 1, K_NONE, 0)
#define SHXD(ik) E(O_SHXD, L_RM, L_GREG, Z_V, Z_V, 1, 1, 0, 1, ik, 0)
#define UN16 UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN, UN
#define SSEM E(O_SSE, 0, 0, 0, 0, 0, 0, 0, 1, K_NONE, 0)
#define SSEI E(O_SSE, 0, 0, 0, 0, 0, 0, 0, 1, K_B, 0)
#define SSE8 SSEM, SSEM, SSEM, SSEM, SSEM, SSEM, SSEM, SSEM
__constant__ u32 kMap2[256] = {
    /*00*/ S2M, E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 1, K_NONE, 0), S2M, S2M, UDE, E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), S2,
    E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), S2, S2, UDE, E(O_UD, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), UDE, NOPM, UDE, UDE,
    /*10*/ SSE8, NOPM, NOPM, NOPM, NOPM, NOPM, NOPM, NOPM, NOPM,
    /*20*/ E(O_SYS, L_RM, 0, Z_Q, Z_Q, 0, 1, 0, 1, K_NONE, 0), S2M, E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 1, K_NONE, 0), S2M, UDE,
    UDE, UDE, UDE, SSEM, SSEM, SSEM, SSEM, SSEM, SSEM, SSEM, SSEM,
    /*30*/ E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0),
    E(O_SYS, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), S2, S2, S2, UDE, UDE, UN, UDE, UN, UDE, UDE, UDE, UDE, UDE,
    /*40*/ CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV, CMOV,
    /*50*/ SSE8, SSE8,
    /*60*/ SSE8, SSE8,
    /*70*/ SSEI, SSEI, SSEI, SSEI, SSEM, SSEM, SSEM, E(O_SSE, 0, 0, 0, 0, 0, 0, 0, 0, K_NONE, 0), SSE8,
    /*80*/ JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32, JCC32,
    /*90*/ SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC, SETCC,
    /*a0*/ S2, S2, S2, E(O_BT, L_RM, L_GREG, Z_V, Z_V, 1, 0, 0, 1, K_NONE, 0), SHXD(K_B), SHXD(K_NONE), UDE, UDE,
    /*a8*/ S2, S2, UDE, BTRW, SHXD(K_B), SHXD(K_NONE), SSEM, E(O_IMUL, L_GREG, L_RM, Z_V, Z_V, 1, 1, 0, 1, K_NONE, 0),
    /*b0*/ E(O_CMPXCHG, L_RM, L_GREG, Z_B, Z_B, 1, 1, 0, 1, K_NONE, 0),
    E(O_CMPXCHG, L_RM, L_GREG, Z_V, Z_V, 1, 1, 0, 1, K_NONE, 0), S2M, BTRW, S2M, S2M,
    E(O_MOVZX, L_GREG, L_RM, Z_V, Z_B, 0, 1, 0, 1, K_NONE, 0), E(O_MOVZX, L_GREG, L_RM, Z_V, Z_W, 0, 1, 0, 1, K_NONE, 0),
    /*b8*/ E(O_POPCNT, L_GREG, L_RM, Z_V, Z_V, 0, 1, 0, 1, K_NONE, 0), UDE,
    E(O_BT, L_RM, L_IMM, Z_V, Z_B, 1, 1, 0, 1, K_B, G_BA), BTRW,
    E(O_BSF, L_GREG, L_RM, Z_V, Z_V, 0, 1, 0, 1, K_NONE, 0), E(O_BSR, L_GREG, L_RM, Z_V, Z_V, 0, 1, 0, 1, K_NONE, 0),
    E(O_MOVSX, L_GREG, L_RM, Z_V, Z_B, 0, 1, 0, 1, K_NONE, 0), E(O_MOVSX, L_GREG, L_RM, Z_V, Z_W, 0, 1, 0, 1, K_NONE, 0),
    /*c0*/ E(O_XADD, L_RM, L_GREG, Z_B, Z_B, 1, 1, 1, 1, K_NONE, 0), E(O_XADD, L_RM, L_GREG, Z_V, Z_V, 1, 1, 1, 1, K_NONE, 0),
    SSEI, SSEM, SSEI, SSEI, SSEI, E(O_SYS, L_RM, 0, Z_V, Z_V, 0, 1, 0, 1, K_NONE, 0),
    BSWAP, BSWAP, BSWAP, BSWAP, BSWAP, BSWAP, BSWAP, BSWAP,
    /*d0*/ SSE8, SSE8,
    /*e0*/ SSE8, SSE8,
    /*f0*/ SSE8, SSE8,
};
constexpr u32 kSseModrm = E(O_SSE, 0, 0, 0, 0, 0, 0, 0, 1, K_NONE, 0);  // 0f 38 / VEX map 2 opcodes
constexpr u32 kSseModrmImm = E(O_SSE, 0, 0, 0, 0, 0, 0, 0, 1, K_B, 0);  // 0f 3a / VEX map 3 opcodes (imm8)
constexpr u32 kUnimpl = UN;
// 32-bit code (U29): 40-4f inc / dec r32, and the one-byte forms 64-bit mode
// leaves #UD that engine_sys.h runs (push / pop es cs ss ds, pusha / popa,
// daa das aaa aas, far call / jmp ptr16:32, into, aam / aad)
constexpr u32 kIncDec32 = E(O_INCDEC, L_OPREG, 0, Z_V, Z_V, 1, 1, 0, 0, K_NONE, 0);
constexpr u32 kSys32 = S2, kSys32B = S2B, kSys32M = S2M;
#undef E
#undef UN
#undef UDE
#undef ALU4
#undef JCC
#undef PUSHR
#undef POPR
#undef XCHGR
#undef MOVR8
#undef MOVRV
#undef STR
#undef FLG
#undef S2
#undef S2M
#undef S2B
#undef LOOPX
#undef NOPM
#undef CMOV
#undef JCC32
#undef SETCC
#undef BSWAP
#undef BTRW
#undef SHXD
#undef UN16
#undef SSEM
#undef SSEI
#undef SSE8

// Instruction bytes as two uniform u64 (SGPR pairs).
struct IBytes {
  u64 lo, hi;
  u32 avail;
};
__device__ __forceinline__ u32 ib_at(const IBytes &b, u32 i) {
  return (u32)((i < 8 ? (b.lo >> (8 * i)) : (b.hi >> (8 * (i - 8)))) & 0xff);
}
__device__ __forceinline__ u64 ib_get(const IBytes &b, u32 pos, u32 n) {
  u64 v = 0;
  for (u32 i = 0; i < n; i++) v |= (u64)ib_at(b, pos + i) << (8 * i);
  return v;
}

__device__ __forceinline__ u32 zsize(u32 z, u32 osz, u32 p66, bool m32) {
  switch (z) {
    case Z_B: return 1;
    case Z_V: return osz;
    case Z_STK: return p66 ? 2 : (m32 ? 4 : 8);
    case Z_Q: return m32 ? 4 : 8;  // near branch targets, return addresses, rbp of leave
    case Z_W: return 2;
    default: return 4;
  }
}

// Decode (uniform). 0 ok, 1 needs bytes beyond avail, 2 longer than 15 (#GP).
// m32: 32-bit code (compatibility mode, U29): no REX, 32-bit operand and
// address size, 32-bit stack slots and branch targets, disp32 absolute.
__device__ __forceinline__ int decode(const IBytes &b, UOp &u, bool m32 = false) {
  u32 pos = 0, p66 = 0, rex = 0, lock = 0, c;
  u.p67 = u.rep = u.seg = 0;
  // operand fields exec reads before it dispatches on the op: defined for the
  // early returns below (#UD / UNIMPLEMENTED decided before the ModRM)
  u.asrc = u.bsrc = L_NONE;
  u.aread = u.awrite = u.bwrite = 0;
  u.is_mem = u.riprel = 0;
  u.reg = u.rm = u.opreg = u.rex = 0;
  u.base = u.index = -1;
  u.scale = 0;
  u.disp = 0;
  for (;;) {
    if (pos >= 15) return 2;
    if (pos >= b.avail) return 1;
    c = ib_at(b, pos++);
    if ((c & 0xf0) == 0x40 && !m32) {  // REX; ignored unless it is the last prefix
      rex = c;
      continue;
    }
    if (c == 0x66) p66 = 1;
    else if (c == 0x67) u.p67 = 1;
    else if (c == 0xf2 || c == 0xf3) u.rep = c;
    else if (c == 0x64) u.seg = 4;
    else if (c == 0x65) u.seg = 5;
    else if (c == 0xf0) lock = 1;
    else if (c != 0x26 && c != 0x2e && c != 0x36 && c != 0x3e) break;
    rex = 0;
  }
  // VEX (c4 / c5; always VEX in 64-bit mode): its fields become the REX bits,
  // the map and `vex` (engine_sse.h: UOp::opreg of an O_SSE op)
  u32 vex = 0, vpp = 0;
  const bool a16 = m32 && u.p67;  // 16-bit addresses in 32-bit code: outside (U29)
  if (m32) u.p67 = 3;
  if (m32 && (c == 0xc4 || c == 0xc5)) {  // les / lds unless the next byte's mod is 11 (VEX)
    if (pos >= 15) return 2;
    if (pos >= b.avail) return 1;
  }
  if ((c == 0xc4 || c == 0xc5) && (!m32 || (ib_at(b, pos) & 0xc0) == 0xc0)) {
    const u32 bad = (p66 || u.rep || rex) ? 1u : 0u;  // a legacy 66 / f2 / f3 / REX before VEX: #UD
    const u32 nb = c == 0xc4 ? 2 : 1;
    if (pos + nb + 1 > 15) return 2;
    if (pos + nb + 1 > b.avail) return 1;
    const u32 b1 = ib_at(b, pos), b2 = c == 0xc4 ? ib_at(b, pos + 1) : b1;
    pos += nb;
    const u32 vr = ((b1 >> 7) & 1) ^ 1;
    const u32 vx = c == 0xc4 ? ((b1 >> 6) & 1) ^ 1 : 0, vb = (c == 0xc4 && !m32) ? ((b1 >> 5) & 1) ^ 1 : 0;
    const u32 vmap = c == 0xc4 ? (b1 & 31) : 1, vw = c == 0xc4 ? (b2 >> 7) & 1 : 0;
    vpp = b2 & 3;
    vex = 1 | (((b2 >> 2) & 1) << 1) | (vw << 2) | ((((~b2) >> 3) & (m32 ? 7 : 15)) << 4) | (vmap << 8) | (bad << 16);
    // VEX.W selects a 64-bit GPR operand in 64-bit mode only ("the operand size
    // is always 32 bits if not in 64-bit mode"; VEX.W1 ignored): it stays in
    // `vex` (bit 2) for the forms whose element size it picks in every mode
    rex = 0x40 | ((m32 ? 0 : vw) << 3) | (vr << 2) | (vx << 1) | vb;
    c = ib_at(b, pos++);  // the opcode
    const bool def = !bad && vmap >= 1 && vmap <= 3 && vex_defined(vmap, c, vpp);
    if (!def || (vmap == 3 && !fp_form(3, c, vpp, true) && !s4_form(3, c, vpp, true) && !x42_form(3, c, vpp, true) &&
                 !gx_form(3, c, vpp, true) && !ax_form(3, c, vpp, true) &&
                 !(kop_bits(3, c, vpp, 0) | kop_bits(3, c, vpp, 1)))) {  // U36: #UD from the opcode byte
      u.len = pos;
      u.op = (lock || !def) ? O_UD : O_UNIMPL;
      u.supported = lock || !def;
      u.opbytes = pos >= 4 ? (u32)b.lo : ((u32)b.lo & ((1u << (8 * pos)) - 1));
      return 0;
    }
  }
  // EVEX (62; 64-bit code only, 32-bit code's bound stays outside, U29):
  // P0 = R X B R' 0 m m m, P1 = W v v v v 1 p p, P2 = z L' L b V' a a a
  // (engine_avx512.h). Its fields become the REX bits and `vex` with EVX set.
  EForm ef{EZ_NONE, 0, 0, false, false, false, false};
  if (c == 0x62 && !m32 && !vex) {  // (after VEX, c is its opcode byte: 62 is vpunpckldq)
    if (pos + 4 > 15) return 2;
    if (pos + 4 > b.avail) return 1;
    const u32 p0 = ib_at(b, pos), p1 = ib_at(b, pos + 1), p2 = ib_at(b, pos + 2);
    pos += 3;
    c = ib_at(b, pos++);
    const u32 emap = p0 & 7, ew = (p1 >> 7) & 1;
    vpp = p1 & 3;
    ef = evex_form(emap, c, vpp, ew);
    // a legacy 66 / f2 / f3 / REX before EVEX or a reserved bit: #UD; maps
    // 1-3 and 5-6 (AVX512-FP16) are defined, the forms outside the subset
    // UNIMPLEMENTED (U36)
    const bool bad = p66 || u.rep || rex || (p0 & 8) || !(p1 & 4) || lock;
    if (bad || !(emap == 1 || emap == 2 || emap == 3 || emap == 5 || emap == 6) || ef.kind == EZ_NONE) {
      const bool ud = bad || emap == 0 || emap == 4 || emap == 7;
      u.len = pos;
      u.op = ud ? O_UD : O_UNIMPL;
      u.supported = ud;
      u.opbytes = (u32)b.lo;
      return 0;
    }
    rex = 0x40 | (ew << 3) | ((((~p0) >> 7) & 1) << 2) | ((((~p0) >> 6) & 1) << 1) | (((~p0) >> 5) & 1);
    vex = 1 | (ew << 2) | ((((~p1) >> 3) & 15) << 4) | (emap << 8) | EVX | (((p2 >> 5) & 3) << 18) |
          (((p2 >> 7) & 1) << 21) | (((p2 >> 4) & 1) << 22) | ((p2 & 7) << 23) | ((((~p2) >> 3) & 1) << 26) |
          ((((~p0) >> 4) & 1) << 27);  // bit 27: R' (moved into UOp::reg below)
  }
  u.rex = rex;
  const u32 rexw = (rex >> 3) & 1, rexr = (rex >> 2) & 1, rexx = (rex >> 1) & 1, rexb = rex & 1;
  u32 e, map2 = 0, smap = 1;
  if (vex & EVX) {
    smap = vex_map(vex);
    map2 = 1;
    e = smap == 3 ? kSseModrmImm : kSseModrm;
  } else if (vex) {
    smap = vex_map(vex);
    map2 = 1;
    e = smap == 1 ? kMap2[c] : smap == 2 ? kSseModrm : kSseModrmImm;
    if (smap == 1 && kop_bits(1, c, vpp, 0) | kop_bits(1, c, vpp, 1)) e = kSseModrm;  // the opmask instructions
    if (smap == 1 && (e & 63) != O_SSE) e = kUnimpl;
  } else if (c == 0x0f) {
    if (pos >= 15) return 2;
    if (pos >= b.avail) return 1;
    c = ib_at(b, pos++);
    if (c == 0x38 || c == 0x3a) {  // three-byte maps: 0f 38 00 (pshufb), 0f 38 17 (ptest), the rest outside the subset
      if (pos >= 15) return 2;
      if (pos >= b.avail) return 1;
      const u32 c3 = ib_at(b, pos++);
      const u32 pfx3 = u.rep == 0xf3 ? 2 : u.rep == 0xf2 ? 3 : p66 ? 1 : 0;
      const u32 m3 = c == 0x38 ? 2 : 3;
      if ((c == 0x38 && (c3 == 0x00 || c3 == 0x17)) || fp_form(m3, c3, pfx3, false) || s4_form(m3, c3, pfx3, false) ||
          x42_form(m3, c3, pfx3, false) || gx_form(m3, c3, pfx3, false) || (pfx3 == 0 && ssse3_mm(m3, c3))) {
        smap = c == 0x38 ? 2 : 3;
        e = smap == 3 ? kSseModrmImm : kSseModrm;
        c = c3;
        map2 = 1;
      } else {
        const bool def = legacy_3byte_defined(c == 0x38 ? 2 : 3, c3, u.rep == 0xf3 ? 2 : u.rep == 0xf2 ? 3 : p66 ? 1 : 0);
        u.len = pos;
        u.op = (lock || !def) ? O_UD : O_UNIMPL;  // U34: lock is #UD first; U36: undefined is #UD
        u.supported = lock || !def;
        u.opbytes = pos >= 4 ? (u32)b.lo : ((u32)b.lo & ((1u << (8 * pos)) - 1));
        return 0;
      }
    } else {
      map2 = 1;
      e = kMap2[c];
      if ((c == 0xb8 && u.rep != 0xf3) || c == 0xff) e = O_UD;  // popcnt needs f3 (jmpe: #UD); ud0
    }
  } else {
    e = kMap1[c];
    if (c == 0x90 && !rexb) e = O_NOP;  // 90 is nop (no zero-extension), f3 90 pause
    if (m32) {
      if (c >= 0x40 && c <= 0x4f) e = kIncDec32;
      else if (c == 0x82) e = kMap1[0x80];
      else if (c == 0xd4 || c == 0xd5) e = kSys32B;
      else if (c == 0x06 || c == 0x07 || c == 0x0e || c == 0x16 || c == 0x17 || c == 0x1e || c == 0x1f ||
               c == 0x27 || c == 0x2f || c == 0x37 || c == 0x3f || c == 0x60 || c == 0x61 || c == 0x9a ||
               c == 0xce || c == 0xea)
        e = kSys32;
      else if (c == 0x62 || c == 0x63 || c == 0xc4 || c == 0xc5)
        e = kSys32M;  // bound, arpl, les / lds (U29): engine_sys.h
      else if (c == 0xd6)
        e = kSys32;  // salc
    }
  }
  const u32 osz = rexw ? 8 : (p66 ? 2 : 4);
  const u32 sstk = p66 ? 2 : (m32 ? 4 : 8);  // a stack slot
  u.op = e & 63;
  u.asrc = (e >> 6) & 15;
  u.bsrc = (e >> 10) & 15;
  u.asz = zsize((e >> 14) & 7, osz, p66, m32);
  u.bsz = zsize((e >> 17) & 7, osz, p66, m32);
  u.aread = (e >> 20) & 1;
  u.awrite = (e >> 21) & 1;
  u.bwrite = (e >> 22) & 1;
  const u32 hasm = (e >> 23) & 1;
  u32 ik = (e >> 24) & 7;
  const u32 grp = (e >> 27) & 15;
  u.sub = c & 0xf;  // cc for jcc/cmov/setcc, string opcode low bits
  if (grp == G_ALU) u.sub = (c >> 3) & 7;
  if (e == kIncDec32 && !map2) u.sub = (c >> 3) & 1;  // 40-47 inc, 48-4f dec
  u.opreg = (c & 7) | (rexb << 3);
  u.is_mem = u.riprel = 0;
  u.reg = u.rm = 0;
  u.base = u.index = -1;
  u.scale = 0;
  u.disp = 0;
  i32 vsib = -1;  // the SIB's raw index register (VSIB: a vector register, 4 included) and scale
  u32 vsib_scale = 0;
  if (hasm) {
    if (pos >= 15) return 2;
    if (pos >= b.avail) return 1;
    const u32 m = ib_at(b, pos++);
    const u32 mod = m >> 6, rm = m & 7;
    u.reg = ((m >> 3) & 7) | (rexr << 3);
    if (mod == 3) {
      u.rm = rm | (rexb << 3);
    } else {
      u.is_mem = 1;
      if (rm == 4) {
        if (pos >= 15) return 2;
        if (pos >= b.avail) return 1;
        const u32 sib = ib_at(b, pos++);
        const u32 idx = ((sib >> 3) & 7) | (rexx << 3), base = sib & 7;
        vsib = (i32)idx;
        vsib_scale = sib >> 6;
        if (idx != 4) {
          u.index = (i32)idx;
          u.scale = sib >> 6;
        }
        if (base == 5 && mod == 0) {
          if (pos + 4 > 15) return 2;
          if (pos + 4 > b.avail) return 1;
          u.disp = sext(ib_get(b, pos, 4), 4);
          pos += 4;
        } else {
          u.base = (i32)(base | (rexb << 3));
        }
      } else if (rm == 5 && mod == 0) {
        if (pos + 4 > 15) return 2;
        if (pos + 4 > b.avail) return 1;
        u.riprel = m32 ? 0 : 1;  // 32-bit code: disp32 absolute
        u.disp = sext(ib_get(b, pos, 4), 4);
        pos += 4;
      } else {
        u.base = (i32)(rm | (rexb << 3));
      }
      if (mod == 1) {
        if (pos + 1 > 15) return 2;
        if (pos + 1 > b.avail) return 1;
        u.disp = sext(ib_get(b, pos, 1), 1);
        if (vex & EVX) u.disp *= (i64)evex_disp8_n(ef, 16u << evex_ll(vex), (vex >> 22) & 1);  // disp8 * N
        pos += 1;
      } else if (mod == 2) {
        if (pos + 4 > 15) return 2;
        if (pos + 4 > b.avail) return 1;
        u.disp = sext(ib_get(b, pos, 4), 4);
        pos += 4;
      }
    }
    if (vex & EVX) {  // 5-bit vector registers: R' above reg, X above a register r/m
      u.reg |= ((vex >> 27) & 1) << 4;
      if (mod == 3) u.rm |= rexx << 4;
      vex &= ~(1u << 27);
    }
    // modrm.reg selected forms
    const u32 r3 = u.reg & 7;
    switch (grp) {
      case G_1:
      case G_2:
        u.sub = r3;
        break;
      case G_3:
        if (r3 <= 1) {
          ik = c == 0xf6 ? K_B : K_Z;
        } else if (r3 == 2 || r3 == 3) {
          u.op = r3 == 2 ? O_NOT : O_NEG;
          u.awrite = 1;
          u.bsrc = L_NONE;
        } else {
          u.op = O_MULDIV;
          u.sub = r3;
          u.bsrc = L_RM;
          u.bsz = u.asz;
          u.asrc = L_NONE;
          u.aread = 0;
          u.awrite = 0;
        }
        break;
      case G_4:
        if (r3 > 1) u.op = O_UD;
        u.sub = r3;
        break;
      case G_5:
        u.sub = r3;
        if (r3 == 2 || r3 == 4) {  // call / jmp near indirect: 64-bit target
          u.op = r3 == 2 ? O_CALL : O_JMP;
          u.asrc = r3 == 2 ? L_PUSH : L_NONE;
          u.asz = m32 ? 4 : 8;
          u.aread = 0;
          u.awrite = r3 == 2;
          u.bsrc = L_RM;
          u.bsz = m32 ? 4 : 8;
        } else if (r3 == 6) {
          u.op = O_PUSH;
          u.asrc = L_PUSH;
          u.asz = u.bsz = sstk;
          u.aread = 0;
          u.awrite = 1;
          u.bsrc = L_RM;
        } else if (r3 == 3 || r3 == 5) {  // far call / jmp m16:osz (engine_sys.h)
          u.op = O_SYS2;
          u.asz = osz;
          u.bsz = sstk;
        } else if (r3 == 7) {
          u.op = O_UD;
        }
        break;
      case G_8F:
      case G_C6:
        if (r3 != 0) u.op = O_UD;  // xop and the reserved forms: #UD
        if (grp == G_C6 && r3 == 7 && !u.is_mem && (u.rm & 7) == 0) {  // xabort / xbegin: RTM (U48)
          u.op = O_SYS2;
          u.asz = osz;
          u.bsz = sstk;
        }
        break;
      case G_BA:
        if (r3 < 4) u.op = O_UD;
        u.sub = r3;
        if (r3 == 4) u.awrite = 0;
        break;
      default:
        break;
    }
  }
  if (u.op == O_ALU && u.sub == 7) u.awrite = 0;  // cmp reads its destination, never writes it
  if (vex && smap == 2 && vpp == 1 && c >= 0x90 && c <= 0x93) {  // gathers (engine_avx2x.h): index -1 = no SIB
    u.index = vsib;
    u.scale = vsib_scale;
  }
  if (map2) {
    const u32 gpc = vex ? vpp : (u.rep == 0xf3 ? 2 : u.rep == 0xf2 ? 3 : p66 ? 1 : 0);
    if (u.op == O_SSE && smap >= 2 && !(vex & EVX) && gx_form(smap, c, gpc, vex != 0)) {  // engine_ext.h (U45)
      u.op = O_GEXT;
      u.sub = c;
      u.bsz = gpc;
      u.opreg = vex ? vex : (smap << 8);
      u.asz = osz;
    } else if (u.op == O_SSE) {  // engine_sse.h: opcode in sub, mandatory-prefix class in bsz, map / VEX in opreg
      u.sub = c;
      if (vex) {
        u.bsz = vpp;
        u.opreg = vex;
        if (vex & EVX) {
          // the subset (evex_form) was checked before the ModRM
        } else if (smap == 1 && c == 0xae && !(vpp == 0 && u.is_mem && ((u.reg & 7) == 2 || (u.reg & 7) == 3)))
          u.op = O_UD;  // U36: vldmxcsr / vstmxcsr are the only VEX group-15 forms
        else if (!vex_valid(smap, c, vpp, u.is_mem, u.reg & 7))
          u.op = O_UNIMPL;
      } else {
        u.bsz = u.rep == 0xf3 ? 2 : u.rep == 0xf2 ? 3 : p66 ? 1 : 0;
        u.opreg = smap << 8;
        if ((smap == 1 && ((u.bsz == 0 && mmx_opcode(c)) || (c == 0xd6 && u.bsz >= 2))) ||
            (u.bsz == 0 && ssse3_mm(smap, c)))
          u.opreg |= kMmxForm;  // U37: engine_sse.h mmx_exec
        else if (!sse_valid(smap, c, u.bsz, u.is_mem, u.reg & 7))
          u.op = (c == 0xae && smap == 1) ? O_SYS2 : O_UNIMPL;
      }
      if (u.op == O_SYS2) {  // group 15 beyond ldmxcsr / stmxcsr / the fences: engine_sys.h
        u.asz = osz;
        u.bsz = sstk;
      }
    }
    if (u.op == O_BT && grp != G_BA) u.sub = c == 0xa3 ? 4 : c == 0xab ? 5 : c == 0xb3 ? 6 : 7;
    if (u.op == O_SHXD) u.sub = (c >= 0xac ? 1u : 0u) | ((c & 1) ? 2u : 0u);  // bit0 shrd, bit1 count in cl
    if (u.op == O_BSF && u.rep == 0xf3) u.op = O_TZCNT;
    if (u.op == O_BSR && u.rep == 0xf3) u.op = O_LZCNT;
    if (u.op == O_SYS) {
      // 0 syscall, 1 sysret (without REX.W: to compatibility mode, U29), 2 swapgs (0f 01 f8),
      // 3 rdrand r (0f c7 /6),
      // 4 mov r64, crN (0f 20 /r), 6 mov crN, r64 (0f 22 /r), 7 wrmsr, 8 rdtsc, 9 rdmsr,
      // 10 rdtscp (0f 01 f9)
      u.sub = c == 0x05 ? 0 : c == 0x07 ? 1 : c == 0x01 ? 2 : c == 0x20 ? 4 : c == 0x22 ? 6 : c == 0x30 ? 7
              : c == 0x31 ? 8 : c == 0x32 ? 9 : 3;
      if ((c == 0x20 || c == 0x22) && u.is_mem) u.op = O_UNIMPL;
      if (c == 0x01 && (u.rm & 7) == 1) u.sub = 10;
      // the rest of groups 7 and 9 (rdrand / rdseed r stay here): engine_sys.h
      if ((c == 0x01 && (u.is_mem || (u.reg & 7) != 7 || (u.rm & 7) > 1)) ||
          (c == 0xc7 && (u.is_mem || (u.reg & 7) < 6 || u.rep))) {
        u.op = O_SYS2;
        u.asz = osz;
        u.bsz = sstk;
      }
    }
  } else if (u.op == O_FLAGOP) {
    u.sub = c;
  } else if (u.op == O_SYS) {  // iretq (48 cf); iret / iretd: engine_sys.h
    u.sub = 5;
    if (!rexw) {
      u.op = O_SYS2;
      u.asz = osz;
      u.bsz = sstk;
    }
  } else if (u.op == O_STRING && c < 0x80) {
    u.sub |= 0x10;  // ins / outs (6c-6f)
  }
  if (u.op == O_SYS2) u.sub = (map2 ? 0x100u : 0u) | c;
  if (lock) {  // U34: lock only on a memory read-modify-write of the lockable forms
    const bool ok = u.is_mem && !vex &&
                    ((u.op == O_ALU && u.asrc == L_RM && u.sub != 7) || (u.op == O_XCHG && u.asrc == L_RM) ||
                     u.op == O_NOT || u.op == O_NEG || u.op == O_INCDEC || (u.op == O_BT && u.sub >= 5) ||
                     u.op == O_CMPXCHG || u.op == O_XADD || (u.op == O_SYS2 && u.sub == 0x1c7 && (u.reg & 7) == 1));
    if (!ok) u.op = O_UD;
  }
  u32 n = 0;
  switch (ik) {
    case K_B: n = 1; break;
    case K_W: n = 2; break;
    case K_Z: n = osz == 2 ? 2 : 4; break;
    case K_V: n = osz; break;
    case K_MOFFS: n = u.p67 ? 4 : 8; break;
    case K_D: n = 4; break;
    case K_ENTER: n = 3; break;
    default: n = 0;
  }
  if (m32 && !map2 && (c == 0x9a || c == 0xea)) n = osz + 2;  // ptr16:32 / ptr16:16
  if (pos + n > 15) return 2;
  if (pos + n > b.avail) return 1;
  const u64 raw = ib_get(b, pos, n);
  // the immediates x86 sign-extends: Ib/Iz of alu/test/push/imul, branch displacements, c7 Iz
  const bool sx = n && (u.op == O_ALU || u.op == O_TEST || u.op == O_PUSH || u.op == O_IMUL || u.op == O_JCC ||
                        u.op == O_LOOP || u.op == O_JMP || u.op == O_CALL || (u.op == O_MOV && c == 0xc7 && !map2));
  u.imm = sx ? sext(raw, n) : raw;
  pos += n;
  u.len = pos;
  u.opbytes = pos >= 4 ? (u32)b.lo : ((u32)b.lo & ((1u << (8 * pos)) - 1));
  // 16-bit addresses, and 16-bit instruction pointers (66 on a near branch), in 32-bit code
  if (a16 || (m32 && p66 && (u.op == O_JCC || u.op == O_JMP || u.op == O_CALL || u.op == O_RET || u.op == O_LOOP)))
    u.op = O_UNIMPL;
  u.supported = u.op != O_UNIMPL;
  return 0;
}

// ---------------------------------------------------------------- arithmetic
// 0 add,1 or,2 adc,3 sbb,4 and,5 sub,6 xor,7 cmp; returns result, status flags in f
__device__ __forceinline__ u64 alu2(u32 op, u64 a, u64 b, u32 sz, u64 rfl, u64 &f) {
  const u64 mk = szmask(sz);
  a &= mk;
  b &= mk;
  u64 res;
  if (op == 0 || op == 2) {
    const u64 c = op == 2 ? (rfl & F_CF) : 0;
    res = (a + b + c) & mk;
    bool carry;
    if (sz == 8) carry = (res < a) || (c && res == a);
    else carry = ((a + b + c) >> (8 * sz)) & 1;
    f = szp(res, sz) | (carry ? F_CF : 0) | (((a ^ b ^ res) & 0x10) ? F_AF : 0) |
        (msb((a ^ res) & (b ^ res), sz) ? F_OF : 0);
  } else if (op == 3 || op == 5 || op == 7) {
    const u64 c = op == 3 ? (rfl & F_CF) : 0;
    res = (a - b - c) & mk;
    const bool borrow = (a < b) || (c && a == b);
    f = szp(res, sz) | (borrow ? F_CF : 0) | (((a ^ b ^ res) & 0x10) ? F_AF : 0) |
        (msb((a ^ b) & (a ^ res), sz) ? F_OF : 0);
  } else {
    res = op == 1 ? (a | b) : (op == 4 ? (a & b) : (a ^ b));
    f = szp(res, sz);
  }
  return res;
}
__device__ __forceinline__ u64 with_status(u64 rfl, u64 f) { return (rfl & ~F_STATUS) | f; }

__device__ __forceinline__ bool cond(u64 fl, u32 cc) {
  const bool cf = fl & F_CF, zf = fl & F_ZF, sf = fl & F_SF, of = fl & F_OF, pf = fl & F_PF;
  bool r;
  switch (cc >> 1) {
    case 0: r = of; break;
    case 1: r = cf; break;
    case 2: r = zf; break;
    case 3: r = cf || zf; break;
    case 4: r = sf; break;
    case 5: r = pf; break;
    case 6: r = sf != of; break;
    default: r = zf || (sf != of); break;
  }
  return (cc & 1) ? !r : r;
}

// shifts / rotates (U2, U3)
__device__ __forceinline__ u64 shift_op(u32 op, u64 v, u32 count, u32 sz, u64 &fl) {
  const u32 bits = 8 * sz;
  const u64 mk = szmask(sz);
  const u32 cnt = count & (sz == 8 ? 0x3f : 0x1f);
  v &= mk;
  if (cnt == 0) return v;
  u64 res = v, f = fl, cf;
  switch (op) {
    case 0: {
      const u32 c = cnt % bits;
      res = c ? ((v << c) | (v >> (bits - c))) & mk : v;
      cf = res & 1;
      f = (f & ~(F_CF | F_OF)) | (cf ? F_CF : 0) | ((msb(res, sz) ^ cf) ? F_OF : 0);
      break;
    }
    case 1: {
      const u32 c = cnt % bits;
      res = c ? ((v >> c) | (v << (bits - c))) & mk : v;
      cf = msb(res, sz);
      f = (f & ~(F_CF | F_OF)) | (cf ? F_CF : 0) | ((msb(res, sz) ^ ((res >> (bits - 2)) & 1)) ? F_OF : 0);
      break;
    }
    case 2: {
      const u32 c = sz == 1 ? cnt % 9 : (sz == 2 ? cnt % 17 : cnt);
      u64 carry = fl & F_CF;
      if (c) {
        const u64 hi_part = c == 1 ? 0 : (v >> (bits - c + 1));
        res = (((v << c) & mk) | (carry << (c - 1)) | hi_part) & mk;
        carry = (v >> (bits - c)) & 1;
      }
      f = (f & ~(F_CF | F_OF)) | (carry ? F_CF : 0) | ((msb(res, sz) ^ carry) ? F_OF : 0);
      break;
    }
    case 3: {
      const u32 c = sz == 1 ? cnt % 9 : (sz == 2 ? cnt % 17 : cnt);
      u64 carry = fl & F_CF;
      if (c) {
        const u64 hi_part = c == 1 ? 0 : ((v << (bits - c + 1)) & mk);
        res = ((v >> c) | (carry << (bits - c)) | hi_part) & mk;
        carry = (v >> (c - 1)) & 1;
      }
      f = (f & ~(F_CF | F_OF)) | (carry ? F_CF : 0) | ((msb(res, sz) ^ ((res >> (bits - 2)) & 1)) ? F_OF : 0);
      break;
    }
    case 4:
    case 6:
      res = (v << cnt) & mk;
      cf = cnt <= bits ? ((v >> (bits - cnt)) & 1) : 0;
      f = (f & ~F_STATUS) | szp(res, sz) | (cf ? F_CF : 0) | ((msb(res, sz) ^ cf) ? F_OF : 0);
      break;
    case 5:
      res = v >> cnt;
      cf = cnt <= bits ? ((v >> (cnt - 1)) & 1) : 0;
      f = (f & ~F_STATUS) | szp(res, sz) | (cf ? F_CF : 0) | (msb(v, sz) ? F_OF : 0);
      break;
    default: {
      const i64 sv = (i64)sext(v, sz);
      res = (u64)(sv >> (cnt >= bits ? bits - 1 : cnt)) & mk;
      cf = ((u64)(sv >> (cnt >= bits ? bits - 1 : cnt - 1))) & 1;
      f = (f & ~F_STATUS) | szp(res, sz) | (cf ? F_CF : 0);
      break;
    }
  }
  fl = f;
  return res;
}

// shld / shrd (U7): sub bit0 = shrd
__device__ __forceinline__ u64 shxd(u32 sub, u64 a, u64 b, u32 cnt, u32 sz, u64 &fl) {
  const u32 bits = 8 * sz;
  const u32 c = cnt & (sz == 8 ? 0x3f : 0x1f);
  if (c == 0) return a;
  const u64 mk = szmask(sz);
  u64 res, cf;
  if (sz == 2) {
    if (!(sub & 1)) {
      const u64 pat = ((a & 0xffff) << 32) | ((b & 0xffff) << 16) | (a & 0xffff);
      res = ((pat << c) >> 32) & 0xffff;
      cf = ((pat << (c - 1)) >> 47) & 1;
    } else {
      const u64 pat = (a & 0xffff) | ((b & 0xffff) << 16) | ((a & 0xffff) << 32);
      res = (pat >> c) & 0xffff;
      cf = (pat >> (c - 1)) & 1;
    }
  } else if (!(sub & 1)) {
    res = ((a << c) | (b >> (bits - c))) & mk;
    cf = (a >> (bits - c)) & 1;
  } else {
    res = ((a >> c) | (b << (bits - c))) & mk;
    cf = (a >> (c - 1)) & 1;
  }
  fl = with_status(fl, szp(res, sz) | (cf ? F_CF : 0) | ((msb(res, sz) ^ msb(a, sz)) ? F_OF : 0));
  return res;
}

// unsigned 128/64 division; requires hi < dv
__device__ __forceinline__ void divu128(u64 hi, u64 lo, u64 dv, u64 &q, u64 &r) {
  if (hi == 0) {
    q = lo / dv;
    r = lo % dv;
    return;
  }
  u64 qq = 0, rem = hi;
  for (int i = 63; i >= 0; i--) {
    const u64 top = rem >> 63;
    rem = (rem << 1) | ((lo >> i) & 1);
    if (top || rem >= dv) {
      rem -= dv;
      qq |= 1ull << i;
    }
  }
  q = qq;
  r = rem;
}

// signed multiply of sz-byte operands: low result + overflow (CF=OF)
__device__ __forceinline__ u64 imul_lo(u64 a, u64 b, u32 sz, bool &ovf) {
  const i64 sa = (i64)sext(a & szmask(sz), sz), sb = (i64)sext(b & szmask(sz), sz);
  if (sz == 8) {
    const u64 lo = (u64)sa * (u64)sb;
    ovf = (u64)__mul64hi(sa, sb) != (u64)((i64)lo >> 63);
    return lo;
  }
  const i64 p = sa * sb;
  const u64 lo = (u64)p & szmask(sz);
  ovf = (i64)sext(lo, sz) != p;
  return lo;
}

// mul / imul / div / idiv (f6/f7 /4../7) into ra (rax or ax) and rd (rdx).
__device__ __forceinline__ bool muldiv(const Lane &L, u32 sub, u32 sz, u64 src, u64 &ra, u64 &rd, u64 &fl) {
  const u64 mk = szmask(sz);
  const u32 bits = 8 * sz;
  src &= mk;
  const u64 a = sz == 1 ? (R(L, 0) & 0xff) : (R(L, 0) & mk);
  if (sub == 4 || sub == 5) {
    u64 lo, hi;
    bool ovf;
    if (sub == 4) {
      if (sz == 8) {
        lo = a * src;
        hi = __umul64hi(a, src);
      } else {
        const u64 p = a * src;
        lo = p & mk;
        hi = (p >> bits) & mk;
      }
      ovf = hi != 0;
    } else {
      const i64 sa = (i64)sext(a, sz), sb = (i64)sext(src, sz);
      if (sz == 8) {
        lo = (u64)sa * (u64)sb;
        hi = (u64)__mul64hi(sa, sb);
        ovf = hi != (u64)((i64)lo >> 63);
      } else {
        const i64 p = sa * sb;
        lo = (u64)p & mk;
        hi = ((u64)p >> bits) & mk;
        ovf = (i64)sext(lo, sz) != p;
      }
    }
    if (sz == 1) ra = (hi << 8) | lo;
    else {
      ra = lo;
      rd = hi;
    }
    fl = with_status(fl, szp(lo, sz) | (ovf ? (F_CF | F_OF) : 0));
    return true;
  }
  if (src == 0) return false;
  if (sub == 6) {
    u64 q, r;
    if (sz == 1) {
      const u64 n = R(L, 0) & 0xffff;
      q = n / src;
      r = n % src;
      if (q > 0xff) return false;
      ra = (r << 8) | q;
      return true;
    }
    const u64 hi = R(L, 2) & mk;
    if (sz == 8) {
      if (hi >= src) return false;
      divu128(hi, a, src, q, r);
    } else {
      const u64 n = (hi << bits) | a;
      q = n / src;
      r = n % src;
      if (q > mk) return false;
    }
    ra = q;
    rd = r;
    return true;
  }
  const i64 dv = (i64)sext(src, sz);
  if (sz != 8) {
    const i64 n = sz == 1 ? (i64)(int16_t)(R(L, 0) & 0xffff) : (i64)sext(((R(L, 2) & mk) << bits) | a, 2 * sz);
    if (dv == -1 && n == INT64_MIN) return false;
    const i64 q = n / dv, r = n % dv;
    if (q < -((i64)1 << (bits - 1)) || q > ((i64)1 << (bits - 1)) - 1) return false;
    if (sz == 1) ra = (((u64)r & 0xff) << 8) | ((u64)q & 0xff);
    else {
      ra = (u64)q;
      rd = (u64)r;
    }
    return true;
  }
  const u64 nhi = R(L, 2), nlo = R(L, 0);
  const bool nneg = (i64)nhi < 0, dneg = dv < 0;
  u64 ahi = nhi, alo = nlo;
  if (nneg) {
    alo = ~nlo + 1;
    ahi = ~nhi + (alo == 0 ? 1 : 0);
  }
  const u64 adv = dneg ? (u64)(-(dv + 1)) + 1 : (u64)dv;
  if (ahi >= adv) return false;
  u64 q, r;
  divu128(ahi, alo, adv, q, r);
  const bool qneg = nneg != dneg;
  if ((!qneg && q > 0x7fffffffffffffffull) || (qneg && q > 0x8000000000000000ull)) return false;
  ra = qneg ? (u64)(-(i64)(q - 1) - 1) : q;
  rd = nneg ? (u64)(-(i64)r) : r;
  return true;
}

// ---------------------------------------------------------------- string ops
__device__ __forceinline__ int string_op(const Dev &P, Lane &L, const UOp &u) {
  // a4 movs, a6 cmps, aa stos, ac lods, ae scas; 6c ins, 6e outs (U31: all
  // ones in, nothing out, #GP(0) at CPL > IOPL checked per iteration)
  const bool io = u.sub & 0x10;
  const u32 op = io ? (0x60 | (u.sub & 0xe)) : (0xa0 | (u.sub & 0xe));
  const u32 sz = io && u.asz == 8 ? 4 : u.asz;
  const u64 amask = u.p67 ? 0xffffffffull : ~0ull;
  const u64 step = (L.rflags & F_DF) ? (u64)(-(i64)sz) : (u64)sz;
  const u64 sb = segbase(P, L, u.seg);
  const bool src = op == 0xa4 || op == 0xa6 || op == 0xac || op == 0x6e;
  const bool dstw = op == 0xa4 || op == 0xaa || op == 0x6c;
  const bool dstr = op == 0xa6 || op == 0xae;
  for (;;) {
    if (u.rep && (R(L, 1) & amask) == 0) break;
    if (io && L.cpl > ((L.rflags >> 12) & 3)) {
      set_fault(L, WTFGPU_VEC_GP, 0, 0);
      return X_KEEP;
    }
    const u64 rsi = R(L, 6) & amask, rdi = R(L, 7) & amask;
    u64 a = op == 0x6c ? ~0ull : R(L, 0), b = 0;
    if (src && !vread(L, sb + rsi, sz, a)) return X_KEEP;
    if (dstr && !vread(L, rdi, sz, b)) return X_KEEP;
    if (dstw && !vwrite(L, rdi, sz, a)) return X_KEEP;
    if (dstr) {
      u64 f;
      alu2(7, op == 0xa6 ? a : R(L, 0), b, sz, L.rflags, f);
      L.rflags = with_status(L.rflags, f);
    }
    if (op == 0xac) setr(L, u.rex, 0, sz, a);
    if (src) RS(L, 6, (rsi + step) & amask);
    if (op != 0xac && op != 0x6e) RS(L, 7, (rdi + step) & amask);
    L.nbytes += L.pend;  // the iteration is architecturally complete
    L.pend = 0;
    tn_commit(L.lane);   // and so are its Tenet accesses
    if (!u.rep) break;
    RS(L, 1, (R(L, 1) - 1) & amask);
    if (dstr) {
      const bool zf = L.rflags & F_ZF;
      if (u.rep == 0xf3 && !zf) break;
      if (u.rep == 0xf2 && zf) break;
    }
  }
  return X_OK;
}

}  // namespace wtfgpu_dev
#include "engine_sys.h"  // sys2_exec: system, far-transfer, I/O and x87-control instructions
namespace wtfgpu_dev {

// ---------------------------------------------------------------- execute
__device__ __forceinline__ bool loc_is_mem(const UOp &u, u32 loc) {
  return (loc == L_RM && u.is_mem) || loc >= L_PUSH;
}
__device__ __forceinline__ u64 loc_reg_read(const Lane &L, const UOp &u, u32 loc, u32 sz) {
  switch (loc) {
    case L_GREG: return getr(L, u.rex, u.reg, sz);
    case L_RM: return getr(L, u.rex, u.rm, sz);
    case L_RAX: return getr(L, u.rex, 0, sz);
    case L_OPREG: return getr(L, u.rex, u.opreg, sz);
    case L_IMM: return u.imm;
    case L_ONE: return 1;
    case L_CL: return R(L, 1) & 0xff;
    default: return 0;
  }
}
__device__ __forceinline__ u32 loc_reg(const UOp &u, u32 loc) {
  return loc == L_GREG ? u.reg : loc == L_RM ? u.rm : loc == L_OPREG ? u.opreg : 0;
}

// One attempt at the instruction; nrip = address of the next instruction.
__device__ __forceinline__ int exec(const Dev &P, Lane &L, const UOp &u, u64 nrip, u64 &next) {
  next = nrip;
  const u32 op = u.op;
  if (op == O_STRING) return string_op(P, L, u);
  if (op == O_SSE) return sse_exec(P, L, u, nrip, next);
  if (op == O_GEXT) return gext_exec(P, L, u, nrip, next);
  if (op == O_LEA && !u.is_mem) {
    set_fault(L, WTFGPU_VEC_UD, 0, 0);
    return X_FAULT;
  }
  // ---- addresses
  const u64 sb = u.seg ? segbase(P, L, u.seg) : 0;
  u64 ea = 0;
  if (u.is_mem) {
    if (u.riprel) {
      ea = nrip + u.disp;
    } else {
      ea = u.disp;
      if (u.base >= 0) ea += R(L, u.base);
      if (u.index >= 0) ea += R(L, u.index) << u.scale;
    }
    if (u.p67) ea &= 0xffffffffull;
  }
  if (op == O_SYS2) return sys2_exec(P, L, u, nrip, next, ea + sb);
  // 32-bit code (U29): esp addresses the stack, branch targets wrap at 4 GiB
  const bool m32 = u.p67 & 2;
  const u64 smask = m32 ? 0xffffffffull : ~0ull;
  const u64 rsp = R(L, 4) & smask;
  // ---- register / immediate operands
  u64 a = (u.aread && !loc_is_mem(u, u.asrc)) ? loc_reg_read(L, u, u.asrc, u.asz) : 0;
  u64 b = loc_is_mem(u, u.bsrc) ? 0 : loc_reg_read(L, u, u.bsrc, u.bsz);
  if (op == O_BT && u.is_mem && u.bsrc == L_GREG) {
    // bit string addressing: the signed register offset selects the word
    const i64 s = (i64)sext(b, u.bsz);
    ea += (u64)((s >> (u.asz == 8 ? 6 : u.asz == 4 ? 5 : 4)) * (i64)u.asz);
  }
  // ---- the memory read
  const bool bmem = loc_is_mem(u, u.bsrc);
  const bool amem = loc_is_mem(u, u.asrc);
  if (bmem || (u.aread && amem)) {
    const u32 rloc = bmem ? u.bsrc : u.asrc;
    u64 addr;
    switch (rloc) {
      case L_RM: addr = ea + sb; break;
      case L_POP: addr = rsp; break;
      case L_MOFFS: addr = u.imm + sb; break;
      case L_RBPMEM: addr = R(L, 5) & smask; break;
      default: {  // xlat
        u64 x = R(L, 3) + (R(L, 0) & 0xff);
        if (u.p67) x &= 0xffffffffull;
        addr = x + sb;
        break;
      }
    }
    const bool rmw = !bmem && u.awrite;
    u64 v = 0;
    if (!vread(L, addr, bmem ? u.bsz : u.asz, v, rmw ? ACC_W : ACC_R)) return X_FAULT;
    if (bmem) b = v;
    else a = v;
  }
  // ---- compute (pure: lane state untouched)
  const u32 asz = u.asz;
  u64 res = 0, resb = 0, fl = L.rflags, f, ra = 0, rd = 0;
  bool wa = u.awrite, wrax = false, wrdx = false;
  u32 raxsz = asz;
  i64 drsp = 0;
  switch (op) {
    case O_ALU:
      res = alu2(u.sub, a, b, asz, fl, f);
      fl = with_status(fl, f);
      wa = u.sub != 7;
      break;
    case O_TEST:
      alu2(4, a, b, asz, fl, f);
      fl = with_status(fl, f);
      break;
    case O_MOV: res = b; break;
    case O_LEA: res = ea; break;
    case O_MOVZX: res = b & szmask(u.bsz); break;
    case O_MOVSX: res = sext(b & szmask(u.bsz), u.bsz); break;
    case O_XCHG:
      res = b;
      resb = a;
      break;
    case O_XADD:
      res = alu2(0, a, b, asz, fl, f);
      fl = with_status(fl, f);
      resb = a;
      break;
    case O_CMPXCHG: {
      const u64 acc = getr(L, u.rex, 0, asz);
      alu2(7, acc, a, asz, fl, f);
      fl = with_status(fl, f);
      if ((acc & szmask(asz)) == (a & szmask(asz))) {
        res = b;
      } else {
        res = a;
        wa = u.is_mem;  // memory is written back; a register destination is untouched
        ra = a;
        wrax = true;
      }
      break;
    }
    case O_INCDEC:
      res = alu2(u.sub ? 5 : 0, a, 1, asz, fl, f);
      fl = (fl & ~(F_STATUS & ~F_CF)) | (f & ~F_CF);
      break;
    case O_NOT: res = ~a; break;
    case O_NEG:
      res = alu2(5, 0, a, asz, fl, f);
      fl = with_status(fl, f);
      break;
    case O_SHIFT: res = shift_op(u.sub, a, (u32)b, asz, fl); break;
    case O_SHXD: res = shxd(u.sub, a, b, (u.sub & 2) ? (u32)(R(L, 1) & 0xff) : (u32)u.imm, asz, fl); break;
    case O_MULDIV:
      if (!muldiv(L, u.sub, u.bsz, b, ra, rd, fl)) {
        set_fault(L, WTFGPU_VEC_DE, 0, 0);
        return X_FAULT;
      }
      wrax = true;
      wrdx = u.bsz != 1;
      raxsz = u.bsz == 1 ? 2 : u.bsz;
      break;
    case O_IMUL: {
      bool ovf;
      // 0f af: dest * r/m ; 69 / 6b: r/m * imm
      res = u.aread ? imul_lo(a, b, asz, ovf) : imul_lo(b, u.imm, asz, ovf);
      fl = with_status(fl, szp(res, asz) | (ovf ? (F_CF | F_OF) : 0));
      break;
    }
    case O_BT: {
      const u64 bitoff = b & (8 * asz - 1);
      res = u.sub == 5 ? (a | (1ull << bitoff)) : u.sub == 6 ? (a & ~(1ull << bitoff)) : (a ^ (1ull << bitoff));
      wa = u.sub != 4;
      fl = (fl & ~F_CF) | ((a >> bitoff) & 1);
      break;
    }
    case O_BSF:
    case O_BSR: {
      const u64 v = b & szmask(u.bsz);
      if (v == 0) {
        fl |= F_ZF;
        wa = false;  // destination unchanged (U6)
      } else {
        res = op == O_BSF ? (u64)__builtin_ctzll(v) : (u64)(63 - __builtin_clzll(v));
        fl &= ~F_ZF;
      }
      break;
    }
    case O_TZCNT:
    case O_LZCNT: {
      const u32 bits = 8 * u.bsz;
      const u64 v = b & szmask(u.bsz);
      if (op == O_TZCNT) res = v ? (u64)__builtin_ctzll(v) : bits;
      else res = v ? (u64)(__builtin_clzll(v) - (64 - bits)) : bits;
      fl = (fl & ~(F_CF | F_ZF)) | (v == 0 ? F_CF : 0) | (res == 0 ? F_ZF : 0);
      break;
    }
    case O_POPCNT: {
      const u64 v = b & szmask(u.bsz);
      res = (u64)__popcll(v);
      fl = with_status(fl, v ? 0 : F_ZF);
      break;
    }
    case O_CMOV: {
      // the source is always read; a false condition still zero-extends a 32-bit destination
      const bool t = cond(fl, u.sub);
      res = t ? b : a;
      wa = t || asz == 4;
      break;
    }
    case O_SETCC: res = cond(fl, u.sub) ? 1 : 0; break;
    case O_BSWAP: res = asz == 8 ? __builtin_bswap64(a) : asz == 4 ? (u64)__builtin_bswap32((u32)a) : 0; break;
    case O_CBW:
      ra = asz == 2 ? sext(R(L, 0), 1) : asz == 4 ? sext(R(L, 0), 2) : sext(R(L, 0), 4);
      wrax = true;
      break;
    case O_CWD:
      rd = msb(R(L, 0), asz) ? ~0ull : 0;
      wrdx = true;
      break;
    case O_LAHF:
      ra = (R(L, 0) & ~0xff00ull) | (((fl & 0xd5) | 2) << 8);
      wrax = true;
      raxsz = 8;
      break;
    case O_SAHF:
      fl = (fl & ~(F_SF | F_ZF | F_AF | F_PF | F_CF)) | ((R(L, 0) >> 8) & (F_SF | F_ZF | F_AF | F_PF | F_CF));
      break;
    case O_FLAGOP:
      if (u.sub == 0xf5) fl ^= F_CF;
      else if (u.sub == 0xf8) fl &= ~F_CF;
      else if (u.sub == 0xf9) fl |= F_CF;
      else if (u.sub == 0xfc) fl &= ~F_DF;
      else fl |= F_DF;
      break;
    case O_NOP: break;
    case O_JCC:
      if (cond(fl, u.sub)) next = nrip + b;
      break;
    case O_JMP: next = u.bsrc == L_IMM ? nrip + b : b; break;
    case O_LOOP: {  // U26: e0 loopne, e1 loope, e2 loop, e3 jrcxz; rcx (ecx with 67), flags untouched
      const u64 amask = u.p67 ? 0xffffffffull : ~0ull;
      bool taken;
      if (u.sub == 3) {
        taken = (R(L, 1) & amask) == 0;
      } else {
        const u64 cnt = (R(L, 1) - 1) & amask;
        RS(L, 1, cnt);
        const bool zf = fl & F_ZF;
        taken = cnt != 0 && (u.sub == 2 || (u.sub == 1 ? zf : !zf));
      }
      if (taken) next = nrip + b;
      break;
    }
    case O_CALL:
      res = nrip;
      next = u.bsrc == L_IMM ? nrip + b : b;
      drsp = -(i64)asz;
      break;
    case O_RET:
      next = b;
      drsp = (i64)u.bsz + (i64)u.imm;
      break;
    case O_PUSH:
      res = b;
      drsp = -(i64)asz;
      break;
    case O_PUSHF:
      res = fl & 0xfcffffull & szmask(asz);
      drsp = -(i64)asz;
      break;
    case O_POP:
      res = b;
      drsp = (i64)u.bsz;
      break;
    case O_POPF: {
      u64 mask = F_STATUS | F_TF | F_DF | 0x4000ull | 0x40000ull | 0x200000ull;
      if (L.cpl == 0) mask |= F_IF | 0x3000ull;
      if (u.bsz == 2) mask &= 0xffff;
      fl = ((fl & ~mask) | (b & mask) | 2) & ~0x10000ull;
      drsp = (i64)u.bsz;
      break;
    }
    case O_LEAVE: break;
    case O_INT3: return X_INT3;
    case O_HLT: return X_HLT;
    case O_UD:
      set_fault(L, WTFGPU_VEC_UD, 0, 0);
      return X_FAULT;
    case O_SYS: {
      // System instructions of the kernel paths (SDM vol. 2):
      // 64-bit SYSCALL / SYSRET with STAR selectors (no descriptor loads),
      // SWAPGS, and a deterministic RDRAND.
      LaneSys &S = P.sys[L.lane];
      if (u.sub == 4) {  // mov r64, crN (ring 0)
        if (L.cpl != 0) {
          set_fault(L, WTFGPU_VEC_GP, 0, 0);
          return X_FAULT;
        }
        const u32 n = u.reg & 15;
        if (n == 0) res = S.cr0;
        else if (n == 2) res = S.cr2;
        else if (n == 3) res = S.cr3;
        else if (n == 4) res = S.cr4;
        else if (n == 8) res = 0;
        else {
          set_fault(L, WTFGPU_VEC_UD, 0, 0);
          return X_FAULT;
        }
        break;
      }
      if (u.sub == 5) {  // iretq (U19): every frame read before any change
        u64 f0, f1, f2, f3, f4;
        if (!vread(L, rsp, 8, f0) || !vread(L, rsp + 8, 8, f1) || !vread(L, rsp + 16, 8, f2) ||
            !vread(L, rsp + 24, 8, f3) || !vread(L, rsp + 32, 8, f4))
          return X_FAULT;
        const u32 ncpl = (u32)f1 & 3;
        if ((f1 & 0xfffc) == 0 || ncpl < L.cpl) {
          set_fault(L, WTFGPU_VEC_GP, (u32)f1 & 0xfffc, 0);
          return X_FAULT;
        }
        if (!canonical(f0)) {
          set_fault(L, WTFGPU_VEC_GP, 0, 0);
          return X_FAULT;
        }
        // SDM IRET: status, TF, DF, NT, RF, AC, ID always; IF if CPL <= IOPL;
        // IOPL, VIF, VIP at CPL 0 only
        u64 mask = 0x254dd5ull;
        if (L.cpl == 0) mask |= 0x200ull | 0x3000ull | 0x80000ull | 0x100000ull;
        else if (L.cpl <= ((fl >> 12) & 3)) mask |= 0x200ull;
        fl = (fl & ~mask) | (f2 & mask) | 2;
        next = f0;
        RS(L, 4, f3);
        set_cs(L, S, (u32)f1 & 0xffff);
        S.ss = (u16)f4;
        if (ncpl != L.cpl) L.flush = 1;  // translations were permission-checked at the old cpl
        L.cpl = S.cpl = ncpl;
        break;
      }
      if (u.sub >= 6) {  // mov crN, r64 / wrmsr / rdtsc / rdmsr / rdtscp (U20, U21)
        if (u.sub == 8 || u.sub == 10) {
          if ((S.cr4 & 4) && L.cpl != 0) {
            set_fault(L, WTFGPU_VEC_GP, 0, 0);
            return X_FAULT;
          }
          const u64 t = P.full[L.lane].tsc + L.icount;
          RS(L, 0, t & 0xffffffffull);
          RS(L, 2, t >> 32);
          if (u.sub == 10) RS(L, 1, P.full[L.lane].tsc_aux & 0xffffffffull);
          break;
        }
        if (L.cpl != 0) {
          set_fault(L, WTFGPU_VEC_GP, 0, 0);
          return X_FAULT;
        }
        if (u.sub == 6) {
          const u32 n = u.reg & 15;
          const u64 v = R(L, u.rm & 15);
          if (n == 0) {
            L.cr0 = S.cr0 = v;
            L.simd = simd_bits(v, S.cr4, P.full[L.lane].xcr0);
            L.flush = 1;
          } else if (n == 2) {
            S.cr2 = v;
          } else if (n == 3) {
            S.cr3 = v;
            L.cr3 = v;
            L.flush = 1;
            if (v != P.cr3_0) {
              L.rflags = fl;
              return X_CR3;  // retires, then the lane stops with Cr3Change_t
            }
          } else if (n == 4) {
            S.cr4 = v;
            L.simd = simd_bits(L.cr0, v, P.full[L.lane].xcr0);
            L.flush = 1;
          } else if (n == 8) {
            P.full[L.lane].cr8 = v & 15;
          } else {
            set_fault(L, WTFGPU_VEC_UD, 0, 0);
            return X_FAULT;
          }
          break;
        }
        // rdmsr / wrmsr: the MSRs CpuState_t carries
        wtfgpu_regs_t &F = P.full[L.lane];
        const u32 idx = (u32)R(L, 1);
        u64 cur = 0;
        int canon = 0, lo32 = 0;
        switch (idx) {
          case 0x10: cur = F.tsc + L.icount; break;
          case 0x1b: cur = F.apic_base; break;
          case 0x174: cur = F.sysenter_cs; break;
          case 0x175: cur = F.sysenter_esp; canon = 1; break;
          case 0x176: cur = F.sysenter_eip; canon = 1; break;
          case 0x277: cur = F.pat; break;
          case 0xc0000080u: cur = L.efer & ~EFER_M32; break;
          case 0xc0000081u: cur = S.star; break;
          case 0xc0000082u: cur = S.lstar; canon = 1; break;
          case 0xc0000083u: cur = F.cstar; canon = 1; break;
          case 0xc0000084u: cur = S.sfmask; lo32 = 1; break;
          case 0xc0000100u: cur = P.fs_base[L.lane]; canon = 1; break;
          case 0xc0000101u: cur = P.gs_base[L.lane]; canon = 1; break;
          case 0xc0000102u: cur = S.kgs; canon = 1; break;
          case 0xc0000103u: cur = F.tsc_aux; lo32 = 1; break;
          default:
            set_fault(L, WTFGPU_VEC_GP, 0, 0);
            return X_FAULT;
        }
        if (u.sub == 9) {
          RS(L, 0, cur & 0xffffffffull);
          RS(L, 2, cur >> 32);
          break;
        }
        const u64 v = (R(L, 0) & 0xffffffffull) | (R(L, 2) << 32);
        if ((canon && !canonical(v)) || (lo32 && (v >> 32))) {
          set_fault(L, WTFGPU_VEC_GP, 0, 0);
          return X_FAULT;
        }
        switch (idx) {
          case 0x10: F.tsc = v - L.icount; break;
          case 0x1b: F.apic_base = v; break;
          case 0x174: F.sysenter_cs = v; break;
          case 0x175: F.sysenter_esp = v; break;
          case 0x176: F.sysenter_eip = v; break;
          case 0x277: F.pat = v; break;
          case 0xc0000080u:
            L.efer = S.efer = (v & ~0x400ull) | (L.efer & (0x400ull | EFER_M32));  // LMA is read-only
            L.flush = 1;
            break;
          case 0xc0000081u: S.star = v; break;
          case 0xc0000082u: S.lstar = v; break;
          case 0xc0000083u: F.cstar = v; break;
          case 0xc0000084u: S.sfmask = v; break;
          case 0xc0000100u: P.fs_base[L.lane] = v; break;
          case 0xc0000101u: P.gs_base[L.lane] = v; break;
          case 0xc0000102u: S.kgs = v; break;
          default: F.tsc_aux = v; break;
        }
        break;
      }
      if (u.sub == 3) {  // rdrand: 0 with CF=1 (U15)
        res = 0;
        fl = with_status(fl, F_CF);
        break;
      }
      if (u.sub == 2) {  // swapgs
        if (L.cpl != 0) {
          set_fault(L, WTFGPU_VEC_GP, 0, 0);
          return X_FAULT;
        }
        const u64 g = P.gs_base[L.lane];
        P.gs_base[L.lane] = S.kgs;
        S.kgs = g;
        break;
      }
      if (!(L.efer & 1)) {  // EFER.SCE
        set_fault(L, WTFGPU_VEC_UD, 0, 0);
        return X_FAULT;
      }
      if (u.sub == 0) {  // syscall (from 32-bit code: to CSTAR, U29)
        RS(L, 1, nrip);
        RS(L, 11, fl & ~0x10000ull);
        fl = ((fl & ~S.sfmask) & ~0x10000ull) | 2;
        next = (u.p67 & 2) ? P.full[L.lane].cstar : S.lstar;
        L.cpl = S.cpl = 0;
        set_cs(L, S, (u32)((S.star >> 32) & 0xfffc));
        S.ss = (u16)(S.cs + 8);
      } else {  // sysretq
        if (L.cpl != 0) {
          set_fault(L, WTFGPU_VEC_GP, 0, 0);
          return X_FAULT;
        }
        if (!(u.rex & 8)) {  // to compatibility mode at ecx (U29)
          const u64 t32 = R(L, 1) & 0xffffffffull;
          fl = (R(L, 11) & 0x3c7fd7ull) | 2;
          next = t32;
          L.cpl = S.cpl = 3;
          set_cs(L, S, (u32)(((S.star >> 48) & 0xffff) | 3));
          S.ss = (u16)((((S.star >> 48) & 0xffff) + 8) | 3);
          L.flush = 1;
          break;
        }
        const u64 target = R(L, 1);
        if (!canonical(target)) {
          set_fault(L, WTFGPU_VEC_GP, 0, 0);
          return X_FAULT;
        }
        fl = (R(L, 11) & 0x3c7fd7ull) | 2;
        next = target;
        L.cpl = S.cpl = 3;
        set_cs(L, S, (u32)((((S.star >> 48) & 0xffff) + 16) | 3));
        S.ss = (u16)((((S.star >> 48) & 0xffff) + 8) | 3);
      }
      L.flush = 1;  // cached translations were permission-checked at the old cpl
      break;
    }
    default: return X_UNIMPL;
  }
  if (m32 && op != O_SYS) next &= 0xffffffffull;
  // ---- the memory write
  if (wa && amem) {
    u64 addr;
    if (u.asrc == L_RM) {
      // pop r/m computes its address with rsp already incremented
      addr = (op == O_POP && u.base == 4 ? ea + u.bsz : ea) + sb;
    } else if (u.asrc == L_PUSH) {
      addr = (rsp - asz) & smask;
    } else {
      addr = u.imm + sb;
    }
    if (!vwrite(L, addr, asz, res)) return X_FAULT;
  }
  // ---- commit
  if (op == O_LEAVE) {
    RS(L, 4, (R(L, 5) + u.bsz) & smask);
    RS(L, 5, m32 ? (b & 0xffffffffull) : b);
  }
  if (drsp) RS(L, 4, (rsp + (u64)drsp) & smask);
  if (u.bwrite && !bmem) setr(L, u.rex, loc_reg(u, u.bsrc), u.bsz, resb);  // xchg / xadd source
  if (wa && !amem) setr(L, u.rex, loc_reg(u, u.asrc), asz, res);  // xadd r,r: DEST := TEMP last (SDM)
  if (wrax) setr(L, u.rex, 0, raxsz, ra);
  if (wrdx) setr(L, u.rex, 2, asz, rd);
  L.rflags = fl;
  return X_OK;
}

}  // namespace wtfgpu_dev
