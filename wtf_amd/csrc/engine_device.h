// engine_device.h — CDNA4 device side of the wtf gpu execution backend.
//
// One lane = one testcase. The kernel runs each wavefront as a RIP-grouped
// SIMT interpreter:
//   1. min-RIP over the wave's running lanes (wave reduction) picks the group;
//   2. the group's instruction is fetched + decoded ONCE, as wave-uniform
//      (scalar) work, from the lane page pool;
//   3. coverage / breakpoint checks are uniform (one lookup per group);
//   4. the semantics execute per lane on the group's exec mask, GPRs held in
//      VGPRs (16 x u64, indexed with s_set_gpr_idx by the uniform register
//      number), memory through a per-lane 4-entry TLB in VGPRs, page walks over
//      the lane's copy-on-write view of guest physical memory.
//
// The semantics mirror the hooks of the reference bochscpu backend
// (src/wtf/bochscpu_backend.cc:445-728) and the conventions U1-U13 written in
// DESIGN.md §5. This header is included by engine.hip only.
#pragma once
#ifndef WTFGPU_HOST_SIM
#include <hip/hip_runtime.h>
#else
#include "../../tests/native/host_sim_shim.h"  // test-only CPU build of the device code
#endif
#include <stdint.h>
#include "../../include/wtfgpu.h"

namespace wtfgpu_dev {

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;
typedef int64_t i64;
typedef int32_t i32;

constexpr u64 F_CF = 0x1, F_PF = 0x4, F_AF = 0x10, F_ZF = 0x40, F_SF = 0x80, F_TF = 0x100,
              F_IF = 0x200, F_DF = 0x400, F_OF = 0x800;
constexpr u64 F_STATUS = F_CF | F_PF | F_AF | F_ZF | F_SF | F_OF;
constexpr u64 EMPTY_KEY = ~0ull;

// TLB entry data: page pointer | permission bits in the low 12 bits.
constexpr u64 T_W = 1, T_U = 2, T_NX = 4, T_PRIV = 8, T_PT = 16;
constexpr int TLB_N = 4;

struct LaneSys {   // rarely touched per-lane system state
  u64 cr0, cr3, cr4, efer;
  u64 star, lstar, sfmask, kgs;  // SYSCALL/SYSRET MSRs, IA32_KERNEL_GS_BASE (SWAPGS)
  u64 idtr, tss, cr2;            // IDT base, TSS base (TR), cr2 (exception delivery)
  u64 deliv_icount;              // retired count at the last delivery (~0: none)
  u32 idtr_limit, pad;
  u32 cpl;
  u16 cs, ss;                    // selectors after SYSCALL/SYSRET (64-bit mode, STAR)
};

// Translation state a lane keeps between k_run launches (regrouped launches
// are short): TLB, code-page cache, overlay filter. tlb_ok[lane] == 0 means
// stale (restore, host writes, injected faults, register / cr writes).
struct LaneTlb {
  u64 tv[TLB_N], td[TLB_N];
  u64 cvpn, cptr, bloom;
  u32 tnext, pad;
};

struct ExitInfo {
  u32 vector, error, opcode, cpl;  // cpl: privilege level the fault was raised at
  u64 addr;
};

// Everything the kernels need, passed by value.
struct Dev {
  // snapshot page pool (index 0 = zero page)
  const u8 *pool;
  const u32 *pfn_map;    // gpfn -> pool page index
  u64 pfn_map_len;
  u64 npool;             // pages in the pool after the zero page
  const u32 *ptbits;     // bitmap over gpfn: page-table pages of the snapshot
  // lanes, SoA
  u32 nlanes;
  u32 K;                 // copy-on-write pages per lane
  u32 lpw;               // lanes per hardware wave (64, 32 or 16): coverage-log wave = lane / lpw
  u64 *gpr;              // [16][nlanes]
  u64 *rip, *rflags, *fs_base, *gs_base, *icount, *nbytes;
  u32 *status, *lflags;  // lflags bit0: skip breakpoint once
  ExitInfo *exinfo;
  LaneSys *sys;
  u32 *ov_count;         // [nlanes]
  u32 *ov_gpfn;          // [K][nlanes]
  u8 *ov_data;           // [nlanes][K][4096]
  // breakpoints (open addressing, EMPTY_KEY)
  const u64 *bp_keys;
  u32 bp_mask;           // table size - 1; 0 with bp_keys==nullptr = none
  // device-side breakpoint actions (own hash table, looked up on a hit only)
  const u64 *act_keys;
  const wtfgpu_bp_action_t *act;
  u32 act_mask;
  // per-lane input feed for WTFGPU_BPACT_FEED: cursor / end into feed_data
  u64 *feed_pos;         // [nlanes], ~0 = no feed
  const u64 *feed_end;   // [nlanes]
  const u8 *feed_data;
  // coverage
  const u64 *code_keys;  // vpn hash table
  const u32 *code_slot;
  u32 code_mask;
  u8 *cov_map;           // [slots][4096]
  u8 *cov_shadow;        // [slots][4096]: the map as of the last absorb
  // new-coverage logs: per lane, an open-addressing set of H rips the lane
  // ran while they were absent from cov_map (bochscpu_backend.cc:501-504)
  u64 *cov_rip;          // [nlanes][H]
  u32 *cov_gen;          // [nlanes][H]: an entry is live when it equals the lane's generation
  u32 *lane_gen;         // [nlanes]: bumped by restore / collection (empties the set in O(1))
  u32 *cov_cnt;          // [nlanes]: live entries
  u32 *cov_overflow;     // [nlanes]: the set filled up (entries were lost)
  u32 H;                 // entries per lane (power of two)
  // lane order of a k_run launch (cross-wave regrouping): hardware wave w runs
  // lanes perm[first + w * lpw ...]; nullptr = identity
  const u32 *perm;
  // device-wide decoded-uop cache (shared by every wave and launch): entries
  // of 3 x 64-byte lines, 14 payload dwords + the key in each line's last 8
  // bytes (a reader takes an entry only when all three tags match)
  u32 *guc;
  u32 guc_mask;
  u8 *warm;  // k_run: per-wave images of the LDS uop cache carried between launches (null: cold start)
  u32 warm_n;  // images in the set (waves a launch can have)
  u64 *rd_seed;           // [nlanes] Rdrand seeds (WTFGPU_BPACT_RDRAND)
  u64 *stop_args;         // [nlanes][6] arguments kept by WTFGPU_BPACT_STOP_ARGS
  // values of the aggregate coverage that are not code bytes of a code page
  // (rips elsewhere, --edges values): an open-addressing set, read-only
  // during k_run, grown by k_cov_commit
  u64 *extra_keys;
  u32 extra_mask;
  u32 edges;              // record branch edges (RecordEdge, bochscpu_backend.cc:699-728)
  u32 *edge_cnt;          // [nlanes][2] with edges: RecordEdge calls, and those new to the lane's set (run stats)
  // rip trace (--trace-type rip / unique_rip, bochscpu_backend.cc:506-520):
  // per lane, the rips about to execute in order, trace_cap of them at most
  u64 *trace;             // [nlanes][trace_cap]
  u32 *trace_cnt;         // [nlanes] rips logged (may exceed trace_cap: truncated)
  u32 trace_cap;
  u64 rd_seed0;           // the initial state's (restore)
  LaneTlb *tlbs;          // [nlanes]
  void *lcopy;            // [nlanes] Lane + 32 u32: the rare path's lane copy (build WTFGPU_LANE_LDS=2 only)
  u32 *tlb_ok;            // [nlanes]
  wtfgpu_regs_t *full;   // [nlanes] cold architectural state (MSRs the hot LaneSys lacks)
  u64 cr3_0;             // the testcases' initial cr3 (Cr3Change_t, bochscpu_backend.cc:628-657)
  u64 limit;
  u64 *stat;             // [0] group steps, [1] retired, [2] lanes still running
};

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ u64 rfl64(u64 v) {
  u32 lo = __builtin_amdgcn_readfirstlane((u32)v);
  u32 hi = __builtin_amdgcn_readfirstlane((u32)(v >> 32));
  return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u32 rfl32(u32 v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ u64 mix64(u64 x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ u64 szmask(u32 sz) { return sz == 8 ? ~0ull : ((1ull << (8 * sz)) - 1); }
__device__ __forceinline__ u64 sext(u64 v, u32 bytes) {
  const u32 s = 64 - 8 * bytes;
  return bytes >= 8 ? v : (u64)(((i64)(v << s)) >> s);
}
__device__ __forceinline__ u64 msb(u64 v, u32 sz) { return (v >> (8 * sz - 1)) & 1; }
__device__ __forceinline__ u64 szp(u64 res, u32 sz) {
  res &= szmask(sz);
  const u64 pf = (__builtin_popcount((u32)(res & 0xff)) & 1) ? 0 : F_PF;
  return (res == 0 ? F_ZF : 0) | (msb(res, sz) ? F_SF : 0) | pf;
}

}  // namespace wtfgpu_dev
