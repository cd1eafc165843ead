// engine.hip — kernels + host implementation of the C ABI in include/wtfgpu.h.
//
// Hot kernel: k_run, the RIP-grouped lane-per-testcase x86-64 interpreter
// (engine_device.h explains the scheme). Everything else here is plumbing:
// lane restore (the dirty-list reset that replaces bochscpu's per-page memcpy,
// bochscpu_backend.cc:730-797), batched guest-memory writes for host-side
// handlers, coverage log compaction and the aggregate coverage map.
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "engine_fast.h"

using namespace wtfgpu_dev;

// ====================================================================== device
namespace {

__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ u64 readlane64(u64 v, int l) {
  const u32 lo = __builtin_amdgcn_readlane((u32)v, l);
  const u32 hi = __builtin_amdgcn_readlane((u32)(v >> 32), l);
  return ((u64)hi << 32) | lo;
}
// Lane masks straight from a compare (one v_cmp writing an SGPR pair), and a
// mask back to a per-lane condition (used as the exec mask as it is): the
// step loop tests and combines groups as masks, where a per-lane bool fed to
// __ballot costs a v_cndmask + v_cmp pair to become a mask again. Every lane
// of the wave runs the step loop, so a compare's mask is the ballot's.
__device__ __forceinline__ u64 m_eq32(u32 a, u32 b) { return __builtin_amdgcn_uicmp(a, b, 32); }
__device__ __forceinline__ u64 m_ne32(u32 a, u32 b) { return __builtin_amdgcn_uicmp(a, b, 33); }
__device__ __forceinline__ u64 m_eq64(u64 a, u64 b) { return __builtin_amdgcn_uicmpl(a, b, 32); }
__device__ __forceinline__ u64 m_ne64(u64 a, u64 b) { return __builtin_amdgcn_uicmpl(a, b, 33); }
__device__ __forceinline__ u64 m_lt64(u64 a, u64 b) { return __builtin_amdgcn_uicmpl(a, b, 36); }
__device__ __forceinline__ u64 m_ge64(u64 a, u64 b) { return __builtin_amdgcn_uicmpl(a, b, 35); }
__device__ __forceinline__ u64 m_ge32(u32 a, u32 b) { return __builtin_amdgcn_uicmp(a, b, 35); }
__device__ __forceinline__ bool in_mask(u64 m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

__device__ __forceinline__ bool hash_find(const u64 *keys, u32 mask, u64 key, u32 &slot) {
  u32 h = (u32)mix64(key) & mask;
  for (u32 i = 0; i <= mask; i++) {
    const u64 k = rfl64(keys[h]);
    if (k == key) {
      slot = h;
      return true;
    }
    if (k == EMPTY_KEY) return false;
    h = (h + 1) & mask;
  }
  return false;
}

// Per-lane (non-uniform) lookup in an open-addressing u64 set.
__device__ __forceinline__ bool set_has(const u64 *keys, u32 mask, u64 key) {
  u32 h = (u32)mix64(key) & mask;
  for (u32 i = 0; i <= mask; i++) {
    const u64 k = keys[h];
    if (k == key) return true;
    if (k == EMPTY_KEY) return false;
    h = (h + 1) & mask;
  }
  return false;
}

// Rip trace: the lane's next entry (the before-execution hook's trace write,
// bochscpu_backend.cc:506-520).
__device__ __forceinline__ void trace_rip(const Dev &P, u32 lane, u64 rip) {
  const u32 n = P.trace_cnt[lane];
  if (n < P.trace_cap) P.trace[(u64)lane * P.trace_cap + n] = rip;
  P.trace_cnt[lane] = n + 1;
}

// RecordEdge's key (bochscpu_backend.cc:699-728): splitmix64's finaliser of
// the branch's rip, xor the rip that follows it.
__device__ __forceinline__ u64 edge_key(u64 rip, u64 next) {
  u64 e = rip;
  e ^= e >> 30;
  e *= 0xbf58476d1ce4e5b9ull;
  e ^= e >> 27;
  e *= 0x94d049bb133111ebull;
  e ^= e >> 31;
  return e ^ next;
}

// The branches RecordEdge sees: conditional near branches taken or not
// (cnear_branch_taken / _not_taken) and indirect near jmp / call
// (ucnear_branch with JMP_INDIRECT / CALL_INDIRECT), :235-257.
__device__ __forceinline__ bool edge_op(u32 op, u32 bsrc) {
  return op == O_JCC || op == O_LOOP || ((op == O_JMP || op == O_CALL) && bsrc != L_IMM);
}

__device__ __forceinline__ void load_lane(const Dev &P, u32 lane, Lane &L) {
  const u64 N = P.nlanes;
#pragma unroll
  for (int i = 0; i < 16; i++) RS(L, i, P.gpr[i * N + lane]);
  L.rip = P.rip[lane];
  L.rflags = P.rflags[lane];
  L.icount = P.icount[lane];
  L.nbytes = P.nbytes[lane];
  L.status = P.status[lane];
  const LaneSys s = P.sys[lane];
  L.cr0 = s.cr0;
  L.cr3 = s.cr3;
  L.efer = s.efer;  // with the 32-bit-code bit (U29)
  L.cpl = s.cpl;
  L.simd = simd_bits(s.cr0, s.cr4, P.full[lane].xcr0);
  L.ovn = P.ov_count[lane];
  L.lane = lane;
  L.cgen = P.lane_gen ? P.lane_gen[lane] : 0;
  L.ccnt = P.cov_cnt ? P.cov_cnt[lane] : 0;
  if (P.tlb_ok && P.tlb_ok[lane]) {
    const LaneTlb &t = P.tlbs[lane];
#pragma unroll
    for (int i = 0; i < TLB_N; i++) {
      L.tv[i] = t.tv[i];
      L.td[i] = t.td[i];
    }
    L.cvpn = t.cvpn;
    L.cptr = t.cptr;
    L.bloom = t.bloom;
    L.tnext = t.tnext;
  } else {
    L.bloom = 0;
    for (u32 k = 0; k < L.ovn; k++) L.bloom |= bloom_bit(P.ov_gpfn[(u64)k * N + lane]);
    tlb_flush(L);
    L.tnext = 0;
  }
  L.exvec = L.exerr = L.exop = 0;
  L.exaddr = 0;
  L.miss = L.miss_acc = L.flush = L.pend = 0;
  L.nodeliver = 0;
  L.miss_va = 0;
}

__device__ __forceinline__ void store_tlb(const Dev &P, const Lane &L) {
  if (!P.tlb_ok) return;
  LaneTlb &t = P.tlbs[L.lane];
#pragma unroll
  for (int i = 0; i < TLB_N; i++) {
    t.tv[i] = L.tv[i];
    t.td[i] = L.td[i];
  }
  t.cvpn = L.cvpn;
  t.cptr = L.cptr;
  t.bloom = L.bloom;
  t.tnext = L.tnext;
  P.tlb_ok[L.lane] = 1;
}
__device__ __forceinline__ void tlb_stale(const Dev &P, u32 lane) {
  if (P.tlb_ok) P.tlb_ok[lane] = 0;
}

__device__ __forceinline__ void store_lane(const Dev &P, const Lane &L) {
  const u64 N = P.nlanes;
  const u32 lane = L.lane;
#pragma unroll
  for (int i = 0; i < 16; i++) P.gpr[i * N + lane] = R(L, i);
  P.rip[lane] = L.rip;
  P.rflags[lane] = L.rflags;
  P.icount[lane] = L.icount;
  P.nbytes[lane] = L.nbytes;
  P.status[lane] = L.status;
  P.ov_count[lane] = L.ovn;
  if (P.cov_cnt) P.cov_cnt[lane] = L.ccnt;
}

__device__ __forceinline__ u32 log_value(const Dev &P, u64 v, bool mine, u32 lane, u32 gen, u32 cnt);

// Coverage (bochscpu_backend.cc:501-504): a rip absent from the aggregate map
// joins the set of every lane that ran it (`mine`). The map check is uniform;
// the set insert is per lane (its own open-addressing table, no contention
// whatever wave runs the lane). Returns the lane's new entry count.
__device__ __noinline__ u32 cover(const Dev &P, u64 rip, bool mine, u32 lane, u32 gen, u32 cnt) {
  if (P.code_keys) {
    u32 s;
    if (hash_find(P.code_keys, P.code_mask, rip >> 12, s)) {
      const u32 cs = rfl32(P.code_slot[s]);
      if (rfl32(P.cov_map[(u64)cs * WTFGPU_PAGE_SIZE + (rip & 0xfff)])) return cnt;
    } else if (P.extra_keys && set_has(P.extra_keys, P.extra_mask, rip)) {
      return cnt;
    }
  }
  return log_value(P, rip, mine, lane, gen, cnt);
}

// Run stats (BochscpuRunStats_t::NumberEdges / NumberUniqueEdges,
// bochscpu_backend.h:17-45): edges recorded, and those new to the lane's set.
__device__ __forceinline__ void count_edge(const Dev &P, u32 lane, bool fresh) {
  if (!P.edge_cnt) return;
  P.edge_cnt[2 * (u64)lane] += 1;
  if (fresh) P.edge_cnt[2 * (u64)lane + 1] += 1;
}

// A branch edge (per-lane value): logged unless the aggregate has it.
__device__ __noinline__ u32 cover_edge(const Dev &P, u64 e, bool mine, u32 lane, u32 gen, u32 cnt) {
  if (!mine) return cnt;
  if (P.extra_keys && set_has(P.extra_keys, P.extra_mask, e)) return cnt;
  return log_value(P, e, true, lane, gen, cnt);
}

__device__ __forceinline__ u32 log_value(const Dev &P, u64 rip, bool mine, u32 lane, u32 gen, u32 cnt) {
  if (!mine) return cnt;
  const u32 H = P.H;
  const u64 base = (u64)lane * H;
  u32 h = (u32)mix64(rip) & (H - 1);
  for (u32 probe = 0; probe < H; probe++) {
    const u64 idx = base + h;
    if (P.cov_gen[idx] != gen) {
      if (cnt >= H - H / 4) {  // keep probes short: a full set drops the rip
        P.cov_overflow[lane] = 1;
        return cnt;
      }
      P.cov_rip[idx] = rip;
      P.cov_gen[idx] = gen;
      return cnt + 1;
    }
    if (P.cov_rip[idx] == rip) return cnt;
    h = (h + 1) & (H - 1);
  }
  return cnt;
}

// Uniform fetch of up to 16 bytes at page pointer p (within one page).
__device__ __forceinline__ void fetch_bytes(u64 pageptr, u32 off, u32 n, u64 &lo, u64 &hi) {
  // n <= 16 and off + n <= 4096
  const u64 a = (pageptr + off) & ~7ull;
  const u32 sh = (u32)((pageptr + off) & 7);
  const u64 pend = pageptr + WTFGPU_PAGE_SIZE;
  const u64 w0 = rfl64(*(const u64 *)a);
  const u64 w1 = (a + 8 < pend) ? rfl64(*(const u64 *)(a + 8)) : 0;
  const u64 w2 = (a + 16 < pend) ? rfl64(*(const u64 *)(a + 16)) : 0;
  if (sh == 0) {
    lo = w0;
    hi = w1;
  } else {
    lo = (w0 >> (8 * sh)) | (w1 << (64 - 8 * sh));
    hi = (w1 >> (8 * sh)) | (w2 << (64 - 8 * sh));
  }
  if (n < 16) {
    if (n <= 8) {
      hi = 0;
      lo = n == 8 ? lo : (lo & ((1ull << (8 * n)) - 1));
    } else {
      hi &= (1ull << (8 * (n - 8))) - 1;
    }
  }
}

// ---------------------------------------------------------------- decoded-uop cache
// Per wave, in LDS, for the lifetime of one k_run launch. Key = page pointer |
// offset of the instruction's first byte; only pages of the read-only snapshot
// pool are cached (a lane's overlay copy can be rewritten by the guest). An
// entry holds the decoded UOp (generic path), its FOp digest (fast path), the
// breakpoint lookup (the set is fixed during a launch), whether the rip is
// already in the aggregate coverage map, and the lanes this wave has already
// logged for it in this launch.
#ifndef WTFGPU_UC_N
#define WTFGPU_UC_N 312  // head-only entries (the UOp lives in the uop slots below)
#endif
// entries per wave: 4 waves x 312 x 64 bytes + the uop slots = 81,792 bytes a
// block, two blocks per CU in 160 KiB (256 entries: tlv's fill passes 16 % of
// wave-steps, 312: 12 %; profiles/r05_stamps_ucindex_ab.txt)
constexpr u32 UC_N = WTFGPU_UC_N;
#ifndef WTFGPU_FILL_INLINE
#define WTFGPU_FILL_INLINE 1  // k_run's fills take the shared-cache hit path inline (uc_fill_shared)
#endif
#ifndef WTFGPU_UC_U
#define WTFGPU_UC_U 4  // 4 x 120 bytes per wave: k_run's LDS (uop cache + lane copies) fits 160 KiB
#endif
constexpr u32 UC_U = WTFGPU_UC_U;  // uop slots per wave (power of two)
constexpr u32 UC_BP = 1, UC_COVERED = 2, UC_CROSS = 4, UC_BADLEN = 8, UC_UNSUP = 16;
struct UCHead {
  u64 key;
  u64 logged;
  u32 flags, pad;
  FOp f;
};
// What the fast loop reads: one LDS entry per cached rip (64 bytes, so a wave
// keeps UC_N of them within the CU's LDS budget at two blocks per CU).
struct UCEntry {
  union {
    UCHead h;
    struct {
      u64 key;
      u64 logged;
      u32 flags, pad;
      FOp f;
    };
  };
  u64 rip;  // the rip that filled it (a warm image re-checks UC_COVERED with it)
};
// The decoded UOp, which only the slow step's generic exec needs: a few
// slots per wave, refilled from the shared cache (or decoded) on demand.
struct UCUop {
  u64 key;
  UOp u;
};
// The shared (device-wide) cache's payload: static flags, FOp, UOp.
struct GPayload {
  u32 flags, pad;
  FOp f;
  UOp u;
};
constexpr u32 GP_HEAD = (sizeof(u32) * 2 + sizeof(FOp)) / 4;  // dwords of flags, pad, FOp
static_assert(sizeof(UOp) % 4 == 0 && sizeof(FOp) % 4 == 0, "copied as dwords");
static_assert(sizeof(UCEntry) == 64, "LDS entry size");
// Warm start: at the end of a launch, every hardware wave stores its LDS uop
// cache as an image; at the start of the next launch on the same queue, wave
// w loads image w (logged masks cleared, UC_COVERED
// re-checked against the coverage map) instead of starting empty. UC_COVERED
// stays true until the coverage map is reset; images are dropped with the
// shared cache (pool, breakpoints, edges / trace) and on a coverage reset.
// One image per wave a launch can have (Dev::warm_n per queue): regrouping
// keeps lanes in rip order, so wave w of the next launch runs much the code
// wave w ran (measured: 64 shared images left tlv's fills at a fifth of
// wave-steps). 16 KB a wave: 32 MB a queue at 131,072 lanes.
constexpr u32 UC_QUEUES = 2;
constexpr u64 UC_IMAGE_BYTES = (u64)UC_N * sizeof(UCEntry);

// WTFGPU_UC_WAYS = 2: two-way sets (entries 2s, 2s + 1), a fill replaces
// way 1 (WTFGPU_UC_MRU) or the way a per-wave counter picks; tlv's 228-instruction loop missed a fifth of
// its wave-steps direct-mapped (scripts: a trace replay gives 23 % direct,
// 14 % two-way at 256 entries).
#ifndef WTFGPU_UC_WAYS
#define WTFGPU_UC_WAYS 2
#endif
constexpr u32 UC_WAYS = WTFGPU_UC_WAYS;
static_assert(UC_N % UC_WAYS == 0, "whole sets");
// WTFGPU_UC_MRU = 1: a fill takes way 0 and moves the old way 0 to way 1, so
// the fast loop's first LDS read finds the newer entry (SYN 4 % shorter
// launches than a counter-picked way; fill passes unchanged)
#ifndef WTFGPU_UC_MRU
#define WTFGPU_UC_MRU 1
#endif
__device__ __forceinline__ bool cacheable_key(u64 lptr, u64 pool_lo, u64 pool_span) {
  return !m_ge64(lptr - pool_lo, pool_span);
}
__device__ __forceinline__ u32 uc_slot(u64 key) {
  if (UC_WAYS == 1) return (u32)((key ^ (key >> 12) * 0x9E3779B1u) % UC_N);
  // multiplicative hash: the offset bits mix into the set index too
  // a 32-bit multiplicative hash (the page bits above 4 GiB folded in), its
  // high bits scaled to the set count by one s_mul_hi (any count); cheaper
  // than the 64-bit product and fewer tlv fill passes (13.0 -> 11.1 %)
  const u32 h = ((u32)key ^ (u32)(key >> 17)) * 0x9E3779B1u;
  return __umulhi(h, UC_N / UC_WAYS) * UC_WAYS;
}
__device__ __forceinline__ u32 uu_slot(u64 key) { return (u32)((key ^ (key >> 12) * 0x9E3779B1u) & (UC_U - 1)); }

template <typename T>
__device__ __forceinline__ void lds_uniform_read(const T *src, T &dst) {
  const u32 *s = (const u32 *)src;
  u32 *d = (u32 *)&dst;
#pragma unroll
  for (u32 i = 0; i < sizeof(T) / 4; i++) d[i] = rfl32(s[i]);
}

// The uop-cache head as the fast loop reads it (wave-uniform): key, flags
// and the FOp words fast_exec uses (not `logged` or the pads).
__device__ __forceinline__ void uc_head_read(const UCEntry *e, UCHead &h) {
  h.key = rfl64(e->key);
  h.flags = rfl32(e->flags);
  h.f.w0 = rfl32(e->f.w0);
  h.f.fl = rfl32(e->f.fl);
  h.f.w2 = rfl32(e->f.w2);
  h.f.disp = rfl64(e->f.disp);
  h.f.imm = rfl64(e->f.imm);
}

__device__ __forceinline__ bool bp_lookup(const Dev &P, u64 rip) {
  u32 s;
  return P.bp_keys && hash_find(P.bp_keys, P.bp_mask, rip, s);
}

// Fill one entry (uniform): fetch + decode from the pool page, digest, lookups.
// Write len bytes at gpa into the lane's overlay (copy-on-write + dirty).
__device__ __forceinline__ bool lane_phys_write(const Dev &P, Lane &L, u64 gpa, const u8 *src, u64 len) {
  while (len) {
    const u64 off = gpa & 0xfff;
    u64 n = 4096 - off;
    if (n > len) n = len;
    bool priv;
    const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, gpa >> 12, priv);
    u8 *dst = (u8 *)pg;
    if (!priv) {
      if (L.ovn >= P.K) return false;
      dst = cow_copy(P, L.lane, L.ovn, gpa >> 12, pg);
      L.ovn++;
      L.bloom |= bloom_bit(gpa >> 12);
    }
    for (u64 i = 0; i < n; i++) dst[off + i] = src[i];
    src += n;
    gpa += n;
    len -= n;
  }
  return true;
}

// One aligned 64-bit word at gpa (copy-on-write + dirty).
__device__ __forceinline__ bool lane_phys_write64(const Dev &P, Lane &L, u64 gpa, u64 v) {
  bool priv;
  const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, gpa >> 12, priv);
  u8 *dst = (u8 *)pg;
  if (!priv) {
    if (L.ovn >= P.K) return false;
    dst = cow_copy(P, L.lane, L.ovn, gpa >> 12, pg);
    L.ovn++;
    L.bloom |= bloom_bit(gpa >> 12);
  }
  *(u64 *)(dst + (gpa & 0xfff)) = v;
  return true;
}

// ---------------------------------------------------------------- exception delivery
// A fault is delivered through the guest IDT when the snapshot has a present
// 64-bit interrupt / trap gate for it (SDM vol. 3 6.12-6.14): stack switch to
// TSS.RSP0 / IST on a privilege change, SS:RSP, RFLAGS, CS:RIP and the error
// code pushed, IF cleared for interrupt gates, cr2 set for #PF. Otherwise (no
// IDT: the ring-3 snapshots; a nested fault while delivering) the lane exits
// with the fault as before.
__device__ __forceinline__ bool has_error_code(u32 vec) {
  return vec == 8 || (vec >= 10 && vec <= 14) || vec == 17 || vec == 21 || vec == 29 || vec == 30;
}
__device__ __forceinline__ bool sup_xlate(const Dev &P, Lane &L, u64 va, int acc, u64 &gpa) {
  u64 td, gpfn;
  if (!walk(P, L, va, acc, td, gpfn)) return false;
  gpa = (gpfn << 12) | (va & 0xfff);
  return true;
}
__device__ __noinline__ bool deliver_fault(const Dev &P, Lane &L) {
  LaneSys &S = P.sys[L.lane];
  const u32 vec = L.exvec, err = L.exerr;
  const u64 cr2 = L.exaddr, frip = L.rip;
  const u32 st0 = L.status, cpl0 = L.cpl;
  bool ok = false;
  do {
    // a fault before any instruction retired since the last delivery (the
    // handler itself faults at once) ends as an exit: the double / triple fault
    // a CPU would raise (U18)
    if (S.deliv_icount == L.icount) break;
    if (!S.idtr || vec > 31 || (u64)vec * 16 + 15 > S.idtr_limit) break;
    u64 ga;
    if (!sup_xlate(P, L, S.idtr + vec * 16, ACC_R, ga) || (ga & 0xfff) > 4096 - 16) break;
    bool priv;
    const u8 *g = phys_page(P, L.lane, L.ovn, L.bloom, ga >> 12, priv) + (ga & 0xfff);
    const u64 lo = *(const u64 *)g, hi = *(const u64 *)(g + 8);
    const u32 attr = (u32)(lo >> 40) & 0xff, type = attr & 0xf, ist = (u32)(lo >> 32) & 7;
    if (!(attr & 0x80) || (type != 0xe && type != 0xf)) break;
    const u64 target = (lo & 0xffff) | ((lo >> 32) & 0xffff0000ull) | (hi << 32);
    const u16 sel = (u16)((lo >> 16) & 0xffff);
    const u32 ncpl = sel & 3;
    if (!canonical(target) || ncpl > L.cpl) break;
    u64 rsp = R(L, 4);
    if (ist || ncpl < L.cpl) {  // TSS64: RSP0 at +4, IST1 at +0x24
      const u64 off = ist ? 0x24 + (u64)(ist - 1) * 8 : 4 + (u64)ncpl * 8;
      u64 ta;
      if (!sup_xlate(P, L, S.tss + off, ACC_R, ta) || (ta & 0xfff) > 4096 - 8) break;
      const u8 *t = phys_page(P, L.lane, L.ovn, L.bloom, ta >> 12, priv) + (ta & 0xfff);
      u64 v = 0;
      for (int i = 0; i < 8; i++) v |= (u64)t[i] << (8 * i);
      rsp = v;
    }
    rsp &= ~0xfull;
    const bool ec = has_error_code(vec);
    const u32 n = ec ? 6 : 5;
    const u64 ors = R(L, 4), orfl = L.rflags, ocs = S.cs, oss = S.ss;
    L.cpl = 0;  // implicit supervisor accesses
    bool wr = true;
    // frame words, lowest address first: [error], rip, cs, rflags, rsp, ss
    for (u32 i = 0; i < n && wr; i++) {
      const u32 k = ec ? i : i + 1;
      const u64 w = k == 0 ? (u64)err : k == 1 ? frip : k == 2 ? ocs : k == 3 ? orfl : k == 4 ? ors : oss;
      u64 pa;
      wr = sup_xlate(P, L, rsp - 8 * n + 8 * i, ACC_W, pa) && (pa & 7) == 0 && lane_phys_write64(P, L, pa, w);
    }
    if (!wr) break;
    if (ncpl < cpl0) S.ss = (u16)ncpl;  // SS := NULL selector at the new privilege level
    set_cs(L, S, sel);
    if (vec == WTFGPU_VEC_PF) S.cr2 = cr2;
    L.cpl = S.cpl = ncpl;
    S.deliv_icount = L.icount;
    RS(L, 4, rsp - 8 * n);
    L.rflags &= ~(0x100ull | 0x4000ull | 0x10000ull | 0x20000ull | (type == 0xe ? 0x200ull : 0));
    L.rip = target;
    L.status = WTFGPU_RUNNING;
    // the frame pushes may have copied the stack page and the cpl changed:
    // drop cached translations now (the handler may run in the fast loop)
    tlb_flush(L);
    L.flush = 0;
    ok = true;
  } while (0);
  if (!ok) {  // keep the original fault
    L.cpl = cpl0;
    L.status = st0;
    L.exvec = vec;
    L.exerr = err;
    L.exaddr = cr2;
    L.nodeliver = 1;
  }
  return ok;
}

constexpr u32 GUC_WORDS = 48;                                  // 3 lines x 16 dwords
constexpr u32 GUC_PAYLOAD = sizeof(GPayload) / 4;  // flags, pad, FOp, UOp
static_assert(GUC_PAYLOAD <= 3 * 14, "global uop cache entry: 3 lines of 14 payload dwords");
__device__ __forceinline__ u32 guc_slot(const Dev &P, u64 key) {
  return (u32)(mix64(key) & P.guc_mask);
}
// payload dword of lane lid (lines of 16 dwords: 14 payload, 2 key tag), or ~0u
__device__ __forceinline__ u32 guc_payload_index(u32 lid) {
  return (lid < GUC_WORDS && (lid & 15) < 14) ? (lid >> 4) * 14 + (lid & 15) : ~0u;
}

// COVERED: the rip's byte in the aggregate coverage map is set (dynamic: not
// part of a shared entry)
__device__ __forceinline__ u32 covered_flag(const Dev &P, u64 rip, u32 off) {
  if (P.code_keys) {
    u32 s;
    if (hash_find(P.code_keys, P.code_mask, rip >> 12, s)) {
      const u32 cs = rfl32(P.code_slot[s]);
      if (rfl32(P.cov_map[(u64)cs * WTFGPU_PAGE_SIZE + off])) return UC_COVERED;
    }
  }
  return 0;
}

// The same per lane (non-uniform rips: a warm image's entries).
__device__ __forceinline__ u32 covered_flag_lane(const Dev &P, u64 rip, u32 off) {
  if (!P.code_keys) return 0;
  u32 h = (u32)mix64(rip >> 12) & P.code_mask;
  for (u32 i = 0; i <= P.code_mask; i++) {
    const u64 k = P.code_keys[h];
    if (k == (rip >> 12)) return P.cov_map[(u64)P.code_slot[h] * WTFGPU_PAGE_SIZE + off] ? UC_COVERED : 0;
    if (k == EMPTY_KEY) return 0;
    h = (h + 1) & P.code_mask;
  }
  return 0;
}

// The FOp of an instruction that always runs in the slow step (its length kept).
__device__ __forceinline__ FOp generic_fop(const UOp &d) {
  FOp f{};
  f.w0 = (d.len & 0x3f) << 20;
  return f;
}

// The shared (device-wide) cache's side of a fill (uniform): one dword per
// lane, the six tag dwords checked; on a hit the head goes to `e` (when
// given) and the UOp to the uop slot `us`. Inline at k_run's fill site (a
// fill is about a fifth of tlv's wave-steps, and a call spills the caller's
// live registers); false = a miss, uc_fill decodes.
__device__ __forceinline__ bool uc_fill_shared(const Dev &P, UCEntry *e, UCUop *us, u64 key, u32 off, u64 rip,
                                               u32 lid) {
  if (!P.guc) return false;
  const u32 pj = guc_payload_index(lid);
  u32 *head = e ? (u32 *)&e->flags : nullptr, *uop = us ? (u32 *)&us->u : nullptr;  // us null: the head only
  u32 *gw = P.guc + (u64)guc_slot(P, key) * GUC_WORDS;
  const u32 w = lid < GUC_WORDS ? gw[lid] : 0;
  const bool tag = lid < GUC_WORDS && (lid & 15) >= 14;
  const bool bad = tag && w != ((lid & 1) ? (u32)(key >> 32) : (u32)key);
  if (__ballot(bad) != 0) return false;
  if (pj < GP_HEAD) {
    if (head) head[pj] = w;
  } else if (pj < GUC_PAYLOAD) {
    if (uop) uop[pj - GP_HEAD] = w;
  }
  // UC_COVERED is cached in the shared entry once seen (coverage only grows
  // until wtfgpu_reset_coverage, which clears the shared cache): most fills
  // skip the map lookup's dependent loads
  const u32 sflags = __builtin_amdgcn_readlane(w, 0);
  u32 flags = sflags;
  if (e && !(sflags & UC_COVERED)) {
    flags |= covered_flag(P, rip, off);
    if ((flags & UC_COVERED) && lid == 0) gw[0] = flags;
  }
  __builtin_amdgcn_wave_barrier();
  if (lid == 0) {
    if (us) us->key = key;
    if (e) {
      e->logged = 0;
      e->flags = flags;
      e->rip = rip;
      e->key = key;
    }
  }
  return true;
}

// Fill one entry (uniform): from the shared cache when it holds the key, else
// fetch + decode from the pool page, digest, lookups, and publish. The head
// goes to `e` (when given), the UOp to the uop slot `us`.
__device__ __noinline__ void uc_fill(const Dev &P, UCEntry *e, UCUop *us, u64 key, u64 lptr, u32 off, u64 rip,
                                     u32 lid, bool shared_checked = false) {
  const u32 pj = guc_payload_index(lid);
  u32 *uop = (u32 *)&us->u;
  if (!shared_checked && uc_fill_shared(P, e, us, key, off, rip, lid)) return;
  u32 *gw = P.guc ? P.guc + (u64)guc_slot(P, key) * GUC_WORDS : nullptr;
  IBytes ib;
  ib.avail = 4096 - off < 16 ? 4096 - off : 16;
  fetch_bytes(lptr, off, ib.avail, ib.lo, ib.hi);
  UOp d;
  const int dr = decode(ib, d);
  u32 flags = dr == 1 ? UC_CROSS : dr == 2 ? UC_BADLEN : 0;
  FOp f;
  if (dr == 0) {
    digest(d, f);
    if (P.edges && edge_op(d.op, d.bsrc)) f = generic_fop(d);  // branches whose edge is recorded run in the slow step
    if (P.trace || g_tn.buf) f = generic_fop(d);               // traced lanes log every rip in the slow step
    if (!d.supported) flags |= UC_UNSUP;
    if (bp_lookup(P, rip)) flags |= UC_BP;
  } else {
    f = FOp{};
  }
  const u32 dyn = (dr == 0 && e) ? covered_flag(P, rip, off) : 0;
  if (lid == 0) {
    us->u = d;
    us->key = key;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (gw) {  // publish (static flags only); one coalesced store of 3 tagged lines
    u32 v = 0;
    if (pj < GP_HEAD) v = pj == 0 ? (flags | dyn) : pj == 1 ? 0u : ((const u32 *)&f)[pj - 2];
    else if (pj < GUC_PAYLOAD) v = uop[pj - GP_HEAD];
    else if (lid < GUC_WORDS && (lid & 15) >= 14) v = (lid & 1) ? (u32)(key >> 32) : (u32)key;
    if (lid < GUC_WORDS) gw[lid] = v;
  }
  if (lid == 0 && e) {
    e->logged = 0;
    e->f = f;
    e->flags = flags | dyn;
    e->rip = rip;
    e->key = key;
  }
}

// The UOp of `key` in the wave's uop slots (the slow step's generic path).
__device__ __forceinline__ const UOp *uc_uop(const Dev &P, UCUop *uu, u64 key, u64 lptr, u32 off, u64 rip, u32 lid) {
  UCUop *us = &uu[uu_slot(key)];
  if (rfl64(us->key) != key) uc_fill(P, nullptr, us, key, lptr, off, rip, lid);
  return &us->u;
}

// Instruction-page translation for lanes whose code-page cache missed.
__device__ __noinline__ void code_xlate(const Dev &P, Lane &L, u64 rip) {
  u64 td;
  const u64 vpn = rip >> 12;
  if (!tlb_get(L, vpn, td) || !perm_ok(L, td, ACC_X)) {
    if (service_miss(P, L, rip & ~0xfffull, ACC_X)) tlb_get(L, vpn, td);
    else td = 0;
    if (td && !perm_ok(L, td, ACC_X)) td = 0;
    if (!td && L.status == WTFGPU_EXIT_FAULT) L.exaddr = rip;
  }
  if (td) {
    L.cvpn = vpn;
    L.cptr = (td & ~0xfffull) | (L.efer & EFER_M32);  // 32-bit code: outside the pool (U29)
  }
}

__device__ __noinline__ bool miss_service(const Dev &P, Lane &L, int attempt) {
  if (attempt >= 16 || !service_miss(P, L, L.miss_va, (int)L.miss_acc)) {
    if (attempt >= 16) set_fault(L, WTFGPU_VEC_GP, 0xffff, L.miss_va);
    return false;
  }
  return true;
}

__device__ __noinline__ int exec_generic(const Dev &P, Lane &L, const UOp *ul, u64 &next) {
  UOp d;
  lds_uniform_read(ul, d);
  return exec(P, L, d, L.rip + d.len, next);
}

// The restartable attempts at one instruction on one lane copy: a TLB miss /
// first write abandons the attempt, miss_service fills the TLB or copies the
// page, the attempt reruns.
__device__ __noinline__ int exec_retry(const Dev &P, Lane &L, const UOp *ul, u64 &next) {
  int x;
  tn_insn_begin(L.lane);
  for (int attempt = 0;; attempt++) {
    L.miss = 0;
    L.pend = 0;
    tn_rollback(L.lane);
    x = exec_generic(P, L, ul, next);
    if (!L.miss || L.status != WTFGPU_RUNNING) break;
    if (!miss_service(P, L, attempt)) break;
  }
  return x;
}

// Retire / exit bookkeeping after the last attempt at an instruction.
__device__ __forceinline__ void retire(const Dev &P, Lane &L, int x, u32 len, u64 next, u32 opbytes) {
  if (L.flush) {
    tlb_flush(L);
    L.flush = 0;
  }
  if ((x == X_OK || x == X_CR3) && L.status == WTFGPU_RUNNING) {
    L.rip = next;
    L.icount++;
    L.nbytes += len + L.pend;
    if (P.limit && L.icount > P.limit) L.status = WTFGPU_EXIT_TIMEOUT;
    else if (x == X_CR3) L.status = WTFGPU_EXIT_CR3;  // bochscpu_backend.cc:628-657 (U20)
  } else if (L.status != WTFGPU_RUNNING) {
    // faulted / overlay full inside exec or service_miss; rip unchanged
  } else if (x == X_UNIMPL) {
    L.status = WTFGPU_EXIT_UNIMPLEMENTED;
    L.exop = len >= 4 ? opbytes : (opbytes & ((1u << (8 * len)) - 1));
  } else if (x == X_INT3) {
    L.status = WTFGPU_EXIT_INT3;
  } else if (x == X_HLT) {
    L.status = WTFGPU_EXIT_HLT;
  }
}

// FEED action: the next chunk of the lane's feed goes to gpr[b] + window -
// size, as fuzzer_tlv_server.cc:83-166 writes the next packet. Writes go
// through the copy-on-write path (the pages are dirtied as VirtWriteDirty
// does). A missing page ends the lane with WTFGPU_EXIT_FEED_FAULT, where the
// module's handler aborts.
// A host-side VirtWriteDirty of n bytes at va (backend.cc:91-121): page by page,
// the stores run as supervisor with CR0.WP clear (translation with
// ValidateRead: only a missing translation stops it, U/S and R/W are not
// checked), through copy-on-write. false = a page did not translate (the
// pages before it are written, as VirtWrite leaves them): the lane ends with
// WTFGPU_EXIT_FEED_FAULT (the host handler's failed write, U43).
__device__ __noinline__ bool host_write(const Dev &P, Lane &L, u64 va, const u8 *__restrict__ src, u64 n) {
  const u32 cpl0 = L.cpl;
  const u64 cr00 = L.cr0;
  L.cpl = 0;
  L.cr0 &= ~(1ull << 16);
  bool ok = true;
  // page by page, as VirtWrite does: translate (copy-on-write on the first
  // write), then copy the page's part, 32 source bytes loaded per round
  for (u64 o = 0; o < n;) {
    const u64 a = va + o, room = 4096 - (a & 0xfff);
    const u32 m = (u32)(n - o < room ? n - o : room);
    u8 *d = nullptr;
    u64 td = 0;
    for (int attempt = 0;; attempt++) {
      L.miss = 0;
      if ((d = xlate(L, a, ACC_W, &td))) break;
      if (L.status != WTFGPU_RUNNING || !L.miss || !miss_service(P, L, attempt)) {
        ok = false;
        break;
      }
    }
    if (!ok) break;
    if (td & T_PT) L.flush = 1;  // a page-table page: cached translations go
    const u8 *__restrict__ sp = src + o;
    u32 k = 0;
    for (; k + 32 <= m; k += 32) {
      u8 t[32];
#pragma unroll
      for (u32 j = 0; j < 32; j++) t[j] = sp[k + j];
#pragma unroll
      for (u32 j = 0; j < 32; j++) d[k + j] = t[j];
    }
    for (; k < m; k++) d[k] = sp[k];
    o += m;
  }
  if (!ok) {
    if (L.status == WTFGPU_RUNNING || L.status == WTFGPU_EXIT_FAULT) L.status = WTFGPU_EXIT_FEED_FAULT;
    L.miss = 0;
  }
  L.cpl = cpl0;
  L.cr0 = cr00;
  L.pend = 0;
  if (ok && L.flush) {
    tlb_flush(L);
    L.flush = 0;
  }
  return ok;
}

__device__ __noinline__ bool feed_apply(const Dev &P, Lane &L, const wtfgpu_bp_action_t &a) {
  if (!P.feed_pos) return false;
  const u64 pos = P.feed_pos[L.lane];
  if (pos == ~0ull) return false;  // no feed: the host handler serves the lane
  const u64 end = P.feed_end[L.lane];
  if (pos + 4 > end) {
    L.status = WTFGPU_EXIT_STOP_OK;
    return true;
  }
  const u8 *src = P.feed_data + pos;
  const u32 n = (u32)src[0] | ((u32)src[1] << 8) | ((u32)src[2] << 16) | ((u32)src[3] << 24);
  P.feed_pos[L.lane] = pos + 4 + n;
  if (n >= a.value || pos + 4 + n > end) {
    L.status = WTFGPU_EXIT_STOP_OK;
    return true;
  }
  const u32 rb = (u32)a.gprs[0] & 15, rn = (u32)a.gprs[1] & 15;
  const u64 dst = R(L, rb) + a.value - n;
  if (!host_write(P, L, dst, src + 4, n)) return true;  // WTFGPU_EXIT_FEED_FAULT
  RS(L, rn, n);
  RS(L, rb, dst);
  return true;
}

// Declared insert (wtfgpu_set_insert; the data form of fuzzer_hevd.cc:20-59's
// InsertTestcase): the lane's feed holds one chunk, the testcase; its first 4
// bytes go to gpr[head_reg], the rest (the payload) is written at
// gpr[ptr_reg], its size goes to gpr[len_reg] and, with len_arg, to
// [rsp + 8 + 8 * len_arg] (GetArgAddress, backend.cc:160-168), in the order
// the module does it. The feed is consumed. A write that does not translate
// ends the lane with WTFGPU_EXIT_FEED_FAULT, where the host handler would
// have failed (U43).
__device__ __noinline__ void insert_apply(const Dev &P, Lane &L, const wtfgpu_insert_t &ins) {
  const u64 pos = P.feed_pos[L.lane], end = P.feed_end[L.lane];
  if (pos == ~0ull) return;
  P.feed_pos[L.lane] = end;
  if (pos + 8 > end) return;
  const u8 *src = P.feed_data + pos;
  const u32 n = (u32)src[0] | ((u32)src[1] << 8) | ((u32)src[2] << 16) | ((u32)src[3] << 24);
  if (n < 4 || pos + 4 + n > end) return;
  const u32 head = (u32)src[4] | ((u32)src[5] << 8) | ((u32)src[6] << 16) | ((u32)src[7] << 24);
  const u64 m = n - 4;
  RS(L, ins.head_reg & 15, head);
  if (!host_write(P, L, R(L, ins.ptr_reg & 15), src + 8, m)) return;
  RS(L, ins.len_reg & 15, m);
  if (ins.len_arg) {
    u8 le[8];
    for (int i = 0; i < 8; i++) le[i] = (u8)(m >> (8 * i));
    host_write(P, L, R(L, WTFGPU_RSP) + 8 + 8 * (u64)ins.len_arg, le, 8);
  }
}

// Device-side breakpoint action (wtfgpu_set_breakpoint_actions) at `grip`.
// true = applied, the lane keeps running at its new rip; false = none
// declared or it could not be applied: the lane exits to the host handler,
// registers untouched. RETURN reads [rsp] as the host's
// SimulateReturnFromFunction does (backend.cc:129-146); a read that would fault
// is left to the host path, whose translation decides the outcome.
// BLAKE3 of an 8-byte input, first 16 output bytes (one chunk, one block:
// CHUNK_START | CHUNK_END | ROOT), for Rdrand's chain.
__device__ __forceinline__ u32 rotr32(u32 x, u32 n) { return (x >> n) | (x << (32 - n)); }
__device__ __forceinline__ void b3_g(u32 *v, int a, int b, int c, int d, u32 x, u32 y) {
  v[a] = v[a] + v[b] + x;
  v[d] = rotr32(v[d] ^ v[a], 16);
  v[c] = v[c] + v[d];
  v[b] = rotr32(v[b] ^ v[c], 12);
  v[a] = v[a] + v[b] + y;
  v[d] = rotr32(v[d] ^ v[a], 8);
  v[c] = v[c] + v[d];
  v[b] = rotr32(v[b] ^ v[c], 7);
}
__device__ __noinline__ void blake3_le64(u64 in, u64 &lo, u64 &hi) {
  const u32 iv[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                     0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
  const u8 perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  u32 m[16] = {(u32)in, (u32)(in >> 32), 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  u32 v[16] = {iv[0], iv[1], iv[2], iv[3], iv[4], iv[5], iv[6], iv[7], iv[0], iv[1], iv[2], iv[3], 0, 0, 8, 1 | 2 | 8};
  for (int r = 0; r < 7; r++) {
    b3_g(v, 0, 4, 8, 12, m[0], m[1]);
    b3_g(v, 1, 5, 9, 13, m[2], m[3]);
    b3_g(v, 2, 6, 10, 14, m[4], m[5]);
    b3_g(v, 3, 7, 11, 15, m[6], m[7]);
    b3_g(v, 0, 5, 10, 15, m[8], m[9]);
    b3_g(v, 1, 6, 11, 12, m[10], m[11]);
    b3_g(v, 2, 7, 8, 13, m[12], m[13]);
    b3_g(v, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      u32 t[16];
      for (int i = 0; i < 16; i++) t[i] = m[perm[i]];
      for (int i = 0; i < 16; i++) m[i] = t[i];
    }
  }
  lo = (u64)(v[0] ^ v[8]) | ((u64)(v[1] ^ v[9]) << 32);
  hi = (u64)(v[2] ^ v[10]) | ((u64)(v[3] ^ v[11]) << 32);
}

__device__ __forceinline__ bool bp_apply_action(const Dev &P, Lane &L, u64 grip, const wtfgpu_bp_action_t *found) {
  u32 s;
  if (!found && (!P.act_keys || !hash_find(P.act_keys, P.act_mask, grip, s))) return false;
  const wtfgpu_bp_action_t &a = found ? *found : P.act[s];
  if (a.kind == WTFGPU_BPACT_SET_GPRS) {
    for (u32 i = 0; i < 16; i++) RS(L, i, a.gprs[i]);
    L.rip = a.gprs[16];
    return true;
  }
  if (a.kind == WTFGPU_BPACT_FEED) return feed_apply(P, L, a);
  if (a.kind == WTFGPU_BPACT_STOP_OK) {
    L.status = WTFGPU_EXIT_STOP_OK;
    return true;
  }
  if (a.kind == WTFGPU_BPACT_RDRAND) {  // Rdrand (bochscpu_backend.cc:874-885); the instruction then runs
    if (!P.rd_seed) return false;
    u64 lo, hi;
    blake3_le64(P.rd_seed[L.lane], lo, hi);
    P.rd_seed[L.lane] = lo;
    RS(L, (u32)a.gprs[0] & 15, hi);
    return true;
  }
  if (a.kind == WTFGPU_BPACT_STOP_ARGS) {  // Win64 arguments 0..5 (backend.cc:168-192), then stop
    if (!P.stop_args) return false;
    const u64 rsp = R(L, WTFGPU_RSP);
    u64 v[6] = {R(L, 1), R(L, 2), R(L, 8), R(L, 9), 0, 0};
    for (u32 i = 4; i < 6 && i < a.value; i++) {
      for (int attempt = 0;; attempt++) {
        L.miss = 0;
        if (vread(L, rsp + 8 + 8 * (u64)i, 8, v[i])) break;
        if (L.status != WTFGPU_RUNNING || !L.miss || !miss_service(P, L, attempt)) {
          L.status = WTFGPU_RUNNING;  // undo a fault: the host handler decides
          L.miss = 0;
          L.pend = 0;
          return false;
        }
      }
    }
    L.pend = 0;
    for (u32 i = 0; i < 6; i++) P.stop_args[(u64)L.lane * 6 + i] = i < a.value ? v[i] : 0;
    L.status = WTFGPU_EXIT_STOP_ARGS;
    return true;
  }
  if (a.kind != WTFGPU_BPACT_RETURN) return false;
  if (a.gprs[0]) {
    // the handler first reads a C string at gpr[gprs[0] - 1], at most gprs[1]
    // bytes (VirtReadString, backend.h:333-430): a byte that does not
    // translate before the terminator leaves the hit to the host handler,
    // whose read then decides (U43)
    // (read as aligned 32-byte blocks, the four words of a block loaded at
    // once: a block never crosses a page, so it translates exactly when the
    // first byte of it the scan needs does)
    const u64 s = R(L, (u32)(a.gprs[0] - 1) & 15);
    const u64 lim = a.gprs[1];
    for (u64 i = 0; i < lim;) {
      const u64 va = s + i, al = va & ~31ull;
      const u8 *p = nullptr;
      for (int attempt = 0;; attempt++) {
        L.miss = 0;
        if ((p = xlate(L, al, ACC_R))) break;
        if (L.status != WTFGPU_RUNNING || !L.miss || !miss_service(P, L, attempt)) {
          L.status = WTFGPU_RUNNING;  // undo a fault: the host handler decides
          L.miss = 0;
          return false;
        }
      }
      const u64 *w = (const u64 *)p;
      const u64 c0 = w[0], c1 = w[1], c2 = w[2], c3 = w[3];
      bool term = false;
      for (u32 b = (u32)(va - al); b < 32 && i < lim && !term; b++, i++) {
        const u64 c = b < 8 ? c0 : b < 16 ? c1 : b < 24 ? c2 : c3;
        term = ((c >> (8 * (b & 7))) & 0xff) == 0;
      }
      if (term) break;
    }
  }
  const u64 rsp = R(L, WTFGPU_RSP);
  u64 ra = 0;
  for (int attempt = 0;; attempt++) {
    L.miss = 0;
    if (vread(L, rsp, 8, ra)) break;
    if (L.status != WTFGPU_RUNNING || !L.miss || !miss_service(P, L, attempt)) {
      L.status = WTFGPU_RUNNING;  // undo a fault: the host handler decides
      L.miss = 0;
      L.pend = 0;
      return false;
    }
  }
  L.pend = 0;
  RS(L, WTFGPU_RAX, a.value);
  RS(L, WTFGPU_RSP, rsp + 8);
  L.rip = ra;
  return true;
}

// The action stands in for a host handler, whose guest-memory reads and writes
// (VirtRead / VirtWrite) are no CPU accesses: Tenet does not log them
// (bochscpu_backend.cc:1215-1323 logs the lin_access hook only).
// found: the action k_run already looked up (nullptr: look it up)
__device__ __noinline__ bool bp_apply(const Dev &P, Lane &L, u64 grip, const wtfgpu_bp_action_t *found = nullptr) {
  tn_mute(L.lane);
  const bool r = bp_apply_action(P, L, grip, found);
  tn_unmute(L.lane, 0, 0, 0, false);
  return r;
}

// A step the uop cache cannot serve: code on a lane overlay page, or an
// instruction that crosses into the next page (translated per lane).
__device__ __noinline__ void slow_step(const Dev &P, Lane &L, u64 grip, u64 lptr, bool ing, bool &skip) {
  const u32 off = (u32)(grip & 0xfff);
  const bool m32 = (lptr & EFER_M32) != 0;  // the group's lanes run 32-bit code (U29)
  lptr &= ~EFER_M32;
  IBytes ib;
  ib.avail = 4096 - off < 16 ? 4096 - off : 16;
  fetch_bytes(lptr, off, ib.avail, ib.lo, ib.hi);
  UOp d;
  int dr = decode(ib, d, m32);
  if (dr == 1) {
    u64 nptr = 0;
    if (ing) {
      const u64 va2 = (grip & ~0xfffull) + 4096;
      u64 td;
      if (!tlb_get(L, va2 >> 12, td) || !perm_ok(L, td, ACC_X)) {
        if (service_miss(P, L, va2, ACC_X)) tlb_get(L, va2 >> 12, td);
        else td = 0;
      }
      if (td) nptr = td & ~0xfffull;
      else ing = false;
    }
    const u64 cm = __ballot(ing);
    if (cm == 0) return;
    const int leader = __ffsll((long long)cm) - 1;
    const u64 lnptr = readlane64(nptr, leader);
    ing = ing && nptr == lnptr;
    const u32 n0 = ib.avail;
    u64 lo2, hi2;
    fetch_bytes(lnptr, 0, 16 - n0, lo2, hi2);
    // splice: bytes [0,n0) from page 1, [n0,16) from page 2
    if (n0 >= 8) {
      ib.hi = (n0 == 8 ? 0 : ib.hi) | (n0 == 8 ? lo2 : (lo2 << (8 * (n0 - 8))));
    } else {
      ib.lo = ib.lo | (lo2 << (8 * n0));
      ib.hi = (lo2 >> (64 - 8 * n0)) | (hi2 << (8 * n0));
    }
    ib.avail = 16;
    dr = decode(ib, d, m32);
  }
  if (dr == 2) {
    if (ing) set_fault(L, WTFGPU_VEC_GP, 0, 0);
    return;
  }
  const u64 gmask = __ballot(ing);
  if (gmask == 0) return;
  if (P.cov_rip) L.ccnt = cover(P, grip, ing, L.lane, L.cgen, L.ccnt);
  if (P.trace && ing && !skip) trace_rip(P, L.lane, grip);  // a resumed breakpoint was logged at its hit
  const bool isbp = bp_lookup(P, grip);
  if (ing) {
    if (isbp && !skip) {
      // breakpoint hit (bochscpu_backend.cc:545-547): device action or host exit;
      // an action that left rip unchanged runs the instruction next step (skip)
      const bool applied = bp_apply(P, L, grip);
      if (!applied) L.status = WTFGPU_EXIT_BREAKPOINT;
      skip = applied && L.rip == grip;
      if (applied && !skip && g_tn.buf) tn_regs(P, L);  // Tenet: the action moved rip
      ing = false;
    } else {
      skip = false;
    }
  }
  if (!d.supported) {
    if (ing) {
      L.status = WTFGPU_EXIT_UNIMPLEMENTED;
      L.exop = d.len >= 4 ? d.opbytes : (d.opbytes & ((1u << (8 * d.len)) - 1));
    }
    return;
  }
  if (ing) {
    u64 next = 0;
    int x;
    tn_insn_begin(L.lane);
    for (int attempt = 0;; attempt++) {
      L.miss = 0;
      L.pend = 0;
      tn_rollback(L.lane);
      x = exec(P, L, d, grip + d.len, next);
      if (!L.miss || L.status != WTFGPU_RUNNING) break;
      if (!miss_service(P, L, attempt)) break;
    }
    retire(P, L, x, d.len, next, d.opbytes);
    if (g_tn.buf && (x == X_OK || x == X_CR3)) tn_regs(P, L);
    // RecordEdge (bochscpu_backend.cc:699-728): the branch ran, whatever the retire hook decided
    if (P.edges && P.cov_rip && edge_op(d.op, d.bsrc) && x == X_OK) {
      const u32 c0 = L.ccnt;
      L.ccnt = cover_edge(P, edge_key(grip, next), true, L.lane, L.cgen, L.ccnt);
      count_edge(P, L.lane, L.ccnt != c0);
    }
  }
}

// Runs `call` on a copy T of lane L whose registers live in arrays of their
// own, so the kernel's register arrays never escape into a called function
// (they stay in VGPRs). WTFGPU_LANE_LDS picks where the copy lives:
//   2 (default) a per-lane slot in HBM (L2-resident while the lane runs),
//     which leaves LDS to a second resident wave per SIMD: k_run launches
//     take 1.25-1.35x less time per lane than with 1 (MI355X, tlv);
//   1 LDS (sLane / sRegs, one slot per thread): one wave per SIMD;
//   0 the stack, i.e. scratch, whose write-backs were most of k_run's HBM traffic.
#ifndef WTFGPU_LANE_LDS
#define WTFGPU_LANE_LDS 2
#endif
#if WTFGPU_LANE_LDS == 1
// the register slots take an odd stride (33 dwords) so a wave's copies spread
// over the LDS banks; the Lane slots (60 dwords) conflict 4-way at most
#define LANE_COPY_DECL            \
  __shared__ Lane sLane[256];     \
  __shared__ u32 sRegs[256][33];
#define LANE_COPY_SLOT                                  \
  Lane &T = sLane[threadIdx.x];                         \
  u32 *const tlo_ = sRegs[threadIdx.x], *const thi_ = sRegs[threadIdx.x] + 16;
#elif WTFGPU_LANE_LDS == 2
// in HBM, one slot per lane (L2-resident while the lane runs): the LDS the
// copy took is left to a second wave per SIMD (measured variant)
struct LaneCopy {
  Lane l;
  u32 r[32];
};
#define LANE_COPY_DECL
#define LANE_COPY_SLOT                                       \
  LaneCopy &C_ = ((LaneCopy *)P.lcopy)[lane];                \
  Lane &T = C_.l;                                            \
  u32 *const tlo_ = C_.r, *const thi_ = C_.r + 16;
#else
#define LANE_COPY_DECL
#define LANE_COPY_SLOT    \
  u32 tlo_[16], thi_[16]; \
  Lane T;
#endif
#define WITH_LANE_COPY(call)                      \
  do {                                            \
    LANE_COPY_SLOT                                \
    _Pragma("unroll") for (int i_ = 0; i_ < 16; i_++) { \
      tlo_[i_] = glo[i_];                         \
      thi_[i_] = ghi[i_];                         \
    }                                             \
    T = L;                                        \
    T.glo = tlo_;                                 \
    T.ghi = thi_;                                 \
    call;                                         \
    L = T;                                        \
    L.glo = glo;                                  \
    L.ghi = ghi;                                  \
    _Pragma("unroll") for (int i_ = 0; i_ < 16; i_++) { \
      glo[i_] = tlo_[i_];                         \
      ghi[i_] = thi_[i_];                         \
    }                                             \
  } while (0)

// Diagnostic build only (-DWTFGPU_STAMPS, `make stamps`): per-phase s_memtime
// cycle totals of the step loop, summed into stat[4..11] (never in the product).
#ifdef WTFGPU_STAMPS
#define STAMP(k)                                   \
  do {                                             \
    const u64 t_ = __builtin_amdgcn_s_memtime();   \
    stamp_[k] += t_ - tprev_;                      \
    tprev_ = t_;                                   \
  } while (0)
// why the fast loop handed the wave to the slow step, counted in stat[12..15]:
// 0 a fast attempt missed (TLB, first write, page crossing, state), 1 the
// code page changed, 2 the rip is not in the wave's LDS uop cache, 3 other
// (generic op, breakpoint, coverage, code outside the pool)
#define WHY(k) why_ = (k)
// and which generic ops the slow step executed (O_* / O_SYS2 etc.), one count per
// group, in stat[16..528): index op | why << 6 | covered << 8
#define OPHIST(op) ophist_[((op) & 63) | (why_ & 3) << 6 | ((op) & 64 ? 256 : 0)]++
constexpr u32 STAT_N = 536;  // + stat[528..535]: cycles in bp_apply by action kind
#else
constexpr u32 STAT_N = 16;
#define OPHIST(op) \
  do {             \
  } while (0)
#define STAMP(k) \
  do {           \
  } while (0)
#define WHY(k) \
  do {         \
  } while (0)
#endif

// The lanes of a per-lane `if` meet again here, before a `continue` or the
// end of the step loop's body. Without it the loop latch is the join of that
// divergent branch, which makes every value the latch merges (the step count,
// the group, `have`) divergent to the compiler, and the step loops become
// exec-masked divergent loops. No instruction is emitted.
#define RECONVERGE() __builtin_amdgcn_wave_barrier()

// ---------------------------------------------------------------- main kernel
// One hardware wave runs P.lpw lanes (64, or 32 / 16 to put more waves on
// each SIMD when the batch is small: the step loop is latency-bound).
// Build knobs (measured variants): WTFGPU_KRUN_WAVES = the
// minimum waves per SIMD the register allocation must allow; WTFGPU_P_BYREF =
// P read from device memory instead of the by-value kernel argument (which is
// copied to scratch because the rare-path functions take it by reference).
#ifndef WTFGPU_KRUN_WAVES
#define WTFGPU_KRUN_WAVES 2
#endif
#ifndef WTFGPU_FAST_REGOPS
#define WTFGPU_FAST_REGOPS 1  // register-only forms skip the fast loop's memory retry rounds
#endif
#ifndef WTFGPU_BP_RESUME_FAST
#define WTFGPU_BP_RESUME_FAST 1  // lanes resuming at a breakpoint run its instruction in the fast loop
#endif
#ifndef WTFGPU_INLINE_ACTIONS
#define WTFGPU_INLINE_ACTIONS 3  // SetGprs (1) / StopOk (2) actions applied without the lane copy
#endif
#ifndef WTFGPU_FILL_PREFETCH
#define WTFGPU_FILL_PREFETCH 8  // entries a fill pass also brings in after the missed one (profiles/r06_ab_fill_prefetch.txt)
#endif
#ifndef WTFGPU_FEED_PREFAULT
#define WTFGPU_FEED_PREFAULT 1
#endif
#ifndef WTFGPU_COVER_FAST
#define WTFGPU_COVER_FAST 1
#endif
#ifndef WTFGPU_FILL_PREFETCH_JUMPS
#define WTFGPU_FILL_PREFETCH_JUMPS 0  // the prefetch chain follows direct jmp / call targets in the page
#endif
#ifndef WTFGPU_ACT_NESTED
#define WTFGPU_ACT_NESTED 0  // the two inline actions in one nested block (the miscompiled form, A/B only)
#endif
#ifndef WTFGPU_FAST_FAULTS
#define WTFGPU_FAST_FAULTS 1  // a fast attempt whose fill would fault raises the fault itself
#endif
#ifndef WTFGPU_P_BYREF
#define WTFGPU_P_BYREF 0
#endif
#if WTFGPU_P_BYREF
__global__ __launch_bounds__(256, WTFGPU_KRUN_WAVES) void k_run(const Dev *__restrict__ Pp, u32 first, u32 count,
                                                                u64 max_steps) {
  const Dev &P = *Pp;
#else
__global__ __launch_bounds__(256, WTFGPU_KRUN_WAVES) void k_run(Dev P, u32 first, u32 count, u64 max_steps) {
#endif
  if (P.perm && rfl64(P.stat[3]) == 0) return;  // regrouped launch with no running lane
  const u32 lid = threadIdx.x & 63;
  const u32 hw = rfl32(blockIdx.x * 4 + (threadIdx.x >> 6));  // hardware wave in the launch (uniform)
  const u32 tid = hw * P.lpw + lid;
  const bool inrange = lid < P.lpw && tid < count && first + tid < P.nlanes;
  // the lane this position runs: identity, or the regrouping order (lanes at
  // the same rip side by side, k_regroup_keys + radix sort)
  const u32 lane = inrange ? (P.perm ? P.perm[first + tid] : first + tid) : 0;
  // a lane that is not running has its final exit already (or waits for the
  // host): it is neither loaded nor stored
  const bool valid = inrange && P.status[lane] == WTFGPU_RUNNING;
  __shared__ UCEntry sUC[4][UC_N];
  __shared__ UCUop sUU[4][UC_U];
  LANE_COPY_DECL
  UCEntry *uc = sUC[threadIdx.x >> 6];
  UCUop *uu = sUU[threadIdx.x >> 6];
  // the LDS uop cache: the warm image of an earlier launch, or empty
  const bool wave_live = __ballot(valid) != 0;
  const UCEntry *img = (P.warm && wave_live) ? (const UCEntry *)P.warm + (u64)(hw % P.warm_n) * UC_N : nullptr;
  if (img) {
    for (u32 i = lid; i < UC_N; i += 64) {
      UCEntry t = img[i];
      t.logged = 0;
      if (P.cov_rip && t.key != EMPTY_KEY && !(t.flags & (UC_COVERED | UC_CROSS | UC_BADLEN)))
        t.flags |= covered_flag_lane(P, t.rip, (u32)(t.rip & 0xfff));
      uc[i] = t;
    }
  } else {
    for (u32 i = lid; i < UC_N; i += 64) uc[i].key = EMPTY_KEY;
  }
  if (lid < UC_U) uu[lid].key = EMPTY_KEY;
  u32 glo[16], ghi[16];
  Lane L;
  L.glo = glo;
  L.ghi = ghi;
  if (valid) {
    load_lane(P, lane, L);
  } else {
    L.status = WTFGPU_EXIT_IDLE;
    L.lane = 0;
    L.rip = 0;
    L.icount = 0;
    L.cvpn = EMPTY_KEY;
  }
  const u64 icount0 = L.icount;
  bool skip = valid && (P.lflags[lane] & 1);
  // Tenet: the registers at the start (first entry), or after a host handler
  // moved rip (resume without skip, lflags bit 1)
  if (valid && g_tn.buf && (g_tn.pos[lane] == 0 || (P.lflags[lane] & 2))) WITH_LANE_COPY(tn_regs(P, T));
  // The fields the step loops read, once: P is address-taken (the rare-path
  // calls take it by reference), so a field read in the loop would be a
  // scratch load each step, and its vmcnt(0) wait would also wait for the
  // previous step's guest stores. A flag that steers uniform control flow
  // goes through readfirstlane (a load from that private copy counts as
  // divergent, and a loop exit on one made the step loop an exec-masked
  // divergent loop). The loop-invariant bounds are kept in VGPRs (the
  // compiler is told nothing of their uniformity) and compared as lane
  // masks: SGPRs are the step loop's scarce registers, and these were
  // spilled to VGPR lanes and reloaded on every wave-step.
  const bool cov_on = rfl32(P.cov_rip != nullptr ? 1u : 0u) != 0;
  u64 pool_lo = (u64)(uintptr_t)P.pool, pool_span = (P.npool + 1) * WTFGPU_PAGE_SIZE;
  u64 limit_v = P.limit ? P.limit : ~0ull;  // icount above it: timeout
  // wave-steps of this launch (a launch is bounded far below 2^32 wave-steps)
  u32 max32 = max_steps > 0xffffffffull ? 0xffffffffu : (u32)max_steps;
  asm volatile("" : "+v"(pool_lo), "+v"(pool_span), "+v"(limit_v), "+v"(max32));
  const FastMem fm = fast_mem(P);
  u32 steps = 0;
#if !WTFGPU_UC_MRU
  u32 fill_way = 0;  // two-way uop cache: the way the next fill replaces (wave-uniform)
#endif
#ifdef WTFGPU_STAMPS
  u64 stamp_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  u64 tprev_ = __builtin_amdgcn_s_memtime();
  u64 whyc_[4] = {0, 0, 0, 0};
  u32 why_ = 3;
  u32 ophist_[512] = {};
  u64 bpcyc_[8] = {};
#endif

  for (;;) {
    // ================= fast loop: the common step, no calls. Leaves with
    // `have` set and `grip` = the group it could not serve.
    u64 grip = 0;
    bool have = false;
    for (;;) {
      if (m_ge32(steps, max32)) break;
      // (a position with no lane is EXIT_IDLE, never running)
      const u64 am = m_eq32(L.status, WTFGPU_RUNNING);
      if (am == 0) break;
      // group = lanes at the min rip; when the wave is converged (the common
      // case) the first active lane's rip is that min and the reduction is skipped
      grip = readlane64(L.rip, __ffsll((long long)am) - 1);
      u64 gm = am & m_eq64(L.rip, grip);
      if (gm != am) {
        for (u64 lo = am & m_lt64(L.rip, grip); lo; lo = am & m_lt64(L.rip, grip))
          grip = readlane64(L.rip, __ffsll((long long)lo) - 1);
        gm = am & m_eq64(L.rip, grip);
      }
      have = true;
      WHY(1);
      // a new code page: the lane's TLB, else a walk, in registers (what
      // code_xlate does); a translation that would fault goes to the slow step
      if (const u64 cxm = gm & m_ne64(L.cvpn, grip >> 12)) {
        if (in_mask(cxm)) {
          u64 td, gp;
          bool ok = tlb_get(L, grip >> 12, td) && perm_ok(L, td, ACC_X);
          if (!ok && walk<false>(P, L, grip & ~0xfffull, ACC_X, td, gp) && perm_ok(L, td, ACC_X)) {
            tlb_put(L, grip >> 12, td);
            ok = true;
          }
          if (ok) {
            L.cvpn = grip >> 12;
            L.cptr = (td & ~0xfffull) | (L.efer & EFER_M32);  // 32-bit code: to slow_step (U29)
          }
        }
        if (gm & m_ne64(L.cvpn, grip >> 12)) break;
      }
      WHY(3);
      const u64 lptr = readlane64(L.cptr, __ffsll((long long)gm) - 1);
      if (m_ge64(lptr - pool_lo, pool_span)) break;
      const u64 ingm = gm & m_eq64(L.cptr, lptr);
      const bool ing = in_mask(ingm);
      const u64 key = lptr | (grip & 0xfff);
      UCEntry *e = &uc[uc_slot(key)];
      // one LDS round trip: key, logged mask, flags and the FOp are contiguous;
      // the second way only when the first misses (reading both at once kept
      // twice the head in flight on every step: SYN 8 % slower than one way)
      // (the words the step needs only: the logged mask is read when the rip
      // is not yet covered, the pads never)
      UCHead h;
      uc_head_read(e, h);
      if (UC_WAYS == 2 && h.key != key) uc_head_read(++e, h);
      WHY(2);
      if (h.key != key) break;
      WHY(3);
      const u32 flags = h.flags;
      if (flags & (UC_CROSS | UC_BADLEN | UC_UNSUP)) break;
      // a breakpoint: the slow step runs its handler; lanes that resume at it
      // (skip: a device action that left rip there, or a host handler's
      // resume) run the instruction here, as the slow step would without
      // calling the handler again
#if WTFGPU_BP_RESUME_FAST
      if ((flags & UC_BP) && (ingm & ~__ballot(skip))) break;
#else
      if (flags & UC_BP) break;
#endif
      if (cov_on && !(flags & UC_COVERED) && (ingm & ~rfl64(e->logged))) break;
      const FOp &f = h.f;
      if (fo_op(f) == FO_GENERIC) break;
#if WTFGPU_PROBE == 1
      // diagnostic build only: a nop retires without the exec pipeline
      if (fo_op(f) == FO_NOP) {
        steps++;
        have = false;
        if (ing) {
          skip = false;
          L.rip = grip + fo_len(f);
          L.icount++;
          L.nbytes += fo_len(f);
          if (L.icount > limit_v) L.status = WTFGPU_EXIT_TIMEOUT;
        }
        continue;
      }
#endif
#if WTFGPU_FAST_REGOPS
      // a form that touches no memory cannot miss: one pass, no retry rounds
      if (!(f.fl & (FF_PUSH | FF_POP | FF_MR_A | FF_MR_B | FF_MW)) && fo_op(f) < FO_VLD) {
        steps++;
        have = false;
        if (ing) {
          skip = false;
          const u32 len = fo_len(f);
          FOp fr = f;
          asm volatile("" : "+s"(fr.w0), "+s"(fr.fl), "+s"(fr.w2), "+s"(fr.disp), "+s"(fr.imm));
          u64 next;
          fast_exec<true>(fm, L, fr, grip + len, next);
          L.rip = next;
          L.icount++;
          L.nbytes += len;
          if (L.icount > limit_v) L.status = WTFGPU_EXIT_TIMEOUT;
        }
        RECONVERGE();
        continue;
      }
#endif
      steps++;
      have = false;
      STAMP(6);
      // a TLB miss or a first write (fxlate: miss 2) is served here, on the
      // lane in registers, and the instruction retried at once, so the group
      // still takes one wave-step (at most 3 fill rounds); anything else (a
      // fault to raise, a page-table write, a page-crossing operand, ...) is
      // left to the slow step, whose exec() raises what it raises. A first
      // write's page copy is made by the whole wave, 64 bytes a position: one
      // memory round trip instead of a lane's 64 dependent ones
      const u32 len = fo_len(f);
      u64 next = 0;
      u64 wantm = ingm;
      if (ing) skip = false;
      for (u32 round = 0;; round++) {
        if (in_mask(wantm)) {
          L.miss = 0;
          L.pend = 0;
          // the FOp as an opaque value each round: otherwise everything
          // fast_exec derives from it (masks, shift counts, every op's
          // conditions) is hoisted out of this loop as invariant, stays live
          // across it and spills to VGPR lanes: ~100 v_writelane and ~280
          // v_readlane on every wave-step
          FOp fr = f;
          asm volatile("" : "+s"(fr.w0), "+s"(fr.fl), "+s"(fr.w2), "+s"(fr.disp), "+s"(fr.imm));
          fast_exec(fm, L, fr, grip + len, next);
        }
        RECONVERGE();
        // lanes to serve and retry: a TLB miss or first write (miss 2), 3 rounds at most
        wantm = round >= 3 ? 0 : wantm & m_eq32(L.miss, 2);
        if (wantm == 0) break;
        u64 csrc = 0, cdst = 0, cgpfn = 0, ctd = 0;
        bool want = in_mask(wantm);
        if (want && !fast_fill_prep(P, L, csrc, cdst, cgpfn, ctd)) {
          want = false;
#if WTFGPU_FAST_FAULTS
          fast_fault(P, L);  // the lane stops with the fault (delivered after the loop)
#endif
        }
        for (u64 cm = __ballot(want && cdst); cm; cm &= cm - 1) {
          const int l = __ffsll((long long)cm) - 1;
          const uint4 *s4 = (const uint4 *)(uintptr_t)readlane64(csrc, l) + lid * 4;
          uint4 *d4 = (uint4 *)(uintptr_t)readlane64(cdst, l) + lid * 4;
          const uint4 a = s4[0], b = s4[1], c = s4[2], d = s4[3];
          d4[0] = a;
          d4[1] = b;
          d4[2] = c;
          d4[3] = d;
        }
        // the copies land before the lanes read their pages (one wave, one CU)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        if (want && cdst) fast_fill_finish(P, L, cdst, cgpfn, ctd);
        wantm = __ballot(want);
      }
      const u64 missm = ingm & m_ne32(L.miss, 0);
      if (in_mask(ingm & ~missm)) {
        L.rip = next;
        L.icount++;
        L.nbytes += len + L.pend;
        if (L.icount > limit_v) L.status = WTFGPU_EXIT_TIMEOUT;
      }
      RECONVERGE();
      STAMP(7);
      // lanes that still missed keep their rip: the slow step services them.
      // The attempt is not a wave-step of its own (the slow step counts the
      // group once): a slice's length in wave-steps must not depend on which
      // path ran a group, since that depends on when other queues' coverage
      // commits landed (U44: fixed-seed campaigns reproduce)
      if (missm & m_eq32(L.status, WTFGPU_RUNNING)) {
        WHY(0);
        steps--;
        have = true;
        break;
      }
      // lanes whose fill raised a fault here (fast_fault): the step counted
      // (as the slow step's would have), the fault is delivered next
      if (missm) break;
    }
    STAMP(0);
    // faults raised by the last slow step: deliver through the guest IDT when
    // it has a gate (the lane resumes at the handler), else the lane exits
    if (__ballot(L.status == WTFGPU_EXIT_FAULT && !L.nodeliver)) {
      if (L.status == WTFGPU_EXIT_FAULT && !L.nodeliver) {
        bool dv;
        WITH_LANE_COPY(dv = deliver_fault(P, T));
        if (dv && g_tn.buf) WITH_LANE_COPY(tn_regs(P, T));  // Tenet: the delivered exception
      }
      RECONVERGE();
      continue;
    }
    if (!have) break;

    // ================= slow step for group `grip`: translation misses, cache
    // fills, page-crossing / overlay code, coverage logging, breakpoints,
    // generic instructions, TLB misses and copy-on-write
    steps++;
#ifdef WTFGPU_STAMPS
    whyc_[why_ & 3]++;
#endif
    const bool active = L.status == WTFGPU_RUNNING;
    bool cand = active && L.rip == grip;
    if (cand && (grip >> 12) != L.cvpn) WITH_LANE_COPY(code_xlate(P, T, grip));
    cand = cand && (grip >> 12) == L.cvpn;
    const u64 cm = __ballot(cand);
    if (cm == 0) continue;
    const int leader = __ffsll((long long)cm) - 1;
    const u64 lptr = readlane64(L.cptr, leader);
    bool ing = cand && L.cptr == lptr;

    const u32 off = (u32)(grip & 0xfff);
    const u64 key = lptr | off;
    UCEntry *e = &uc[uc_slot(key)];
    if (UC_WAYS == 2 && rfl64(e->key) != key) {
      if (rfl64(e[1].key) == key) e += 1;
#if WTFGPU_UC_MRU
      else if (cacheable_key(lptr, pool_lo, pool_span)) {
        // the newest fill takes way 0 (the fast loop's first read), the old
        // way 0 moves to way 1 (whose entry is the one dropped)
        if (lid < 16) ((u32 *)&e[1])[lid] = ((const u32 *)e)[lid];
        __builtin_amdgcn_wave_barrier();
      }
#else
      else e += (fill_way++ & 1);  // the way a fill replaces
#endif
    }
    const bool cacheable = !m_ge64(lptr - pool_lo, pool_span);
    if (cacheable && rfl64(e->key) != key) {
#if WTFGPU_FILL_INLINE
      if (!uc_fill_shared(P, e, &uu[uu_slot(key)], key, off, grip, lid))
        uc_fill(P, e, &uu[uu_slot(key)], key, lptr, off, grip, lid, true);
#else
      uc_fill(P, e, &uu[uu_slot(key)], key, lptr, off, grip, lid);
#endif
#if WTFGPU_FILL_PREFETCH
      // sequential prefetch: the instructions after this one in the page, from
      // the shared cache into their sets' second (older) way, while the wave
      // is in the slow step anyway; stops at the first that is cached, absent
      // from the shared cache, or crosses the page
      if (UC_WAYS == 2) {
        const UCEntry *pe = e;
        u64 prip = grip;
        for (u32 k = 0; k < WTFGPU_FILL_PREFETCH; k++) {
          const u32 pf = rfl32(pe->flags), pw0 = rfl32(pe->f.w0), plen = (pw0 >> 20) & 0x3f;
          if ((pf & (UC_CROSS | UC_BADLEN)) || !plen) break;
          u64 nxt = prip + plen;  // the fall-through; a direct jmp / call: its target (same page only)
#if WTFGPU_FILL_PREFETCH_JUMPS
          const u32 pop = pw0 & 0xff;
          if ((pop == FO_JMP || pop == FO_CALL) && !(rfl32(pe->f.fl) & FF_BREG)) nxt += rfl64(pe->f.imm);
          if (pop == FO_RET || ((pop == FO_JMP || pop == FO_CALL) && (rfl32(pe->f.fl) & FF_BREG))) break;
#endif
          if ((nxt >> 12) != (grip >> 12) || (nxt & 0xfff) > 4096 - 16) break;
          const u32 poff = (u32)(nxt & 0xfff);
          const u64 pkey = lptr | poff;
          UCEntry *ps = &uc[uc_slot(pkey)];
          if (rfl64(ps->key) == pkey || rfl64(ps[1].key) == pkey) break;
          if (!uc_fill_shared(P, ps + 1, nullptr, pkey, poff, nxt, lid)) break;
          pe = ps + 1;
          prip = nxt;
        }
      }
#endif
      // an entry the fast loop can run (a common op, nothing to log, no
      // breakpoint): back to it, this pass was only the fill
      const u32 ff = rfl32(e->flags);
      if (!(ff & (UC_BP | UC_CROSS | UC_BADLEN | UC_UNSUP)) && (!cov_on || (ff & UC_COVERED)) &&
          (rfl32(e->f.w0) & 0xff) != FO_GENERIC) {  // read uniformly: a divergent exit here made the whole step loop divergent
        steps--;
        STAMP(2);
        continue;
      }
    }
    STAMP(2);
    const u32 flags = cacheable ? rfl32(e->flags) : UC_CROSS;
    if (flags & (UC_CROSS | UC_BADLEN)) {
      if (flags & UC_BADLEN) {
        if (ing) set_fault(L, WTFGPU_VEC_GP, 0, 0);
      } else if (L.status != WTFGPU_EXIT_IDLE) {  // a position with no lane has no copy slot of its own
        bool sk = skip;  // skip stays a register (a reference would put it in scratch for the whole loop)
        WITH_LANE_COPY(slow_step(P, T, grip, lptr, ing, sk));
        skip = sk;
      }
      RECONVERGE();
      STAMP(5);
      continue;
    }
    const u32 len = (rfl32(e->f.w0) >> 20) & 0x3f;  // fo_len, read once for the wave
    const u64 gmask = __ballot(ing);

    // ---- coverage, then breakpoint (bochscpu_backend.cc:501-547)
    if (P.trace && ing && !skip) trace_rip(P, L.lane, grip);  // a resumed breakpoint was logged at its hit
    bool logged_now = false;  // wave-uniform
    if (cov_on && !(flags & UC_COVERED)) {
      const u64 logged = rfl64(e->logged);
      if (gmask & ~logged) {
        L.ccnt = cover(P, grip, ing && !((logged >> lid) & 1), L.lane, L.cgen, L.ccnt);
        if (lid == 0) e->logged = logged | gmask;
        logged_now = true;
      }
    }
    STAMP(3);
#if WTFGPU_COVER_FAST
    // the group has just logged the rip (its lanes are all in the entry's mask
    // now): an op the fast loop runs goes back to it, not to the generic exec.
    // Only right after logging, so a group the fast loop hands back (a miss
    // to serve) finds nothing to log and takes the generic path: no ping-pong
    if (logged_now && !(flags & (UC_BP | UC_UNSUP)) && (rfl32(e->f.w0) & 0xff) != FO_GENERIC) {
      steps--;
      continue;
    }
#endif
    // a register-only device action (SetGprs, StopOk: the same for every lane)
    // is applied here, without the lane copy and call the others take
    u32 act_kind = ~0u;
    const wtfgpu_bp_action_t *act = nullptr;
    if (WTFGPU_INLINE_ACTIONS && (flags & UC_BP) && P.act_keys && !g_tn.buf) {
      u32 slot;
      if (hash_find(P.act_keys, P.act_mask, grip, slot)) {
        act = &P.act[slot];
        act_kind = rfl32(act->kind);
      }
    }
#ifdef WTFGPU_STAMPS
    // breakpoint hits by action kind (56 + kind; 63: none found)
    if (__ballot(ing && (flags & UC_BP) && !skip)) OPHIST(56 + (act_kind < 7 ? act_kind : 7));
#endif
    // (one block per kind: with the two kinds nested in one per-lane if/else
    // the build ran wrong on MI355X, tlv's lanes stopping Ok at their SetGprs
    // breakpoint, although either kind alone ran right; WTFGPU_ACT_NESTED=1
    // builds that form for the A/B in DESIGN.md §3)
#if WTFGPU_ACT_NESTED
    if (WTFGPU_INLINE_ACTIONS == 3 && (act_kind == WTFGPU_BPACT_SET_GPRS || act_kind == WTFGPU_BPACT_STOP_OK) && ing &&
        !skip) {
      if (act_kind == WTFGPU_BPACT_SET_GPRS) {
#pragma unroll
        for (u32 i = 0; i < 16; i++) RS(L, i, act->gprs[i]);
        L.rip = act->gprs[16];
        skip = L.rip == grip;
      } else {
        L.status = WTFGPU_EXIT_STOP_OK;
        skip = true;
      }
      ing = false;
    }
#else
    if ((WTFGPU_INLINE_ACTIONS & 1) && act_kind == WTFGPU_BPACT_SET_GPRS && ing && !skip) {
#pragma unroll
      for (u32 i = 0; i < 16; i++) RS(L, i, act->gprs[i]);
      L.rip = act->gprs[16];
      skip = L.rip == grip;
      ing = false;
    }
    if ((WTFGPU_INLINE_ACTIONS & 2) && act_kind == WTFGPU_BPACT_STOP_OK && ing && !skip) {
      L.status = WTFGPU_EXIT_STOP_OK;
      skip = true;
      ing = false;
    }
#endif
#if WTFGPU_FEED_PREFAULT
    // a Feed action about to write a packet (feed_apply's checks) whose first
    // page is not yet the lane's own: that page's copy-on-write is made here
    // by the whole wave, 64 bytes a position (as the fast loop's first writes),
    // instead of by each lane's 16-round copy inside host_write. Same walk
    // (supervisor, CR0.WP clear, as host_write), same overlay slot, same page:
    // host_write then finds it private. Anything else is left to host_write.
    if (act_kind == WTFGPU_BPACT_FEED && P.feed_pos) {
      bool want = false;
      if (ing && !skip) {
        const u64 pos = P.feed_pos[L.lane];
        const u64 end = P.feed_end[L.lane];
        if (pos != ~0ull && pos + 4 <= end) {
          const u8 *src = P.feed_data + pos;
          const u32 n = (u32)src[0] | ((u32)src[1] << 8) | ((u32)src[2] << 16) | ((u32)src[3] << 24);
          const u64 win = act->value;
          if (n && n < win && pos + 4 + n <= end) {
            const u64 va = R(L, (u32)act->gprs[0] & 15) + win - n;
            u64 td;
            if (!(tlb_get(L, va >> 12, td) && (td & T_PRIV))) {
              L.miss_va = va;
              L.miss_acc = ACC_W;
              want = true;
            }
          }
        }
      }
      u64 csrc = 0, cdst = 0, cgpfn = 0, ctd = 0;
      if (want) {
        const u32 cpl0 = L.cpl;
        const u64 cr00 = L.cr0;
        L.cpl = 0;
        L.cr0 &= ~(1ull << 16);
        want = fast_fill_prep(P, L, csrc, cdst, cgpfn, ctd);
        L.cpl = cpl0;
        L.cr0 = cr00;
      }
      RECONVERGE();
      for (u64 cm = __ballot(want && cdst); cm; cm &= cm - 1) {
        const int l = __ffsll((long long)cm) - 1;
        const uint4 *s4 = (const uint4 *)(uintptr_t)readlane64(csrc, l) + lid * 4;
        uint4 *d4 = (uint4 *)(uintptr_t)readlane64(cdst, l) + lid * 4;
        const uint4 a = s4[0], b = s4[1], c = s4[2], d = s4[3];
        d4[0] = a;
        d4[1] = b;
        d4[2] = c;
        d4[3] = d;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      if (want && cdst) fast_fill_finish(P, L, cdst, cgpfn, ctd);
      RECONVERGE();
    }
#endif
    if (ing) {
      if ((flags & UC_BP) && !skip) {
        // breakpoint hit: device action (the lane keeps running) or host exit
        bool applied = false;
#ifdef WTFGPU_STAMPS
        const u64 tb_ = __builtin_amdgcn_s_memtime();
#endif
        if (P.act_keys) WITH_LANE_COPY(applied = bp_apply(P, T, grip, act));
#ifdef WTFGPU_STAMPS
        bpcyc_[act_kind < 7 ? act_kind : 7] += __builtin_amdgcn_s_memtime() - tb_;
#endif
        if (!applied) L.status = WTFGPU_EXIT_BREAKPOINT;
        skip = applied && L.rip == grip;
        if (applied && !skip && g_tn.buf) WITH_LANE_COPY(tn_regs(P, T));  // Tenet: the action moved rip
        ing = false;
      } else {
        skip = false;
      }
    }
    STAMP(4);
    // the UOp for the generic path (wave-uniform: the slot fill is a wave operation)
    const UOp *u = nullptr;
    if (__ballot(ing)) u = uc_uop(P, uu, key, lptr, off, grip, lid);
    if (__ballot(ing) && !(flags & UC_UNSUP)) OPHIST(rfl32(u->op) + (flags & UC_COVERED ? 64 : 0));
    if (ing && (flags & UC_UNSUP)) {
      const u32 ob = u->opbytes, n = len;
      L.status = WTFGPU_EXIT_UNIMPLEMENTED;
      L.exop = n >= 4 ? ob : (ob & ((1u << (8 * n)) - 1));
      ing = false;
    }
    if (ing) {
      // restartable attempts (exec_retry), all on one copy of the lane
      u64 next = 0;
      int x;
      WITH_LANE_COPY(x = exec_retry(P, T, u, next));
      u32 opbytes = 0;
      if (x == X_UNIMPL) opbytes = u->opbytes;
      retire(P, L, x, len, next, opbytes);
      if (g_tn.buf && (x == X_OK || x == X_CR3)) WITH_LANE_COPY(tn_regs(P, T));  // Tenet: the retired instruction
      // RecordEdge (bochscpu_backend.cc:699-728): the branch ran, whatever the retire hook decided
      if (P.edges && P.cov_rip && x == X_OK && edge_op(rfl32(u->op), rfl32(u->bsrc))) {
        const u32 c0 = L.ccnt;
        L.ccnt = cover_edge(P, edge_key(grip, next), true, L.lane, L.cgen, L.ccnt);
        count_edge(P, L.lane, L.ccnt != c0);
      }
    }
    RECONVERGE();
    STAMP(1);
  }

  if (P.warm && wave_live && hw < P.warm_n) {  // this wave's cache for the next launch
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    UCEntry *out = (UCEntry *)P.warm + (u64)hw * UC_N;
    for (u32 i = lid; i < UC_N; i += 64) out[i] = uc[i];
  }
  // Tenet: a lane that stopped with accesses still open (an undelivered fault,
  // an unimplemented instruction) closes them with a REGS entry
  if (valid && g_tn.buf && L.status != WTFGPU_RUNNING && L.status != WTFGPU_EXIT_BREAKPOINT &&
      g_tn.pos[lane] > g_tn.ipos[lane])
    WITH_LANE_COPY(tn_regs(P, T));
  if (valid) {
    store_lane(P, L);
    store_tlb(P, L);
    if (L.status == WTFGPU_EXIT_FAULT || L.status == WTFGPU_EXIT_UNIMPLEMENTED) {
      ExitInfo ei;
      ei.vector = L.exvec;
      ei.error = L.exerr;
      ei.opcode = L.exop;
      ei.cpl = L.cpl;
      ei.addr = L.exaddr;
      P.exinfo[lane] = ei;
    }
    P.lflags[lane] = skip ? 1u : 0u;
  }
  const u64 retired = wave_sum(valid ? L.icount - icount0 : 0);
  const u64 running = wave_sum((valid && L.status == WTFGPU_RUNNING) ? 1 : 0);
  if (lid == 0) {
    atomicAdd((unsigned long long *)&P.stat[0], (unsigned long long)steps);
    atomicAdd((unsigned long long *)&P.stat[1], (unsigned long long)retired);
    if (running) atomicAdd((unsigned long long *)&P.stat[2], (unsigned long long)running);
#ifdef WTFGPU_STAMPS
    for (int k = 0; k < 8; k++) atomicAdd((unsigned long long *)&P.stat[4 + k], (unsigned long long)stamp_[k]);
    for (int k = 0; k < 4; k++) atomicAdd((unsigned long long *)&P.stat[12 + k], (unsigned long long)whyc_[k]);
    for (int k = 0; k < 512; k++)
      if (ophist_[k]) atomicAdd((unsigned long long *)&P.stat[16 + k], (unsigned long long)ophist_[k]);
    for (int k = 0; k < 8; k++) atomicAdd((unsigned long long *)&P.stat[528 + k], (unsigned long long)bpcyc_[k]);
#endif
  }
}

// ---------------------------------------------------------------- restore
struct InitState {
  u64 g[16];
  u64 rip, rflags, fsb, gsb;
  LaneSys sys;
};

// Registers, system state and overlay of one lane back to the snapshot (the
// dirty-list reset: overlays dropped, nothing copied).
__device__ __forceinline__ void restore_lane(const Dev &P, const InitState &s, const wtfgpu_regs_t *full0,
                                             wtfgpu_regs_t *full, u32 lane) {
  const u64 N = P.nlanes;
  full[lane] = *full0;
#pragma unroll
  for (int i = 0; i < 16; i++) P.gpr[i * N + lane] = s.g[i];
  P.rip[lane] = s.rip;
  P.rflags[lane] = s.rflags;
  P.fs_base[lane] = s.fsb;
  P.gs_base[lane] = s.gsb;
  P.icount[lane] = 0;
  P.nbytes[lane] = 0;
  P.status[lane] = WTFGPU_RUNNING;
  P.lflags[lane] = 0;
  P.sys[lane] = s.sys;
  P.ov_count[lane] = 0;
  tlb_stale(P, lane);
  if (P.rd_seed) P.rd_seed[lane] = P.rd_seed0;  // bochscpu_backend.cc:1030
  if (P.trace_cnt) P.trace_cnt[lane] = 0;
  if (P.edge_cnt) P.edge_cnt[2 * (u64)lane] = P.edge_cnt[2 * (u64)lane + 1] = 0;
  if (g_tn.buf) {
    g_tn.pos[lane] = g_tn.ipos[lane] = g_tn.cpos[lane] = 0;
    g_tn.last[lane] = ~0ull;
    g_tn.mute[lane] = 0;
  }
  if (P.cov_rip) {
    P.lane_gen[lane] += 1;
    P.cov_cnt[lane] = 0;
    P.cov_overflow[lane] = 0;
  }
}

// Streaming form: a lane list.
__global__ void k_restore_list(Dev P, const InitState *S, const wtfgpu_regs_t *full0, wtfgpu_regs_t *full,
                               const u32 *lanes, u32 n) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const InitState s = *S;
  restore_lane(P, s, full0, full, lanes[t]);
}

__global__ void k_restore(Dev P, const InitState *S, const wtfgpu_regs_t *full0, wtfgpu_regs_t *full, u32 first,
                          u32 count) {
  const u32 tid = blockIdx.x * blockDim.x + threadIdx.x;
  const u32 lane = first + tid;
  if (tid >= count || lane >= P.nlanes) return;
  const u64 N = P.nlanes;
  const InitState s = *S;
  full[lane] = *full0;  // cold architectural state (read/write_regs only)
#pragma unroll
  for (int i = 0; i < 16; i++) P.gpr[i * N + lane] = s.g[i];
  P.rip[lane] = s.rip;
  P.rflags[lane] = s.rflags;
  P.fs_base[lane] = s.fsb;
  P.gs_base[lane] = s.gsb;
  P.icount[lane] = 0;
  P.nbytes[lane] = 0;
  P.status[lane] = WTFGPU_RUNNING;
  P.lflags[lane] = 0;
  P.sys[lane] = s.sys;
  P.ov_count[lane] = 0;  // the dirty-list reset: overlays dropped, nothing copied
  tlb_stale(P, lane);
  if (P.rd_seed) P.rd_seed[lane] = P.rd_seed0;  // bochscpu_backend.cc:1030
  if (P.trace_cnt) P.trace_cnt[lane] = 0;
  if (P.edge_cnt) P.edge_cnt[2 * (u64)lane] = P.edge_cnt[2 * (u64)lane + 1] = 0;
  if (g_tn.buf) {
    g_tn.pos[lane] = g_tn.ipos[lane] = g_tn.cpos[lane] = 0;
    g_tn.last[lane] = ~0ull;
    g_tn.mute[lane] = 0;
  }
  if (P.cov_rip) {       // the lane's coverage set empties
    P.lane_gen[lane] += 1;
    P.cov_cnt[lane] = 0;
    P.cov_overflow[lane] = 0;
  }
}

// ---------------------------------------------------------------- host-driven lane memory
// One thread per lane with pending writes (records sorted by lane). op: 0 write virt.
struct WriteRec {
  u32 lane, len;
  u64 gva, data_off;
};

__device__ __forceinline__ void lane_min_load(const Dev &P, u32 lane, Lane &L) {
  const LaneSys s = P.sys[lane];
  L.cr0 = s.cr0;
  L.cr3 = s.cr3;
  L.efer = s.efer;
  L.cpl = 0;  // host accesses are not subject to user checks (VirtTranslate has none)
  L.simd = 0;
  L.ovn = P.ov_count[lane];
  L.bloom = 0;
  for (u32 k = 0; k < L.ovn; k++) L.bloom |= bloom_bit(P.ov_gpfn[(u64)k * P.nlanes + lane]);
  L.lane = lane;
  L.status = WTFGPU_RUNNING;
  L.nbytes = 0;
  tlb_flush(L);
  L.tnext = 0;
  L.miss = L.miss_acc = L.flush = L.pend = 0;
  L.nodeliver = 0;
}

// Host-side translation (bochscpu_mem_virt_translate semantics: present bits
// only, no permission checks).
__device__ __forceinline__ bool host_walk(const Dev &P, Lane &L, u64 va, u64 &gpa) {
  u64 table = L.cr3 & 0x000ffffffffff000ull;
  bool priv;
  u64 e = 0, pmask = 0xfff;
  for (int level = 3; level >= 0; level--) {
    const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, table >> 12, priv);
    e = *(const u64 *)(pg + ((va >> (12 + 9 * level)) & 0x1ff) * 8);
    if (!(e & 1)) return false;
    if ((level == 1 || level == 2) && (e & 0x80)) {
      pmask = level == 2 ? 0x3fffffffull : 0x1fffffull;
      break;
    }
    table = e & 0x000ffffffffff000ull;
  }
  gpa = ((e & 0x000ffffffffff000ull) & ~pmask) | (va & pmask);
  return true;
}

// The same write by one 64-thread block (the control is uniform, every
// thread computes it; the page copy and the bytes are spread over the block).
__device__ __forceinline__ bool lane_phys_write_block(const Dev &P, Lane &L, u64 gpa, const u8 *src, u64 len, u32 lid) {
  while (len) {
    const u64 off = gpa & 0xfff;
    u64 n = 4096 - off;
    if (n > len) n = len;
    bool priv;
    const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, gpa >> 12, priv);
    u8 *dst = (u8 *)pg;
    if (!priv) {
      if (L.ovn >= P.K) return false;
      dst = P.ov_data + ((u64)L.lane * P.K + L.ovn) * WTFGPU_PAGE_SIZE;
      const uint4 *s4 = (const uint4 *)pg;
      uint4 *d4 = (uint4 *)dst;
      for (u32 i = lid; i < 256; i += 64) d4[i] = s4[i];
      if (lid == 0) P.ov_gpfn[(u64)L.ovn * P.nlanes + L.lane] = (u32)(gpa >> 12);
      __syncthreads();  // the copy before the patch (and the slot before later lookups)
      L.ovn++;
      L.bloom |= bloom_bit(gpa >> 12);
    }
    for (u64 i = lid; i < n; i += 64) dst[off + i] = src[i];
    __syncthreads();
    src += n;
    gpa += n;
    len -= n;
  }
  return true;
}

// Host-handler writes, one 64-thread block per lane, records in order.
__global__ void k_apply_writes(Dev P, const WriteRec *recs, const u32 *starts, u32 nlanes_w, const u8 *data,
                               i32 *status_out, u32 phys) {
  const u32 t = blockIdx.x, lid = threadIdx.x;
  if (t >= nlanes_w) return;
  const u32 r0 = starts[t], r1 = starts[t + 1];
  const u32 lane = recs[r0].lane;
  Lane L;
  lane_min_load(P, lane, L);
  for (u32 r = r0; r < r1; r++) {
    const WriteRec w = recs[r];
    u64 va = w.gva, left = w.len;
    const u8 *src = data + w.data_off;
    i32 st = 0;
    while (left) {
      const u64 off = va & 0xfff;
      u64 n = 4096 - off;
      if (n > left) n = left;
      u64 gpa = va;
      if (!phys && !host_walk(P, L, va, gpa)) {
        st = WTFGPU_ERR_TRANSLATE;
        break;
      }
      if (!lane_phys_write_block(P, L, gpa, src, n, lid)) {
        st = WTFGPU_ERR_OOM;
        break;
      }
      va += n;
      src += n;
      left -= n;
    }
    if (lid == 0) status_out[r] = st;
  }
  if (lid == 0) {
    P.ov_count[lane] = L.ovn;
    tlb_stale(P, lane);
  }
}

// Host-injected exception per lane (PageFaultsMemoryIfNeeded): delivered
// through the guest IDT now; the lane resumes at the handler.
__global__ void k_inject_fault(Dev P, const u32 *lanes, const u64 *addrs, u32 n, u32 vector, u32 error, i32 *ok) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const u32 lane = lanes[t];
  u32 glo[16], ghi[16];
  Lane L;
  L.glo = glo;
  L.ghi = ghi;
  load_lane(P, lane, L);
  L.status = WTFGPU_EXIT_FAULT;
  L.exvec = vector;
  L.exerr = error;
  L.exaddr = addrs[t];
  const bool d = deliver_fault(P, L);
  ok[t] = d ? 1 : 0;
  if (d && g_tn.buf) {  // Tenet: the injected exception
    g_tn.ipos[lane] = g_tn.pos[lane];
    tn_regs(P, L);
  }
  if (d) {
    store_lane(P, L);
    tlb_stale(P, lane);
    P.lflags[lane] = 0;
  }
}

// The declared insert of a lane list (wtfgpu_set_insert), after the feed
// scatter: lanes without a feed are left alone. The writes are not CPU
// accesses (Tenet does not log them).
__global__ void k_insert(Dev P, wtfgpu_insert_t ins, const u32 *lanes, u32 first, u32 n) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const u32 lane = lanes ? lanes[t] : first + t;
  if (P.feed_pos[lane] == ~0ull || P.status[lane] != WTFGPU_RUNNING) return;
  u32 glo[16], ghi[16];
  Lane L;
  L.glo = glo;
  L.ghi = ghi;
  load_lane(P, lane, L);
  if (g_tn.buf) tn_mute(lane);
  insert_apply(P, L, ins);
  if (g_tn.buf) tn_unmute(lane, 0, 0, 0, false);
  store_lane(P, L);
  store_tlb(P, L);
}

// Lane status (+ skip-breakpoint-once flag) for a lane list (resume / stop).
__global__ void k_set_status(Dev P, const u32 *lanes, u32 n, u32 status, const u8 *skip) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const u32 lane = lanes[t];
  P.status[lane] = status;
  if (skip) P.lflags[lane] = skip[t] ? 1u : (g_tn.buf ? 2u : 0u);  // 2: Tenet entry at the next launch
}

// Single-lane memory services for the host proxy.
// op 0: translate (out u64 gpa), 1: read phys, 2: write phys, 3: read virt, 4: write virt
__global__ void k_lane_mem(Dev P, u32 lane, u32 op, u64 addr, u64 len, u8 *buf, i64 *result) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Lane L;
  lane_min_load(P, lane, L);
  i64 rc = 0;
  if (op == 0) {
    u64 gpa;
    rc = host_walk(P, L, addr, gpa) ? (i64)gpa : -1;
  } else if (op == 1 || op == 3) {
    u64 a = addr;
    for (u64 i = 0; i < len;) {
      u64 gpa = a;
      if (op == 3 && !host_walk(P, L, a, gpa)) {
        rc = -1;
        break;
      }
      u64 n = 4096 - (a & 0xfff);
      if (n > len - i) n = len - i;
      bool priv;
      const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, gpa >> 12, priv);
      for (u64 k = 0; k < n; k++) buf[i + k] = pg[(gpa & 0xfff) + k];
      i += n;
      a += n;
    }
  } else {
    u64 a = addr;
    for (u64 i = 0; i < len;) {
      u64 gpa = a;
      if (op == 4 && !host_walk(P, L, a, gpa)) {
        rc = -1;
        break;
      }
      u64 n = 4096 - (a & 0xfff);
      if (n > len - i) n = len - i;
      if (!lane_phys_write(P, L, gpa, buf + i, n)) {
        rc = -2;
        break;
      }
      i += n;
      a += n;
    }
    P.ov_count[lane] = L.ovn;
    tlb_stale(P, lane);
  }
  *result = rc;
}

// ---------------------------------------------------------------- bulk lane services
// GPRs + rip + rflags (18 u64, that order) of a lane list, gathered / scattered.
__global__ void k_gather_gprs(Dev P, const u32 *lanes, u32 n, u64 *out) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const u64 N = P.nlanes, l = lanes[t];
  for (int i = 0; i < 16; i++) out[(u64)t * 18 + i] = P.gpr[i * N + l];
  out[(u64)t * 18 + 16] = P.rip[l];
  out[(u64)t * 18 + 17] = P.rflags[l];
}
__global__ void k_scatter_gprs(Dev P, const u32 *lanes, u32 n, const u64 *in) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const u64 N = P.nlanes, l = lanes[t];
  for (int i = 0; i < 16; i++) P.gpr[i * N + l] = in[(u64)t * 18 + i];
  P.rip[l] = in[(u64)t * 18 + 16];
  P.rflags[l] = in[(u64)t * 18 + 17];
}
// Dirty lists of a lane list: out[t * (K + 1)] = count, then the gpfns.
__global__ void k_gather_dirty(Dev P, const u32 *lanes, u32 n, u32 *out) {
  const u32 t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const u32 l = lanes[t], cnt = P.ov_count[l];
  u32 *o = out + (u64)t * (P.K + 1);
  o[0] = cnt;
  for (u32 k = 0; k < cnt && k < P.K; k++) o[1 + k] = P.ov_gpfn[(u64)k * P.nlanes + l];
}
// Lane views of physical pages (overlay copy, else snapshot, else zeros): one
// 256-thread block per (lane, gpa) request, 16 bytes per thread.
// `len` bytes (<= 256, within one page) at (lane, gpa) from each lane's view:
// one 64-thread block per record, 4 bytes per thread.
__global__ void k_gather_bytes(Dev P, const u32 *lanes, const u64 *gpas, u32 n, u32 len, u8 *out) {
  const u32 r = blockIdx.x;
  if (r >= n) return;
  const u32 l = lanes[r];
  const u64 gpa = gpas[r];
  const u32 ovn = P.ov_count[l];
  u64 bloom = 0;
  for (u32 k = 0; k < ovn; k++) bloom |= bloom_bit(P.ov_gpfn[(u64)k * P.nlanes + l]);
  bool priv;
  const u8 *src = phys_page(P, l, ovn, bloom, gpa >> 12, priv) + (gpa & 0xfff);
  for (u32 i = threadIdx.x; i < len; i += blockDim.x) out[(u64)r * len + i] = src[i];
}

__global__ void k_gather_pages(Dev P, const u32 *lanes, const u64 *gpas, u32 n, u8 *out) {
  const u32 r = blockIdx.x;
  if (r >= n) return;
  const u32 l = lanes[r];
  const u64 gpfn = gpas[r] >> 12;
  const u32 ovn = P.ov_count[l];
  u64 bloom = 0;
  for (u32 k = 0; k < ovn; k++) bloom |= bloom_bit(P.ov_gpfn[(u64)k * P.nlanes + l]);
  bool priv;
  const uint4 *src = (const uint4 *)phys_page(P, l, ovn, bloom, gpfn, priv);
  ((uint4 *)(out + (u64)r * WTFGPU_PAGE_SIZE))[threadIdx.x] = src[threadIdx.x];
}

// ---------------------------------------------------------------- coverage services
// The coverage sets of a lane list (lanes == nullptr: lanes first + i), one
// block per lane, compacted into (lane, rip) pairs.
__global__ void k_cov_collect(Dev P, const u32 *lanes, u32 first, u32 n, u32 *out_lane, u64 *out_rip, u64 cap,
                              unsigned long long *n_out, u32 *ovf) {
  const u32 i = blockIdx.x;
  if (i >= n) return;
  const u32 lane = lanes ? lanes[i] : first + i;
  const u32 g = P.lane_gen[lane];
  const u64 base = (u64)lane * P.H;
  for (u32 k = threadIdx.x; k < P.H; k += blockDim.x) {
    if (P.cov_gen[base + k] != g) continue;
    const unsigned long long pos = atomicAdd(n_out, 1ull);
    if (pos < cap) {
      out_lane[pos] = lane;
      out_rip[pos] = P.cov_rip[base + k];
    }
  }
  if (threadIdx.x == 0 && P.cov_overflow[lane]) atomicOr(ovf, 1u);
}

// The coverage sets of the stopped lanes of [first, first + count) (status
// neither RUNNING nor IDLE: the lanes a slice finished or left at a host
// breakpoint), compacted as k_cov_collect does (wtfgpu_prefetch_coverage).
// One wave per lane; an empty set (cov_cnt 0, the common case once the
// coverage has settled) costs one load.
__global__ void k_cov_collect_stopped(Dev P, u32 first, u32 count, u32 *out_lane, u64 *out_rip, u64 cap,
                                      unsigned long long *n_out, u32 *ovf) {
  const u32 i = blockIdx.x * 4 + (threadIdx.x >> 6), lid = threadIdx.x & 63;
  if (i >= count) return;
  const u32 lane = first + i;
  const u32 st = P.status[lane];
  if (st == WTFGPU_RUNNING || st == WTFGPU_EXIT_IDLE) return;
  if (P.cov_overflow[lane] && lid == 0) atomicOr(ovf, 1u);
  if (P.cov_cnt[lane] == 0) return;
  const u32 g = P.lane_gen[lane];
  const u64 base = (u64)lane * P.H;
  for (u32 k = lid; k < P.H; k += 64) {
    if (P.cov_gen[base + k] != g) continue;
    const unsigned long long pos = atomicAdd(n_out, 1ull);
    if (pos < cap) {
      out_lane[pos] = lane;
      out_rip[pos] = P.cov_rip[base + k];
    }
  }
}

// Rdrand seeds of a lane list: gathered into / scattered from buf.
__global__ void k_lane_seeds(Dev P, const u32 *lanes, u32 n, u64 *buf, int write) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (write) P.rd_seed[lanes[i]] = buf[i];
  else buf[i] = P.rd_seed[lanes[i]];
}

// STOP_ARGS arguments of a lane list (6 u64 each).
__global__ void k_stop_args(Dev P, const u32 *lanes, u32 n, u64 *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * 6) return;
  out[i] = P.stop_args[(u64)lanes[i / 6] * 6 + i % 6];
}

// Exit records of lanes [first, first + count) (wtfgpu_read_exits).
__global__ void k_pack_exits(Dev P, u32 first, u32 count, wtfgpu_exit_t *out) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const u32 lane = first + i;
  wtfgpu_exit_t e;
  e.status = P.status[lane];
  e.vector = e.error = e.opcode = 0;
  e.addr = 0;
  if (e.status == WTFGPU_EXIT_FAULT) {
    const ExitInfo x = P.exinfo[lane];
    e.vector = x.vector;
    e.error = x.error;
    e.addr = x.addr;
    e.opcode = x.cpl;
  } else if (e.status == WTFGPU_EXIT_UNIMPLEMENTED) {
    e.opcode = P.exinfo[lane].opcode;
  }
  e.rip = P.rip[lane];
  e.icount = P.icount[lane];
  out[i] = e;
}

// Regrouping keys: running lanes by rip (lanes at one rip become neighbours,
// so one wave step serves them all), every other lane after them (their
// waves find nothing to run and leave at once).
// They also count the running lanes (P.stat[3]): a launch with none returns at once.
__global__ void k_regroup_keys(Dev P, u32 first, u32 count, u32 *keys, u32 *lanes) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = i < count;
  const u32 lane = first + (in ? i : 0);
  const bool run = in && P.status[lane] == WTFGPU_RUNNING;
  const u64 m = __ballot(run);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd((unsigned long long *)&P.stat[3], (unsigned long long)__popcll(m));
  if (!in) return;
  const u32 r = (u32)P.rip[lane] & 0xffffffu;  // 24 key bits: three radix passes
  keys[i] = run ? (r == 0xffffffu ? r - 1 : r) : 0xffffffu;
  lanes[i] = lane;
}

// Empty the coverage sets of a lane list (generation bump: O(1) per lane).
__global__ void k_cov_clear(Dev P, const u32 *lanes, u32 n) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32 lane = lanes[i];
  P.lane_gen[lane] += 1;
  P.cov_cnt[lane] = 0;
  P.cov_overflow[lane] = 0;
}

// Bytes set in the coverage map but not in its shadow (what a MAX all-reduce
// brought in from other shards since the last look), as byte indices; with
// `write`, the shadow catches up with the map. Sixteen bytes per thread.
__global__ void k_cov_absorb(const u8 *map, u8 *shadow, u64 n16, u64 *out_idx, u64 cap,
                             unsigned long long *count, int write) {
  const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n16) return;
  const uint4 m = ((const uint4 *)map)[t], s = ((const uint4 *)shadow)[t];
  if (m.x == s.x && m.y == s.y && m.z == s.z && m.w == s.w) return;
  const u32 mw[4] = {m.x, m.y, m.z, m.w}, sw[4] = {s.x, s.y, s.z, s.w};
  for (int w = 0; w < 4; w++)
    for (int b = 0; b < 4; b++)
      if (((mw[w] >> (8 * b)) & 0xff) && !((sw[w] >> (8 * b)) & 0xff)) {
        const unsigned long long pos = atomicAdd(count, 1ull);
        if (write && pos < cap) out_idx[pos] = t * 16 + w * 4 + b;
      }
  if (write) ((uint4 *)shadow)[t] = m;
}

// A merged map from the other shards (bytes are 0 / 1, so OR is the MAX):
// the deferred shard merge (CoverageExchange_t::MergeEnd); k_cov_absorb then
// reports what it added.
__global__ void k_cov_merge_in(uint4 *map, const uint4 *src, u64 n16) {
  const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n16) return;
  const uint4 a = map[t], b = src[t];
  if ((b.x & ~a.x) | (b.y & ~a.y) | (b.z & ~a.z) | (b.w & ~a.w)) map[t] = uint4{a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w};
}

// Per-lane feed regions (streaming): `n` lanes, lane lanes[i] gets
// len[i] bytes from src + off[i] at its region.
// Lane i's feed: bytes [off[i], off[i + 1]) of src into the lane's region, its
// read position and end set; a lane without a feed (has[i] = 0) or with one
// larger than its region keeps none (the host handler serves it).
__global__ void k_feed_scatter(u8 *feed, u64 stride, const u32 *lanes, const u64 *off, const u8 *has, u32 n,
                               const u8 *src, u64 *feed_pos, u64 *feed_end) {
  const u32 i = blockIdx.x;
  if (i >= n) return;
  const u32 lane = lanes[i];
  const u64 o = off[i], len = off[i + 1] - o;
  const bool keep = (!has || has[i]) && len <= stride;
  if (threadIdx.x == 0) {
    feed_pos[lane] = keep ? (u64)lane * stride : ~0ull;
    feed_end[lane] = keep ? (u64)lane * stride + len : 0;
  }
  if (!keep) return;
  u8 *dst = feed + (u64)lane * stride;
  const u8 *sp = src + o;
  for (u64 k = threadIdx.x; k < len; k += blockDim.x) dst[k] = sp[k];
}

__global__ void k_cov_commit(Dev P, const u64 *rips, u64 n) {
  const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n || !P.code_keys) return;
  const u64 rip = rips[t];
  u32 h = (u32)mix64(rip >> 12) & P.code_mask;
  for (u32 i = 0; i <= P.code_mask; i++) {
    const u64 k = P.code_keys[h];
    if (k == rip >> 12) {
      const u64 at = (u64)P.code_slot[h] * WTFGPU_PAGE_SIZE + (rip & 0xfff);
      P.cov_map[at] = 1;
      P.cov_shadow[at] = 1;  // this shard's own find: not reported by absorb
      return;
    }
    if (k == EMPTY_KEY) break;
    h = (h + 1) & P.code_mask;
  }
  // not a code byte of a code page (a rip elsewhere, an edge): the extra set,
  // kept at most 3/4 full (a value that does not fit is logged again later)
  if (!P.extra_keys || rip == EMPTY_KEY) return;
  u32 g = (u32)mix64(rip) & P.extra_mask;
  for (u32 i = 0; i <= P.extra_mask / 4; i++) {
    const unsigned long long prev = atomicCAS((unsigned long long *)&P.extra_keys[g], EMPTY_KEY, rip);
    if (prev == EMPTY_KEY || prev == rip) return;
    g = (g + 1) & P.extra_mask;
  }
}

}  // namespace

// ====================================================================== host
#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      fprintf(stderr, "wtfgpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                                 \
      return WTFGPU_ERR_HIP;                                                             \
    }                                                                                    \
  } while (0)

// What a queue owns (wtfgpu_select_queue): its stream and the scratch a call
// on it stages through, so that work queued on one (a k_run slice) runs while
// the host drives the other.
struct QueueRes {
  hipStream_t stream = nullptr;
  u8 *d_scratch = nullptr;
  u64 scratch_bytes = 0;
  u8 *h_stage = nullptr;  // pinned host staging of the queue's asynchronous uploads
  u64 stage_bytes = 0;
  u64 *d_stat = nullptr;
  Dev *d_dev = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  u32 *d_rkeys = nullptr, *d_rkeys2 = nullptr, *d_rlanes = nullptr;
  void *d_rtemp = nullptr;
  size_t rtemp_bytes = 0;
  u32 async_launches = 0;  // wtfgpu_run_async in flight (0 = none)
  // asynchronous plumbing (see ring_put / wtfgpu_prefetch_*): the pinned
  // upload ring, the prefetched exits / coverage entries, the event after the
  // queue's plumbing of its last run (another queue's work is ordered after it)
  u8 *h_ring = nullptr;
  u64 ring_cap = 0, ring_off = 0;
  wtfgpu_exit_t *d_exq = nullptr;
  u64 exq_cap = 0;
  u8 *d_pcov = nullptr;
  hipEvent_t ev_pre = nullptr;
  bool pre_valid = false;
};

struct wtfgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  Dev P{};
  // pool
  u8 *d_pool = nullptr;
  u32 *d_pfnmap = nullptr;
  u32 *d_ptbits = nullptr;
  u64 npool = 0;
  // lanes
  u64 *d_gpr = nullptr, *d_rip = nullptr, *d_rflags = nullptr, *d_fsb = nullptr, *d_gsb = nullptr,
      *d_icount = nullptr, *d_nbytes = nullptr;
  u32 *d_status = nullptr, *d_lflags = nullptr, *d_ovcount = nullptr, *d_ovgpfn = nullptr;
  ExitInfo *d_exinfo = nullptr;
  LaneSys *d_sys = nullptr;
  u32 *d_guc = nullptr;       // device-wide decoded-uop cache (Dev::guc)
  u8 *d_warm = nullptr;       // LDS uop-cache images, UC_QUEUES sets of warm_n (Dev::warm)
  u32 warm_n = 0;
  u64 *d_rdseed = nullptr;    // per-lane Rdrand seeds (Dev::rd_seed)
  u64 *d_stopargs = nullptr;  // per-lane STOP_ARGS arguments (Dev::stop_args)
  u64 *d_extra = nullptr;     // coverage values outside code pages (Dev::extra_keys)
  u8 *d_tn_buf = nullptr;     // Tenet traces (g_tn)
  u64 *d_tn_pos = nullptr, *d_tn_cpos = nullptr, *d_tn_ipos = nullptr, *d_tn_last = nullptr;
  u32 *d_tn_mute = nullptr;
  u64 tn_cap = 0;
  u64 *d_trace = nullptr;     // rip traces (Dev::trace)
  u32 *d_tracecnt = nullptr;
  u32 *d_edgecnt = nullptr;  // [nlanes][2] (wtfgpu_set_edges)
  LaneTlb *d_tlbs = nullptr;  // translation state kept between k_run launches
  u8 *d_lcopy = nullptr;      // WTFGPU_LANE_LDS=2: the rare path's lane copies
  u32 *d_tlbok = nullptr;
  u8 *d_ovdata = nullptr;
  wtfgpu_regs_t *d_full = nullptr;  // full per-lane architectural state (cold fields)
  // breakpoints
  u64 *d_bp = nullptr;
  u64 *d_actkeys = nullptr;
  wtfgpu_bp_action_t *d_act = nullptr;
  u64 *d_feedpos = nullptr, *d_feedend = nullptr;
  u8 *d_feeddata = nullptr;
  u64 feed_cap = 0;
  u64 feed_stride = 0;  // streaming: bytes of feed region per lane (0 = one packed feed)
  bool ins_on = false;  // a declared insert (wtfgpu_set_insert) runs after each feed upload
  wtfgpu_insert_t ins{};
  // coverage
  u64 *d_codekeys = nullptr;
  u32 *d_codeslot = nullptr;
  u8 *d_covmap = nullptr;
  u8 *d_covshadow = nullptr;  // the map as of the last absorb / own commit
  u64 ncovslots = 0;
  u64 *d_covrip = nullptr;
  u32 *d_covgen = nullptr, *d_lanegen = nullptr, *d_covcnt = nullptr, *d_covovf = nullptr;
  std::vector<u64> code_vpns;
  // host copy of the pool (page-table marking, host-side reads)
  std::vector<u8> h_pool;
  std::vector<u32> h_map;
  // misc
  u64 *d_stat = nullptr;
  InitState *d_init = nullptr;
  wtfgpu_regs_t *d_init_full = nullptr;  // initial architectural state, copied per lane by k_restore
  Dev *d_dev = nullptr;                  // device copy of P for k_run
  wtfgpu_regs_t initial{};
  bool have_initial = false;
  u8 *d_scratch = nullptr;
  u8 *h_stage = nullptr;
  u64 stage_bytes = 0;
  // cross-wave regrouping (wtfgpu_run): sort keys, the lane order, radix-sort scratch
  u32 *d_rkeys = nullptr, *d_rkeys2 = nullptr, *d_rlanes = nullptr, *d_perm = nullptr;
  void *d_rtemp = nullptr;
  size_t rtemp_bytes = 0;
  u64 scratch_bytes = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  u64 regroup_steps = 1024;
  // regrouping pays only while lanes diverge from their wave neighbours:
  // regroup_now() measures both schedules (lanes retired per wave-step) and
  // runs the better one, probing the other every kProbe-th run; all counts,
  // no clocks, so a fixed-seed campaign schedules the same way every time
  // (WTFGPU_REGROUP_AUTO=0: always regroup)
  // A synchronous run to completion (wtfgpu_run with no step bound) ends
  // with the same lane states in either order, so there the choice is by
  // measured kernel time per retired instruction instead: a run whose longest
  // lane sets its length (SYN) gains nothing from denser wave-steps and pays
  // for the sorts and the shorter launches.
  bool regroup_auto = true;
  double lps_sched[2] = {0, 0};  // lanes per wave-step, EMA: [0] fixed order, [1] regrouped
  u64 rg_runs = 0;
  u8 rg_used[2] = {2, 2};  // per queue: its run in flight regroups (1), not (0), unmeasured (2)
  double nspi_sched[2] = {0, 0};  // run-to-completion runs: kernel ns per retired instruction, EMA
  u64 rg_sync_runs = 0;
  u32 async_launches = 0;
  u8 *h_ring = nullptr;
  u64 ring_cap = 0, ring_off = 0;
  wtfgpu_exit_t *d_exq = nullptr;
  u64 exq_cap = 0;
  u8 *d_pcov = nullptr;
  hipEvent_t ev_pre = nullptr;
  bool pre_valid = false;
  // the current queue's resources live in the members above; the others here
  QueueRes queues[2];
  u32 cur_queue = 0;
};

namespace {

template <typename T>
int dalloc(T **p, u64 count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void **)p, count * sizeof(T));
  if (e != hipSuccess) {
    fprintf(stderr, "wtfgpu: hipMalloc(%llu bytes) failed: %s\n", (unsigned long long)(count * sizeof(T)),
            hipGetErrorString(e));
    return WTFGPU_ERR_OOM;
  }
  return WTFGPU_OK;
}
template <typename T>
void dfree(T *&p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// The current queue's device scratch, at least `bytes`. Growth is geometric
// and stream-ordered (hipFreeAsync / hipMallocAsync on the queue's stream):
// the old buffer is released after the queue's earlier work that reads it
// (e.g. an asynchronous k_feed_scatter) and nothing synchronises the device,
// so the other queue's k_run slice keeps running.
int ensure_scratch(wtfgpu_ctx *c, u64 bytes) {
  if (c->scratch_bytes >= bytes) return WTFGPU_OK;
  const u64 want = std::max<u64>(std::max<u64>(bytes, 2 * c->scratch_bytes), 1ull << 20);
  if (c->d_scratch) HIPCHK(hipFreeAsync(c->d_scratch, c->stream));
  c->d_scratch = nullptr;
  c->scratch_bytes = 0;
  if (hipMallocAsync((void **)&c->d_scratch, want, c->stream) != hipSuccess) return WTFGPU_ERR_OOM;
  c->scratch_bytes = want;
  return WTFGPU_OK;
}

// The current queue's pinned staging buffer, at least `bytes`. Only for a
// call that synchronised the queue's stream first (no DMA still reads it).
int ensure_stage(wtfgpu_ctx *c, u64 bytes) {
  if (bytes <= c->stage_bytes) return WTFGPU_OK;
  if (c->h_stage) HIPCHK(hipHostFree(c->h_stage));
  c->h_stage = nullptr;
  c->stage_bytes = 0;
  const u64 want = std::max<u64>(bytes * 2, 1 << 20);
  if (hipHostMalloc((void **)&c->h_stage, want, hipHostMallocDefault) != hipSuccess) return WTFGPU_ERR_OOM;
  c->stage_bytes = want;
  return WTFGPU_OK;
}

// Pinned staging for an asynchronous upload on the current queue: the bytes
// are copied into the queue's pinned ring and the caller queues the DMA from
// there, so the call returns without waiting for the queue's stream (whose
// earlier kernels may wait behind the other queue's k_run for free compute
// units: every VGPR of a SIMD is taken by two k_run waves). The ring restarts
// after each synchronisation of the stream (wtfgpu_run_wait, or here when
// full): no DMA still reads it then.
u8 *ring_put(wtfgpu_ctx *c, const void *src, u64 bytes) {
  const u64 need = (bytes + 255) & ~255ull;
  if (c->ring_off + need > c->ring_cap) {
    if (hipStreamSynchronize(c->stream) != hipSuccess) return nullptr;
    c->ring_off = 0;
    if (need > c->ring_cap) {
      if (c->h_ring) (void)hipHostFree(c->h_ring);
      c->h_ring = nullptr;
      c->ring_cap = 0;
      const u64 want = std::max<u64>(need * 2, 4ull << 20);
      if (hipHostMalloc((void **)&c->h_ring, want, hipHostMallocDefault) != hipSuccess) return nullptr;
      c->ring_cap = want;
    }
  }
  u8 *p = c->h_ring + c->ring_off;
  if (src && bytes) memcpy(p, src, bytes);
  c->ring_off += need;
  return p;
}
// the current queue's stream is idle: the ring may be reused from its start
void ring_reset(wtfgpu_ctx *c) { c->ring_off = 0; }

void queue_save(wtfgpu_ctx *c, QueueRes &q) {
  q.stream = c->stream;
  q.d_scratch = c->d_scratch;
  q.scratch_bytes = c->scratch_bytes;
  q.h_stage = c->h_stage;
  q.stage_bytes = c->stage_bytes;
  q.d_stat = c->d_stat;
  q.d_dev = c->d_dev;
  q.ev0 = c->ev0;
  q.ev1 = c->ev1;
  q.d_rkeys = c->d_rkeys;
  q.d_rkeys2 = c->d_rkeys2;
  q.d_rlanes = c->d_rlanes;
  q.d_rtemp = c->d_rtemp;
  q.rtemp_bytes = c->rtemp_bytes;
  q.async_launches = c->async_launches;
  q.h_ring = c->h_ring;
  q.ring_cap = c->ring_cap;
  q.ring_off = c->ring_off;
  q.d_exq = c->d_exq;
  q.exq_cap = c->exq_cap;
  q.d_pcov = c->d_pcov;
  q.ev_pre = c->ev_pre;
  q.pre_valid = c->pre_valid;
}
void queue_load(wtfgpu_ctx *c, const QueueRes &q) {
  c->stream = q.stream;
  c->d_scratch = q.d_scratch;
  c->scratch_bytes = q.scratch_bytes;
  c->h_stage = q.h_stage;
  c->stage_bytes = q.stage_bytes;
  c->d_stat = q.d_stat;
  c->d_dev = q.d_dev;
  c->ev0 = q.ev0;
  c->ev1 = q.ev1;
  c->d_rkeys = q.d_rkeys;
  c->d_rkeys2 = q.d_rkeys2;
  c->d_rlanes = q.d_rlanes;
  c->d_rtemp = q.d_rtemp;
  c->rtemp_bytes = q.rtemp_bytes;
  c->async_launches = q.async_launches;
  c->h_ring = q.h_ring;
  c->ring_cap = q.ring_cap;
  c->ring_off = q.ring_off;
  c->d_exq = q.d_exq;
  c->exq_cap = q.exq_cap;
  c->d_pcov = q.d_pcov;
  c->ev_pre = q.ev_pre;
  c->pre_valid = q.pre_valid;
}
int queue_create(QueueRes &q) {
  HIPCHK(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreate(&q.ev0));
  HIPCHK(hipEventCreate(&q.ev1));
  HIPCHK(hipEventCreateWithFlags(&q.ev_pre, hipEventDisableTiming));
  if (dalloc(&q.d_stat, STAT_N) || dalloc(&q.d_dev, 1)) return WTFGPU_ERR_OOM;
  return WTFGPU_OK;
}
void regroup_free(u32 *&k, u32 *&k2, u32 *&l, void *&t, size_t &tb) {
  dfree(k);
  dfree(k2);
  dfree(l);
  if (t) (void)hipFree(t);
  t = nullptr;
  tb = 0;
}
void queue_destroy(QueueRes &q) {
  if (q.stream) (void)hipStreamSynchronize(q.stream);
  regroup_free(q.d_rkeys, q.d_rkeys2, q.d_rlanes, q.d_rtemp, q.rtemp_bytes);
  dfree(q.d_stat);
  dfree(q.d_dev);
  dfree(q.d_scratch);
  dfree(q.d_exq);
  dfree(q.d_pcov);
  if (q.h_stage) (void)hipHostFree(q.h_stage);
  q.h_stage = nullptr;
  if (q.h_ring) (void)hipHostFree(q.h_ring);
  q.h_ring = nullptr;
  if (q.ev_pre) (void)hipEventDestroy(q.ev_pre);
  if (q.ev0) (void)hipEventDestroy(q.ev0);
  if (q.ev1) (void)hipEventDestroy(q.ev1);
  if (q.stream) (void)hipStreamDestroy(q.stream);
  q = QueueRes{};
}

u64 hmix(u64 x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

u32 table_size(u64 n) {
  u32 s = 16;
  while (s < 2 * n + 2) s <<= 1;
  return s;
}

InitState make_init(const wtfgpu_regs_t &r) {
  InitState s{};
  for (int i = 0; i < 16; i++) s.g[i] = r.gpr[i];
  s.rip = r.rip;
  s.rflags = r.rflags;
  s.fsb = r.seg[WTFGPU_FS].base;
  s.gsb = r.seg[WTFGPU_GS].base;
  s.sys.cr0 = r.cr0;
  s.sys.cr3 = r.cr3;
  s.sys.cr4 = r.cr4;
  s.sys.efer = (r.efer & ~EFER_M32) | (compat_sel(r.star, r.seg[WTFGPU_CS].selector) ? EFER_M32 : 0);  // U29
  s.sys.cpl = r.seg[WTFGPU_CS].selector & 3;
  s.sys.star = r.star;
  s.sys.lstar = r.lstar;
  s.sys.sfmask = r.sfmask;
  s.sys.kgs = r.kernel_gs_base;
  s.sys.cs = r.seg[WTFGPU_CS].selector;
  s.sys.idtr = r.idtr_base;
  s.sys.idtr_limit = r.idtr_limit;
  s.sys.tss = r.seg[WTFGPU_TR].base;
  s.sys.cr2 = r.cr2;
  s.sys.deliv_icount = ~0ull;
  s.sys.ss = r.seg[WTFGPU_SS].selector;
  return s;
}

bool lanes_ok(wtfgpu_ctx *c, u32 first, u32 count) {
  return c && c->d_gpr && (u64)first + count <= c->P.nlanes;
}

template <typename T>
int d2h(wtfgpu_ctx *c, T *dst, const T *src, u64 n) {
  HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyDeviceToHost, c->stream));
  return WTFGPU_OK;
}
template <typename T>
int h2d(wtfgpu_ctx *c, T *dst, const T *src, u64 n) {
  HIPCHK(hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return WTFGPU_OK;
}

constexpr u32 kExtraEntries = 1u << 20;

// The warm images of every queue dropped (rare: setup-time changes). Every
// queue is drained first: a launch in flight on another queue reads or
// writes its set.
int warm_clear(wtfgpu_ctx *c) {
  if (!c->d_warm) return WTFGPU_OK;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemset(c->d_warm, 0xff, UC_IMAGE_BYTES * c->warm_n * UC_QUEUES));
  return WTFGPU_OK;
}

// Entries depend on the pool pages and the breakpoint set: cleared with them.
int guc_clear(wtfgpu_ctx *c) {
  if (c->d_guc) HIPCHK(hipMemsetAsync(c->d_guc, 0, (u64)(c->P.guc_mask + 1) * GUC_WORDS * 4, c->stream));
  return warm_clear(c);
}

}  // namespace

extern "C" {

int wtfgpu_abi_version(void) { return WTFGPU_ABI_VERSION; }

int wtfgpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int wtfgpu_create(int device, wtfgpu_ctx **out) {
  if (!out) return WTFGPU_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return WTFGPU_ERR_NODEV;
  HIPCHK(hipSetDevice(device));
  wtfgpu_ctx *c = new (std::nothrow) wtfgpu_ctx();
  if (!c) return WTFGPU_ERR_OOM;
  c->device = device;
  // regrouped launches of 1024 wave-steps by default (measured on MI355X:
  // HEVD 0.73M -> 1.9M execs/s, tlv 2.0M -> 2.1-2.3M, SYN 0.88M -> 0.81M)
  c->regroup_steps = 1024;
  if (const char *e = getenv("WTFGPU_REGROUP_STEPS")) c->regroup_steps = strtoull(e, nullptr, 0);
  if (const char *e = getenv("WTFGPU_REGROUP_AUTO")) c->regroup_auto = e[0] != '0';
  {
    // shared decoded-uop cache: 256K entries of 192 bytes, 48 MB (WTFGPU_GUC=0:
    // off; 32K entries had HEVD I/O launches 2-3 % longer, profiles/r06_ab_guc_size.txt)
    const char *e = getenv("WTFGPU_GUC");
    const u32 n = e ? (u32)strtoul(e, nullptr, 0) : 262144u;
    if (n && !(n & (n - 1))) {
      if (dalloc(&c->d_guc, (u64)n * GUC_WORDS)) {
        delete c;
        return WTFGPU_ERR_OOM;
      }
      HIPCHK(hipMemset(c->d_guc, 0, (u64)n * GUC_WORDS * 4));
      c->P.guc = c->d_guc;
      c->P.guc_mask = n - 1;
    }
  }
  if (queue_create(c->queues[0]) || dalloc(&c->d_init, 1) || dalloc(&c->d_init_full, 1)) {
    wtfgpu_destroy(c);
    return WTFGPU_ERR_OOM;
  }
  queue_load(c, c->queues[0]);
  *out = c;
  return WTFGPU_OK;
}

void *wtfgpu_stream(wtfgpu_ctx *c) { return c ? (void *)c->stream : nullptr; }

static void free_lanes(wtfgpu_ctx *c) {
  dfree(c->d_feedpos);  // sized by the lane count
  dfree(c->d_feedend);
  c->d_feedpos = c->d_feedend = nullptr;
  c->P.feed_pos = nullptr;
  c->P.feed_end = nullptr;
  dfree(c->d_gpr);
  dfree(c->d_rip);
  dfree(c->d_rflags);
  dfree(c->d_fsb);
  dfree(c->d_gsb);
  dfree(c->d_icount);
  dfree(c->d_nbytes);
  dfree(c->d_status);
  dfree(c->d_lflags);
  dfree(c->d_ovcount);
  dfree(c->d_ovgpfn);
  dfree(c->d_exinfo);
  dfree(c->d_sys);
  dfree(c->d_tlbs);
  dfree(c->d_lcopy);
  dfree(c->d_tlbok);
  dfree(c->d_rdseed);
  dfree(c->d_stopargs);
  dfree(c->d_extra);
  dfree(c->d_trace);
  dfree(c->d_tracecnt);
  dfree(c->d_edgecnt);
  c->d_trace = nullptr;
  c->d_tracecnt = nullptr;
  c->d_edgecnt = nullptr;
  c->P.trace = nullptr;
  c->P.trace_cnt = nullptr;
  c->P.edge_cnt = nullptr;
  c->P.trace_cap = 0;
  if (c->d_tn_buf) {  // Tenet buffers are sized by the lane count
    dfree(c->d_tn_buf);
    dfree(c->d_tn_pos);
    dfree(c->d_tn_cpos);
    dfree(c->d_tn_ipos);
    dfree(c->d_tn_last);
    dfree(c->d_tn_mute);
    c->d_tn_buf = nullptr, c->d_tn_pos = c->d_tn_cpos = c->d_tn_ipos = c->d_tn_last = nullptr, c->d_tn_mute = nullptr;
    c->tn_cap = 0;
    const TenetDev T{};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tn), &T, sizeof(T));
  }
  dfree(c->d_ovdata);
  dfree(c->d_full);
  dfree(c->d_perm);
  // regrouping buffers are sized by the lane count: every queue's
  regroup_free(c->d_rkeys, c->d_rkeys2, c->d_rlanes, c->d_rtemp, c->rtemp_bytes);
  for (u32 q = 0; q < 2; q++)
    if (q != c->cur_queue) {
      QueueRes &Q = c->queues[q];
      regroup_free(Q.d_rkeys, Q.d_rkeys2, Q.d_rlanes, Q.d_rtemp, Q.rtemp_bytes);
    }
  dfree(c->d_covrip);
  dfree(c->d_covgen);
  dfree(c->d_lanegen);
  dfree(c->d_covcnt);
  dfree(c->d_covovf);
}

int wtfgpu_destroy(wtfgpu_ctx *c) {
  if (!c) return WTFGPU_OK;
  (void)hipSetDevice(c->device);
  for (QueueRes &q : c->queues)
    if (q.stream) (void)hipStreamSynchronize(q.stream);
  free_lanes(c);
  dfree(c->d_guc);
  if (c->d_warm) (void)hipFree(c->d_warm);
  dfree(c->d_pool);
  dfree(c->d_pfnmap);
  dfree(c->d_ptbits);
  dfree(c->d_bp);
  dfree(c->d_actkeys);
  dfree(c->d_act);
  dfree(c->d_feedpos);
  dfree(c->d_feedend);
  dfree(c->d_feeddata);
  dfree(c->d_codekeys);
  dfree(c->d_codeslot);
  dfree(c->d_covmap);
  dfree(c->d_covshadow);
  dfree(c->d_init);
  dfree(c->d_init_full);
  queue_save(c, c->queues[c->cur_queue]);
  for (QueueRes &q : c->queues) queue_destroy(q);
  delete c;
  return WTFGPU_OK;
}

static int mark_pt_pages(wtfgpu_ctx *c);

// Snapshot page pool. Also marks page-table pages reachable from the
// initial cr3 (set later by wtfgpu_set_initial_state).
int wtfgpu_load_pool(wtfgpu_ctx *c, const uint64_t *gpfns, const uint8_t *pages, uint64_t npages) {
  if (!c || (npages && (!gpfns || !pages))) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  dfree(c->d_pool);
  dfree(c->d_pfnmap);
  dfree(c->d_ptbits);
  u64 maxpfn = 0;
  for (u64 i = 0; i < npages; i++) maxpfn = std::max<u64>(maxpfn, gpfns[i]);
  const u64 maplen = npages ? maxpfn + 1 : 1;
  std::vector<u32> map(maplen, 0);
  for (u64 i = 0; i < npages; i++)
    if (map[gpfns[i]] == 0) map[gpfns[i]] = (u32)(i + 1);  // first occurrence wins (try_emplace)
  if (dalloc(&c->d_pool, (npages + 1) * WTFGPU_PAGE_SIZE)) return WTFGPU_ERR_OOM;
  // TLB entries pack permission bits into the low 12 bits of page pointers
  if ((uintptr_t)c->d_pool & 0xfff) {
    fprintf(stderr, "wtfgpu: page pool not 4 KiB aligned\n");
    return WTFGPU_ERR_OOM;
  }
  if (dalloc(&c->d_pfnmap, maplen)) return WTFGPU_ERR_OOM;
  if (dalloc(&c->d_ptbits, (maplen + 31) / 32)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemsetAsync(c->d_pool, 0, WTFGPU_PAGE_SIZE, c->stream));
  if (npages)
    HIPCHK(hipMemcpyAsync(c->d_pool + WTFGPU_PAGE_SIZE, pages, npages * WTFGPU_PAGE_SIZE, hipMemcpyHostToDevice,
                          c->stream));
  HIPCHK(hipMemcpyAsync(c->d_pfnmap, map.data(), maplen * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(c->d_ptbits, 0, (maplen + 31) / 32 * 4, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));

  c->npool = npages;
  c->h_pool.assign(pages, pages + npages * WTFGPU_PAGE_SIZE);
  c->h_map = std::move(map);
  c->P.pool = c->d_pool;
  c->P.pfn_map = c->d_pfnmap;
  c->P.pfn_map_len = maplen;
  c->P.npool = npages;
  c->P.ptbits = c->d_ptbits;
  if (c->d_tlbok) HIPCHK(hipMemsetAsync(c->d_tlbok, 0, (u64)c->P.nlanes * 4, c->stream));  // old page pointers
  if (guc_clear(c)) return WTFGPU_ERR_HIP;
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->have_initial) return mark_pt_pages(c);
  return WTFGPU_OK;
}

int wtfgpu_alloc_lanes(wtfgpu_ctx *c, uint32_t nlanes, uint32_t overlay_pages, uint32_t cov_entries) {
  if (!c || nlanes == 0 || overlay_pages == 0) return WTFGPU_ERR_INVALID;
  if (cov_entries & (cov_entries - 1)) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  free_lanes(c);
  const u64 N = nlanes;
  // lanes per wave: 64. Measured on MI355X (SYN, 64K lanes): 32 and 16 lanes
  // per wave take 2x / 4x the time: the step loop's cost is per wave-step,
  // more resident waves do not overlap it (WTFGPU_LPW overrides, for tests)
  u32 lpw = 64;
  if (const char *e = getenv("WTFGPU_LPW")) {
    const u32 v = (u32)atoi(e);
    if (v == 64 || v == 32 || v == 16) lpw = v;
  }
  int rc = 0;
  rc |= dalloc(&c->d_gpr, 16 * N);
  rc |= dalloc(&c->d_rip, N);
  rc |= dalloc(&c->d_rflags, N);
  rc |= dalloc(&c->d_fsb, N);
  rc |= dalloc(&c->d_gsb, N);
  rc |= dalloc(&c->d_icount, N);
  rc |= dalloc(&c->d_nbytes, N);
  rc |= dalloc(&c->d_status, N);
  rc |= dalloc(&c->d_lflags, N);
  rc |= dalloc(&c->d_ovcount, N);
  rc |= dalloc(&c->d_ovgpfn, (u64)overlay_pages * N);
  rc |= dalloc(&c->d_exinfo, N);
  rc |= dalloc(&c->d_sys, N);
  rc |= dalloc(&c->d_ovdata, N * overlay_pages * WTFGPU_PAGE_SIZE);
  if (!rc && ((uintptr_t)c->d_ovdata & 0xfff)) {
    fprintf(stderr, "wtfgpu: overlay pages not 4 KiB aligned\n");
    return WTFGPU_ERR_OOM;
  }
  rc |= dalloc(&c->d_full, N);
  rc |= dalloc(&c->d_tlbs, N);
#if WTFGPU_LANE_LDS == 2
  rc |= dalloc(&c->d_lcopy, N * sizeof(LaneCopy));
#endif
  rc |= dalloc(&c->d_tlbok, N);
  rc |= dalloc(&c->d_rdseed, N);
  rc |= dalloc(&c->d_stopargs, 6 * N);
  if (!c->d_extra) {  // the aggregate's values outside code pages (Dev::extra_keys): 1M entries
    rc |= dalloc(&c->d_extra, (u64)kExtraEntries);
    if (!rc) HIPCHK(hipMemset(c->d_extra, 0xff, (u64)kExtraEntries * 8));
  }
  if (cov_entries) {
    rc |= dalloc(&c->d_covrip, N * cov_entries);
    rc |= dalloc(&c->d_covgen, N * cov_entries);
    rc |= dalloc(&c->d_lanegen, N);
    rc |= dalloc(&c->d_covcnt, N);
    rc |= dalloc(&c->d_covovf, N);
  }
  if (rc) return WTFGPU_ERR_OOM;
  std::vector<u32> idle(N, WTFGPU_EXIT_IDLE);
  HIPCHK(hipMemcpyAsync(c->d_status, idle.data(), N * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(c->d_ovcount, 0, N * 4, c->stream));
  HIPCHK(hipMemsetAsync(c->d_lflags, 0, N * 4, c->stream));
  HIPCHK(hipMemsetAsync(c->d_tlbok, 0, N * 4, c->stream));
  HIPCHK(hipMemsetAsync(c->d_rdseed, 0, N * 8, c->stream));  // CpuState_t::Seed = 0 (globals.h:1084)
  HIPCHK(hipMemsetAsync(c->d_icount, 0, N * 8, c->stream));
  HIPCHK(hipMemsetAsync(c->d_nbytes, 0, N * 8, c->stream));
  HIPCHK(hipMemsetAsync(c->d_exinfo, 0, N * sizeof(ExitInfo), c->stream));
  if (cov_entries) {
    HIPCHK(hipMemsetAsync(c->d_covgen, 0, N * cov_entries * 4, c->stream));
    std::vector<u32> one(N, 1);  // generation 1: every entry (0) is empty
    HIPCHK(hipMemcpyAsync(c->d_lanegen, one.data(), N * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->d_covcnt, 0, N * 4, c->stream));
    HIPCHK(hipMemsetAsync(c->d_covovf, 0, N * 4, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  Dev &P = c->P;
  P.nlanes = nlanes;
  P.K = overlay_pages;
  P.lpw = lpw;
  P.gpr = c->d_gpr;
  P.rip = c->d_rip;
  P.rflags = c->d_rflags;
  P.fs_base = c->d_fsb;
  P.gs_base = c->d_gsb;
  P.icount = c->d_icount;
  P.nbytes = c->d_nbytes;
  P.status = c->d_status;
  P.lflags = c->d_lflags;
  P.exinfo = c->d_exinfo;
  P.sys = c->d_sys;
  P.tlbs = c->d_tlbs;
  P.lcopy = c->d_lcopy;
  P.tlb_ok = c->d_tlbok;
  P.rd_seed = c->d_rdseed;
  P.stop_args = c->d_stopargs;
  P.extra_keys = c->d_extra;
  P.extra_mask = kExtraEntries - 1;
  P.rd_seed0 = 0;
  P.ov_count = c->d_ovcount;
  P.ov_gpfn = c->d_ovgpfn;
  P.ov_data = c->d_ovdata;
  P.full = c->d_full;
  P.cov_rip = c->d_covrip;
  P.cov_gen = c->d_covgen;
  P.lane_gen = c->d_lanegen;
  P.cov_cnt = c->d_covcnt;
  P.cov_overflow = c->d_covovf;
  P.H = cov_entries;
  P.stat = c->d_stat;
  if (P.edges) return wtfgpu_set_edges(c, 1);  // the counters follow the lane count
  return WTFGPU_OK;
}

uint32_t wtfgpu_lane_count(wtfgpu_ctx *c) { return c ? c->P.nlanes : 0; }

// Walks the initial page tables on the host copy of the pool to mark
// page-table pages (a guest write to one invalidates the lane TLB).
static int mark_pt_pages(wtfgpu_ctx *c) {
  if (!c->d_ptbits) return WTFGPU_OK;
  const u64 maplen = c->h_map.size();
  if (maplen == 0) return WTFGPU_OK;
  std::vector<u32> bits((maplen + 31) / 32, 0);
  auto page = [&](u64 gpfn) -> const u8 * {
    const u32 idx = gpfn < maplen ? c->h_map[gpfn] : 0;
    return idx ? c->h_pool.data() + (u64)(idx - 1) * WTFGPU_PAGE_SIZE : nullptr;
  };
  auto mark = [&](u64 gpfn) {
    if (gpfn < maplen) bits[gpfn >> 5] |= 1u << (gpfn & 31);
  };
  std::vector<std::pair<u64, int>> work;
  work.push_back({c->initial.cr3 >> 12 & 0xffffffffffull, 3});
  while (!work.empty()) {
    auto [pfn, level] = work.back();
    work.pop_back();
    if (pfn < maplen && (bits[pfn >> 5] >> (pfn & 31)) & 1) continue;
    mark(pfn);
    const u8 *pg = page(pfn);
    if (!pg || level == 0) continue;
    for (int i = 0; i < 512; i++) {
      u64 e;
      memcpy(&e, pg + 8 * i, 8);
      if (!(e & 1)) continue;
      if ((level == 1 || level == 2) && (e & 0x80)) continue;  // large leaf
      work.push_back({(e & 0x000ffffffffff000ull) >> 12, level - 1});
    }
  }
  HIPCHK(hipMemcpyAsync(c->d_ptbits, bits.data(), bits.size() * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_set_initial_state(wtfgpu_ctx *c, const wtfgpu_regs_t *regs) {
  if (!c || !regs) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  c->initial = *regs;
  c->have_initial = true;
  c->P.cr3_0 = regs->cr3;
  if (c->d_tlbok) HIPCHK(hipMemsetAsync(c->d_tlbok, 0, (u64)c->P.nlanes * 4, c->stream));  // page-table pages change
  const InitState s = make_init(*regs);
  HIPCHK(hipMemcpyAsync(c->d_init, &s, sizeof(s), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_init_full, regs, sizeof(*regs), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return mark_pt_pages(c);
}

int wtfgpu_set_regroup(wtfgpu_ctx *c, uint64_t steps) {
  if (!c) return WTFGPU_ERR_INVALID;
  c->regroup_steps = steps;
  return WTFGPU_OK;
}

int wtfgpu_set_limit(wtfgpu_ctx *c, uint64_t limit) {
  if (!c) return WTFGPU_ERR_INVALID;
  c->P.limit = limit;
  return WTFGPU_OK;
}

int wtfgpu_set_breakpoints(wtfgpu_ctx *c, const uint64_t *gvas, uint32_t n) {
  if (!c || (n && !gvas)) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  dfree(c->d_bp);
  c->P.bp_keys = nullptr;
  c->P.bp_mask = 0;
  if (guc_clear(c)) return WTFGPU_ERR_HIP;  // shared entries carry the breakpoint flag
  if (n == 0) {
    HIPCHK(hipStreamSynchronize(c->stream));
    return WTFGPU_OK;
  }
  const u32 sz = table_size(n);
  std::vector<u64> t(sz, EMPTY_KEY);
  for (u32 i = 0; i < n; i++) {
    u32 h = (u32)hmix(gvas[i]) & (sz - 1);
    while (t[h] != EMPTY_KEY && t[h] != gvas[i]) h = (h + 1) & (sz - 1);
    t[h] = gvas[i];
  }
  if (dalloc(&c->d_bp, sz)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_bp, t.data(), sz * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->P.bp_keys = c->d_bp;
  c->P.bp_mask = sz - 1;
  return WTFGPU_OK;
}

int wtfgpu_set_breakpoint_actions(wtfgpu_ctx *c, const wtfgpu_bp_action_t *acts, uint32_t n) {
  if (!c || (n && !acts)) return WTFGPU_ERR_INVALID;
  for (u32 i = 0; i < n; i++) {
    if (acts[i].kind > WTFGPU_BPACT_STOP_ARGS || acts[i].gva == EMPTY_KEY) return WTFGPU_ERR_INVALID;
    if (acts[i].kind == WTFGPU_BPACT_STOP_ARGS && acts[i].value > 6) return WTFGPU_ERR_INVALID;
  }
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  dfree(c->d_actkeys);
  dfree(c->d_act);
  c->P.act_keys = nullptr;
  c->P.act = nullptr;
  c->P.act_mask = 0;
  if (n == 0) return WTFGPU_OK;
  const u32 sz = table_size(n);
  std::vector<u64> t(sz, EMPTY_KEY);
  std::vector<wtfgpu_bp_action_t> a(sz);
  memset(a.data(), 0, sz * sizeof(wtfgpu_bp_action_t));
  for (u32 i = 0; i < n; i++) {
    u32 h = (u32)hmix(acts[i].gva) & (sz - 1);
    while (t[h] != EMPTY_KEY && t[h] != acts[i].gva) h = (h + 1) & (sz - 1);
    t[h] = acts[i].gva;
    a[h] = acts[i];
  }
  if (dalloc(&c->d_actkeys, sz) || dalloc(&c->d_act, sz)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_actkeys, t.data(), sz * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_act, a.data(), sz * sizeof(wtfgpu_bp_action_t), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->P.act_keys = c->d_actkeys;
  c->P.act = c->d_act;
  c->P.act_mask = sz - 1;
  return WTFGPU_OK;
}

int wtfgpu_set_feed(wtfgpu_ctx *c, uint32_t first, uint32_t count, const uint64_t *offsets, const uint8_t *has_feed,
                    const uint8_t *bytes, uint64_t nbytes) {
  if (!lanes_ok(c, first, count) || !offsets || (nbytes && !bytes)) return WTFGPU_ERR_INVALID;
  for (u32 i = 0; i < count; i++)
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] > nbytes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  const u64 N = c->P.nlanes;
  if (!c->d_feedpos) {
    if (dalloc(&c->d_feedpos, N) || dalloc(&c->d_feedend, N)) return WTFGPU_ERR_OOM;
    std::vector<u64> none(N, ~0ull);
    HIPCHK(hipMemcpy(c->d_feedpos, none.data(), N * 8, hipMemcpyHostToDevice));
  }
  // the data of one call is the whole feed (earlier feeds are replaced)
  c->feed_stride = 0;  // packed layout (per-lane regions: wtfgpu_set_feed_lanes)
  if (nbytes > c->feed_cap) {
    dfree(c->d_feeddata);
    c->d_feeddata = nullptr;
    c->feed_cap = 0;
    if (dalloc(&c->d_feeddata, nbytes)) return WTFGPU_ERR_OOM;
    c->feed_cap = nbytes;
  }
  std::vector<u64> pos(count), end(count);
  for (u32 i = 0; i < count; i++) {
    const bool has = !has_feed || has_feed[i];
    pos[i] = has ? offsets[i] : ~0ull;
    end[i] = offsets[i + 1];
  }
  if (nbytes) HIPCHK(hipMemcpyAsync(c->d_feeddata, bytes, nbytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_feedpos + first, pos.data(), count * 8ull, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_feedend + first, end.data(), count * 8ull, hipMemcpyHostToDevice, c->stream));
  c->P.feed_pos = c->d_feedpos;
  c->P.feed_end = c->d_feedend;
  c->P.feed_data = c->d_feeddata;
  if (c->ins_on && count) {
    k_insert<<<(count + 63) / 64, 64, 0, c->stream>>>(c->P, c->ins, nullptr, first, count);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_set_insert(wtfgpu_ctx *c, const wtfgpu_insert_t *ins) {
  if (!c) return WTFGPU_ERR_INVALID;
  if (ins && (ins->head_reg > 15 || ins->ptr_reg > 15 || ins->len_reg > 15 || ins->len_arg > 64))
    return WTFGPU_ERR_INVALID;
  c->ins_on = ins != nullptr;
  if (ins) c->ins = *ins;
  return WTFGPU_OK;
}

int wtfgpu_set_code_pages(wtfgpu_ctx *c, const uint64_t *vpns, uint32_t n) {
  if (!c || (n && !vpns)) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  dfree(c->d_codekeys);
  dfree(c->d_codeslot);
  dfree(c->d_covmap);
  dfree(c->d_covshadow);
  c->P.code_keys = nullptr;
  c->P.code_slot = nullptr;
  c->P.cov_map = nullptr;
  c->P.cov_shadow = nullptr;
  c->P.code_mask = 0;
  c->code_vpns.assign(vpns, vpns + n);
  c->ncovslots = n;
  if (n == 0) return WTFGPU_OK;
  const u32 sz = table_size(n);
  std::vector<u64> keys(sz, EMPTY_KEY);
  std::vector<u32> slots(sz, 0);
  for (u32 i = 0; i < n; i++) {
    u32 h = (u32)hmix(vpns[i]) & (sz - 1);
    while (keys[h] != EMPTY_KEY && keys[h] != vpns[i]) h = (h + 1) & (sz - 1);
    keys[h] = vpns[i];
    slots[h] = i;
  }
  if (dalloc(&c->d_codekeys, sz) || dalloc(&c->d_codeslot, sz) || dalloc(&c->d_covmap, (u64)n * WTFGPU_PAGE_SIZE) ||
      dalloc(&c->d_covshadow, (u64)n * WTFGPU_PAGE_SIZE))
    return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_codekeys, keys.data(), sz * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_codeslot, slots.data(), sz * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(c->d_covmap, 0, (u64)n * WTFGPU_PAGE_SIZE, c->stream));
  HIPCHK(hipMemsetAsync(c->d_covshadow, 0, (u64)n * WTFGPU_PAGE_SIZE, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (int rc = warm_clear(c)) return rc;  // images carry UC_COVERED
  c->P.cov_shadow = c->d_covshadow;
  c->P.code_keys = c->d_codekeys;
  c->P.code_slot = c->d_codeslot;
  c->P.code_mask = sz - 1;
  c->P.cov_map = c->d_covmap;
  return WTFGPU_OK;
}

int wtfgpu_restore(wtfgpu_ctx *c, uint32_t first, uint32_t count) {
  if (!lanes_ok(c, first, count) || !c->have_initial) return WTFGPU_ERR_STATE;
  if (count == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  k_restore<<<(count + 255) / 256, 256, 0, c->stream>>>(c->P, c->d_init, c->d_init_full, c->d_full, first, count);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_restore_lanes(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n) {
  if (!c || !c->d_gpr || !c->have_initial || (n && !lanes)) return WTFGPU_ERR_INVALID;
  if (n == 0) return WTFGPU_OK;
  for (u32 i = 0; i < n; i++)
    if (lanes[i] >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  // queued without a wait (ordered before the queue's later work, see ring_put)
  const u8 *st = ring_put(c, lanes, (u64)n * 4);
  if (!st || ensure_scratch(c, (u64)n * 4)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, st, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  k_restore_list<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, c->d_init, c->d_init_full, c->d_full,
                                                         (const u32 *)c->d_scratch, n);
  HIPCHK(hipGetLastError());
  return WTFGPU_OK;
}

int wtfgpu_set_feed_lanes(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, const uint64_t *offsets,
                          const uint8_t *has_feed, const uint8_t *bytes, uint64_t nbytes) {
  if (!c || !c->d_gpr || (n && (!lanes || !offsets)) || (nbytes && !bytes)) return WTFGPU_ERR_INVALID;
  {  // one branch-light pass: lanes in range, offsets ascending within the bytes
    u32 bad = 0;
    for (u32 i = 0; i < n; i++)
      bad |= (u32)(lanes[i] >= c->P.nlanes) | (u32)(offsets[i + 1] < offsets[i]) | (u32)(offsets[i + 1] > nbytes);
    if (bad) return WTFGPU_ERR_INVALID;
  }
  if (n == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  const u64 N = c->P.nlanes;
  if (!c->d_feedpos || c->feed_stride == 0) HIPCHK(hipDeviceSynchronize());  // first use: buffers change under every queue
  if (!c->d_feedpos) {
    if (dalloc(&c->d_feedpos, N) || dalloc(&c->d_feedend, N)) return WTFGPU_ERR_OOM;
    std::vector<u64> none(N, ~0ull);
    HIPCHK(hipMemcpy(c->d_feedpos, none.data(), N * 8, hipMemcpyHostToDevice));
  }
  if (c->feed_stride == 0) {  // switch to per-lane regions (a packed feed's lanes are finished by now)
    const u64 stride = 16384;
    dfree(c->d_feeddata);
    c->d_feeddata = nullptr;
    c->feed_cap = 0;
    if (dalloc(&c->d_feeddata, N * stride)) return WTFGPU_ERR_OOM;
    c->feed_cap = N * stride;
    c->feed_stride = stride;
  }
  // one staging upload of the lane list, the offsets and the flags (the
  // scatter derives each lane's length, position and end), one of the bytes
  // (straight from the caller's buffer: pinned memory DMAs), then one scatter
  const u64 o_off = ((u64)n * 4 + 255) & ~255ull, o_has = (o_off + (u64)(n + 1) * 8 + 255) & ~255ull,
            o_data = (o_has + n + 255) & ~255ull;
  if (ensure_scratch(c, o_data + nbytes)) return WTFGPU_ERR_OOM;
  u8 *stage = ring_put(c, nullptr, o_data);  // (see ring_put: no wait for the queue)
  if (!stage) return WTFGPU_ERR_OOM;
  memcpy(stage, lanes, (u64)n * 4);
  memcpy(stage + o_off, offsets, (u64)(n + 1) * 8);
  if (has_feed) memcpy(stage + o_has, has_feed, n);
  HIPCHK(hipMemcpyAsync(c->d_scratch, stage, o_data, hipMemcpyHostToDevice, c->stream));
  if (nbytes) HIPCHK(hipMemcpyAsync(c->d_scratch + o_data, bytes, nbytes, hipMemcpyHostToDevice, c->stream));
  k_feed_scatter<<<n, 128, 0, c->stream>>>(c->d_feeddata, c->feed_stride, (const u32 *)c->d_scratch,
                                           (const u64 *)(c->d_scratch + o_off), has_feed ? c->d_scratch + o_has : nullptr,
                                           n, c->d_scratch + o_data, c->d_feedpos, c->d_feedend);
  HIPCHK(hipGetLastError());
  // no wait: the queue's later work (its k_run slice) is ordered after the
  // scatter, and the next call on this queue synchronises first
  c->P.feed_pos = c->d_feedpos;
  c->P.feed_end = c->d_feedend;
  c->P.feed_data = c->d_feeddata;
  if (c->ins_on) {  // the declared insert of the listed lanes, ordered after the scatter
    k_insert<<<(n + 63) / 64, 64, 0, c->stream>>>(c->P, c->ins, (const u32 *)c->d_scratch, 0, n);
    HIPCHK(hipGetLastError());
  }
  return WTFGPU_OK;
}

// ---- register I/O

int wtfgpu_read_gprs(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint64_t *out18) {
  if (!lanes_ok(c, first, count) || !out18) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u64 N = c->P.nlanes;
  std::vector<u64> tmp((u64)18 * count);
  int rc = 0;
  for (int i = 0; i < 16; i++) rc |= d2h(c, tmp.data() + (u64)i * count, c->d_gpr + i * N + first, count);
  rc |= d2h(c, tmp.data() + (u64)16 * count, c->d_rip + first, count);
  rc |= d2h(c, tmp.data() + (u64)17 * count, c->d_rflags + first, count);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  for (u64 l = 0; l < count; l++)
    for (int i = 0; i < 18; i++) out18[l * 18 + i] = tmp[(u64)i * count + l];
  return WTFGPU_OK;
}

int wtfgpu_write_gprs(wtfgpu_ctx *c, uint32_t first, uint32_t count, const uint64_t *in18) {
  if (!lanes_ok(c, first, count) || !in18) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u64 N = c->P.nlanes;
  std::vector<u64> tmp((u64)18 * count);
  for (u64 l = 0; l < count; l++)
    for (int i = 0; i < 18; i++) tmp[(u64)i * count + l] = in18[l * 18 + i];
  int rc = 0;
  for (int i = 0; i < 16; i++) rc |= h2d(c, c->d_gpr + i * N + first, tmp.data() + (u64)i * count, count);
  rc |= h2d(c, c->d_rip + first, tmp.data() + (u64)16 * count, count);
  rc |= h2d(c, c->d_rflags + first, tmp.data() + (u64)17 * count, count);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_read_regs(wtfgpu_ctx *c, uint32_t first, uint32_t count, wtfgpu_regs_t *out) {
  if (!lanes_ok(c, first, count) || !out) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  std::vector<u64> g((u64)18 * count);
  int rc = wtfgpu_read_gprs(c, first, count, g.data());
  if (rc) return rc;
  std::vector<u64> fsb(count), gsb(count);
  std::vector<LaneSys> sys(count);
  rc |= d2h(c, out, c->d_full + first, count);
  rc |= d2h(c, fsb.data(), c->d_fsb + first, count);
  rc |= d2h(c, gsb.data(), c->d_gsb + first, count);
  rc |= d2h(c, sys.data(), c->d_sys + first, count);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  for (u64 l = 0; l < count; l++) {
    wtfgpu_regs_t &r = out[l];
    for (int i = 0; i < 16; i++) r.gpr[i] = g[l * 18 + i];
    r.rip = g[l * 18 + 16];
    r.rflags = g[l * 18 + 17];
    r.seg[WTFGPU_FS].base = fsb[l];
    r.seg[WTFGPU_GS].base = gsb[l];
    r.cr0 = sys[l].cr0;
    r.cr3 = sys[l].cr3;
    r.cr4 = sys[l].cr4;
    r.efer = sys[l].efer & ~EFER_M32;
    r.kernel_gs_base = sys[l].kgs;
    r.star = sys[l].star;
    r.lstar = sys[l].lstar;
    r.sfmask = sys[l].sfmask;
    r.cr2 = sys[l].cr2;
    r.seg[WTFGPU_CS].selector = sys[l].cs;
    r.seg[WTFGPU_SS].selector = sys[l].ss;
  }
  return WTFGPU_OK;
}

int wtfgpu_write_regs(wtfgpu_ctx *c, uint32_t first, uint32_t count, const wtfgpu_regs_t *in) {
  if (!lanes_ok(c, first, count) || !in) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  std::vector<u64> g((u64)18 * count), fsb(count), gsb(count);
  std::vector<LaneSys> sys(count);
  for (u64 l = 0; l < count; l++) {
    const wtfgpu_regs_t &r = in[l];
    for (int i = 0; i < 16; i++) g[l * 18 + i] = r.gpr[i];
    g[l * 18 + 16] = r.rip;
    g[l * 18 + 17] = r.rflags;
    fsb[l] = r.seg[WTFGPU_FS].base;
    gsb[l] = r.seg[WTFGPU_GS].base;
    sys[l] = make_init(r).sys;
  }
  int rc = wtfgpu_write_gprs(c, first, count, g.data());
  if (rc) return rc;
  rc |= h2d(c, c->d_full + first, in, count);
  rc |= h2d(c, c->d_fsb + first, fsb.data(), count);
  rc |= h2d(c, c->d_gsb + first, gsb.data(), count);
  rc |= h2d(c, c->d_sys + first, sys.data(), count);
  if (c->d_tlbok) HIPCHK(hipMemsetAsync(c->d_tlbok + first, 0, (u64)count * 4, c->stream));
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_read_exits(wtfgpu_ctx *c, uint32_t first, uint32_t count, wtfgpu_exit_t *out) {
  if (!lanes_ok(c, first, count) || !out) return WTFGPU_ERR_INVALID;
  if (count == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  // packed on the device, one copy back
  const u64 bytes = (u64)count * sizeof(wtfgpu_exit_t);
  if (ensure_scratch(c, bytes)) return WTFGPU_ERR_OOM;
  k_pack_exits<<<(count + 255) / 256, 256, 0, c->stream>>>(c->P, first, count, (wtfgpu_exit_t *)c->d_scratch);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->d_scratch, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

static int set_status_list(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint32_t status, const uint8_t *skip) {
  if (!c || !c->d_status || (n && !lanes)) return WTFGPU_ERR_INVALID;
  if (n == 0) return WTFGPU_OK;
  for (u32 i = 0; i < n; i++)
    if (lanes[i] >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  // lane list (+ skip flags) -> scratch, one scatter kernel: no whole-array round trips
  // queued without a wait (ordered before the queue's later work, see ring_put)
  const u64 o_skip = ((u64)n * 4 + 255) & ~255ull;
  u8 *st = ring_put(c, nullptr, o_skip + n);
  if (!st || ensure_scratch(c, o_skip + n)) return WTFGPU_ERR_OOM;
  memcpy(st, lanes, (u64)n * 4);
  if (skip) memcpy(st + o_skip, skip, n);
  HIPCHK(hipMemcpyAsync(c->d_scratch, st, skip ? o_skip + n : (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  k_set_status<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n, status,
                                                      skip ? c->d_scratch + o_skip : nullptr);
  HIPCHK(hipGetLastError());
  return WTFGPU_OK;
}

int wtfgpu_resume(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, const uint8_t *skip_bp) {
  std::vector<u8> zeros;
  if (!skip_bp) {
    zeros.assign(n, 0);
    skip_bp = zeros.data();
  }
  return set_status_list(c, lanes, n, WTFGPU_RUNNING, skip_bp);
}

int wtfgpu_stop(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint32_t status) {
  return set_status_list(c, lanes, n, status, nullptr);
}

// Regrouping buffers of the current queue (sized by the lane count).
static int regroup_buffers(wtfgpu_ctx *c) {
  if (c->d_rkeys) return WTFGPU_OK;
  const u64 N = c->P.nlanes;
  if (!c->d_perm && dalloc(&c->d_perm, N)) return WTFGPU_ERR_OOM;
  if (dalloc(&c->d_rkeys, N) || dalloc(&c->d_rkeys2, N) || dalloc(&c->d_rlanes, N)) return WTFGPU_ERR_OOM;
  size_t bytes = 0;
  HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, c->d_rkeys, c->d_rkeys2, c->d_rlanes, c->d_perm, (int)N, 0,
                                            24, c->stream));
  HIPCHK(hipMalloc(&c->d_rtemp, bytes));
  c->rtemp_bytes = bytes;
  return WTFGPU_OK;
}

// The kernel parameters of a run on the current queue.
static Dev run_params(wtfgpu_ctx *c, bool regroup) {
  Dev Q = c->P;
  Q.perm = regroup ? c->d_perm : nullptr;
  Q.stat = c->d_stat;
  // warm-started LDS uop caches (WTFGPU_WARM=0: every launch starts empty)
  const char *w = getenv("WTFGPU_WARM");
  if (!(w && atoi(w) == 0)) {
    const u32 need = (u32)((c->P.nlanes + c->P.lpw - 1) / c->P.lpw);  // the most waves a launch can have
    if (c->d_warm && c->warm_n < need) {
      (void)hipDeviceSynchronize();
      (void)hipFree(c->d_warm);
      c->d_warm = nullptr;
    }
    if (!c->d_warm) {
      c->warm_n = need;
      const u64 bytes = UC_IMAGE_BYTES * need * UC_QUEUES;
      if (hipMalloc((void **)&c->d_warm, bytes) != hipSuccess) {
        c->d_warm = nullptr;
      } else if (hipMemset(c->d_warm, 0xff, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(c->d_warm);
        c->d_warm = nullptr;
      }
    }
    Q.warm = c->d_warm ? c->d_warm + (u64)(c->cur_queue % UC_QUEUES) * UC_IMAGE_BYTES * c->warm_n : nullptr;
    Q.warm_n = c->warm_n;
  } else {
    Q.warm = nullptr;
  }
  return Q;
}

// Whether this run regroups (see wtfgpu_ctx::regroup_auto): measure each
// schedule once, then run the one that retires more lanes per wave-step
// (regrouping must win by kMargin: its sorts and shorter launches cost time a
// wave-step count does not show), probing the other every kProbe-th run.
static u64 regroup_now(wtfgpu_ctx *c, u32 count) {
  c->rg_used[c->cur_queue & 1] = 2;  // not a measured choice
  if (!c->regroup_steps || count < 2 * c->P.lpw) return 0;
  if (!c->regroup_auto) return c->regroup_steps;
  static constexpr double kMargin = 1.1;
  static constexpr u64 kProbe = 32;
  const u64 i = c->rg_runs++;
  bool on;
  if (c->lps_sched[1] == 0) on = true;
  else if (c->lps_sched[0] == 0) on = false;
  else {
    on = c->lps_sched[1] > kMargin * c->lps_sched[0];
    if (i % kProbe == kProbe - 1) on = !on;
  }
  c->rg_used[c->cur_queue & 1] = on;
  return on ? c->regroup_steps : 0;
}
// The same choice for a synchronous run to completion, by kernel time per
// retired instruction (its result does not depend on the lane order).
static u64 regroup_now_timed(wtfgpu_ctx *c, u32 count, int &used) {
  used = 2;
  if (!c->regroup_steps || count < 2 * c->P.lpw) return 0;
  if (!c->regroup_auto) return c->regroup_steps;
  static constexpr u64 kProbe = 32;
  const u64 i = c->rg_sync_runs++;
  bool on;
  if (c->nspi_sched[1] == 0) on = true;
  else if (c->nspi_sched[0] == 0) on = false;
  else {
    on = c->nspi_sched[1] < c->nspi_sched[0];
    if (i % kProbe == kProbe - 1) on = !on;
  }
  used = on;
  return on ? c->regroup_steps : 0;
}
static void regroup_observe_timed(wtfgpu_ctx *c, int used, double ms, u64 retired) {
  if (used > 1 || retired < 4096) return;
  const double v = ms * 1e6 / (double)retired;
  double &e = c->nspi_sched[used];
  e = e == 0 ? v : 0.75 * e + 0.25 * v;
}
static void regroup_observe(wtfgpu_ctx *c, u64 group_steps, u64 retired) {
  const u8 used = c->rg_used[c->cur_queue & 1];
  if (used > 1 || group_steps < 64) return;
  const double lps = (double)retired / (double)group_steps;
  double &e = c->lps_sched[used];
  e = e == 0 ? lps : 0.75 * e + 0.25 * lps;
}

// One k_run launch of `steps` wave-steps over [first, first + count), after
// the regrouping sort when on.
static int launch_chunk(wtfgpu_ctx *c, const Dev &Q, u32 first, u32 count, u64 steps, bool regroup) {
  const u32 hwaves = (count + c->P.lpw - 1) / c->P.lpw;
  if (regroup) {
    HIPCHK(hipMemsetAsync(c->d_stat + 2, 0, 16, c->stream));  // running lanes: this launch's (2: after, 3: before)
    k_regroup_keys<<<(count + 255) / 256, 256, 0, c->stream>>>(Q, first, count, c->d_rkeys, c->d_rlanes);
    HIPCHK(hipGetLastError());
    size_t bytes = c->rtemp_bytes;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(c->d_rtemp, bytes, c->d_rkeys, c->d_rkeys2, c->d_rlanes,
                                              c->d_perm + first, (int)count, 0, 24, c->stream));
  }
#if WTFGPU_P_BYREF
  k_run<<<(hwaves + 3) / 4, 256, 0, c->stream>>>(c->d_dev, first, count, steps);
#else
  k_run<<<(hwaves + 3) / 4, 256, 0, c->stream>>>(Q, first, count, steps);
#endif
  HIPCHK(hipGetLastError());
  return WTFGPU_OK;
}

// Diagnostic build only: the per-phase cycle totals of one run (stat[4..11]).
static void print_stamps(const u64 *s) {
#ifdef WTFGPU_STAMPS
  if (s[0])
    fprintf(stderr,
            "wtfgpu stamps (cycles per wave-step, %llu steps): fast loop %.0f, slow: xlate+fill %.0f, coverage %.0f, "
            "exec %.0f, cross-page %.0f; slow steps: miss %llu, codepage %llu, ucmiss %llu, other %llu; "
            "fast lookup %.0f, fast exec %.0f, bp %.0f\n",
            (unsigned long long)s[0], (double)s[4] / s[0], (double)s[6] / s[0], (double)s[7] / s[0],
            (double)s[5] / s[0], (double)s[9] / s[0], (unsigned long long)s[12], (unsigned long long)s[13],
            (unsigned long long)s[14], (unsigned long long)s[15], (double)s[10] / s[0], (double)s[11] / s[0], (double)s[8] / s[0]);
  fprintf(stderr, "wtfgpu stamps generic ops:");
  for (int k = 0; k < 512; k++)
    if (s[16 + k]) fprintf(stderr, " %d:%llu", k, (unsigned long long)s[16 + k]);
  fprintf(stderr, "\n");
  fprintf(stderr, "wtfgpu stamps bp_apply cycles by kind:");
  for (int k = 0; k < 8; k++) fprintf(stderr, " %d:%llu", k, (unsigned long long)s[528 + k]);
  fprintf(stderr, "\n");
#else
  (void)s;
#endif
}

int wtfgpu_run(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint64_t max_steps, wtfgpu_run_stats_t *stats) {
  if (!lanes_ok(c, first, count) || (first % c->P.lpw)) return WTFGPU_ERR_INVALID;
  if (!c->P.pool) return WTFGPU_ERR_STATE;
  if (c->async_launches) return WTFGPU_ERR_STATE;  // wtfgpu_run_wait first
  HIPCHK(hipSetDevice(c->device));
  wtfgpu_run_stats_t st{};
  u64 chunk = 1ull << 20;  // wave-steps per launch: keeps every launch short
  // Cross-wave regrouping: launches of `regroup` wave-steps, between them the
  // lanes are sorted by rip so that lanes that diverged from their wave
  // neighbours meet lanes at the same rip in another wave (wtfgpu_set_regroup,
  // WTFGPU_REGROUP_STEPS; 0 = fixed lane order; regroup_now).
  // (no step bound: a run to completion, see wtfgpu_ctx::nspi_sched)
  const bool to_end = max_steps >= (1ull << 32);
  int used_timed = 2;
  const u64 regroup = to_end ? regroup_now_timed(c, count, used_timed) : regroup_now(c, count);
  if (regroup) {
    chunk = regroup;
    if (int rc = regroup_buffers(c)) return rc;
  }
  const Dev Q = run_params(c, regroup != 0);
#if WTFGPU_P_BYREF
  HIPCHK(hipMemcpyAsync(c->d_dev, &Q, sizeof(Dev), hipMemcpyHostToDevice, c->stream));
#endif
  // launches per host synchronisation: regrouped chunks are short, so a
  // group of them is queued at once (one stats read-back per group)
  const u32 group = regroup ? (u32)std::max<u64>(1, 4096 / regroup) : 1;
  u64 done = 0;
  float ms_total = 0;
  for (;;) {
    HIPCHK(hipMemsetAsync(c->d_stat, 0, STAT_N * 8, c->stream));
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    u32 k = 0;
    for (; k < group && done < max_steps; k++) {
      const u64 steps = std::min<u64>(chunk, max_steps - done);
      if (int rc = launch_chunk(c, Q, first, count, steps, regroup != 0)) return rc;
      done += steps;
    }
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    u64 s[STAT_N];
    HIPCHK(hipMemcpyAsync(s, c->d_stat, sizeof(s), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    ms_total += ms;
    st.kernel_launches += k;
    st.group_steps += s[0];
    st.lane_retired += s[1];
    print_stamps(s);
    if (s[2] == 0 || done >= max_steps) break;
  }
  if (to_end) regroup_observe_timed(c, used_timed, ms_total, st.lane_retired);
  else regroup_observe(c, st.group_steps, st.lane_retired);
  st.kernel_ms = ms_total;
  if (stats) *stats = st;
  return WTFGPU_OK;
}

int wtfgpu_run_async(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint64_t max_steps) {
  if (!lanes_ok(c, first, count) || (first % c->P.lpw) || max_steps == 0 || max_steps > (1ull << 32))
    return WTFGPU_ERR_INVALID;
  if (!c->P.pool) return WTFGPU_ERR_STATE;
  if (c->async_launches) return WTFGPU_ERR_STATE;
  HIPCHK(hipSetDevice(c->device));
  const u64 regroup = regroup_now(c, count);
  const u64 chunk = regroup ? regroup : max_steps;
  if (regroup)
    if (int rc = regroup_buffers(c)) return rc;
  const Dev Q = run_params(c, regroup != 0);
#if WTFGPU_P_BYREF
  HIPCHK(hipMemcpyAsync(c->d_dev, &Q, sizeof(Dev), hipMemcpyHostToDevice, c->stream));
#endif
  HIPCHK(hipEventRecord(c->ev_pre, c->stream));  // the plumbing before this run (wtfgpu_select_queue)
  c->pre_valid = true;
  HIPCHK(hipMemsetAsync(c->d_stat, 0, STAT_N * 8, c->stream));
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  u32 k = 0;
  for (u64 done = 0; done < max_steps; done += chunk, k++) {
    if (int rc = launch_chunk(c, Q, first, count, std::min<u64>(chunk, max_steps - done), regroup != 0)) return rc;
  }
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  c->async_launches = k;
  return WTFGPU_OK;
}

int wtfgpu_run_wait(wtfgpu_ctx *c, wtfgpu_run_stats_t *stats) {
  if (!c) return WTFGPU_ERR_INVALID;
  wtfgpu_run_stats_t st{};
  if (c->async_launches) {
    HIPCHK(hipSetDevice(c->device));
    u64 s[STAT_N];
    HIPCHK(hipMemcpyAsync(s, c->d_stat, sizeof(s), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    ring_reset(c);
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    st.kernel_launches = c->async_launches;
    st.group_steps = s[0];
    st.lane_retired = s[1];
    st.kernel_ms = ms;
    c->async_launches = 0;
    regroup_observe(c, st.group_steps, st.lane_retired);
    print_stamps(s);
  }
  if (stats) *stats = st;
  return WTFGPU_OK;
}

int wtfgpu_prefetch_results(wtfgpu_ctx *c, uint32_t first, uint32_t count, wtfgpu_exit_t *exits, uint64_t *bytes,
                            uint32_t *dirty, uint64_t *stop_args) {
  if (!lanes_ok(c, first, count) || !exits) return WTFGPU_ERR_INVALID;
  if (count == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  if (c->exq_cap < count) {  // stream-ordered, as ensure_scratch
    if (c->d_exq) HIPCHK(hipFreeAsync(c->d_exq, c->stream));
    c->d_exq = nullptr;
    c->exq_cap = 0;
    if (hipMallocAsync((void **)&c->d_exq, (u64)count * sizeof(wtfgpu_exit_t), c->stream) != hipSuccess)
      return WTFGPU_ERR_OOM;
    c->exq_cap = count;
  }
  k_pack_exits<<<(count + 255) / 256, 256, 0, c->stream>>>(c->P, first, count, c->d_exq);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(exits, c->d_exq, (u64)count * sizeof(wtfgpu_exit_t), hipMemcpyDeviceToHost, c->stream));
  if (bytes) HIPCHK(hipMemcpyAsync(bytes, c->d_nbytes + first, (u64)count * 8, hipMemcpyDeviceToHost, c->stream));
  if (dirty) HIPCHK(hipMemcpyAsync(dirty, c->d_ovcount + first, (u64)count * 4, hipMemcpyDeviceToHost, c->stream));
  if (stop_args && c->d_stopargs)
    HIPCHK(hipMemcpyAsync(stop_args, c->d_stopargs + (u64)first * 6, (u64)count * 48, hipMemcpyDeviceToHost,
                          c->stream));
  return WTFGPU_OK;
}

constexpr u64 kPcovCap = 1ull << 22;  // prefetched coverage entries per queue
constexpr u64 kPcovLanes = 256, kPcovRips = kPcovLanes + kPcovCap * 4;

int wtfgpu_prefetch_coverage(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint64_t *hdr) {
  if (!lanes_ok(c, first, count) || !hdr) return WTFGPU_ERR_INVALID;
  if (!c->d_covrip || count == 0) {
    hdr[0] = hdr[1] = 0;
    return WTFGPU_ERR_STATE;  // nothing to prefetch: the caller reads the sets itself
  }
  HIPCHK(hipSetDevice(c->device));
  if (!c->d_pcov && hipMallocAsync((void **)&c->d_pcov, kPcovRips + kPcovCap * 8, c->stream) != hipSuccess) {
    c->d_pcov = nullptr;
    return WTFGPU_ERR_OOM;
  }
  HIPCHK(hipMemsetAsync(c->d_pcov, 0, 16, c->stream));
  k_cov_collect_stopped<<<(count + 3) / 4, 256, 0, c->stream>>>(
      c->P, first, count, (u32 *)(c->d_pcov + kPcovLanes), (u64 *)(c->d_pcov + kPcovRips), kPcovCap,
      (unsigned long long *)c->d_pcov, (u32 *)(c->d_pcov + 8));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(hdr, c->d_pcov, 16, hipMemcpyDeviceToHost, c->stream));
  return WTFGPU_OK;
}

int wtfgpu_prefetched_coverage(wtfgpu_ctx *c, uint32_t *out_lanes, uint64_t *out_rips, uint64_t n) {
  if (!c || (n && (!out_lanes || !out_rips)) || n > kPcovCap || (n && !c->d_pcov)) return WTFGPU_ERR_INVALID;
  if (n == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(out_lanes, c->d_pcov + kPcovLanes, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(out_rips, c->d_pcov + kPcovRips, n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_clear_coverage_lanes(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n) {
  if (!c || (n && !lanes)) return WTFGPU_ERR_INVALID;
  if (!c->d_covrip || n == 0) return WTFGPU_OK;
  for (u32 i = 0; i < n; i++)
    if (lanes[i] >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u8 *st = ring_put(c, lanes, (u64)n * 4);
  if (!st || ensure_scratch(c, (u64)n * 4)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, st, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  k_cov_clear<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n);
  HIPCHK(hipGetLastError());
  return WTFGPU_OK;
}

int wtfgpu_lane_seeds(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint64_t *seeds, int write) {
  if (!c || (n && (!lanes || !seeds)) || !c->d_rdseed) return WTFGPU_ERR_INVALID;
  if (n == 0) return WTFGPU_OK;
  for (u32 i = 0; i < n; i++)
    if (lanes[i] >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u64 o_s = ((u64)n * 4 + 255) & ~255ull;
  if (ensure_scratch(c, o_s + (u64)n * 8)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  if (write) HIPCHK(hipMemcpyAsync(c->d_scratch + o_s, seeds, (u64)n * 8, hipMemcpyHostToDevice, c->stream));
  k_lane_seeds<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n, (u64 *)(c->d_scratch + o_s),
                                                       write);
  HIPCHK(hipGetLastError());
  if (!write) HIPCHK(hipMemcpyAsync(seeds, c->d_scratch + o_s, (u64)n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_read_stop_args(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint64_t *out6) {
  if (!c || (n && (!lanes || !out6)) || !c->d_stopargs) return WTFGPU_ERR_INVALID;
  if (n == 0) return WTFGPU_OK;
  for (u32 i = 0; i < n; i++)
    if (lanes[i] >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u64 o_s = ((u64)n * 4 + 255) & ~255ull;
  if (ensure_scratch(c, o_s + (u64)n * 48)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  k_stop_args<<<(n * 6 + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n,
                                                        (u64 *)(c->d_scratch + o_s));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out6, c->d_scratch + o_s, (u64)n * 48, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_select_queue(wtfgpu_ctx *c, uint32_t queue) {
  if (!c || queue >= 2) return WTFGPU_ERR_INVALID;
  if (queue == c->cur_queue) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  QueueRes &next = c->queues[queue];
  if (!next.stream)
    if (int rc = queue_create(next)) return rc;
  // The plumbing queued on the old queue without a wait (restores, status
  // and feed uploads, wtfgpu_restore_lanes ...) may touch lanes the new
  // queue runs: the new queue's later work is ordered after it. Only after
  // the plumbing: with a run in flight, after the event wtfgpu_run_async
  // recorded before its launches (the two queues' slices still overlap);
  // without one, after everything the old queue holds.
  if (!c->async_launches) {
    HIPCHK(hipEventRecord(c->ev_pre, c->stream));
    c->pre_valid = true;
  }
  if (c->pre_valid) HIPCHK(hipStreamWaitEvent(next.stream, c->ev_pre, 0));
  queue_save(c, c->queues[c->cur_queue]);
  queue_load(c, next);
  c->cur_queue = queue;
  return WTFGPU_OK;
}

// ---- lane memory services
static int lane_mem(wtfgpu_ctx *c, uint32_t lane, u32 op, u64 addr, void *buf, u64 len, i64 *result) {
  if (!c || lane >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  if (ensure_scratch(c, len + 64)) return WTFGPU_ERR_OOM;
  i64 *d_res = (i64 *)c->d_scratch;
  u8 *d_buf = c->d_scratch + 64;
  if ((op == 2 || op == 4) && len) HIPCHK(hipMemcpyAsync(d_buf, buf, len, hipMemcpyHostToDevice, c->stream));
  k_lane_mem<<<1, 64, 0, c->stream>>>(c->P, lane, op, addr, len, d_buf, d_res);
  HIPCHK(hipGetLastError());
  if ((op == 1 || op == 3) && len) HIPCHK(hipMemcpyAsync(buf, d_buf, len, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(result, d_res, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_lane_translate(wtfgpu_ctx *c, uint32_t lane, uint64_t gva, uint64_t *gpa) {
  i64 r = 0;
  int rc = lane_mem(c, lane, 0, gva, nullptr, 0, &r);
  if (rc) return rc;
  if (r < 0) return WTFGPU_ERR_TRANSLATE;
  if (gpa) *gpa = (u64)r;
  return WTFGPU_OK;
}
int wtfgpu_lane_read_phys(wtfgpu_ctx *c, uint32_t lane, uint64_t gpa, void *buf, uint64_t len) {
  i64 r = 0;
  int rc = lane_mem(c, lane, 1, gpa, buf, len, &r);
  return rc ? rc : (r < 0 ? WTFGPU_ERR_TRANSLATE : WTFGPU_OK);
}
int wtfgpu_lane_write_phys(wtfgpu_ctx *c, uint32_t lane, uint64_t gpa, const void *buf, uint64_t len) {
  i64 r = 0;
  int rc = lane_mem(c, lane, 2, gpa, (void *)buf, len, &r);
  return rc ? rc : (r == -2 ? WTFGPU_ERR_OOM : (r < 0 ? WTFGPU_ERR_TRANSLATE : WTFGPU_OK));
}
int wtfgpu_lane_read_virt(wtfgpu_ctx *c, uint32_t lane, uint64_t gva, void *buf, uint64_t len) {
  i64 r = 0;
  int rc = lane_mem(c, lane, 3, gva, buf, len, &r);
  return rc ? rc : (r < 0 ? WTFGPU_ERR_TRANSLATE : WTFGPU_OK);
}
int wtfgpu_lane_write_virt(wtfgpu_ctx *c, uint32_t lane, uint64_t gva, const void *buf, uint64_t len) {
  i64 r = 0;
  int rc = lane_mem(c, lane, 4, gva, (void *)buf, len, &r);
  return rc ? rc : (r == -2 ? WTFGPU_ERR_OOM : (r < 0 ? WTFGPU_ERR_TRANSLATE : WTFGPU_OK));
}

static int apply_writes(wtfgpu_ctx *c, const wtfgpu_write_t *writes, uint32_t n, const uint8_t *data,
                        uint64_t data_len, int32_t *status_out, u32 phys) {
  if (!c || (n && (!writes || !data))) return WTFGPU_ERR_INVALID;
  if (n == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  std::vector<u32> order(n);
  for (u32 i = 0; i < n; i++) {
    order[i] = i;
    if (writes[i].lane >= c->P.nlanes || writes[i].data_off + writes[i].len > data_len) return WTFGPU_ERR_INVALID;
  }
  bool grouped = true;  // records of a lane already consecutive and lanes ascending: no sort
  for (u32 i = 1; i < n && grouped; i++) grouped = writes[i - 1].lane <= writes[i].lane;
  if (!grouped)
    std::stable_sort(order.begin(), order.end(), [&](u32 a, u32 b) { return writes[a].lane < writes[b].lane; });
  std::vector<WriteRec> recs(n);
  std::vector<u32> starts;
  for (u32 i = 0; i < n; i++) {
    const wtfgpu_write_t &w = writes[order[i]];
    recs[i] = WriteRec{w.lane, w.len, w.gva, w.data_off};
    if (i == 0 || w.lane != recs[i - 1].lane) starts.push_back(i);
  }
  const u32 nl = (u32)starts.size();
  starts.push_back(n);
  const u64 b_recs = (u64)n * sizeof(WriteRec), b_starts = starts.size() * 4ull, b_st = (u64)n * 4;
  const u64 o_starts = (b_recs + 255) & ~255ull, o_st = (o_starts + b_starts + 255) & ~255ull,
            o_data = (o_st + b_st + 255) & ~255ull;
  if (ensure_scratch(c, o_data + data_len)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, recs.data(), b_recs, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_scratch + o_starts, starts.data(), b_starts, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_scratch + o_data, data, data_len, hipMemcpyHostToDevice, c->stream));
  k_apply_writes<<<nl, 64, 0, c->stream>>>(c->P, (const WriteRec *)c->d_scratch,
                                                       (const u32 *)(c->d_scratch + o_starts), nl,
                                                       c->d_scratch + o_data, (i32 *)(c->d_scratch + o_st), phys);
  HIPCHK(hipGetLastError());
  std::vector<i32> st(n);
  HIPCHK(hipMemcpyAsync(st.data(), c->d_scratch + o_st, b_st, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  int rc = WTFGPU_OK;
  for (u32 i = 0; i < n; i++) {
    if (status_out) status_out[order[i]] = st[i];
    if (st[i]) rc = st[i];
  }
  return rc;
}

int wtfgpu_apply_writes(wtfgpu_ctx *c, const wtfgpu_write_t *writes, uint32_t n, const uint8_t *data,
                        uint64_t data_len, int32_t *status_out) {
  return apply_writes(c, writes, n, data, data_len, status_out, 0);
}
int wtfgpu_apply_phys_writes(wtfgpu_ctx *c, const wtfgpu_write_t *writes, uint32_t n, const uint8_t *data,
                             uint64_t data_len, int32_t *status_out) {
  return apply_writes(c, writes, n, data, data_len, status_out, 1);
}

static int check_lane_list(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n) {
  if (!c || !c->d_gpr || (n && !lanes)) return WTFGPU_ERR_INVALID;
  for (uint32_t i = 0; i < n; i++)
    if (lanes[i] >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  return WTFGPU_OK;
}

int wtfgpu_read_gprs_list(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint64_t *out18) {
  if (int rc = check_lane_list(c, lanes, n)) return rc;
  if (n == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  const u64 o_out = ((u64)n * 4 + 255) & ~255ull;
  if (ensure_scratch(c, o_out + (u64)n * 18 * 8)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  k_gather_gprs<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n,
                                                         (u64 *)(c->d_scratch + o_out));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out18, c->d_scratch + o_out, (u64)n * 18 * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_write_gprs_list(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, const uint64_t *in18) {
  if (int rc = check_lane_list(c, lanes, n)) return rc;
  if (n == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  const u64 o_in = ((u64)n * 4 + 255) & ~255ull;
  if (ensure_scratch(c, o_in + (u64)n * 18 * 8)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_scratch + o_in, in18, (u64)n * 18 * 8, hipMemcpyHostToDevice, c->stream));
  k_scatter_gprs<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n,
                                                          (const u64 *)(c->d_scratch + o_in));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_read_dirty_list(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint32_t *out) {
  if (int rc = check_lane_list(c, lanes, n)) return rc;
  if (n == 0) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  const u64 stride = (u64)c->P.K + 1;
  const u64 o_out = ((u64)n * 4 + 255) & ~255ull;
  if (ensure_scratch(c, o_out + (u64)n * stride * 4)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  k_gather_dirty<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n,
                                                          (u32 *)(c->d_scratch + o_out));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->d_scratch + o_out, (u64)n * stride * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

uint32_t wtfgpu_overlay_pages(wtfgpu_ctx *c) { return c ? c->P.K : 0; }

int wtfgpu_gather_pages(wtfgpu_ctx *c, const uint32_t *lanes, const uint64_t *gpas, uint32_t n, uint8_t *out) {
  if (int rc = check_lane_list(c, lanes, n)) return rc;
  if (n == 0) return WTFGPU_OK;
  if (!gpas || !out || !c->P.pool) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u64 o_gpa = ((u64)n * 4 + 255) & ~255ull, o_out = (o_gpa + (u64)n * 8 + 4095) & ~4095ull;
  if (ensure_scratch(c, o_out + (u64)n * WTFGPU_PAGE_SIZE)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_scratch + o_gpa, gpas, (u64)n * 8, hipMemcpyHostToDevice, c->stream));
  k_gather_pages<<<n, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, (const u64 *)(c->d_scratch + o_gpa), n,
                                           c->d_scratch + o_out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->d_scratch + o_out, (u64)n * WTFGPU_PAGE_SIZE, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_inject_fault(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint32_t vector, uint32_t error,
                        const uint64_t *addrs, int32_t *delivered) {
  if (int rc = check_lane_list(c, lanes, n)) return rc;
  if (n == 0) return WTFGPU_OK;
  if (!addrs || !delivered || vector > 31) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u64 o_a = ((u64)n * 4 + 255) & ~255ull, o_ok = (o_a + (u64)n * 8 + 255) & ~255ull;
  if (ensure_scratch(c, o_ok + (u64)n * 4)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_scratch + o_a, addrs, (u64)n * 8, hipMemcpyHostToDevice, c->stream));
  k_inject_fault<<<(n + 63) / 64, 64, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch,
                                                     (const u64 *)(c->d_scratch + o_a), n, vector, error,
                                                     (i32 *)(c->d_scratch + o_ok));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(delivered, c->d_scratch + o_ok, (u64)n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_gather_bytes(wtfgpu_ctx *c, const uint32_t *lanes, const uint64_t *gpas, uint32_t n, uint32_t len,
                        uint8_t *out) {
  if (int rc = check_lane_list(c, lanes, n)) return rc;
  if (n == 0) return WTFGPU_OK;
  if (!gpas || !out || !c->P.pool || len == 0 || len > 256) return WTFGPU_ERR_INVALID;
  for (u32 i = 0; i < n; i++)
    if ((gpas[i] & 0xfff) + len > WTFGPU_PAGE_SIZE) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  const u64 o_gpa = ((u64)n * 4 + 255) & ~255ull, o_out = (o_gpa + (u64)n * 8 + 255) & ~255ull;
  if (ensure_scratch(c, o_out + (u64)n * len)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->d_scratch + o_gpa, gpas, (u64)n * 8, hipMemcpyHostToDevice, c->stream));
  k_gather_bytes<<<n, 64, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, (const u64 *)(c->d_scratch + o_gpa), n,
                                          len, c->d_scratch + o_out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->d_scratch + o_out, (u64)n * len, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

static int lane_cr_ptr(wtfgpu_ctx *c, uint32_t lane, uint32_t cr, u8 **p) {
  if (!c || !c->d_sys || lane >= c->P.nlanes || (cr != 2 && cr != 3)) return WTFGPU_ERR_INVALID;
  *p = (u8 *)(c->d_sys + lane) + (cr == 2 ? offsetof(LaneSys, cr2) : offsetof(LaneSys, cr3));
  return WTFGPU_OK;
}

int wtfgpu_lane_get_cr(wtfgpu_ctx *c, uint32_t lane, uint32_t cr, uint64_t *value) {
  u8 *p = nullptr;
  if (!value || lane_cr_ptr(c, lane, cr, &p)) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(value, p, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_lane_set_cr(wtfgpu_ctx *c, uint32_t lane, uint32_t cr, uint64_t value) {
  u8 *p = nullptr;
  if (lane_cr_ptr(c, lane, cr, &p)) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(p, &value, 8, hipMemcpyHostToDevice, c->stream));
  if (cr == 3) HIPCHK(hipMemsetAsync(c->d_tlbok + lane, 0, 4, c->stream));  // translations of the old cr3
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

// Page-locked host memory for staging buffers: device<->host copies into it
// are plain DMA (no bounce through a driver staging buffer).
int wtfgpu_host_alloc(wtfgpu_ctx *c, uint64_t bytes, void **out) {
  if (!c || !out || !bytes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) return WTFGPU_ERR_OOM;
  return WTFGPU_OK;
}

int wtfgpu_host_free(wtfgpu_ctx *c, void *p) {
  if (!c) return WTFGPU_ERR_INVALID;
  if (p) HIPCHK(hipHostFree(p));
  return WTFGPU_OK;
}

int wtfgpu_read_dirty(wtfgpu_ctx *c, uint32_t lane, uint64_t *gpas, uint32_t cap, uint32_t *n) {
  if (!c || lane >= c->P.nlanes || !n) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  u32 cnt = 0;  // (on the queue's stream: after its queued restores)
  HIPCHK(hipMemcpyAsync(&cnt, c->d_ovcount + lane, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *n = cnt;
  for (u32 k = 0; k < cnt && k < cap; k++) {
    u32 g = 0;
    HIPCHK(hipMemcpyAsync(&g, c->d_ovgpfn + (u64)k * c->P.nlanes + lane, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    gpas[k] = (u64)g << 12;
  }
  return WTFGPU_OK;
}

// The coverage sets of a lane list (lanes == nullptr: first .. first+n),
// compacted into (lane, rip) pairs; `clear` empties the sets read.
static int collect_sets(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t first, uint32_t n, uint32_t *out_lanes,
                        uint64_t *out_rips, uint64_t cap, uint64_t *total, uint32_t *overflow, int clear) {
  HIPCHK(hipSetDevice(c->device));
  const u64 room = std::max<u64>(cap, 1);
  const u64 o_n = ((u64)(lanes ? n : 0) * 4 + 255) & ~255ull, o_l = o_n + 256, o_r = (o_l + room * 4 + 255) & ~255ull;
  if (ensure_scratch(c, o_r + room * 8)) return WTFGPU_ERR_OOM;
  if (lanes) HIPCHK(hipMemcpyAsync(c->d_scratch, lanes, (u64)n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemsetAsync(c->d_scratch + o_n, 0, 16, c->stream));
  k_cov_collect<<<n, 256, 0, c->stream>>>(c->P, lanes ? (const u32 *)c->d_scratch : nullptr, first, n,
                                          (u32 *)(c->d_scratch + o_l), (u64 *)(c->d_scratch + o_r), cap,
                                          (unsigned long long *)(c->d_scratch + o_n), (u32 *)(c->d_scratch + o_n + 8));
  HIPCHK(hipGetLastError());
  u64 hdr[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(hdr, c->d_scratch + o_n, 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (clear && lanes && hdr[0] <= cap) {  // everything was read: the sets empty (ordered before later work)
    k_cov_clear<<<(n + 255) / 256, 256, 0, c->stream>>>(c->P, (const u32 *)c->d_scratch, n);
    HIPCHK(hipGetLastError());
  }
  const u64 m = std::min(hdr[0], cap);
  if (m) {
    HIPCHK(hipMemcpyAsync(out_lanes, c->d_scratch + o_l, m * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out_rips, c->d_scratch + o_r, m * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  if (overflow) *overflow = (u32)hdr[1] & 1;
  *total = hdr[0];
  return WTFGPU_OK;
}

int wtfgpu_read_coverage(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint32_t *lanes, uint64_t *rips,
                         uint64_t cap, uint64_t *n, uint32_t *overflow) {
  if (!lanes_ok(c, first, count) || !n || (cap && (!lanes || !rips))) return WTFGPU_ERR_INVALID;
  *n = 0;
  if (overflow) *overflow = 0;
  if (!c->d_covrip || count == 0) return WTFGPU_OK;
  return collect_sets(c, nullptr, first, count, lanes, rips, cap, n, overflow, 0);
}

int wtfgpu_collect_coverage_lanes(wtfgpu_ctx *c, const uint32_t *lanes, uint32_t n, uint32_t *out_lanes,
                                  uint64_t *out_rips, uint64_t cap, uint64_t *total, uint32_t *overflow) {
  if (!c || !total || (n && !lanes) || (cap && (!out_lanes || !out_rips))) return WTFGPU_ERR_INVALID;
  *total = 0;
  if (overflow) *overflow = 0;
  if (!c->d_covrip || n == 0) return WTFGPU_OK;
  for (u32 i = 0; i < n; i++)
    if (lanes[i] >= c->P.nlanes) return WTFGPU_ERR_INVALID;
  return collect_sets(c, lanes, 0, n, out_lanes, out_rips, cap, total, overflow, 1);
}

int wtfgpu_commit_coverage(wtfgpu_ctx *c, const uint64_t *rips, uint64_t n) {
  if (!c || (n && !rips)) return WTFGPU_ERR_INVALID;
  if (n == 0 || !c->d_covmap) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  if (ensure_scratch(c, n * 8)) return WTFGPU_ERR_OOM;
  HIPCHK(hipMemcpyAsync(c->d_scratch, rips, n * 8, hipMemcpyHostToDevice, c->stream));
  k_cov_commit<<<(u32)((n + 255) / 256), 256, 0, c->stream>>>(c->P, (const u64 *)c->d_scratch, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_reset_coverage(wtfgpu_ctx *c) {
  if (!c) return WTFGPU_ERR_INVALID;
  if (!c->d_covmap) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemsetAsync(c->d_covmap, 0, c->ncovslots * WTFGPU_PAGE_SIZE, c->stream));
  HIPCHK(hipMemsetAsync(c->d_covshadow, 0, c->ncovslots * WTFGPU_PAGE_SIZE, c->stream));
  if (c->d_extra) HIPCHK(hipMemsetAsync(c->d_extra, 0xff, (u64)kExtraEntries * 8, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return guc_clear(c);  // shared entries and images carry UC_COVERED
}

int wtfgpu_set_trace(wtfgpu_ctx *c, uint32_t per_lane) {
  if (!c || !c->P.nlanes) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  dfree(c->d_trace);
  dfree(c->d_tracecnt);
  c->d_trace = nullptr;
  c->d_tracecnt = nullptr;
  c->P.trace = nullptr;
  c->P.trace_cnt = nullptr;
  c->P.trace_cap = 0;
  if (per_lane) {
    const u64 N = c->P.nlanes;
    if (dalloc(&c->d_trace, N * per_lane) || dalloc(&c->d_tracecnt, N)) return WTFGPU_ERR_OOM;
    HIPCHK(hipMemset(c->d_tracecnt, 0, N * 4));
    c->P.trace = c->d_trace;
    c->P.trace_cnt = c->d_tracecnt;
    c->P.trace_cap = per_lane;
  }
  return guc_clear(c);  // cached entries were digested for the other setting
}

int wtfgpu_read_trace(wtfgpu_ctx *c, uint32_t lane, uint64_t *rips, uint64_t cap, uint64_t *n) {
  if (!c || !n || (cap && !rips) || lane >= c->P.nlanes || !c->d_trace) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  u32 cnt = 0;
  HIPCHK(hipMemcpyAsync(&cnt, c->d_tracecnt + lane, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *n = cnt;
  const u64 k = std::min<u64>(std::min<u64>(cnt, c->P.trace_cap), cap);
  if (k) HIPCHK(hipMemcpyAsync(rips, c->d_trace + (u64)lane * c->P.trace_cap, k * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

// Tenet traces (engine_exec.h TenetDev): bytes_per_lane of entries per lane, 0 = off.
int wtfgpu_set_tenet(wtfgpu_ctx *c, uint64_t bytes_per_lane) {
  if (!c || !c->d_gpr || (bytes_per_lane & 7)) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  dfree(c->d_tn_buf);
  dfree(c->d_tn_pos);
  dfree(c->d_tn_cpos);
  dfree(c->d_tn_ipos);
  dfree(c->d_tn_last);
  dfree(c->d_tn_mute);
  c->d_tn_buf = nullptr, c->d_tn_pos = c->d_tn_cpos = c->d_tn_ipos = c->d_tn_last = nullptr, c->d_tn_mute = nullptr;
  TenetDev T{};
  c->tn_cap = 0;
  if (bytes_per_lane) {
    const u64 N = c->P.nlanes;
    if (dalloc(&c->d_tn_buf, N * bytes_per_lane) || dalloc(&c->d_tn_pos, N) || dalloc(&c->d_tn_cpos, N) ||
        dalloc(&c->d_tn_ipos, N) || dalloc(&c->d_tn_last, N) || dalloc(&c->d_tn_mute, N))
      return WTFGPU_ERR_OOM;
    HIPCHK(hipMemset(c->d_tn_pos, 0, N * 8));
    HIPCHK(hipMemset(c->d_tn_cpos, 0, N * 8));
    HIPCHK(hipMemset(c->d_tn_ipos, 0, N * 8));
    HIPCHK(hipMemset(c->d_tn_last, 0xff, N * 8));
    HIPCHK(hipMemset(c->d_tn_mute, 0, N * 4));
    T = TenetDev{c->d_tn_buf, bytes_per_lane, c->d_tn_pos, c->d_tn_cpos, c->d_tn_ipos, c->d_tn_last, c->d_tn_mute};
    c->tn_cap = bytes_per_lane;
  }
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_tn), &T, sizeof(T)));
  return guc_clear(c);  // cached entries were digested for the other setting
}

int wtfgpu_read_tenet(wtfgpu_ctx *c, uint32_t lane, uint8_t *buf, uint64_t cap, uint64_t *n) {
  if (!c || !n || (cap && !buf) || lane >= c->P.nlanes || !c->d_tn_buf) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  u64 pos = 0;
  HIPCHK(hipMemcpyAsync(&pos, c->d_tn_pos + lane, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *n = pos;
  const u64 k = std::min<u64>(std::min<u64>(pos, c->tn_cap), cap);
  if (k) HIPCHK(hipMemcpyAsync(buf, c->d_tn_buf + (u64)lane * c->tn_cap, k, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_set_edges(wtfgpu_ctx *c, int on) {
  if (!c) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  c->P.edges = on ? 1 : 0;
  if (on && !c->d_edgecnt && c->P.nlanes) {
    if (dalloc(&c->d_edgecnt, 2ull * c->P.nlanes)) return WTFGPU_ERR_OOM;
    HIPCHK(hipMemset(c->d_edgecnt, 0, 8ull * c->P.nlanes));
  }
  c->P.edge_cnt = on ? c->d_edgecnt : nullptr;
  return guc_clear(c);  // cached entries were digested for the other setting
}

int wtfgpu_coverage_absorb(wtfgpu_ctx *c, uint64_t *rips, uint64_t cap, uint64_t *n) {
  if (!c || !n || (cap && !rips)) return WTFGPU_ERR_INVALID;
  *n = 0;
  if (!c->d_covmap || !c->ncovslots) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  const u64 bytes = c->ncovslots * WTFGPU_PAGE_SIZE, n16 = bytes / 16;
  if (ensure_scratch(c, 256 + cap * 8)) return WTFGPU_ERR_OOM;
  unsigned long long *d_count = (unsigned long long *)c->d_scratch;
  u64 *d_idx = (u64 *)(c->d_scratch + 256);
  HIPCHK(hipMemsetAsync(d_count, 0, 8, c->stream));
  k_cov_absorb<<<(u32)((n16 + 255) / 256), 256, 0, c->stream>>>(c->d_covmap, c->d_covshadow, n16, d_idx, cap, d_count,
                                                                 cap ? 1 : 0);
  HIPCHK(hipGetLastError());
  u64 total = 0;
  HIPCHK(hipMemcpyAsync(&total, d_count, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const u64 m = std::min(total, cap);
  if (m) {
    std::vector<u64> idx(m);
    HIPCHK(hipMemcpyAsync(idx.data(), d_idx, m * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    std::sort(idx.begin(), idx.end());
    for (u64 i = 0; i < m; i++) rips[i] = (c->code_vpns[idx[i] / WTFGPU_PAGE_SIZE] << 12) | (idx[i] % WTFGPU_PAGE_SIZE);
  }
  *n = total;
  return WTFGPU_OK;
}

int wtfgpu_coverage_merge_in(wtfgpu_ctx *c, const void *dev_src, uint64_t bytes) {
  if (!c || (bytes && !dev_src)) return WTFGPU_ERR_INVALID;
  if (!c->d_covmap || !c->ncovslots) return bytes ? WTFGPU_ERR_INVALID : WTFGPU_OK;
  const u64 mb = c->ncovslots * WTFGPU_PAGE_SIZE, n16 = mb / 16;
  if (bytes != mb) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  k_cov_merge_in<<<(u32)((n16 + 255) / 256), 256, 0, c->stream>>>((uint4 *)c->d_covmap, (const uint4 *)dev_src, n16);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_coverage_device_map(wtfgpu_ctx *c, void **dev_ptr, uint64_t *bytes) {
  if (!c || !dev_ptr || !bytes) return WTFGPU_ERR_INVALID;
  *dev_ptr = c->d_covmap;
  *bytes = c->ncovslots * WTFGPU_PAGE_SIZE;
  return WTFGPU_OK;
}

int wtfgpu_coverage_rips(wtfgpu_ctx *c, uint64_t *rips, uint64_t cap, uint64_t *n) {
  if (!c || !n) return WTFGPU_ERR_INVALID;
  *n = 0;
  if (!c->d_covmap) return WTFGPU_OK;
  HIPCHK(hipSetDevice(c->device));
  std::vector<u8> m(c->ncovslots * WTFGPU_PAGE_SIZE);
  HIPCHK(hipMemcpyAsync(m.data(), c->d_covmap, m.size(), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  u64 k = 0;
  for (u64 s = 0; s < c->ncovslots; s++)
    for (u64 o = 0; o < WTFGPU_PAGE_SIZE; o++)
      if (m[s * WTFGPU_PAGE_SIZE + o]) {
        if (k < cap && rips) rips[k] = (c->code_vpns[s] << 12) | o;
        k++;
      }
  *n = k;
  return WTFGPU_OK;
}

int wtfgpu_read_bytes(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint64_t *out) {
  if (!lanes_ok(c, first, count) || !out) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(out, c->d_nbytes + first, (u64)count * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_read_edge_counts(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint32_t *out2) {
  if (!lanes_ok(c, first, count) || !out2) return WTFGPU_ERR_INVALID;
  if (!c->d_edgecnt) {
    memset(out2, 0, 8ull * count);
    return WTFGPU_OK;
  }
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(out2, c->d_edgecnt + 2ull * first, 8ull * count, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

int wtfgpu_read_dirty_counts(wtfgpu_ctx *c, uint32_t first, uint32_t count, uint32_t *out) {
  if (!lanes_ok(c, first, count) || !out) return WTFGPU_ERR_INVALID;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(out, c->d_ovcount + first, (u64)count * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WTFGPU_OK;
}

}  // extern "C"
