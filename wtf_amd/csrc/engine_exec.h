// engine_exec.h — per-lane state, guest memory, decode and execute for the
// RIP-grouped interpreter (see engine_device.h). Included by engine.hip only.
#pragma once
#include "engine_device.h"

namespace wtfgpu_dev {

// ------------------------------------------------------------------ lane state

struct Lane {
  u32 *glo, *ghi;            // guest GPRs: two 16 x u32 arrays local to the kernel (VGPRs)
  u64 rip, rflags, icount, nbytes;
  u64 tv[TLB_N], td[TLB_N];  // TLB: vpn tags, page pointer | T_* bits
  u64 bloom;                 // overlay membership filter
  u64 cvpn, cptr;            // code-page cache: vpn of the last instruction page, its page pointer
  u64 cr0, cr3, efer;
  u64 exaddr;
  u64 miss_va;               // pending translation (TLB miss or copy-on-write)
  u32 tnext, ovn, cpl, status, lane, exvec, exerr, exop;
  u32 miss, miss_acc, flush, pend;  // pend: bytes accessed by the attempt in flight
  u32 nodeliver;                    // this fault could not be delivered through the guest IDT
  u32 cgen, ccnt;                   // coverage set: generation, live entries
  u32 simd;                         // bit 0: SSE usable, bit 1: AVX usable, bit 2: AVX-512 state on (simd_bits)
};

// Which vector state the lane's cr0 / cr4 / xcr0 enable without a fault: bit 0
// legacy SSE (CR0.EM = 0, CR0.TS = 0, CR4.OSFXSR), bit 1 VEX (CR4.OSXSAVE,
// XCR0[2:1] = 11, CR0.TS = 0). The fast path runs vector moves only then.
// Bit 2: EVEX usable (CR4.OSXSAVE, XCR0[7:5] = 111 with [2:1] = 11, CR0.TS = 0;
// U47): a VEX write then also zeroes the register's bits 511:256.
__device__ __forceinline__ u32 simd_bits(u64 cr0, u64 cr4, u64 xcr0) {
  const bool ts = (cr0 >> 3) & 1;
  const u32 sse = !((cr0 >> 2) & 1) && !ts && ((cr4 >> 9) & 1);
  const u32 avx = !ts && ((cr4 >> 18) & 1) && (xcr0 & 6) == 6;
  const u32 z = avx && (xcr0 & 0xe0) == 0xe0;
  return sse | avx << 1 | z << 2;
}

// GPR r of the lane. r is wave-uniform and the halves live in two u32 arrays
// that the compiler keeps in VGPRs, indexed with s_set_gpr_idx (32-bit moves
// only: no memory, no per-register select chains).
__device__ __forceinline__ u64 R(const Lane &L, u32 r) { return ((u64)L.ghi[r & 15] << 32) | L.glo[r & 15]; }
__device__ __forceinline__ void RS(Lane &L, u32 r, u64 v) {
  L.glo[r & 15] = (u32)v;
  L.ghi[r & 15] = (u32)(v >> 32);
}

// ------------------------------------------------------------------ TLB
__device__ __forceinline__ bool tlb_get(const Lane &L, u64 vpn, u64 &td) {
  bool hit = false;
  u64 r = 0;
#pragma unroll
  for (int i = 0; i < TLB_N; i++) {
    if (L.tv[i] == vpn) {
      hit = true;
      r = L.td[i];
    }
  }
  td = r;
  return hit;
}
__device__ __forceinline__ void tlb_put(Lane &L, u64 vpn, u64 td) {
#pragma unroll
  for (int i = 0; i < TLB_N; i++) {
    if (L.tnext == (u32)i) {
      L.tv[i] = vpn;
      L.td[i] = td;
    }
  }
  L.tnext = (L.tnext + 1) & (TLB_N - 1);
}
__device__ __forceinline__ void tlb_flush(Lane &L) {
#pragma unroll
  for (int i = 0; i < TLB_N; i++) L.tv[i] = EMPTY_KEY;
  L.cvpn = EMPTY_KEY;
}

// ------------------------------------------------------------------ compatibility mode (U29)
// A lane runs 32-bit code when CS is SYSRET's 32-bit selector, STAR[63:48]
// (Windows' and Linux' layout: the only CS.L = 0 code segment; descriptors are
// not read, U19). The mode is bit 63 of the lane's efer copy (never of
// LaneSys::efer, never reported: EFER bits 63:16 are reserved) and of its code
// pointer L.cptr, which puts the pointer outside the page pool: the fast loop's
// pool check and the slow step's cacheable test send every 32-bit instruction
// to slow_step, which decodes it in 32-bit mode. LaneSys::efer carries the
// bit too (set by make_init from the snapshot's CS, stripped from every
// register read-back), so load_lane copies it with efer. (bochscpu.hpp:119-182:
// the reference state is the full segment cache; its CS.L picks the mode.)
constexpr u64 EFER_M32 = 1ull << 63;
__host__ __device__ __forceinline__ bool compat_sel(u64 star, u32 sel) {
  return ((sel ^ (u32)(star >> 48)) & 0xfffc) == 0;
}
// CS := sel, with the mode it selects; a mode change drops the code-page cache
// (its pointer carries the mode)
__device__ __forceinline__ void set_cs(Lane &L, LaneSys &S, u32 sel) {
  S.cs = (u16)sel;
  const u64 m = compat_sel(S.star, sel) ? EFER_M32 : 0;
  if ((L.efer & EFER_M32) != m) {
    L.efer ^= EFER_M32;
    S.efer ^= EFER_M32;
    L.cvpn = EMPTY_KEY;
  }
}

// ------------------------------------------------------------------ physical memory
__device__ __forceinline__ u64 bloom_bit(u64 gpfn) { return 1ull << ((gpfn * 0x9E3779B97F4A7C15ull) >> 58); }

// Lane view of a guest physical page: private overlay copy if the lane wrote
// it, else the snapshot pool page, else the zero page (bochscpu_backend.cc:124-131).
__device__ __forceinline__ const u8 *phys_page(const Dev &P, u32 lane, u32 ovn, u64 bloom, u64 gpfn, bool &priv) {
  priv = false;
  if (bloom & bloom_bit(gpfn)) {
    for (u32 k = 0; k < ovn; k++) {
      if (P.ov_gpfn[(u64)k * P.nlanes + lane] == (u32)gpfn) {
        priv = true;
        return P.ov_data + ((u64)lane * P.K + k) * WTFGPU_PAGE_SIZE;
      }
    }
  }
  const u32 idx = gpfn < P.pfn_map_len ? P.pfn_map[gpfn] : 0u;
  return P.pool + (u64)idx * WTFGPU_PAGE_SIZE;
}

__device__ __forceinline__ bool is_ptpage(const Dev &P, u64 gpfn) {
  if (gpfn >= P.pfn_map_len) return false;
  return (P.ptbits[gpfn >> 5] >> (gpfn & 31)) & 1;
}

// Little-endian load of sz bytes that do not cross a page: aligned u64 pair + funnel.
__device__ __forceinline__ u64 load_le(const u8 *p, u32 sz) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)7;
  const u32 off = (u32)((uintptr_t)p & 7);
  const u64 lo = *(const u64 *)a;
  u64 v = lo >> (8 * off);
  if (off + sz > 8) {
    const u64 hi = *(const u64 *)(a + 8);
    v |= hi << (64 - 8 * off);
  }
  return v & szmask(sz);
}
__device__ __forceinline__ void store_le(u8 *p, u32 sz, u64 v) {
  const uintptr_t a = (uintptr_t)p;
  if ((a & (sz - 1)) == 0) {
    if (sz == 8) *(u64 *)p = v;
    else if (sz == 4) *(u32 *)p = (u32)v;
    else if (sz == 2) *(u16 *)p = (u16)v;
    else *p = (u8)v;
    return;
  }
  for (u32 i = 0; i < sz; i++) p[i] = (u8)(v >> (8 * i));
}

enum { ACC_R = 0, ACC_W = 1, ACC_X = 2, ACC_WPROBE = 3 };  // WPROBE: write permission check only

__device__ __forceinline__ void set_fault(Lane &L, u32 vec, u32 err, u64 addr) {
  L.status = WTFGPU_EXIT_FAULT;
  L.exvec = vec;
  L.exerr = err;
  L.exaddr = addr;
}

__device__ __forceinline__ bool canonical(u64 va) { return (u64)(((i64)(va << 16)) >> 16) == va; }

__device__ __forceinline__ u32 pf_error(const Lane &L, int acc, bool present) {
  const bool nxe = (L.efer >> 11) & 1;
  return (present ? 1u : 0u) | (acc == ACC_W || acc == ACC_WPROBE ? 2u : 0u) | (L.cpl == 3 ? 4u : 0u) |
         (acc == ACC_X && nxe ? 16u : 0u);
}

// Permission check of a translation (SDM 4.6): U/S, R/W (+CR0.WP), NX.
__device__ __forceinline__ bool perm_ok(const Lane &L, u64 td, int acc) {
  const bool user = L.cpl == 3;
  const bool wp = (L.cr0 >> 16) & 1;
  const bool w = acc == ACC_W || acc == ACC_WPROBE;
  return !((user && !(td & T_U)) || (w && !(td & T_W) && (user || wp)) || (acc == ACC_X && (td & T_NX)));
}

// 4-level walk through the lane's physical view (kdmp-parser.h:269-345 shape,
// SDM permission bits accumulated). No A/D updates (U8). Faults set on L
// (kFault); without kFault a walk that would fault only returns false.
template <bool kFault = true>
__device__ __forceinline__ bool walk(const Dev &P, Lane &L, u64 va, int acc, u64 &td, u64 &gpfn) {
  const bool nxe = (L.efer >> 11) & 1;
  if (!canonical(va)) {
    if (kFault) set_fault(L, WTFGPU_VEC_GP, 0, va);
    return false;
  }
  u64 table = L.cr3 & 0x000ffffffffff000ull;
  bool aw = true, au = true, nx = false;
  u64 e = 0, pmask = 0xfff;
  bool priv;
  for (int level = 3; level >= 0; level--) {
    const u64 idx = (va >> (12 + 9 * level)) & 0x1ff;
    const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, table >> 12, priv);
    e = *(const u64 *)(pg + idx * 8);
    if (!(e & 1)) {
      if (kFault) set_fault(L, WTFGPU_VEC_PF, pf_error(L, acc, false), va);
      return false;
    }
    aw &= (e & 2) != 0;
    au &= (e & 4) != 0;
    if (nxe && (e >> 63)) nx = true;
    if ((level == 2 || level == 1) && (e & 0x80)) {
      pmask = level == 2 ? 0x3fffffffull : 0x1fffffull;
      break;
    }
    table = e & 0x000ffffffffff000ull;
  }
  const u64 gpa = ((e & 0x000ffffffffff000ull) & ~pmask) | (va & pmask);
  gpfn = gpa >> 12;
  const u8 *pg = phys_page(P, L.lane, L.ovn, L.bloom, gpfn, priv);
  td = (u64)(uintptr_t)pg | (aw ? T_W : 0) | (au ? T_U : 0) | (nx ? T_NX : 0) | (priv ? T_PRIV : 0) |
       (is_ptpage(P, gpfn) ? T_PT : 0);
  return true;
}

// Copy-on-write into overlay slot `slot` of `lane`: the page joins the dirty
// list (bochscpu_backend.cc:887-889 DirtyGpa; dropped again by restore :751-772).
// One lane's copy (the slow path; k_run's fast loop copies with the whole
// wave): 256 bytes in flight per round, 16 rounds.
__device__ __forceinline__ u8 *cow_copy(const Dev &P, u32 lane, u32 slot, u64 gpfn, const u8 *src) {
  u8 *dst = P.ov_data + ((u64)lane * P.K + slot) * WTFGPU_PAGE_SIZE;
  const uint4 *__restrict__ s4 = (const uint4 *)src;
  uint4 *__restrict__ d4 = (uint4 *)dst;
  for (int i = 0; i < 256; i += 16) {
    uint4 t[16];
#pragma unroll
    for (int j = 0; j < 16; j++) t[j] = s4[i + j];
#pragma unroll
    for (int j = 0; j < 16; j++) d4[i + j] = t[j];
  }
  P.ov_gpfn[(u64)slot * P.nlanes + lane] = (u32)gpfn;
  return dst;
}

// Slow path of a translation (one call site in the kernel): walk, permission
// check, copy-on-write, TLB fill. false = the lane faulted / ran out of overlay.
__device__ __forceinline__ bool service_miss(const Dev &P, Lane &L, u64 va, int acc) {
  u64 td, gpfn;
  if (!walk(P, L, va, acc, td, gpfn)) return false;
  if (!perm_ok(L, td, acc)) {
    set_fault(L, WTFGPU_VEC_PF, pf_error(L, acc, true), va);
    return false;
  }
  if (acc == ACC_W && !(td & T_PRIV)) {
    if (L.ovn >= P.K) {
      L.status = WTFGPU_EXIT_OVERLAY_FULL;
      return false;
    }
    u8 *np = cow_copy(P, L.lane, L.ovn, gpfn, (const u8 *)(uintptr_t)(td & ~0xfffull));
    L.ovn++;
    L.bloom |= bloom_bit(gpfn);
    tlb_flush(L);  // other vpns may alias the old page
    td = (u64)(uintptr_t)np | (td & 0xfff) | T_PRIV;
  }
  tlb_put(L, va >> 12, td);
  return true;
}

// The fast loop's own miss service (k_run): the TLB fill or first-write copy
// service_miss would make, done in registers when it raises nothing. false =
// the walk or the permission check would fault, the page is a page-table page
// (exec() flushes after such a write) or the overlay is full: exec() in the
// slow step then takes the instruction and raises exactly what it raises.
__device__ __forceinline__ bool fast_fill(const Dev &P, Lane &L) {
  const u64 va = L.miss_va;
  const int acc = (int)L.miss_acc;
  u64 td, gpfn;
  if (!walk<false>(P, L, va, acc, td, gpfn) || !perm_ok(L, td, acc)) return false;
  if (acc == ACC_W && !(td & T_PRIV)) {
    if ((td & T_PT) || L.ovn >= P.K) return false;
    u8 *np = cow_copy(P, L.lane, L.ovn, gpfn, (const u8 *)(uintptr_t)(td & ~0xfffull));
    L.ovn++;
    L.bloom |= bloom_bit(gpfn);
    tlb_flush(L);  // other vpns may alias the old page
    td = (u64)(uintptr_t)np | (td & 0xfff) | T_PRIV;
  }
  tlb_put(L, va >> 12, td);
  return true;
}

// fast_fill in two halves around a copy the whole wave makes (k_run): the
// walk and checks, then either the TLB fill (nothing to copy: dst = 0) or the
// page to copy (src, dst: the lane's next overlay slot, taken now); after the
// copy, fast_fill_finish records the page as the lane's own. false = as
// fast_fill's false.
__device__ __forceinline__ bool fast_fill_prep(const Dev &P, Lane &L, u64 &src, u64 &dst, u64 &gpfn, u64 &td) {
  const u64 va = L.miss_va;
  const int acc = (int)L.miss_acc;
  dst = 0;
  if (!walk<false>(P, L, va, acc, td, gpfn) || !perm_ok(L, td, acc)) return false;
  if (acc == ACC_W && !(td & T_PRIV)) {
    if ((td & T_PT) || L.ovn >= P.K) return false;
    src = td & ~0xfffull;
    dst = (u64)(uintptr_t)(P.ov_data + ((u64)L.lane * P.K + L.ovn) * WTFGPU_PAGE_SIZE);
    return true;
  }
  tlb_put(L, va >> 12, td);
  return true;
}
// When fast_fill_prep declines because the access faults (the walk fails or
// the permission check does), raise the fault service_miss would raise for
// the same access, so the lane leaves the step loop with it instead of
// re-running the instruction through exec() only to fault there (a
// page-table page or a full overlay stays for the slow step: no fault).
__device__ __forceinline__ void fast_fault(const Dev &P, Lane &L) {
  const u64 va = L.miss_va;
  const int acc = (int)L.miss_acc;
  u64 td, gpfn;
  if (!walk(P, L, va, acc, td, gpfn)) return;  // (walk<true> set the fault)
  if (!perm_ok(L, td, acc)) set_fault(L, WTFGPU_VEC_PF, pf_error(L, acc, true), va);
}
__device__ __forceinline__ void fast_fill_finish(const Dev &P, Lane &L, u64 dst, u64 gpfn, u64 td) {
  P.ov_gpfn[(u64)L.ovn * P.nlanes + L.lane] = (u32)gpfn;
  L.ovn++;
  L.bloom |= bloom_bit(gpfn);
  tlb_flush(L);  // other vpns may alias the old page
  tlb_put(L, L.miss_va >> 12, dst | (td & 0xfff) | T_PRIV);
}

// Fast path: TLB hit + permission check. A miss (or a write to a shared page)
// records the address in L.miss and returns nullptr: the instruction is
// abandoned and re-executed after service_miss. Real faults set L.status.
__device__ __forceinline__ u8 *xlate(Lane &L, u64 va, int acc, u64 *tdo = nullptr) {
  u64 td;
  if (!tlb_get(L, va >> 12, td)) {
    L.miss = 1;
    L.miss_va = va;
    L.miss_acc = (u32)acc;
    return nullptr;
  }
  if (!perm_ok(L, td, acc)) {
    set_fault(L, WTFGPU_VEC_PF, pf_error(L, acc, true), va);
    return nullptr;
  }
  if (acc == ACC_W && !(td & T_PRIV)) {  // first write: copy-on-write in service_miss
    L.miss = 1;
    L.miss_va = va;
    L.miss_acc = (u32)acc;
    return nullptr;
  }
  if (tdo) *tdo = td;
  return (u8 *)(uintptr_t)(td & ~0xfffull) + (va & 0xfff);
}

// [va, va + n) (n <= 4096) writable and in the lane's overlay: false = a miss
// (the caller restarts after service_miss) or a fault. Every page passes the
// write check before any of them is copied (a fault dirties nothing).
__device__ __forceinline__ bool span_w(Lane &L, u64 va, u32 n) {
  const u64 last = (va + n - 1) & ~0xfffull;
  const bool two = ((va ^ (va + n - 1)) >> 12) != 0;
  if (!xlate(L, va, ACC_WPROBE) || (two && !xlate(L, last, ACC_WPROBE))) return false;
  return xlate(L, va, ACC_W) && (!two || xlate(L, last, ACC_W));
}

// ------------------------------------------------------------------ Tenet trace
// (wtfgpu_set_tenet; bochscpu_backend.cc:1215-1323; U38 in DESIGN.md). Per
// lane a byte stream of 8-byte-aligned entries:
//   ACC  {u64 va; u64 meta = 1 << 56 | type << 32 | len; data, len bytes
//         rounded up to 8}: one data access of an instruction (the operand as
//         a whole, up to 32 bytes; an RMW operand once, as read-write); the
//         data is the memory after the instruction, filled at its REGS entry;
//   REGS {u64 meta = 2 << 56; u64 gpr[16]; u64 rip}: the registers at the
//         start, after each retired instruction, after each delivered
//         exception, after a breakpoint action that moved rip, and when a
//         lane stops with accesses still open.
// pos: bytes written (past cap: truncated); cpos: the committed position a
// restarted attempt rolls back to (string ops commit per iteration); ipos: the
// current instruction's first ACC entry; mute: nested accesses of an operand
// already logged as a whole.
struct TenetDev {
  u8 *buf;
  u64 cap;
  u64 *pos, *cpos, *ipos, *last;  // last: the instruction's latest ACC entry (~0: none)
  u32 *mute;
};
__device__ TenetDev g_tn;
enum : u32 { TN_R = 1, TN_W = 2, TN_RW = 3 };
constexpr u64 TN_ACC = 1ull << 56, TN_REGS = 2ull << 56;

__device__ __noinline__ void tn_access(u32 lane, u64 va, u32 len, u32 type) {
  if (g_tn.mute[lane]) return;
  const u64 p = g_tn.pos[lane], last = g_tn.last[lane];
  u8 *const base = g_tn.buf + (u64)lane * g_tn.cap;
  // the write of a read-modify-write operand: its read entry is the latest one
  if (type == TN_W && last != ~0ull && last + 16 <= g_tn.cap && *(const u64 *)(base + last) == va &&
      *(const u64 *)(base + last + 8) == (TN_ACC | (u64)TN_RW << 32 | len))
    return;
  const u64 n = 16 + ((u64)len + 7) / 8 * 8;
  if (p + n <= g_tn.cap) {
    *(u64 *)(base + p) = va;
    *(u64 *)(base + p + 8) = TN_ACC | (u64)type << 32 | len;
  } else if (p + 16 <= g_tn.cap) {
    *(u64 *)(base + p) = 0;  // truncated here: readers stop at this zero header
    *(u64 *)(base + p + 8) = 0;
  }
  g_tn.last[lane] = p;
  g_tn.pos[lane] = p + n;
}
// An operand wider than one vread / vwrite (16 / 32 bytes): its pieces are
// muted and, once every piece succeeded, it is logged once as a whole.
__device__ __forceinline__ void tn_mute(u32 lane) {
  if (g_tn.buf) g_tn.mute[lane]++;
}
__device__ __forceinline__ bool tn_unmute(u32 lane, u64 va, u32 len, u32 type, bool ok) {
  if (g_tn.buf) {
    g_tn.mute[lane]--;
    if (ok) tn_access(lane, va, len, type);
  }
  return ok;
}
// instruction start / attempt restart / iteration commit
__device__ __forceinline__ void tn_insn_begin(u32 lane) {
  if (!g_tn.buf) return;
  g_tn.ipos[lane] = g_tn.cpos[lane] = g_tn.pos[lane];
  g_tn.last[lane] = ~0ull;
  g_tn.mute[lane] = 0;
}
__device__ __forceinline__ void tn_rollback(u32 lane) {
  if (!g_tn.buf) return;
  g_tn.pos[lane] = g_tn.cpos[lane];
  g_tn.last[lane] = ~0ull;
  g_tn.mute[lane] = 0;
}
__device__ __forceinline__ void tn_commit(u32 lane) {
  if (g_tn.buf) g_tn.cpos[lane] = g_tn.pos[lane];
}

// Guest virtual reads / writes of 1..8 bytes (page crossing handled).
__device__ __forceinline__ bool vread(Lane &L, u64 va, u32 sz, u64 &out, int acc = ACC_R) {
  const u32 off = (u32)(va & 0xfff);
  if (off + sz <= 4096) {
    const u8 *p = xlate(L, va, acc);
    if (!p) return false;
    out = load_le(p, sz);
  } else {
    const u32 n0 = 4096 - off;
    if (acc == ACC_W) {  // both pages must pass the write check before either is copied
      if (!xlate(L, va, ACC_WPROBE) || !xlate(L, va + n0, ACC_WPROBE)) return false;
    }
    const u8 *p0 = xlate(L, va, acc);
    if (!p0) return false;
    const u8 *p1 = xlate(L, va + n0, acc);
    if (!p1) return false;
    u64 v = 0;
    for (u32 i = 0; i < sz; i++) v |= (u64)(i < n0 ? p0[i] : p1[i - n0]) << (8 * i);
    out = v;
  }
  L.pend += sz;
  if (g_tn.buf) tn_access(L.lane, va, sz, acc == ACC_W ? TN_RW : TN_R);
  return true;
}

__device__ __forceinline__ bool vwrite(Lane &L, u64 va, u32 sz, u64 v) {
  const u32 off = (u32)(va & 0xfff);
  u64 td0 = 0, td1 = 0;
  if (off + sz <= 4096) {
    u8 *p = xlate(L, va, ACC_W, &td0);
    if (!p) return false;
    store_le(p, sz, v);
  } else {
    const u32 n0 = 4096 - off;
    if (!xlate(L, va, ACC_WPROBE) || !xlate(L, va + n0, ACC_WPROBE)) return false;
    u8 *p0 = xlate(L, va, ACC_W, &td0);
    if (!p0) return false;
    u8 *p1 = xlate(L, va + n0, ACC_W, &td1);
    if (!p1) return false;
    for (u32 i = 0; i < sz; i++) {
      if (i < n0) p0[i] = (u8)(v >> (8 * i));
      else p1[i - n0] = (u8)(v >> (8 * i));
    }
  }
  // a write into a page-table page invalidates cached translations (applied
  // when the instruction retires, so a restart cannot livelock)
  if ((td0 | td1) & T_PT) L.flush = 1;
  L.pend += sz;
  if (g_tn.buf) tn_access(L.lane, va, sz, TN_W);
  return true;
}

// Tenet (engine_exec.h TenetDev): fills the data of the ACC entries the
// current instruction logged with the memory as it is now (translation by
// present bits, as the oracle's orc_read_virt; a page that no longer
// translates reads as zeros), then appends a REGS entry with the lane's
// registers. The lane's state is left as it was.
__device__ __noinline__ void tn_regs(const Dev &P, Lane &L) {
  const u32 lane = L.lane;
  const u64 cap = g_tn.cap, end = g_tn.pos[lane];
  u8 *const base = g_tn.buf + (u64)lane * cap;
  const u32 st = L.status, ev = L.exvec, ee = L.exerr, cpl = L.cpl, pend = L.pend, miss = L.miss;
  const u64 ea = L.exaddr, cr0 = L.cr0;
  L.cpl = 0;  // supervisor reads, CR0.WP clear: only the present bits decide
  L.cr0 &= ~(1ull << 16);
  for (u64 q = g_tn.ipos[lane]; q + 16 <= end && q + 16 <= cap;) {
    const u64 va = *(const u64 *)(base + q), meta = *(const u64 *)(base + q + 8);
    if (meta >> 56 != 1) break;  // the truncation mark (tn_access)
    const u32 len = (u32)(meta & 0xffffffffull);
    const u64 n = 16 + ((u64)len + 7) / 8 * 8;
    if (q + n > cap) break;
    {
      u8 *out = base + q + 16;
      for (u32 i = 0; i < len; i++) {
        u8 b = 0;
        for (int attempt = 0;; attempt++) {
          L.miss = 0;
          L.status = WTFGPU_RUNNING;
          const u8 *p = xlate(L, va + i, ACC_R);
          if (p) {
            b = *p;
            break;
          }
          if (!L.miss || attempt >= 16 || !service_miss(P, L, L.miss_va, (int)L.miss_acc)) break;
        }
        out[i] = b;
      }
    }
    q += n;
  }
  L.status = st, L.exvec = ev, L.exerr = ee, L.exaddr = ea, L.cpl = cpl, L.pend = pend, L.miss = miss, L.cr0 = cr0;
  const u64 n = 8 + 17 * 8;
  if (end + n <= cap) {
    u64 *r = (u64 *)(base + end);
    r[0] = TN_REGS;
    for (u32 i = 0; i < 16; i++) r[1 + i] = R(L, i);
    r[17] = L.rip;
  } else if (end + 16 <= cap) {
    *(u64 *)(base + end) = 0;  // truncation mark
    *(u64 *)(base + end + 8) = 0;
  }
  g_tn.pos[lane] = g_tn.ipos[lane] = g_tn.cpos[lane] = end + n;
  g_tn.last[lane] = ~0ull;
}

}  // namespace wtfgpu_dev
