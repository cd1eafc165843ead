// sim_lane.cc — TEST INFRASTRUCTURE ONLY: one lane of the GPU interpreter's
// per-step logic (engine.hip k_run: code translation, fetch, decode, exec with
// miss/retry, retire) compiled for the host, for divergence debugging. With
// `fast` set, each instruction first tries the fast loop's form (digest +
// fast_exec, engine_fast.h) and falls back to exec() on a miss, as k_run does.
#include <cstdlib>
#include <vector>
#include "../../wtf_amd/csrc/engine_fast.h"
using namespace wtfgpu_dev;

// Tenet stream of the next sim_run_full (sim_set_tenet; engine_exec.h TenetDev)
static std::vector<uint8_t> g_tn_store;
static uint64_t g_tn_pos, g_tn_cpos, g_tn_ipos, g_tn_last;
static uint32_t g_tn_mute;

extern "C" {
void sim_set_tenet(uint64_t cap) { g_tn_store.assign(cap, 0); }
uint64_t sim_tenet(uint8_t *out, uint64_t cap) {
  const uint64_t n = g_tn_pos < g_tn_store.size() ? g_tn_pos : g_tn_store.size();
  memcpy(out, g_tn_store.data(), n < cap ? n : cap);
  return g_tn_pos;
}

struct SimResult {
  uint64_t gpr[16], rip, rflags, icount, nbytes;
  uint32_t status, vector, error, ovn;
  uint64_t addr;
  uint64_t dirty[64];
  uint64_t xmm[32];
  uint32_t mxcsr, pad;
  uint64_t ymmh[32];
  uint8_t win[512];  // the lane's view of [win_va, win_va + 512) at the end (zeros where unmapped)
};

// final (optional): the lane's whole architectural state at the end, hot
// fields merged into the cold copy as wtfgpu_read_regs does
int sim_run_full(const uint64_t *gpfns, const uint8_t *pages, uint64_t npages, const wtfgpu_regs_t *r0,
                 uint64_t limit, SimResult *out, int fast, uint64_t *fast_count, uint64_t win_va,
                 wtfgpu_regs_t *final, uint8_t *ovpages) {
  uint64_t maxpfn = 0;
  for (uint64_t i = 0; i < npages; i++) maxpfn = gpfns[i] > maxpfn ? gpfns[i] : maxpfn;
  // page pointers carry flags in their low 12 bits: storage must be 4 KiB aligned
  uint8_t *pool = (uint8_t *)aligned_alloc(4096, (npages + 1) * 4096);
  memset(pool, 0, 4096);
  memcpy(pool + 4096, pages, npages * 4096);
  std::vector<uint32_t> map(maxpfn + 1, 0);
  for (uint64_t i = 0; i < npages; i++) if (!map[gpfns[i]]) map[gpfns[i]] = (uint32_t)(i + 1);
  std::vector<uint32_t> ptbits((maxpfn + 32) / 32, 0);
  const uint32_t K = 64;
  uint8_t *ov = (uint8_t *)aligned_alloc(4096, K * 4096);
  std::vector<uint32_t> ovg(K), ovc(1);
  std::vector<uint64_t> fsb(1, r0->seg[WTFGPU_FS].base), gsb(1, r0->seg[WTFGPU_GS].base);
  Dev P{};
  P.pool = pool;
  P.pfn_map = map.data();
  P.pfn_map_len = map.size();
  P.ptbits = ptbits.data();
  P.nlanes = 1;
  P.K = K;
  P.ov_count = ovc.data();
  P.ov_gpfn = ovg.data();
  P.ov_data = ov;
  P.fs_base = fsb.data();
  P.gs_base = gsb.data();
  P.limit = limit;
  wtfgpu_regs_t full = *r0;  // cold state: XMM registers, MXCSR
  LaneSys sys{};  // as engine.hip make_init
  sys.cr0 = r0->cr0;
  sys.cr3 = r0->cr3;
  sys.cr4 = r0->cr4;
  sys.efer = (r0->efer & ~EFER_M32) | (compat_sel(r0->star, r0->seg[WTFGPU_CS].selector) ? EFER_M32 : 0);  // make_init
  sys.cpl = r0->seg[WTFGPU_CS].selector & 3;
  sys.star = r0->star;
  sys.lstar = r0->lstar;
  sys.sfmask = r0->sfmask;
  sys.kgs = r0->kernel_gs_base;
  sys.cs = r0->seg[WTFGPU_CS].selector;
  sys.ss = r0->seg[WTFGPU_SS].selector;
  sys.idtr = r0->idtr_base;
  sys.idtr_limit = r0->idtr_limit;
  sys.tss = r0->seg[WTFGPU_TR].base;
  sys.cr2 = r0->cr2;
  sys.deliv_icount = ~0ull;
  P.full = &full;
  P.sys = &sys;
  uint32_t glo[16], ghi[16];
  Lane L{};
  L.glo = glo;
  L.ghi = ghi;
  for (int i = 0; i < 16; i++) RS(L, i, r0->gpr[i]);
  L.rip = r0->rip;
  L.rflags = r0->rflags;
  L.cr0 = r0->cr0;
  L.cr3 = r0->cr3;
  L.efer = sys.efer;  // as load_lane (U29)
  L.cpl = r0->seg[WTFGPU_CS].selector & 3;
  L.status = WTFGPU_RUNNING;
  L.simd = simd_bits(r0->cr0, r0->cr4, r0->xcr0);
  tlb_flush(L);
  g_tn = TenetDev{};
  if (!g_tn_store.empty()) {
    g_tn_pos = g_tn_cpos = g_tn_ipos = 0;
    g_tn_last = ~0ull;
    g_tn_mute = 0;
    g_tn = TenetDev{g_tn_store.data(), g_tn_store.size(), &g_tn_pos, &g_tn_cpos, &g_tn_ipos, &g_tn_last, &g_tn_mute};
    tn_regs(P, L);  // the registers at the start
  }
  for (uint64_t steps = 0; steps < 100000000 && L.status == WTFGPU_RUNNING; steps++) {
    const uint64_t grip = L.rip;
    uint64_t td;
    if (!tlb_get(L, grip >> 12, td) || !perm_ok(L, td, ACC_X)) {
      if (service_miss(P, L, grip & ~0xfffull, ACC_X)) tlb_get(L, grip >> 12, td);
      else td = 0;
      if (!td && L.status == WTFGPU_EXIT_FAULT) L.exaddr = grip;
    }
    if (!td) break;
    const uint8_t *page = (const uint8_t *)(uintptr_t)(td & ~0xfffull);
    const uint32_t off = grip & 0xfff;
    IBytes ib;
    ib.avail = 4096 - off < 16 ? 4096 - off : 16;
    uint8_t bytes[16] = {0};
    memcpy(bytes, page + off, ib.avail);
    UOp d;
    memcpy(&ib.lo, bytes, 8);
    memcpy(&ib.hi, bytes + 8, 8);
    const bool m32 = (L.efer & EFER_M32) != 0;  // 32-bit code: slow_step's decode, never the fast path (U29)
    int dr = decode(ib, d, m32);
    if (dr == 1) {
      const uint64_t va2 = (grip & ~0xfffull) + 4096;
      if (!tlb_get(L, va2 >> 12, td) || !perm_ok(L, td, ACC_X)) {
        if (service_miss(P, L, va2, ACC_X)) tlb_get(L, va2 >> 12, td);
        else td = 0;
      }
      if (!td) break;
      memcpy(bytes + ib.avail, (const uint8_t *)(uintptr_t)(td & ~0xfffull), 16 - ib.avail);
      memcpy(&ib.lo, bytes, 8);
      memcpy(&ib.hi, bytes + 8, 8);
      ib.avail = 16;
      dr = decode(ib, d, m32);
    }
    if (dr == 2) {
      set_fault(L, WTFGPU_VEC_GP, 0, 0);
      break;
    }
    if (!d.supported) {
      L.status = WTFGPU_EXIT_UNIMPLEMENTED;
      break;
    }
    uint64_t next = 0;
    if (fast && !m32) {
      FOp f;
      digest(d, f);
      if (fo_op(f) != FO_GENERIC) {
        bool done = false;
        for (int fills = 0;; fills++) {  // k_run: a TLB miss / first write served in place (fast_fill)
          L.miss = 0;
          L.pend = 0;
          fast_exec(P, L, f, grip + d.len, next);
          if (!L.miss) {
            done = true;
            break;
          }
          if (L.miss != 2 || fills >= 3 || !fast_fill(P, L)) break;
        }
        if (done) {
          if (fast_count) ++*fast_count;
          L.rip = next;
          L.icount++;
          L.nbytes += d.len + L.pend;
          if (P.limit && L.icount > P.limit) L.status = WTFGPU_EXIT_TIMEOUT;
          continue;
        }
      }
    }
    int x;
    tn_insn_begin(L.lane);
    for (int attempt = 0;; attempt++) {
      L.miss = 0;
      L.pend = 0;
      tn_rollback(L.lane);
      x = exec(P, L, d, grip + d.len, next);
      if (!L.miss || L.status != WTFGPU_RUNNING) break;
      if (attempt >= 16 || !service_miss(P, L, L.miss_va, (int)L.miss_acc)) break;
    }
    if (L.flush) {
      tlb_flush(L);
      L.flush = 0;
    }
    if (x == X_OK && L.status == WTFGPU_RUNNING) {
      L.rip = next;
      L.icount++;
      L.nbytes += d.len + L.pend;
      if (P.limit && L.icount > P.limit) L.status = WTFGPU_EXIT_TIMEOUT;
      if (g_tn.buf) tn_regs(P, L);
    } else if (L.status != WTFGPU_RUNNING) {
    } else if (x == X_UNIMPL) {
      L.status = WTFGPU_EXIT_UNIMPLEMENTED;
    } else if (x == X_INT3) {
      L.status = WTFGPU_EXIT_INT3;
    } else if (x == X_HLT) {
      L.status = WTFGPU_EXIT_HLT;
    }
  }
  if (g_tn.buf && g_tn_pos > g_tn_ipos) tn_regs(P, L);  // open accesses of the stopping instruction
  g_tn = TenetDev{};
  for (int i = 0; i < 16; i++) out->gpr[i] = R(L, i);
  out->rip = L.rip;
  out->rflags = L.rflags;
  out->icount = L.icount;
  out->nbytes = L.nbytes;
  out->status = L.status;
  out->vector = L.exvec;
  out->error = L.exerr;
  out->addr = L.exaddr;
  out->ovn = L.ovn;
  for (uint32_t k = 0; k < L.ovn && k < 64; k++) out->dirty[k] = (uint64_t)ovg[k] << 12;
  for (int k = 0; k < 16; k++) out->xmm[2 * k] = full.xmm[k][0], out->xmm[2 * k + 1] = full.xmm[k][1];
  out->mxcsr = full.mxcsr;
  for (int k = 0; k < 16; k++) out->ymmh[2 * k] = full.ymmh[k][0], out->ymmh[2 * k + 1] = full.ymmh[k][1];
  if (ovpages) memcpy(ovpages, ov, (size_t)(L.ovn < 64 ? L.ovn : 64) * 4096);  // the dirty pages, in out->dirty order
  if (final) {
    wtfgpu_regs_t f = full;
    for (int i = 0; i < 16; i++) f.gpr[i] = R(L, i);
    f.rip = L.rip;
    f.rflags = L.rflags;
    f.seg[WTFGPU_FS].base = fsb[0];
    f.seg[WTFGPU_GS].base = gsb[0];
    f.cr0 = sys.cr0;
    f.cr3 = sys.cr3;
    f.cr4 = sys.cr4;
    f.efer = sys.efer & ~EFER_M32;
    f.kernel_gs_base = sys.kgs;
    f.star = sys.star;
    f.lstar = sys.lstar;
    f.sfmask = sys.sfmask;
    f.cr2 = sys.cr2;
    f.seg[WTFGPU_CS].selector = sys.cs;
    f.seg[WTFGPU_SS].selector = sys.ss;
    *final = f;
  }
  memset(out->win, 0, sizeof(out->win));
  if (win_va) {
    L.cpl = 0;
    const uint32_t st = L.status;
    for (uint32_t i = 0; i < sizeof(out->win); i++) {
      uint64_t td, gpfn;
      if (walk(P, L, win_va + i, ACC_R, td, gpfn)) out->win[i] = ((const uint8_t *)(uintptr_t)(td & ~0xfffull))[(win_va + i) & 0xfff];
    }
    L.status = st;
  }
  free(pool);
  free(ov);
  return 0;
}

// Decode + digest of up to 16 instruction bytes (diagnostic: which forms the
// fast path leaves generic). out: decode result, UOp op, sub, FOp op, length,
// seg, p67, rep, rex, asz, bsz, asrc, bsrc, is_mem, supported.
int sim_digest(const uint8_t *bytes, uint32_t avail, uint32_t *out) {
  IBytes ib;
  ib.avail = avail > 16 ? 16 : avail;
  uint8_t b[16] = {};
  memcpy(b, bytes, ib.avail);
  memcpy(&ib.lo, b, 8);
  memcpy(&ib.hi, b + 8, 8);
  UOp d;
  const int dr = decode(ib, d);
  FOp f{};
  if (dr == 0) digest(d, f);
  const uint32_t v[15] = {(uint32_t)dr, d.op, d.sub, fo_op(f), d.len, d.seg, d.p67, d.rep, d.rex,
                          d.asz, d.bsz, d.asrc, d.bsrc, d.is_mem, d.supported};
  memcpy(out, v, sizeof(v));
  return dr;
}
int sim_run_mode(const uint64_t *gpfns, const uint8_t *pages, uint64_t npages, const wtfgpu_regs_t *r0,
                 uint64_t limit, SimResult *out, int fast, uint64_t *fast_count, uint64_t win_va) {
  return sim_run_full(gpfns, pages, npages, r0, limit, out, fast, fast_count, win_va, nullptr, nullptr);
}
int sim_run(const uint64_t *gpfns, const uint8_t *pages, uint64_t npages, const wtfgpu_regs_t *r0,
            uint64_t limit, SimResult *out) {
  return sim_run_mode(gpfns, pages, npages, r0, limit, out, 0, nullptr, 0);
}
}
