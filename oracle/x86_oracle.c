/*
 * x86_oracle.c — scalar CPU restatement of the wtf execution hot path.
 * TEST INFRASTRUCTURE ONLY (see x86_oracle.h). Plain C99, one lane, no tricks:
 * decode with a classic byte switch, execute, account hooks.
 *
 * Semantic conventions for behaviour the SDM leaves undefined (SURVEY.md
 * H1 / Appendix C). The GPU engine implements the same choices; DESIGN.md §5
 * lists them:
 *   U1 logic ops (and/or/xor/test): CF=OF=AF=0.
 *   U2 shl/shr/sar, count!=0: AF=0; OF = (shl) msb(res)^CF, (shr) msb(orig),
 *      (sar) 0 for every count; CF=0 when count > operand bits.
 *   U3 rol/ror: OF = msb(res)^lsb(res) (rol), msb(res)^msb-1(res) (ror), any count.
 *      rcl/rcr: OF = msb(res)^CF (rcl), msb(res)^msb-1(res) (rcr), any count.
 *   U4 mul/imul: SF/ZF/PF from the low half of the product, AF=0.
 *   U5 div/idiv: flags unchanged.
 *   U6 bsf/bsr: only ZF written; zero source leaves the destination unchanged.
 *      tzcnt/lzcnt: only CF and ZF written. bt/bts/btr/btc: only CF written.
 *   U7 shld/shrd: AF=0, OF = msb(res)^msb(orig); count > operand bits (16-bit
 *      forms) shifts through the 32-bit concatenation modulo 32.
 *   U8 no accessed/dirty bit updates during page walks; no TLB (every access walks).
 *   U9 a rep string instruction is one retired instruction whatever the count.
 *   U10 a breakpoint handler that stops the lane or moves rip cancels the
 *      hooked instruction (not executed, not counted).
 *   U11 an exception is delivered through the guest IDT when the snapshot has
 *      a present 64-bit interrupt / trap gate for its vector (TSS RSP0 / IST
 *      stack switch, frame push, cr2 for #PF, IF cleared by interrupt gates);
 *      otherwise the lane exits FAULT with vector / error code / cr2 and the
 *      faulting instruction not retired. A fault raised before any instruction
 *      retired since the previous delivery exits too (the double / triple
 *      fault a CPU would raise, U18).
 *   U12 int3 and hlt exit before retiring.
 *   U13 16-bit bswap writes 0.
 *   U15 RDRAND r returns 0 with CF=1 (the value is unpinned: bochs draws a host
 *       random number; the hevd module overwrites it, fuzzer_hevd.cc:96-108).
 *   U16 SYSCALL / SYSRETQ (64-bit forms; 32-bit SYSRET is unimplemented) load
 *       CS/SS selectors from STAR without descriptor-table reads; SWAPGS swaps
 *       GS.base with IA32_KERNEL_GS_BASE.
 *   U19 IRETQ (64-bit operand size) pops rip, cs, rflags, rsp, ss and loads the
 *       selectors without descriptor-table reads; the new CPL is cs.RPL (a
 *       return to an inner ring, or a null cs, is #GP); rflags bits change as
 *       the SDM's IRET lists for the current CPL / IOPL.
 *   U20 MOV crN, r64 at CPL 0: cr0 / cr2 / cr4 / cr8 are written; a cr3 other
 *       than the testcase's initial cr3 retires the instruction and ends the
 *       testcase with Cr3Change_t (bochscpu_backend.cc:628-657; the limit
 *       check of the retire hook runs after it and wins).
 *   U21 RDTSC / RDTSCP return the snapshot's Tsc + the instructions retired
 *       so far (bochs' tick counter advances one per instruction); RDMSR /
 *       WRMSR at CPL 0 reach the MSRs CpuState_t carries (TSC, APIC_BASE,
 *       SYSENTER_*, PAT, EFER, STAR, LSTAR, CSTAR, SFMASK, FS/GS/KERNEL_GS
 *       base, TSC_AUX); any other MSR, a non-canonical base / entry point or
 *       upper bits in SFMASK / TSC_AUX is #GP(0); EFER.LMA is read-only.
 *   U22 SSE / SSE2: the legacy-encoded integer and data-movement subset (see
 *       exec_sse) plus pshufb and ptest; SSE floating-point arithmetic and
 *       the rest of SSE3+ are UNIMPLEMENTED. MMX: U37 (exec_mmx). #UD if CR0.EM or !CR4.OSFXSR, #NM if CR0.TS, #GP(0) for a
 *       misaligned 16-byte operand of an aligned form; the checks run in that
 *       order, before any memory access.
 *   U23 AVX / AVX2 (VEX): the same subset at 128 / 256 bits plus vzeroupper,
 *       vzeroall, vpshufb, vptest, vpbroadcast (see exec_vex); VEX.128 zeroes
 *       bits 255:128; legacy SSE leaves them. 16- / 32-byte operands: every
 *       page is checked before any byte moves, a fault is reported at the
 *       operand's start or at the page boundary it crosses.
 */
#include "x86_oracle.h"
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;
typedef int64_t i64;

/* ---------------- small open-addressing hash map u64 -> pointer ---------------- */
typedef struct {
  u64 *keys;
  void **vals;
  u8 *used;
  u64 cap, n;
} hmap;

static u64 hmix(u64 x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

static void hm_init(hmap *h, u64 cap) {
  h->cap = cap;
  h->n = 0;
  h->keys = (u64 *)calloc(cap, sizeof(u64));
  h->vals = (void **)calloc(cap, sizeof(void *));
  h->used = (u8 *)calloc(cap, 1);
}
static void hm_free(hmap *h) {
  free(h->keys);
  free(h->vals);
  free(h->used);
  memset(h, 0, sizeof(*h));
}
static void **hm_slot(hmap *h, u64 k, int insert);
static void hm_grow(hmap *h) {
  hmap n;
  hm_init(&n, h->cap * 2);
  for (u64 i = 0; i < h->cap; i++)
    if (h->used[i]) *hm_slot(&n, h->keys[i], 1) = h->vals[i];
  hm_free(h);
  *h = n;
}
static void **hm_slot(hmap *h, u64 k, int insert) {
  if (insert && (h->n + 1) * 2 > h->cap) hm_grow(h);
  u64 i = hmix(k) & (h->cap - 1);
  for (;;) {
    if (!h->used[i]) {
      if (!insert) return NULL;
      h->used[i] = 1;
      h->keys[i] = k;
      h->vals[i] = NULL;
      h->n++;
      return &h->vals[i];
    }
    if (h->keys[i] == k) return &h->vals[i];
    i = (i + 1) & (h->cap - 1);
  }
}
static void *hm_get(hmap *h, u64 k) {
  void **s = hm_slot(h, k, 0);
  return s ? *s : NULL;
}
static int hm_has(hmap *h, u64 k) { return hm_slot(h, k, 0) != NULL; }

/* growable u64 vector */
typedef struct {
  u64 *v;
  u64 n, cap;
} vec;
static void vec_push(vec *a, u64 x) {
  if (a->n == a->cap) {
    a->cap = a->cap ? a->cap * 2 : 64;
    a->v = (u64 *)realloc(a->v, a->cap * sizeof(u64));
  }
  a->v[a->n++] = x;
}

/* ---------------- machine ---------------- */
struct orc_machine {
  hmap snap;    /* gpfn -> const page (owned copy) */
  hmap overlay; /* gpfn -> private page */
  vec dirty;    /* gpfns in first-write order */
  hmap bps;     /* gva -> (void*)1 */
  hmap cov;     /* rip -> (void*)1 */
  vec covlist;
  wtfgpu_regs_t r;
  u64 initial_cr3;
  u64 limit;
  u64 icount;
  u64 bytes;
  u64 deliv_icount; /* retired count at the last IDT delivery (valid if deliv_valid) */
  int deliv_valid;
  int edges; /* record branch edges into the coverage (RecordEdge) */
  u64 edges_run, edges_new; /* RecordEdge calls of the testcase, and those whose edge joined its set (run stats) */
  int trace, resumed; /* rip trace on; the next instruction resumes a breakpoint hit */
  vec tracelist;
  /* Tenet (U38, wtfgpu_set_tenet's stream): entries as u64 words */
  int tn, tn_mute;
  u32 xm_flags; /* MXCSR flags of an instruction that faulted with #XM (U40) */
  vec tnlist;
  u64 tn_ipos, tn_last; /* the current instruction's first entry / latest ACC entry (~0: none) */
  /* per-instruction scratch */
  wtfgpu_exit_t *ex;
  int faulted;
};

static const u8 kZeroPage[4096];

#define RF_CF 0x1ULL
#define RF_PF 0x4ULL
#define RF_AF 0x10ULL
#define RF_ZF 0x40ULL
#define RF_SF 0x80ULL
#define RF_TF 0x100ULL
#define RF_IF 0x200ULL
#define RF_DF 0x400ULL
#define RF_OF 0x800ULL
#define RF_STATUS (RF_CF | RF_PF | RF_AF | RF_ZF | RF_SF | RF_OF)

orc_machine *orc_create(void) {
  orc_machine *m = (orc_machine *)calloc(1, sizeof(*m));
  hm_init(&m->snap, 1024);
  hm_init(&m->overlay, 64);
  hm_init(&m->bps, 64);
  hm_init(&m->cov, 1024);
  return m;
}

void orc_destroy(orc_machine *m) {
  if (!m) return;
  for (u64 i = 0; i < m->snap.cap; i++)
    if (m->snap.used[i]) free(m->snap.vals[i]);
  for (u64 i = 0; i < m->overlay.cap; i++)
    if (m->overlay.used[i]) free(m->overlay.vals[i]);
  hm_free(&m->snap);
  hm_free(&m->overlay);
  hm_free(&m->bps);
  hm_free(&m->cov);
  free(m->dirty.v);
  free(m->covlist.v);
  free(m->tracelist.v);
  free(m->tnlist.v);
  free(m);
}

int orc_add_page(orc_machine *m, u64 gpfn, const u8 *page) {
  void **s = hm_slot(&m->snap, gpfn, 1);
  if (!*s) *s = malloc(4096);
  memcpy(*s, page, 4096);
  return 0;
}

void orc_set_regs(orc_machine *m, const wtfgpu_regs_t *r) { m->r = *r; }
void orc_get_regs(orc_machine *m, wtfgpu_regs_t *r) { *r = m->r; }
void orc_set_limit(orc_machine *m, u64 limit) { m->limit = limit; }
void orc_set_edges(orc_machine *m, int on) { m->edges = on; }

int orc_set_breakpoints(orc_machine *m, const u64 *gvas, u32 n) {
  hm_free(&m->bps);
  hm_init(&m->bps, 64);
  for (u32 i = 0; i < n; i++) *hm_slot(&m->bps, gvas[i], 1) = (void *)1;
  return 0;
}

void orc_restore(orc_machine *m, const wtfgpu_regs_t *r) {
  for (u64 i = 0; i < m->overlay.cap; i++)
    if (m->overlay.used[i]) free(m->overlay.vals[i]);
  hm_free(&m->overlay);
  hm_init(&m->overlay, 64);
  m->dirty.n = 0;
  hm_free(&m->cov);
  hm_init(&m->cov, 1024);
  m->covlist.n = 0;
  m->tracelist.n = 0;
  m->tnlist.n = 0;
  m->tn_ipos = 0;
  m->tn_last = ~0ULL;
  m->tn_mute = 0;
  m->r = *r;
  m->initial_cr3 = r->cr3;
  m->icount = 0;
  m->bytes = 0;
  m->edges_run = m->edges_new = 0;
  m->deliv_valid = 0;
}

uint64_t orc_icount(orc_machine *m) { return m->icount; }
uint64_t orc_bytes(orc_machine *m) { return m->bytes; }
uint64_t orc_edges(orc_machine *m, uint64_t *unique) {
  if (unique) *unique = m->edges_new;
  return m->edges_run;
}

uint64_t orc_coverage(orc_machine *m, u64 *out, u64 cap) {
  for (u64 i = 0; i < m->covlist.n && i < cap; i++) out[i] = m->covlist.v[i];
  return m->covlist.n;
}
uint64_t orc_dirty(orc_machine *m, u64 *out, u64 cap) {
  for (u64 i = 0; i < m->dirty.n && i < cap; i++) out[i] = m->dirty.v[i] << 12;
  return m->dirty.n;
}

/* ---------------- physical memory ---------------- */
static const u8 *phys_ro(orc_machine *m, u64 gpfn) {
  const u8 *p = (const u8 *)hm_get(&m->overlay, gpfn);
  if (p) return p;
  p = (const u8 *)hm_get(&m->snap, gpfn);
  return p ? p : kZeroPage;
}
/* Copy-on-write: the page joins the lane's dirty set (bochscpu_backend.cc:887-889). */
static u8 *phys_rw(orc_machine *m, u64 gpfn) {
  void **s = hm_slot(&m->overlay, gpfn, 1);
  if (!*s) {
    u8 *p = (u8 *)malloc(4096);
    const u8 *src = (const u8 *)hm_get(&m->snap, gpfn);
    memcpy(p, src ? src : kZeroPage, 4096);
    *s = p;
    vec_push(&m->dirty, gpfn);
  }
  return (u8 *)*s;
}
static u64 phys_read64(orc_machine *m, u64 pa) {
  u64 v;
  memcpy(&v, phys_ro(m, pa >> 12) + (pa & 0xfff), 8);
  return v;
}


int orc_read_phys(orc_machine *m, u64 gpa, void *buf, u64 len) {
  u8 *o = (u8 *)buf;
  while (len) {
    u64 off = gpa & 0xfff, n = 4096 - off;
    if (n > len) n = len;
    memcpy(o, phys_ro(m, gpa >> 12) + off, n);
    o += n;
    gpa += n;
    len -= n;
  }
  return 0;
}
int orc_write_phys(orc_machine *m, u64 gpa, const void *buf, u64 len) {
  const u8 *i = (const u8 *)buf;
  while (len) {
    u64 off = gpa & 0xfff, n = 4096 - off;
    if (n > len) n = len;
    memcpy(phys_rw(m, gpa >> 12) + off, i, n);
    i += n;
    gpa += n;
    len -= n;
  }
  return 0;
}

/* ---------------- page walk ---------------- */
enum { ACC_R = 0, ACC_W = 1, ACC_X = 2 };
#define PTE_P 0x1ULL
#define PTE_W 0x2ULL
#define PTE_U 0x4ULL
#define PTE_PS 0x80ULL
#define PTE_NX (1ULL << 63)
#define PTE_ADDR 0x000ffffffffff000ULL

static int cpl(orc_machine *m) { return m->r.seg[WTFGPU_CS].selector & 3; }
/* 32-bit code (compatibility mode, U29): CS is SYSRET's 32-bit selector,
 * STAR[63:48] (the one CS.L = 0 code segment of Windows' and Linux' GDTs;
 * descriptors are not read, U19). bochscpu.hpp:119-182 carries the segment
 * cache whose CS.L the reference's core reads. */
static int is_m32(orc_machine *m) {
  return ((m->r.seg[WTFGPU_CS].selector ^ (u32)(m->r.star >> 48)) & 0xfffc) == 0;
}

static int is_canonical(u64 va) {
  i64 s = (i64)(va << 16) >> 16;
  return (u64)s == va;
}


/* 4-level walk; check: perform permission checks. Returns 0 ok, else sets fault. */
static int walk(orc_machine *m, u64 va, int acc, int check, u64 *pa) {
  const int user = cpl(m) == 3;
  const int nxe = (m->r.efer >> 11) & 1;
  const int wp = (m->r.cr0 >> 16) & 1;
  u64 table = m->r.cr3 & PTE_ADDR;
  int allow_w = 1, allow_u = 1, nx = 0;
  u64 e = 0;
  int level;
  u64 page_mask = 0xfff;
  if (check && !is_canonical(va)) {
    m->faulted = 1;
    m->ex->status = WTFGPU_EXIT_FAULT;
    m->ex->vector = WTFGPU_VEC_GP;
    m->ex->error = 0;
    m->ex->addr = va;
    return -1;
  }
  for (level = 3; level >= 0; level--) {
    const u64 idx = (va >> (12 + 9 * level)) & 0x1ff;
    e = phys_read64(m, table + idx * 8);
    if (!(e & PTE_P)) goto pf_notpresent;
    allow_w &= (e & PTE_W) != 0;
    allow_u &= (e & PTE_U) != 0;
    if (nxe && (e & PTE_NX)) nx = 1;
    if (level > 0 && level < 3 && (e & PTE_PS)) {
      page_mask = level == 2 ? 0x3fffffffULL : 0x1fffffULL;
      break;
    }
    table = e & PTE_ADDR;
  }
  if (check) {
    int bad = 0;
    if (user && !allow_u) bad = 1;
    if (acc == ACC_W && !allow_w && (user || wp)) bad = 1;
    if (acc == ACC_X && nx) bad = 1;
    if (bad) {
      m->faulted = 1;
      m->ex->status = WTFGPU_EXIT_FAULT;
      m->ex->vector = WTFGPU_VEC_PF;
      m->ex->error = 1 | (acc == ACC_W ? 2 : 0) | (user ? 4 : 0) | (acc == ACC_X && nxe ? 16 : 0);
      m->ex->addr = va;
      return -1;
    }
  }
  *pa = ((e & PTE_ADDR) & ~page_mask) | (va & page_mask);
  return 0;
pf_notpresent:
  if (check) {
    m->faulted = 1;
    m->ex->status = WTFGPU_EXIT_FAULT;
    m->ex->vector = WTFGPU_VEC_PF;
    m->ex->error = (acc == ACC_W ? 2 : 0) | (user ? 4 : 0) | (acc == ACC_X && nxe ? 16 : 0);
    m->ex->addr = va;
  }
  return -1;
}

int orc_translate(orc_machine *m, u64 gva, u64 *gpa) {
  wtfgpu_exit_t dummy;
  wtfgpu_exit_t *save = m->ex;
  m->ex = &dummy;
  int rc = walk(m, gva, ACC_R, 0, gpa);
  m->ex = save;
  return rc;
}
int orc_read_virt(orc_machine *m, u64 gva, void *buf, u64 len) {
  u8 *o = (u8 *)buf;
  while (len) {
    u64 off = gva & 0xfff, n = 4096 - off, pa;
    if (n > len) n = len;
    if (orc_translate(m, gva, &pa)) return -1;
    orc_read_phys(m, pa, o, n);
    o += n;
    gva += n;
    len -= n;
  }
  return 0;
}
int orc_write_virt(orc_machine *m, u64 gva, const void *buf, u64 len) {
  const u8 *i = (const u8 *)buf;
  while (len) {
    u64 off = gva & 0xfff, n = 4096 - off, pa;
    if (n > len) n = len;
    if (orc_translate(m, gva, &pa)) return -1;
    orc_write_phys(m, pa, i, n);
    i += n;
    gva += n;
    len -= n;
  }
  return 0;
}

/* ---------------- Tenet (U38) ----------------
 * The stream wtfgpu_set_tenet documents (include/wtfgpu.h), as u64 words:
 * ACC {va, 1 << 56 | type << 32 | len, data words} for each data access of an
 * instruction (an operand as a whole, an RMW operand once as type 3), REGS
 * {2 << 56, gpr[16], rip} at the start, after each retired instruction,
 * delivered exception and rip-moving breakpoint handler, and when the run
 * stops with accesses open. ACC data = the memory after the instruction, read
 * byte by byte through present-bit translation (zero where none). Implicit
 * supervisor accesses (descriptor tables, exception frames) are not logged. */
#define TN_R 1u
#define TN_W 2u
#define TN_RW 3u
static void tn_access(orc_machine *m, u64 va, u32 len, u32 type) {
  if (!m->tn || m->tn_mute) return;
  if (type == TN_W && m->tn_last != ~0ULL && m->tnlist.v[m->tn_last] == va &&
      m->tnlist.v[m->tn_last + 1] == ((1ULL << 56) | ((u64)TN_RW << 32) | len))
    return; /* the write of a read-modify-write operand */
  m->tn_last = m->tnlist.n;
  vec_push(&m->tnlist, va);
  vec_push(&m->tnlist, (1ULL << 56) | ((u64)type << 32) | len);
  for (u32 i = 0; i < (len + 7) / 8; i++) vec_push(&m->tnlist, 0);
}
static void tn_regs(orc_machine *m) {
  if (!m->tn) return;
  for (u64 q = m->tn_ipos; q + 2 <= m->tnlist.n;) {
    const u64 va = m->tnlist.v[q], len = m->tnlist.v[q + 1] & 0xffffffffULL;
    u8 *out = (u8 *)&m->tnlist.v[q + 2];
    for (u64 i = 0; i < len; i++) {
      u64 pa;
      u8 b = 0;
      if (orc_translate(m, va + i, &pa) == 0) orc_read_phys(m, pa, &b, 1);
      out[i] = b;
    }
    q += 2 + (len + 7) / 8;
  }
  vec_push(&m->tnlist, 2ULL << 56);
  for (int i = 0; i < 16; i++) vec_push(&m->tnlist, m->r.gpr[i]);
  vec_push(&m->tnlist, m->r.rip);
  m->tn_ipos = m->tnlist.n;
  m->tn_last = ~0ULL;
}

/* ---------------- guest virtual access with permission checks ---------------- */
/* Translate [va, va+len) (len <= 16) for acc; fills up to two physical spans. */
static int vprobe(orc_machine *m, u64 va, u32 len, int acc, u64 pa[2], u32 n[2]) {
  u64 off = va & 0xfff;
  if (walk(m, va, acc, 1, &pa[0])) return -1;
  if (off + len <= 4096) {
    n[0] = len;
    n[1] = 0;
    return 0;
  }
  n[0] = (u32)(4096 - off);
  n[1] = len - n[0];
  if (walk(m, va + n[0], acc, 1, &pa[1])) return -1;
  return 0;
}
static int vread(orc_machine *m, u64 va, u32 len, void *out) {
  u64 pa[2];
  u32 n[2];
  if (vprobe(m, va, len, ACC_R, pa, n)) return -1;
  orc_read_phys(m, pa[0], out, n[0]);
  if (n[1]) orc_read_phys(m, pa[1], (u8 *)out + n[0], n[1]);
  m->bytes += len;
  tn_access(m, va, len, TN_R);
  return 0;
}
static int vwrite(orc_machine *m, u64 va, u32 len, const void *in) {
  u64 pa[2];
  u32 n[2];
  if (vprobe(m, va, len, ACC_W, pa, n)) return -1;
  orc_write_phys(m, pa[0], in, n[0]);
  if (n[1]) orc_write_phys(m, pa[1], (const u8 *)in + n[0], n[1]);
  m->bytes += len;
  tn_access(m, va, len, TN_W);
  return 0;
}
/* Read for a read-modify-write: write permission required, pages dirtied at
 * read time like bochs' read_RMW (reported as BOCHSCPU_HOOK_MEM_RW). */
static int vread_rmw(orc_machine *m, u64 va, u32 len, void *out) {
  u64 pa[2];
  u32 n[2];
  if (vprobe(m, va, len, ACC_W, pa, n)) return -1;
  memcpy(out, phys_rw(m, pa[0] >> 12) + (pa[0] & 0xfff), n[0]);
  if (n[1]) memcpy((u8 *)out + n[0], phys_rw(m, pa[1] >> 12) + (pa[1] & 0xfff), n[1]);
  m->bytes += len;
  tn_access(m, va, len, TN_RW);
  return 0;
}

/* up to 32 bytes: every page checked before any byte moves (a 32-byte
 * operand crosses at most one page boundary; the fault is at its start or
 * at the boundary) */
static int vread_n(orc_machine *m, u64 va, u32 len, void *out) {
  if (len <= 16) return vread(m, va, len, out);
  u64 pa[2];
  u32 nn[2];
  if (vprobe(m, va, 16, ACC_R, pa, nn) || vprobe(m, va + 16, len - 16, ACC_R, pa, nn)) return -1;
  m->tn_mute++; /* Tenet: one access of len bytes */
  const int rc = vread(m, va, 16, out) || vread(m, va + 16, len - 16, (u8 *)out + 16);
  m->tn_mute--;
  if (!rc) tn_access(m, va, len, TN_R);
  return rc;
}
static int vwrite_n(orc_machine *m, u64 va, u32 len, const void *in) {
  if (len <= 16) return vwrite(m, va, len, in);
  u64 pa[2];
  u32 nn[2];
  if (vprobe(m, va, 16, ACC_W, pa, nn) || vprobe(m, va + 16, len - 16, ACC_W, pa, nn)) return -1;
  m->tn_mute++;
  const int rc = vwrite(m, va, 16, in) || vwrite(m, va + 16, len - 16, (const u8 *)in + 16);
  m->tn_mute--;
  if (!rc) tn_access(m, va, len, TN_W);
  return rc;
}

/* ---------------- decode ---------------- */
typedef struct {
  u64 start;
  u32 len;
  u32 pfx66, pfx67, rep, lock, seg; /* seg: 0 none, 4 fs, 5 gs */
  u32 rex, rexw, rexr, rexx, rexb;
  u32 opmap; /* 0 one-byte, 1 = 0F, 2 = 0F38, 3 = 0F3A */
  u32 m32, a16; /* 32-bit code (U29); a 67 prefix there (16-bit addresses: outside) */
  u32 undef; /* U36: an encoding the emulated CPU does not define (#UD) */
  u32 vex, vl, vw, vvvv, vpp, vbad; /* VEX prefix: present, L, W, vvvv (decoded), pp; a legacy prefix before it */
  u32 evex, ell, ez, eb, eaaa, er2; /* EVEX (U47): L'L, z, b, aaa, R' (vvvv has V' as bit 4) */
  u32 op;
  u32 has_modrm, mod, reg, rm; /* reg, rm include REX extension */
  u32 is_mem;
  u64 ea; /* effective address (linear, seg base included) */
  int vsib_idx, vsib_base; /* the SIB's raw index register (-1: no SIB) and base (-1: none), for VSIB */
  u32 vsib_ss;
  u64 vsib_disp;
  u8 bytes[16];
  u32 pos;
  int fetch_fail;
} insn;

static u8 fetch8(orc_machine *m, insn *d) {
  if (d->pos >= 15) {
    d->fetch_fail = 2; /* too long -> #GP */
    return 0;
  }
  u64 va = d->start + d->pos;
  u64 pa;
  if (walk(m, va, ACC_X, 1, &pa)) {
    d->fetch_fail = 1;
    return 0;
  }
  u8 b = phys_ro(m, pa >> 12)[pa & 0xfff];
  d->bytes[d->pos++] = b;
  return b;
}
static u64 fetchn(orc_machine *m, insn *d, int n) {
  u64 v = 0;
  for (int i = 0; i < n; i++) v |= (u64)fetch8(m, d) << (8 * i);
  return v;
}
static u64 sxn(u64 v, int bytes) {
  int s = 64 - 8 * bytes;
  return (u64)(((i64)(v << s)) >> s);
}

static u64 seg_base(orc_machine *m, u32 seg) {
  if (seg == 4) return m->r.seg[WTFGPU_FS].base;
  if (seg == 5) return m->r.seg[WTFGPU_GS].base;
  return 0;
}

/* Decode modrm (+sib, disp). ea computed relative to rip of next insn later
 * (rip-relative needs final length) -> store components. */
typedef struct {
  int riprel;
  u64 disp;
  int base, index, scale;
} memref;

static void decode_modrm(orc_machine *m, insn *d, memref *mr) {
  u8 b = fetch8(m, d);
  d->has_modrm = 1;
  d->mod = b >> 6;
  d->reg = ((b >> 3) & 7) | (d->rexr << 3);
  u32 rm = b & 7;
  memset(mr, 0, sizeof(*mr));
  mr->base = -1;
  mr->index = -1;
  d->vsib_idx = -1;
  if (d->mod == 3) {
    d->rm = rm | (d->rexb << 3);
    d->is_mem = 0;
    return;
  }
  d->is_mem = 1;
  if (rm == 4) {
    u8 sib = fetch8(m, d);
    u32 ss = sib >> 6, idx = ((sib >> 3) & 7) | (d->rexx << 3), base = sib & 7;
    d->vsib_idx = (int)idx;
    d->vsib_ss = ss;
    if (idx != 4) {
      mr->index = (int)idx;
      mr->scale = 1 << ss;
    }
    if (base == 5 && d->mod == 0) {
      mr->disp = sxn(fetchn(m, d, 4), 4);
    } else {
      mr->base = (int)(base | (d->rexb << 3));
    }
  } else if (rm == 5 && d->mod == 0) {
    mr->riprel = !d->m32; /* 32-bit code: disp32 absolute */
    mr->disp = sxn(fetchn(m, d, 4), 4);
  } else {
    mr->base = (int)(rm | (d->rexb << 3));
  }
  if (d->mod == 1) mr->disp = sxn(fetchn(m, d, 1), 1);
  if (d->mod == 2) mr->disp = sxn(fetchn(m, d, 4), 4);
  d->vsib_base = mr->base;
  d->vsib_disp = mr->disp;
}

static void finish_ea(orc_machine *m, insn *d, memref *mr) {
  if (!d->is_mem) return;
  u64 ea;
  if (mr->riprel) {
    ea = d->start + d->len + mr->disp;
  } else {
    ea = mr->disp;
    if (mr->base >= 0) ea += m->r.gpr[mr->base];
    if (mr->index >= 0) ea += m->r.gpr[mr->index] * (u64)mr->scale;
  }
  if (d->pfx67) ea &= 0xffffffffULL;
  d->ea = ea + seg_base(m, d->seg);
}

/* ---------------- registers ---------------- */
static u64 szmask(int sz) { return sz == 8 ? ~0ULL : ((1ULL << (8 * sz)) - 1); }

static u64 getreg(orc_machine *m, insn *d, u32 r, int sz) {
  if (sz == 1) {
    if (!d->rex && r >= 4 && r < 8) return (m->r.gpr[r - 4] >> 8) & 0xff;
    return m->r.gpr[r] & 0xff;
  }
  return m->r.gpr[r] & szmask(sz);
}
static void setreg(orc_machine *m, insn *d, u32 r, int sz, u64 v) {
  if (sz == 1) {
    if (!d->rex && r >= 4 && r < 8) {
      m->r.gpr[r - 4] = (m->r.gpr[r - 4] & ~0xff00ULL) | ((v & 0xff) << 8);
    } else {
      m->r.gpr[r] = (m->r.gpr[r] & ~0xffULL) | (v & 0xff);
    }
  } else if (sz == 2) {
    m->r.gpr[r] = (m->r.gpr[r] & ~0xffffULL) | (v & 0xffff);
  } else if (sz == 4) {
    m->r.gpr[r] = v & 0xffffffffULL;
  } else {
    m->r.gpr[r] = v;
  }
}

/* rm operand access */
static int rd_rm(orc_machine *m, insn *d, int sz, u64 *v) {
  if (!d->is_mem) {
    *v = getreg(m, d, d->rm, sz);
    return 0;
  }
  *v = 0;
  return vread(m, d->ea, (u32)sz, v);
}
static int rd_rm_rmw(orc_machine *m, insn *d, int sz, u64 *v) {
  if (!d->is_mem) {
    *v = getreg(m, d, d->rm, sz);
    return 0;
  }
  *v = 0;
  return vread_rmw(m, d->ea, (u32)sz, v);
}
static int wr_rm(orc_machine *m, insn *d, int sz, u64 v) {
  if (!d->is_mem) {
    setreg(m, d, d->rm, sz, v);
    return 0;
  }
  return vwrite(m, d->ea, (u32)sz, &v);
}

/* ---------------- flags ---------------- */
static int parity8(u64 v) { return !__builtin_parity((unsigned)(v & 0xff)); }
static u64 msb(u64 v, int sz) { return (v >> (8 * sz - 1)) & 1; }

static void set_flags(orc_machine *m, u64 mask, u64 vals) {
  m->r.rflags = (m->r.rflags & ~mask) | (vals & mask);
}
static u64 szp(u64 res, int sz) {
  res &= szmask(sz);
  return (res == 0 ? RF_ZF : 0) | (msb(res, sz) ? RF_SF : 0) | (parity8(res) ? RF_PF : 0);
}
static int CF(orc_machine *m) { return (m->r.rflags & RF_CF) != 0; }

/* ALU binary op: 0 add,1 or,2 adc,3 sbb,4 and,5 sub,6 xor,7 cmp. Returns result. */
static u64 alu2(orc_machine *m, int op, u64 a, u64 b, int sz) {
  const u64 mk = szmask(sz);
  a &= mk;
  b &= mk;
  u64 res = 0, f = 0;
  u64 c = 0;
  switch (op) {
  case 0:
  case 2: {
    c = (op == 2) ? (u64)CF(m) : 0;
    res = (a + b + c) & mk;
    int carry;
    if (sz == 8)
      carry = (res < a) || (c && res == a);
    else
      carry = ((a + b + c) >> (8 * sz)) & 1;
    f = szp(res, sz) | (carry ? RF_CF : 0) | (((a ^ b ^ res) & 0x10) ? RF_AF : 0) |
        (msb((a ^ res) & (b ^ res), sz) ? RF_OF : 0);
    break;
  }
  case 3:
  case 5:
  case 7: {
    c = (op == 3) ? (u64)CF(m) : 0;
    res = (a - b - c) & mk;
    int borrow = (a < b) || (c && a == b);
    f = szp(res, sz) | (borrow ? RF_CF : 0) | (((a ^ b ^ res) & 0x10) ? RF_AF : 0) |
        (msb((a ^ b) & (a ^ res), sz) ? RF_OF : 0);
    break;
  }
  case 1:
    res = a | b;
    f = szp(res, sz);
    break;
  case 4:
    res = a & b;
    f = szp(res, sz);
    break;
  case 6:
    res = a ^ b;
    f = szp(res, sz);
    break;
  }
  set_flags(m, RF_STATUS, f);
  return res;
}

static int cond(orc_machine *m, u32 cc) {
  const u64 f = m->r.rflags;
  const int cf = (f & RF_CF) != 0, zf = (f & RF_ZF) != 0, sf = (f & RF_SF) != 0,
            of = (f & RF_OF) != 0, pf = (f & RF_PF) != 0;
  int r;
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

/* shifts/rotates: op = modrm.reg (0 rol,1 ror,2 rcl,3 rcr,4 shl,5 shr,6 sal=shl,7 sar) */
static u64 shift_op(orc_machine *m, int op, u64 v, u32 count, int sz) {
  const int bits = 8 * sz;
  const u64 mk = szmask(sz);
  u32 cnt = count & (sz == 8 ? 0x3f : 0x1f);
  v &= mk;
  if (cnt == 0) return v;
  u64 res = v;
  u64 f = m->r.rflags;
  int cf;
  switch (op) {
  case 0: { /* rol */
    u32 c = cnt % bits;
    res = c ? ((v << c) | (v >> (bits - c))) & mk : v;
    cf = res & 1;
    f = (f & ~(RF_CF | RF_OF)) | (cf ? RF_CF : 0) | ((msb(res, sz) ^ cf) ? RF_OF : 0);
    break;
  }
  case 1: { /* ror */
    u32 c = cnt % bits;
    res = c ? ((v >> c) | (v << (bits - c))) & mk : v;
    cf = (int)msb(res, sz);
    f = (f & ~(RF_CF | RF_OF)) | (cf ? RF_CF : 0) |
        ((msb(res, sz) ^ ((res >> (bits - 2)) & 1)) ? RF_OF : 0);
    break;
  }
  case 2: { /* rcl */
    u32 c = (sz == 1) ? cnt % 9 : (sz == 2) ? cnt % 17 : cnt;
    int carry = CF(m);
    for (u32 i = 0; i < c; i++) {
      int out = (int)msb(res, sz);
      res = ((res << 1) | (u64)carry) & mk;
      carry = out;
    }
    f = (f & ~(RF_CF | RF_OF)) | (carry ? RF_CF : 0) | ((msb(res, sz) ^ (u64)carry) ? RF_OF : 0);
    break;
  }
  case 3: { /* rcr */
    u32 c = (sz == 1) ? cnt % 9 : (sz == 2) ? cnt % 17 : cnt;
    int carry = CF(m);
    for (u32 i = 0; i < c; i++) {
      int out = (int)(res & 1);
      res = (res >> 1) | ((u64)carry << (bits - 1));
      carry = out;
    }
    f = (f & ~(RF_CF | RF_OF)) | (carry ? RF_CF : 0) |
        ((msb(res, sz) ^ ((res >> (bits - 2)) & 1)) ? RF_OF : 0);
    break;
  }
  case 4:
  case 6: { /* shl */
    res = cnt >= 64 ? 0 : (v << cnt) & mk;
    cf = cnt <= (u32)bits ? (int)((v >> (bits - cnt)) & 1) : 0;
    f = (f & ~RF_STATUS) | szp(res, sz) | (cf ? RF_CF : 0) | ((msb(res, sz) ^ (u64)cf) ? RF_OF : 0);
    break;
  }
  case 5: { /* shr */
    res = cnt >= 64 ? 0 : v >> cnt;
    cf = cnt <= (u32)bits ? (int)((v >> (cnt - 1)) & 1) : 0;
    f = (f & ~RF_STATUS) | szp(res, sz) | (cf ? RF_CF : 0) | (msb(v, sz) ? RF_OF : 0);
    break;
  }
  case 7: { /* sar */
    i64 sv = (i64)sxn(v, sz);
    u32 c = cnt >= (u32)bits ? (u32)bits - 1 : cnt;
    res = (u64)(sv >> c) & mk;
    cf = (int)(((u64)(sv >> (cnt >= (u32)bits ? (u32)bits - 1 : cnt - 1))) & 1);
    f = (f & ~RF_STATUS) | szp(res, sz) | (cf ? RF_CF : 0);
    break;
  }
  }
  m->r.rflags = f;
  return res;
}

/* ---------------- stack ---------------- */
/* 32-bit code addresses the stack with esp (U29: the result zero-extends) */
static u64 smask(orc_machine *m) { return is_m32(m) ? 0xffffffffULL : ~0ULL; }
static int push64(orc_machine *m, u64 v, int sz) {
  u64 rsp = (m->r.gpr[WTFGPU_RSP] - (u64)sz) & smask(m);
  if (vwrite(m, rsp, (u32)sz, &v)) return -1;
  m->r.gpr[WTFGPU_RSP] = rsp;
  return 0;
}
static int pop64(orc_machine *m, u64 *v, int sz) {
  u64 t = 0;
  const u64 sm = smask(m);
  if (vread(m, m->r.gpr[WTFGPU_RSP] & sm, (u32)sz, &t)) return -1;
  m->r.gpr[WTFGPU_RSP] = ((m->r.gpr[WTFGPU_RSP] & sm) + (u64)sz) & sm;
  *v = t;
  return 0;
}

static void fault(orc_machine *m, u32 vec, u32 err) {
  m->faulted = 1;
  m->ex->status = WTFGPU_EXIT_FAULT;
  m->ex->vector = vec;
  m->ex->error = err;
  m->ex->addr = 0;
}

/* ---------------- string instructions ---------------- */
static int string_op(orc_machine *m, insn *d, u32 op, int sz) {
  /* op: a4 movs, a6 cmps, aa stos, ac lods, ae scas (sz from low bit) */
  const u64 amask = d->pfx67 ? 0xffffffffULL : ~0ULL;
  const int df = (m->r.rflags & RF_DF) != 0;
  const u64 step = df ? (u64)-(i64)sz : (u64)sz;
  const u64 srcbase = seg_base(m, d->seg);
  for (;;) {
    if (d->rep) {
      if ((m->r.gpr[WTFGPU_RCX] & amask) == 0) break;
    }
    u64 rsi = m->r.gpr[WTFGPU_RSI] & amask, rdi = m->r.gpr[WTFGPU_RDI] & amask;
    u64 a = 0, b = 0;
    int stop_rep = 0;
    const u64 bytes0 = m->bytes; /* a faulting iteration accounts no bytes */
    switch (op) {
    case 0xa4:
      if (vread(m, srcbase + rsi, (u32)sz, &a)) { m->bytes = bytes0; return -1; }
      if (vwrite(m, rdi, (u32)sz, &a)) { m->bytes = bytes0; return -1; }
      break;
    case 0xa6:
      if (vread(m, srcbase + rsi, (u32)sz, &a)) { m->bytes = bytes0; return -1; }
      if (vread(m, rdi, (u32)sz, &b)) { m->bytes = bytes0; return -1; }
      alu2(m, 7, a, b, sz);
      break;
    case 0xaa:
      a = m->r.gpr[WTFGPU_RAX];
      if (vwrite(m, rdi, (u32)sz, &a)) { m->bytes = bytes0; return -1; }
      break;
    case 0xac:
      if (vread(m, srcbase + rsi, (u32)sz, &a)) { m->bytes = bytes0; return -1; }
      setreg(m, d, WTFGPU_RAX, sz, a);
      break;
    case 0xae:
      if (vread(m, rdi, (u32)sz, &b)) { m->bytes = bytes0; return -1; }
      alu2(m, 7, m->r.gpr[WTFGPU_RAX], b, sz);
      break;
    }
    if (op == 0xa4 || op == 0xa6 || op == 0xac) {
      u64 n = (rsi + step) & amask;
      m->r.gpr[WTFGPU_RSI] = n;
    }
    if (op != 0xac) {
      u64 n = (rdi + step) & amask;
      m->r.gpr[WTFGPU_RDI] = n;
    }
    if (!d->rep) break;
    {
      u64 c = (m->r.gpr[WTFGPU_RCX] - 1) & amask;
      m->r.gpr[WTFGPU_RCX] = c;
    }
    if (op == 0xa6 || op == 0xae) {
      const int zf = (m->r.rflags & RF_ZF) != 0;
      if (d->rep == 0xf3 && !zf) stop_rep = 1;
      if (d->rep == 0xf2 && zf) stop_rep = 1;
    }
    if (stop_rep) break;
  }
  return 0;
}

/* ---------------- mul / div ---------------- */
static int muldiv(orc_machine *m, insn *d, int sub, int sz, u64 src) {
  const u64 mk = szmask(sz);
  const int bits = 8 * sz;
  u64 a = m->r.gpr[WTFGPU_RAX] & mk;
  if (sz == 1) a = m->r.gpr[WTFGPU_RAX] & 0xff;
  switch (sub) {
  case 4: { /* mul */
    unsigned __int128 p = (unsigned __int128)a * (src & mk);
    u64 lo = (u64)p & mk, hi = (u64)(p >> bits) & mk;
    if (sz == 8) hi = (u64)(p >> 64);
    if (sz == 1) {
      setreg(m, d, WTFGPU_RAX, 2, (u64)p & 0xffff);
    } else {
      setreg(m, d, WTFGPU_RAX, sz, lo);
      setreg(m, d, WTFGPU_RDX, sz, hi);
    }
    u64 f = szp(lo, sz) | (hi ? (RF_CF | RF_OF) : 0);
    set_flags(m, RF_STATUS, f);
    return 0;
  }
  case 5: { /* imul */
    __int128 p = (__int128)(i64)sxn(a, sz) * (__int128)(i64)sxn(src & mk, sz);
    u64 lo = (u64)p & mk;
    u64 hi = (u64)(p >> bits) & mk;
    if (sz == 8) hi = (u64)(p >> 64);
    int ovf = (__int128)(i64)sxn(lo, sz) != p;
    if (sz == 1) {
      setreg(m, d, WTFGPU_RAX, 2, (u64)p & 0xffff);
    } else {
      setreg(m, d, WTFGPU_RAX, sz, lo);
      setreg(m, d, WTFGPU_RDX, sz, hi);
    }
    set_flags(m, RF_STATUS, szp(lo, sz) | (ovf ? (RF_CF | RF_OF) : 0));
    return 0;
  }
  case 6: { /* div */
    u64 dv = src & mk;
    if (dv == 0) {
      fault(m, WTFGPU_VEC_DE, 0);
      return -1;
    }
    unsigned __int128 n;
    if (sz == 1)
      n = m->r.gpr[WTFGPU_RAX] & 0xffff;
    else
      n = ((unsigned __int128)(m->r.gpr[WTFGPU_RDX] & mk) << bits) | a;
    unsigned __int128 q = n / dv, r = n % dv;
    if (q > mk) {
      fault(m, WTFGPU_VEC_DE, 0);
      return -1;
    }
    if (sz == 1) {
      setreg(m, d, WTFGPU_RAX, 2, ((u64)r << 8) | (u64)q);
    } else {
      setreg(m, d, WTFGPU_RAX, sz, (u64)q);
      setreg(m, d, WTFGPU_RDX, sz, (u64)r);
    }
    return 0;
  }
  case 7: { /* idiv */
    i64 dv = (i64)sxn(src & mk, sz);
    if (dv == 0) {
      fault(m, WTFGPU_VEC_DE, 0);
      return -1;
    }
    __int128 n;
    if (sz == 1)
      n = (__int128)(int16_t)(m->r.gpr[WTFGPU_RAX] & 0xffff);
    else if (sz == 8)
      n = (__int128)(((unsigned __int128)m->r.gpr[WTFGPU_RDX] << 64) | a);
    else
      n = (__int128)(i64)sxn(((m->r.gpr[WTFGPU_RDX] & mk) << bits) | a, 2 * sz);
    /* overflow: quotient out of range (also INT_MIN / -1) */
    __int128 q, r;
    if (dv == -1) {
      if (n < -(((__int128)1 << (bits - 1)) - 1)) { /* -n would leave the range */
        fault(m, WTFGPU_VEC_DE, 0);
        return -1;
      }
      q = -n;
      r = 0;
    } else {
      q = n / dv;
      r = n % dv;
    }
    __int128 lo = -((__int128)1 << (bits - 1)), hi = ((__int128)1 << (bits - 1)) - 1;
    if (q < lo || q > hi) {
      fault(m, WTFGPU_VEC_DE, 0);
      return -1;
    }
    if (sz == 1) {
      setreg(m, d, WTFGPU_RAX, 2, (((u64)r & 0xff) << 8) | ((u64)q & 0xff));
    } else {
      setreg(m, d, WTFGPU_RAX, sz, (u64)q);
      setreg(m, d, WTFGPU_RDX, sz, (u64)r);
    }
    return 0;
  }
  }
  return 0;
}

/* ---------------- execute one instruction ---------------- */
/* X_FAULT_KEEP: rep progress stays; X_FAULT_PARTIAL: a gather's completed
 * elements stay in its registers (U46), its bytes are not counted */
enum { X_OK = 0, X_FAULT = 1, X_UNIMPL = 2, X_INT3 = 3, X_HLT = 4, X_CR3 = 5, X_FAULT_KEEP = 6, X_FAULT_PARTIAL = 7 };

#define CHK(x)                                                                                   \
  do {                                                                                           \
    if (x) return X_FAULT;                                                                       \
  } while (0)

/* ---------------- SSE / SSE2 (U22) ----------------
 * The legacy-encoded integer and data-movement subset compilers emit for
 * x86-64 (SSE2 baseline): 128-bit moves, scalar / half moves, movd / movq,
 * logic, integer add / sub / saturate / compare / min / max / multiply,
 * shifts, shuffles, unpacks, packs, mask extraction, ldmxcsr / stmxcsr, fences,
 * movnti, plus pshufb (0f 38 00) and ptest (0f 38 17). MMX (no-prefix 0f 6x /
 * dx-fx), SSE floating-point arithmetic and the rest of SSE3+ are outside the
 * subset (UNIMPLEMENTED); VEX forms are exec_vex's. Faults: #UD when CR0.EM = 1
 * or CR4.OSFXSR = 0, #NM when CR0.TS = 1, #GP(0) for a 16-byte memory operand
 * that is not 16-byte aligned (all but movups / movupd / movdqu). */
typedef struct { u8 b[16]; } x128;

static x128 xreg(orc_machine *m, u32 r) {
  x128 v;
  memcpy(v.b, m->r.xmm[r & 15], 16);
  return v;
}
static void xput(orc_machine *m, u32 r, x128 v) { memcpy(m->r.xmm[r & 15], v.b, 16); }
static u64 el(const x128 *v, int i, int w) {
  u64 x = 0;
  memcpy(&x, v->b + i * w, (size_t)w);
  return x;
}
static void elput(x128 *v, int i, int w, u64 x) { memcpy(v->b + i * w, &x, (size_t)w); }
static i64 sel(const x128 *v, int i, int w) { return (i64)sxn(el(v, i, w), w); }
static u64 satu(i64 x, int w) {
  const i64 hi = (i64)szmask(w);
  return (u64)(x < 0 ? 0 : x > hi ? hi : x);
}
static u64 sats(i64 x, int w) {
  const i64 hi = (i64)(szmask(w) >> 1), lo = -hi - 1;
  return (u64)(x < lo ? lo : x > hi ? hi : x) & szmask(w);
}

/* element-wise op `k` on w-byte elements */
enum { EW_ADD, EW_SUB, EW_ADDUS, EW_SUBUS, EW_ADDS, EW_SUBS, EW_MINU, EW_MAXU, EW_MINS, EW_MAXS, EW_EQ, EW_GT,
       EW_AVG, EW_MULLO, EW_MULHS, EW_MULHU };
static x128 ewise(int k, int w, const x128 *a, const x128 *b) {
  x128 r;
  for (int i = 0; i < 16 / w; i++) {
    const u64 x = el(a, i, w), y = el(b, i, w);
    const i64 sx = sel(a, i, w), sy = sel(b, i, w);
    u64 v = 0;
    switch (k) {
    case EW_ADD: v = x + y; break;
    case EW_SUB: v = x - y; break;
    case EW_ADDUS: v = satu((i64)(x + y), w); break;
    case EW_SUBUS: v = satu((i64)x - (i64)y, w); break;
    case EW_ADDS: v = sats(sx + sy, w); break;
    case EW_SUBS: v = sats(sx - sy, w); break;
    case EW_MINU: v = x < y ? x : y; break;
    case EW_MAXU: v = x > y ? x : y; break;
    case EW_MINS: v = sx < sy ? x : y; break;
    case EW_MAXS: v = sx > sy ? x : y; break;
    case EW_EQ: v = x == y ? ~0ULL : 0; break;
    case EW_GT: v = sx > sy ? ~0ULL : 0; break;
    case EW_AVG: v = (x + y + 1) >> 1; break;
    case EW_MULLO: v = (u64)(sx * sy); break;
    case EW_MULHS: v = (u64)((sx * sy) >> 16); break;
    default: v = (x * y) >> 16; break;
    }
    elput(&r, i, w, v & szmask(w));
  }
  return r;
}
/* interleave the low (hi = 0) or high halves of a and b in w-byte elements */
static x128 unpack(int w, int hi, const x128 *a, const x128 *b) {
  x128 r;
  const int n = 8 / w;
  for (int i = 0; i < n; i++) {
    elput(&r, 2 * i, w, el(a, i + hi * n, w));
    elput(&r, 2 * i + 1, w, el(b, i + hi * n, w));
  }
  return r;
}
/* shift every w-byte element by cnt: 0 logical right, 1 arithmetic right, 2 left */
static x128 shift_el(int kind, int w, const x128 *a, u64 cnt) {
  x128 r;
  const u64 bits = 8 * (u64)w;
  for (int i = 0; i < 16 / w; i++) {
    const u64 x = el(a, i, w);
    u64 v;
    if (kind == 1) v = (u64)(sel(a, i, w) >> (cnt >= bits ? bits - 1 : cnt));
    else if (cnt >= bits) v = 0;
    else v = kind == 0 ? x >> cnt : x << cnt;
    elput(&r, i, w, v & szmask(w));
  }
  return r;
}

/* the r/m operand as 128 bits: an xmm register, or n bytes of memory
 * (zero-extended; n = 16 needs 16-byte alignment when `align`) */
static int xsrc(orc_machine *m, insn *d, int n, int align, x128 *v) {
  memset(v->b, 0, 16);
  if (!d->is_mem) {
    *v = xreg(m, d->rm);
    return 0;
  }
  if (align && (d->ea & 15)) {
    fault(m, WTFGPU_VEC_GP, 0);
    return -1;
  }
  return vread(m, d->ea, (u32)n, v->b);
}
static int xstore(orc_machine *m, insn *d, int n, int align, const x128 *v) {
  if (align && (d->ea & 15)) {
    fault(m, WTFGPU_VEC_GP, 0);
    return -1;
  }
  return vwrite(m, d->ea, (u32)n, v->b);
}

static int sse_opcode(u32 op) {
  return (op >= 0x10 && op <= 0x17) || (op >= 0x28 && op <= 0x2f) || op == 0xc2 || (op >= 0x50 && op <= 0x7f) ||
         op == 0xae || op == 0xc3 || (op >= 0xc4 && op <= 0xc6) || op >= 0xd0;
}

/* pshufb of one lane */
static x128 pshufb(const x128 *a, const x128 *b) {
  x128 r;
  for (int i = 0; i < 16; i++) r.b[i] = (b->b[i] & 0x80) ? 0 : a->b[b->b[i] & 15];
  return r;
}
/* ptest over n bytes: ZF = (a & b) == 0, CF = (~a & b) == 0, AF OF PF SF = 0 */
static void ptest(orc_machine *m, const u8 *a, const u8 *b, int n) {
  int z = 1, c = 1;
  for (int i = 0; i < n; i++) {
    if (a[i] & b[i]) z = 0;
    if (~a[i] & b[i]) c = 0;
  }
  m->r.rflags = (m->r.rflags & ~RF_STATUS) | (z ? RF_ZF : 0) | (c ? RF_CF : 0);
}

/* ---------------- MMX (U37) ----------------
 * The MMX and SSE-integer-on-MMX forms of 0f 60-7f, c4 / c5, d1-fe (no
 * mandatory prefix), emms, and movq2dq / movdq2q (f3 / f2 0f d6). mm i is
 * physical x87 register R(i); fpst holds ST(0..7), so mm i = fpst[(i - TOS) & 7].
 * A completed MMX instruction sets TOS = 0 (fpst rotated to R order) and every
 * tag valid (fptw = 0); emms sets every tag empty (fptw = 0xffff). Checks in
 * order: #UD if CR0.EM, #NM if CR0.TS, #MF if an unmasked x87 flag is set, then the operand's
 * memory faults (8-byte operands, no alignment check). ModRM's mm fields
 * ignore REX. maskmovq, the SSSE3 (0f 38 / 0f 3a) and the floating-point
 * MMX forms are UNIMPLEMENTED; 0f 6c / 6d / d0 / d6 / e6 / f0 without a prefix
 * are #UD. */
static int mmx_opcode(u32 op) {
  return (op >= 0x60 && op <= 0x7f && op != 0x78 && op != 0x79 && op != 0x7a && op != 0x7b && op != 0x7c &&
          op != 0x7d) ||
         op == 0xc4 || op == 0xc5 || (op >= 0xd0 && op <= 0xfe);
}
static u64 mmx_read(const orc_machine *m, u32 i) { return m->r.fpst[(i - ((m->r.fpsw >> 11) & 7)) & 7]; }
/* a completed MMX instruction: TOS = 0 (fpst rotated to R order), tags valid */
static void mmx_commit(orc_machine *m) {
  const u32 tos = (m->r.fpsw >> 11) & 7;
  if (tos) {
    u64 t[8];
    u16 e[8];
    for (u32 j = 0; j < 8; j++) t[j] = m->r.fpst[(j - tos) & 7], e[j] = m->r.fpse[(j - tos) & 7];
    memcpy(m->r.fpst, t, sizeof(t));
    memcpy(m->r.fpse, e, sizeof(e));
  }
  m->r.fpsw &= (u16)~0x3800;
  m->r.fptw = 0;
}
/* an MMX register write: the significand, sign and exponent all ones */
static void mmx_put(orc_machine *m, u32 i, u64 v) {
  m->r.fpst[i] = v;
  m->r.fpse[i] = 0xffff;
}
static x128 x64(u64 v) {
  x128 r;
  memset(r.b, 0, 16);
  memcpy(r.b, &v, 8);
  return r;
}

/* The SSSE3 instructions on mm registers (no prefix; 0f 38 00-0b / 1c-1e, 0f 3a 0f), after the SDM's
 * operation sections: d = the destination's quadword, s = the source's. */
static int ssse3_mm(u32 map, u32 op) { return map == 2 ? (op <= 0x0b || (op >= 0x1c && op <= 0x1e)) : (map == 3 && op == 0x0f); }
static u64 ssse3_mm_op(u32 map, u32 op, u64 d, u64 s, u32 imm) {
  u64 r = 0;
  if (map == 3) { /* palignr: ((d << 64) | s) >> (imm * 8), low 64 bits */
    for (u32 i = 0; i < 8; i++) {
      const u32 k = i + imm; /* byte k of the 16-byte concatenation (0-7: s, 8-15: d) */
      const u64 byte = k < 8 ? (s >> (8 * k)) & 0xff : k < 16 ? (d >> (8 * (k - 8))) & 0xff : 0;
      r |= byte << (8 * i);
    }
    return r;
  }
  switch (op) {
  case 0x00: /* pshufb */
    for (u32 i = 0; i < 8; i++) {
      const u32 k = (u32)(s >> (8 * i)) & 0xff;
      if (!(k & 0x80)) r |= ((d >> (8 * (k & 7))) & 0xff) << (8 * i);
    }
    return r;
  case 0x01: case 0x02: case 0x03: case 0x05: case 0x06: case 0x07: { /* phadd / phsub w, d, sw */
    const u32 w = op == 0x02 || op == 0x06 ? 4 : 2, n = 8 / w;
    for (u32 i = 0; i < n; i++) { /* result i: pair i of d (i < n / 2), else pair i - n / 2 of s */
      const u64 src = i < n / 2 ? d : s;
      const u32 j = 2 * (i % (n / 2));
      const i64 x = (i64)sxn((src >> (8 * w * j)) & szmask((int)w), (int)w);
      const i64 y = (i64)sxn((src >> (8 * w * (j + 1))) & szmask((int)w), (int)w);
      i64 v = op >= 0x05 ? x - y : x + y;
      if (op == 0x03 || op == 0x07) v = v > 32767 ? 32767 : v < -32768 ? -32768 : v;
      r |= ((u64)v & szmask((int)w)) << (8 * w * i);
    }
    return r;
  }
  case 0x04: /* pmaddubsw: unsigned bytes of d times signed bytes of s, pairs, saturated */
    for (u32 i = 0; i < 4; i++) {
      const i64 v = (i64)((d >> (16 * i)) & 0xff) * (int8_t)(s >> (16 * i)) +
                    (i64)((d >> (16 * i + 8)) & 0xff) * (int8_t)(s >> (16 * i + 8));
      r |= (u64)(u16)(v > 32767 ? 32767 : v < -32768 ? -32768 : v) << (16 * i);
    }
    return r;
  case 0x08: case 0x09: case 0x0a: { /* psignb / w / d */
    const u32 w = 1u << (op - 8);
    for (u32 i = 0; i < 8 / w; i++) {
      const i64 sv = (i64)sxn((s >> (8 * w * i)) & szmask((int)w), (int)w);
      const u64 dv = (d >> (8 * w * i)) & szmask((int)w);
      const u64 v = sv < 0 ? (0 - dv) : sv == 0 ? 0 : dv;
      r |= (v & szmask((int)w)) << (8 * w * i);
    }
    return r;
  }
  case 0x0b: /* pmulhrsw */
    for (u32 i = 0; i < 4; i++) {
      const int32_t t = (int32_t)(int16_t)(d >> (16 * i)) * (int32_t)(int16_t)(s >> (16 * i));
      r |= (u64)(u16)(((t >> 14) + 1) >> 1) << (16 * i);
    }
    return r;
  default: { /* 1c-1e pabsb / w / d of s */
    const u32 w = 1u << (op - 0x1c);
    for (u32 i = 0; i < 8 / w; i++) {
      const i64 sv = (i64)sxn((s >> (8 * w * i)) & szmask((int)w), (int)w);
      r |= ((u64)(sv < 0 ? -sv : sv) & szmask((int)w)) << (8 * w * i);
    }
    return r;
  }
  }
}

static int exec_mmx(orc_machine *m, insn *d, int pc) {
  const u32 op = d->op, r3 = d->reg & 7, mr = d->reg & 7, mm_rm = d->rm & 7;
  const int mem = d->is_mem;
  const u8 imm = d->bytes[d->len - 1];
  if (d->opmap == 1 && pc == 0 && (op == 0xd0 || op == 0xd6 || op == 0xe6 || op == 0xf0 || op == 0x6c || op == 0x6d)) {
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (d->opmap == 1 && op == 0xf7 && mem) { /* maskmovq: register operands only */
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (d->opmap == 1 && (op >= 0x71 && op <= 0x73) &&
      (mem || !((op == 0x73) ? (r3 == 2 || r3 == 6) : (r3 == 2 || r3 == 4 || r3 == 6)))) {
    fault(m, WTFGPU_VEC_UD, 0); /* register forms /2 /4 /6 (73: /2 /6) only */
    return X_FAULT;
  }
  if (d->opmap == 1 && (op == 0xc5 || op == 0xd7 || (op == 0xd6 && pc)) && mem) {
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (d->opmap == 1 && op == 0xe7 && !mem) {
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (m->r.cr0 & 4) { /* CR0.EM */
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (m->r.cr0 & 8) { /* CR0.TS */
    fault(m, 7, 0);
    return X_FAULT;
  }
  if (m->r.fpsw & ~m->r.fpcw & 0x3f) { /* a pending unmasked x87 exception */
    fault(m, 16, 0);
    return X_FAULT;
  }
  if (d->opmap == 1 && op == 0x77) { /* emms */
    m->r.fptw = 0xffff;
    return X_OK;
  }
  if (d->opmap >= 2) { /* SSSE3 on mm registers (U41) */
    const u64 dv = mmx_read(m, mr);
    u64 sv = 0;
    if (mem) {
      if (vread(m, d->ea, 8, &sv)) return X_FAULT;
    } else {
      sv = mmx_read(m, mm_rm);
    }
    const u64 res = ssse3_mm_op(d->opmap, op, dv, sv, imm);
    mmx_commit(m);
    mmx_put(m, mr, res);
    return X_OK;
  }
  if (op == 0xf7) { /* maskmovq mm1, mm2: mm1's bytes whose mm2 byte has bit 7 set, to [rdi] (seg override applies) */
    const u64 dv = mmx_read(m, mr), sel = mmx_read(m, mm_rm);
    u64 di = m->r.gpr[7];
    if (d->pfx67) di &= 0xffffffffULL;
    di += seg_base(m, d->seg);
    u64 pa[2];
    u32 nn[2];
    for (u32 i = 0; i < 8; i++) /* every written byte's page first */
      if (((sel >> (8 * i + 7)) & 1) && vprobe(m, di + i, 1, ACC_W, pa, nn)) return X_FAULT;
    int rc = 0;
    m->tn_mute++;
    for (u32 i = 0; !rc && i < 8; i++)
      if ((sel >> (8 * i + 7)) & 1) {
        const u8 b = (u8)(dv >> (8 * i));
        rc = vwrite(m, di + i, 1, &b);
      }
    m->tn_mute--;
    if (rc) return X_FAULT;
    tn_access(m, di, 8, TN_W);
    mmx_commit(m);
    return X_OK;
  }
  if (op == 0xd6) { /* f3: movq2dq xmm, mm; f2: movdq2q mm, xmm */
    if (pc == 2) {
      const u64 v = mmx_read(m, mm_rm);
      mmx_commit(m);
      xput(m, d->reg, x64(v));
    } else {
      const x128 x = xreg(m, d->rm);
      mmx_commit(m);
      mmx_put(m, mr, el(&x, 0, 8));
    }
    return X_OK;
  }
  const u64 av = mmx_read(m, mr);
  u64 bv = 0;
  /* the r/m source (not for the forms whose r/m is a destination or a GPR) */
  const int rm_src = !(op == 0x7e || op == 0x7f || op == 0xe7 || op == 0x6e || op == 0xc4);
  if (rm_src) {
    if (mem) {
      if (vread(m, d->ea, 8, &bv)) return X_FAULT;
    } else {
      bv = mmx_read(m, mm_rm);
    }
  }
  x128 a = x64(av), b = x64(bv), r;
  u64 res;
  int to_gpr = -1;
  switch (op) {
  case 0x6e: { /* movd / movq mm, r/m */
    const int n = d->rexw ? 8 : 4;
    u64 v = 0;
    if (mem) {
      if (vread(m, d->ea, (u32)n, &v)) return X_FAULT;
    } else {
      v = m->r.gpr[d->rm] & szmask(n);
    }
    res = v;
    break;
  }
  case 0x7e: { /* movd / movq r/m, mm */
    const int n = d->rexw ? 8 : 4;
    const u64 v = av & szmask(n);
    if (mem) {
      if (vwrite(m, d->ea, (u32)n, &v)) return X_FAULT;
      mmx_commit(m);
      return X_OK;
    }
    mmx_commit(m);
    m->r.gpr[d->rm] = v;
    return X_OK;
  }
  case 0x6f: res = bv; break;
  case 0x7f: case 0xe7: /* movq mm/m64, mm; movntq m64, mm */
    if (mem) {
      if (vwrite(m, d->ea, 8, &av)) return X_FAULT;
      mmx_commit(m);
      return X_OK;
    }
    mmx_commit(m);
    mmx_put(m, mm_rm, av);
    return X_OK;
  case 0x60: case 0x61: case 0x62: /* punpckl*: the low halves */
    r = unpack(1 << (op - 0x60), 0, &a, &b);
    res = el(&r, 0, 8);
    break;
  case 0x68: case 0x69: case 0x6a: { /* punpckh*: the high halves */
    const x128 ah = x64(av >> 32), bh = x64(bv >> 32);
    r = unpack(1 << (op - 0x68), 0, &ah, &bh);
    res = el(&r, 0, 8);
    break;
  }
  case 0x63: case 0x67: case 0x6b: { /* packsswb, packuswb, packssdw: a's elements, then b's */
    const int w = op == 0x6b ? 4 : 2, n = 8 / w;
    r = x64(0);
    for (int i = 0; i < 2 * n; i++) {
      const i64 x = i < n ? sel(&a, i, w) : sel(&b, i - n, w);
      elput(&r, i, w / 2, op == 0x67 ? satu(x, 1) : sats(x, w / 2));
    }
    res = el(&r, 0, 8);
    break;
  }
  case 0x64: case 0x65: case 0x66: case 0x74: case 0x75: case 0x76:
    r = ewise(op >= 0x74 ? EW_EQ : EW_GT, 1 << ((op & 0xf) % 4), &a, &b);
    res = el(&r, 0, 8);
    break;
  case 0x70: /* pshufw */
    res = 0;
    for (int i = 0; i < 4; i++) res |= ((bv >> (16 * ((imm >> (2 * i)) & 3))) & 0xffff) << (16 * i);
    break;
  case 0x71: case 0x72: case 0x73: { /* shifts by imm8 of mm (r/m) */
    const int w = op == 0x71 ? 2 : op == 0x72 ? 4 : 8;
    r = shift_el(r3 == 2 ? 0 : r3 == 4 ? 1 : 2, w, &b, imm);
    mmx_commit(m);
    mmx_put(m, mm_rm, el(&r, 0, 8));
    return X_OK;
  }
  case 0xc4: { /* pinsrw mm, r32/m16, imm8 */
    u64 v = 0;
    if (mem) {
      if (vread(m, d->ea, 2, &v)) return X_FAULT;
    } else {
      v = m->r.gpr[d->rm];
    }
    const int k = imm & 3;
    res = (av & ~(0xffffULL << (16 * k))) | ((v & 0xffff) << (16 * k));
    break;
  }
  case 0xc5: /* pextrw r32, mm, imm8 */
    to_gpr = 1;
    res = (bv >> (16 * (imm & 3))) & 0xffff;
    break;
  case 0xd7: /* pmovmskb r32, mm */
    to_gpr = 1;
    res = 0;
    for (int i = 0; i < 8; i++) res |= ((bv >> (8 * i + 7)) & 1) << i;
    break;
  case 0xd1: case 0xd2: case 0xd3: r = shift_el(0, op == 0xd1 ? 2 : op == 0xd2 ? 4 : 8, &a, bv); res = el(&r, 0, 8); break;
  case 0xe1: case 0xe2: r = shift_el(1, op == 0xe1 ? 2 : 4, &a, bv); res = el(&r, 0, 8); break;
  case 0xf1: case 0xf2: case 0xf3: r = shift_el(2, op == 0xf1 ? 2 : op == 0xf2 ? 4 : 8, &a, bv); res = el(&r, 0, 8); break;
  case 0xd4: res = av + bv; break;
  case 0xfb: res = av - bv; break;
  case 0xfc: case 0xfd: case 0xfe: r = ewise(EW_ADD, 1 << (op - 0xfc), &a, &b); res = el(&r, 0, 8); break;
  case 0xf8: case 0xf9: case 0xfa: r = ewise(EW_SUB, 1 << (op - 0xf8), &a, &b); res = el(&r, 0, 8); break;
  case 0xd5: r = ewise(EW_MULLO, 2, &a, &b); res = el(&r, 0, 8); break;
  case 0xe5: r = ewise(EW_MULHS, 2, &a, &b); res = el(&r, 0, 8); break;
  case 0xe4: r = ewise(EW_MULHU, 2, &a, &b); res = el(&r, 0, 8); break;
  case 0xd8: case 0xd9: r = ewise(EW_SUBUS, op - 0xd7, &a, &b); res = el(&r, 0, 8); break;
  case 0xdc: case 0xdd: r = ewise(EW_ADDUS, op - 0xdb, &a, &b); res = el(&r, 0, 8); break;
  case 0xe8: case 0xe9: r = ewise(EW_SUBS, op - 0xe7, &a, &b); res = el(&r, 0, 8); break;
  case 0xec: case 0xed: r = ewise(EW_ADDS, op - 0xeb, &a, &b); res = el(&r, 0, 8); break;
  case 0xda: r = ewise(EW_MINU, 1, &a, &b); res = el(&r, 0, 8); break;
  case 0xde: r = ewise(EW_MAXU, 1, &a, &b); res = el(&r, 0, 8); break;
  case 0xea: r = ewise(EW_MINS, 2, &a, &b); res = el(&r, 0, 8); break;
  case 0xee: r = ewise(EW_MAXS, 2, &a, &b); res = el(&r, 0, 8); break;
  case 0xe0: r = ewise(EW_AVG, 1, &a, &b); res = el(&r, 0, 8); break;
  case 0xe3: r = ewise(EW_AVG, 2, &a, &b); res = el(&r, 0, 8); break;
  case 0xdb: res = av & bv; break;
  case 0xdf: res = ~av & bv; break;
  case 0xeb: res = av | bv; break;
  case 0xef: res = av ^ bv; break;
  case 0xf4: res = (av & 0xffffffffULL) * (bv & 0xffffffffULL); break; /* pmuludq */
  case 0xf5: /* pmaddwd */
    r = x64(0);
    for (int i = 0; i < 2; i++)
      elput(&r, i, 4, (u64)(sel(&a, 2 * i, 2) * sel(&b, 2 * i, 2) + sel(&a, 2 * i + 1, 2) * sel(&b, 2 * i + 1, 2)) & 0xffffffffULL);
    res = el(&r, 0, 8);
    break;
  case 0xf6: { /* psadbw */
    u64 sum = 0;
    for (int i = 0; i < 8; i++) {
      const u32 x = (u32)((av >> (8 * i)) & 0xff), y = (u32)((bv >> (8 * i)) & 0xff);
      sum += x > y ? x - y : y - x;
    }
    res = sum;
    break;
  }
  default:
    return X_UNIMPL;
  }
  mmx_commit(m);
  if (to_gpr >= 0) m->r.gpr[d->reg] = res; /* zero-extended into the 64-bit register */
  else mmx_put(m, mr, res);
  return X_OK;
}

static int fp_form_o(u32 map, u32 c, int pp, int vex); /* x86_oracle_fp.inc */
static int exec_fp(orc_machine *m, insn *d);
static int s4_form_o(u32 map, u32 c, int pp, int vex); /* x86_oracle_sse4.inc */
static int exec_s4(orc_machine *m, insn *d);
static int gx_form_o(u32 map, u32 c, int pp, int vex); /* x86_oracle_ext.inc */
static int x42_form_o(u32 map, u32 c, int pp, int vex);
static int exec_gext(orc_machine *m, insn *d);
static int exec_x42(orc_machine *m, insn *d);
static int ax_form_o(u32 map, u32 c, int pp, int vex); /* x86_oracle_avx2x.inc */
static int exec_ax(orc_machine *m, insn *d);

static int exec_sse(orc_machine *m, insn *d) {
  const u32 op = d->op, r3 = d->reg & 7;
  const int pc = d->rep == 0xf3 ? 2 : d->rep == 0xf2 ? 3 : d->pfx66 ? 1 : 0; /* none, 66, f3, f2 */
  const int mem = d->is_mem;
  const u8 imm = d->bytes[d->len - 1];
  x128 a, b, r;
  u64 v;
  if (d->opmap == 1 && ((pc == 0 && mmx_opcode(op)) || (op == 0xd6 && pc >= 2))) return exec_mmx(m, d, pc);
  if (pc == 0 && ssse3_mm(d->opmap, op)) return exec_mmx(m, d, pc); /* U41: SSSE3 on mm registers */
  if (fp_form_o(d->opmap, op, pc, 0)) return exec_fp(m, d); /* U39 / U40 */
  if (s4_form_o(d->opmap, op, pc, 0)) return exec_s4(m, d); /* U41 */
  if (gx_form_o(d->opmap, op, pc, 0)) return exec_gext(m, d); /* U45 */
  if (x42_form_o(d->opmap, op, pc, 0)) return exec_x42(m, d);
  if (d->opmap == 2) { /* 66 0f 38 00 pshufb, 66 0f 38 17 ptest */
    if (pc != 1) return X_UNIMPL;
    if (m->r.cr0 & 4 || !(m->r.cr4 & 0x200)) {
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    }
    if (m->r.cr0 & 8) {
      fault(m, 7, 0);
      return X_FAULT;
    }
    a = xreg(m, d->reg);
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    if (op == 0x17) ptest(m, a.b, b.b, 16);
    else xput(m, d->reg, pshufb(&a, &b));
    return X_OK;
  }
  if (op == 0xc3) { /* movnti m32/64, r (SSE2 general-register store) */
    if (pc != 0) return X_UNIMPL;
    if (!mem) {
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    }
    const int sz = d->rexw ? 8 : 4;
    v = m->r.gpr[d->reg] & szmask(sz);
    return vwrite(m, d->ea, (u32)sz, &v) ? X_FAULT : X_OK;
  }
  if (op == 0xae) {
    if (pc != 0) return X_UNIMPL;
    if (!mem) return r3 >= 5 ? X_OK : X_UNIMPL; /* lfence / mfence / sfence */
    if (r3 != 2 && r3 != 3) return X_UNIMPL;
  }
  /* encodings outside the subset */
  {
    int ok;
    if (op >= 0x60 && op <= 0x6d) ok = pc == 1;
    else if (op == 0x6e || op == 0x74 || op == 0x75 || op == 0x76 || op == 0xc4 || op == 0xc5 || op == 0xd6)
      ok = pc == 1;
    else if (op == 0x6f || op == 0x7f) ok = pc == 1 || pc == 2;
    else if (op == 0x70) ok = pc != 0;
    else if (op >= 0x71 && op <= 0x73) ok = pc == 1;
    else if (op == 0x7e) ok = pc == 1 || pc == 2;
    else if (op == 0x10 || op == 0x11) ok = 1;
    else if ((op >= 0x12 && op <= 0x17) || op == 0x28 || op == 0x29 || op == 0x2b || op == 0x50 || op == 0xc6 ||
             (op >= 0x54 && op <= 0x57))
      ok = pc <= 1;
    else if (op == 0xae) ok = 1;
    else if (op >= 0xd0) {
      ok = pc == 1 && op != 0xd0 && op != 0xd6 && op != 0xe6 && op != 0xe7 && op != 0xf0 && op != 0xf7 &&
           op != 0xff;
      if (op == 0xd6 || op == 0xe7) ok = pc == 1;
    } else ok = 0;
    if (!ok) return X_UNIMPL;
  }
  /* register-only and memory-only forms */
  {
    const int reg_only = (op >= 0x71 && op <= 0x73) || op == 0x50 || op == 0xd7 || op == 0xc5;
    const int mem_only = op == 0x13 || op == 0x17 || op == 0x2b || op == 0xe7 || op == 0xae ||
                         ((op == 0x12 || op == 0x16) && pc == 1);
    if ((reg_only && mem) || (mem_only && !mem)) {
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    }
    if (op >= 0x71 && op <= 0x73 && !((r3 == 2 || r3 == 4 || r3 == 6) && op != 0x73) &&
        !(op == 0x73 && (r3 == 2 || r3 == 3 || r3 == 6 || r3 == 7)))
      return X_UNIMPL;
  }
  if (m->r.cr0 & 4 || !(m->r.cr4 & 0x200)) {
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (m->r.cr0 & 8) {
    fault(m, 7, 0); /* #NM */
    return X_FAULT;
  }
  a = xreg(m, d->reg);
  switch (op) {
  case 0x10: /* movups / movupd / movss / movsd load */
    if (pc <= 1) {
      if (xsrc(m, d, 16, 0, &b)) return X_FAULT;
      xput(m, d->reg, b);
    } else {
      const int n = pc == 2 ? 4 : 8;
      if (xsrc(m, d, n, 0, &b)) return X_FAULT;
      if (mem) xput(m, d->reg, b); /* zero-extended */
      else {
        memcpy(a.b, b.b, (size_t)n);
        xput(m, d->reg, a);
      }
    }
    return X_OK;
  case 0x11: /* stores of 0x10 */
    if (pc <= 1) {
      if (mem) return xstore(m, d, 16, 0, &a) ? X_FAULT : X_OK;
      xput(m, d->rm, a);
    } else {
      const int n = pc == 2 ? 4 : 8;
      if (mem) return xstore(m, d, n, 0, &a) ? X_FAULT : X_OK;
      r = xreg(m, d->rm);
      memcpy(r.b, a.b, (size_t)n);
      xput(m, d->rm, r);
    }
    return X_OK;
  case 0x12: /* movlps / movlpd m64; movhlps */
  case 0x16: /* movhps / movhpd m64; movlhps */
    if (xsrc(m, d, 8, 0, &b)) return X_FAULT;
    if (op == 0x12) memcpy(a.b, b.b + (mem ? 0 : 8), 8);
    else memcpy(a.b + 8, b.b, 8);
    xput(m, d->reg, a);
    return X_OK;
  case 0x13:
  case 0x17:
    if (op == 0x17) memcpy(a.b, a.b + 8, 8);
    return xstore(m, d, 8, 0, &a) ? X_FAULT : X_OK;
  case 0x14:
  case 0x15:
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    xput(m, d->reg, unpack(pc ? 8 : 4, op == 0x15, &a, &b));
    return X_OK;
  case 0x28:
  case 0x6f:
    if (xsrc(m, d, 16, op == 0x28 || pc == 1, &b)) return X_FAULT;
    xput(m, d->reg, b);
    return X_OK;
  case 0x29:
  case 0x2b:
  case 0x7f:
  case 0xe7:
    if (mem) return xstore(m, d, 16, op != 0x7f || pc == 1, &a) ? X_FAULT : X_OK;
    xput(m, d->rm, a);
    return X_OK;
  case 0x50: { /* movmskps / movmskpd */
    b = xreg(m, d->rm);
    const int w = pc ? 8 : 4;
    v = 0;
    for (int i = 0; i < 16 / w; i++) v |= (el(&b, i, w) >> (8 * w - 1)) << i;
    m->r.gpr[d->reg] = v;
    return X_OK;
  }
  case 0xd7: /* pmovmskb */
    b = xreg(m, d->rm);
    v = 0;
    for (int i = 0; i < 16; i++) v |= (u64)(b.b[i] >> 7) << i;
    m->r.gpr[d->reg] = v;
    return X_OK;
  case 0x54: case 0x55: case 0x56: case 0x57: case 0xdb: case 0xdf: case 0xeb: case 0xef:
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    for (int i = 0; i < 16; i++) {
      const u8 x = a.b[i], y = b.b[i];
      r.b[i] = (op == 0x54 || op == 0xdb) ? (u8)(x & y) : (op == 0x55 || op == 0xdf) ? (u8)(~x & y)
             : (op == 0x56 || op == 0xeb) ? (u8)(x | y) : (u8)(x ^ y);
    }
    xput(m, d->reg, r);
    return X_OK;
  case 0x60: case 0x61: case 0x62: case 0x6c:
  case 0x68: case 0x69: case 0x6a: case 0x6d: {
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    const u32 lo = op & 0xf7;
    const int w = lo == 0x60 ? 1 : lo == 0x61 ? 2 : lo == 0x62 ? 4 : 8;
    xput(m, d->reg, unpack(w, op == 0x68 || op == 0x69 || op == 0x6a || op == 0x6d, &a, &b));
    return X_OK;
  }
  case 0x63: case 0x67: case 0x6b: { /* packsswb, packuswb, packssdw */
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    const int w = op == 0x6b ? 4 : 2, n = 16 / w;
    for (int i = 0; i < 2 * n; i++) {
      const i64 x = i < n ? sel(&a, i, w) : sel(&b, i - n, w);
      elput(&r, i, w / 2, op == 0x67 ? satu(x, 1) : sats(x, w / 2));
    }
    xput(m, d->reg, r);
    return X_OK;
  }
  case 0x64: case 0x65: case 0x66: case 0x74: case 0x75: case 0x76:
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    xput(m, d->reg, ewise(op >= 0x74 ? EW_EQ : EW_GT, 1 << ((op & 0xf) % 4), &a, &b));
    return X_OK;
  case 0x6e: /* movd / movq xmm, r/m */
  case 0x7e: {
    const int n = d->rexw ? 8 : 4;
    if (op == 0x7e && pc == 2) { /* movq xmm, xmm/m64 */
      if (xsrc(m, d, 8, 0, &b)) return X_FAULT;
      memset(b.b + 8, 0, 8);
      xput(m, d->reg, b);
      return X_OK;
    }
    if (op == 0x6e) {
      memset(r.b, 0, 16);
      if (mem) {
        if (vread(m, d->ea, (u32)n, r.b)) return X_FAULT;
      } else {
        v = m->r.gpr[d->rm] & szmask(n);
        memcpy(r.b, &v, 8);
      }
      xput(m, d->reg, r);
      return X_OK;
    }
    v = el(&a, 0, n);
    if (mem) return vwrite(m, d->ea, (u32)n, &v) ? X_FAULT : X_OK;
    m->r.gpr[d->rm] = v;
    return X_OK;
  }
  case 0x70: { /* pshufd / pshufhw / pshuflw */
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    r = b;
    if (pc == 1)
      for (int i = 0; i < 4; i++) elput(&r, i, 4, el(&b, (imm >> (2 * i)) & 3, 4));
    else
      for (int i = 0; i < 4; i++) elput(&r, i + (pc == 2 ? 4 : 0), 2, el(&b, ((imm >> (2 * i)) & 3) + (pc == 2 ? 4 : 0), 2));
    xput(m, d->reg, r);
    return X_OK;
  }
  case 0x71: case 0x72: case 0x73: {
    b = xreg(m, d->rm);
    const int w = op == 0x71 ? 2 : op == 0x72 ? 4 : 8;
    if (op == 0x73 && (r3 == 3 || r3 == 7)) { /* psrldq / pslldq: bytes */
      memset(r.b, 0, 16);
      for (int i = 0; i < 16; i++) {
        const int src = r3 == 3 ? i + imm : i - imm;
        if (src >= 0 && src < 16) r.b[i] = b.b[src];
      }
    } else {
      r = shift_el(r3 == 2 ? 0 : r3 == 4 ? 1 : 2, w, &b, imm);
    }
    xput(m, d->rm, r);
    return X_OK;
  }
  case 0xc4: /* pinsrw */
    if (mem) {
      v = 0;
      if (vread(m, d->ea, 2, &v)) return X_FAULT;
    } else {
      v = m->r.gpr[d->rm];
    }
    elput(&a, imm & 7, 2, v & 0xffff);
    xput(m, d->reg, a);
    return X_OK;
  case 0xc5: /* pextrw */
    b = xreg(m, d->rm);
    m->r.gpr[d->reg] = el(&b, imm & 7, 2);
    return X_OK;
  case 0xc6: /* shufps / shufpd */
    if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
    if (pc == 0) {
      elput(&r, 0, 4, el(&a, imm & 3, 4));
      elput(&r, 1, 4, el(&a, (imm >> 2) & 3, 4));
      elput(&r, 2, 4, el(&b, (imm >> 4) & 3, 4));
      elput(&r, 3, 4, el(&b, (imm >> 6) & 3, 4));
    } else {
      elput(&r, 0, 8, el(&a, imm & 1, 8));
      elput(&r, 1, 8, el(&b, (imm >> 1) & 1, 8));
    }
    xput(m, d->reg, r);
    return X_OK;
  case 0xd6: /* movq xmm/m64, xmm */
    if (mem) return xstore(m, d, 8, 0, &a) ? X_FAULT : X_OK;
    memset(a.b + 8, 0, 8);
    xput(m, d->rm, a);
    return X_OK;
  case 0xae: { /* ldmxcsr / stmxcsr */
    u32 mx = 0;
    if (r3 == 3) return vwrite(m, d->ea, 4, &m->r.mxcsr) ? X_FAULT : X_OK;
    if (vread(m, d->ea, 4, &mx)) return X_FAULT;
    if (mx & ~(m->r.mxcsr_mask ? m->r.mxcsr_mask : 0xffbfu)) {
      fault(m, WTFGPU_VEC_GP, 0);
      return X_FAULT;
    }
    m->r.mxcsr = mx;
    return X_OK;
  }
  default:
    break;
  }
  /* 66 0f d1-fe: integer arithmetic on xmm, xmm/m128 */
  if (xsrc(m, d, 16, 1, &b)) return X_FAULT;
  switch (op) {
  case 0xd1: case 0xd2: case 0xd3: r = shift_el(0, op == 0xd1 ? 2 : op == 0xd2 ? 4 : 8, &a, el(&b, 0, 8)); break;
  case 0xe1: case 0xe2: r = shift_el(1, op == 0xe1 ? 2 : 4, &a, el(&b, 0, 8)); break;
  case 0xf1: case 0xf2: case 0xf3: r = shift_el(2, op == 0xf1 ? 2 : op == 0xf2 ? 4 : 8, &a, el(&b, 0, 8)); break;
  case 0xd4: r = ewise(EW_ADD, 8, &a, &b); break;
  case 0xfb: r = ewise(EW_SUB, 8, &a, &b); break;
  case 0xfc: case 0xfd: case 0xfe: r = ewise(EW_ADD, 1 << (op - 0xfc), &a, &b); break;
  case 0xf8: case 0xf9: case 0xfa: r = ewise(EW_SUB, 1 << (op - 0xf8), &a, &b); break;
  case 0xd5: r = ewise(EW_MULLO, 2, &a, &b); break;
  case 0xe5: r = ewise(EW_MULHS, 2, &a, &b); break;
  case 0xe4: r = ewise(EW_MULHU, 2, &a, &b); break;
  case 0xd8: case 0xd9: r = ewise(EW_SUBUS, op - 0xd7, &a, &b); break;
  case 0xdc: case 0xdd: r = ewise(EW_ADDUS, op - 0xdb, &a, &b); break;
  case 0xe8: case 0xe9: r = ewise(EW_SUBS, op - 0xe7, &a, &b); break;
  case 0xec: case 0xed: r = ewise(EW_ADDS, op - 0xeb, &a, &b); break;
  case 0xda: r = ewise(EW_MINU, 1, &a, &b); break;
  case 0xde: r = ewise(EW_MAXU, 1, &a, &b); break;
  case 0xea: r = ewise(EW_MINS, 2, &a, &b); break;
  case 0xee: r = ewise(EW_MAXS, 2, &a, &b); break;
  case 0xe0: r = ewise(EW_AVG, 1, &a, &b); break;
  case 0xe3: r = ewise(EW_AVG, 2, &a, &b); break;
  case 0xf4: /* pmuludq */
    elput(&r, 0, 8, el(&a, 0, 4) * el(&b, 0, 4));
    elput(&r, 1, 8, el(&a, 2, 4) * el(&b, 2, 4));
    break;
  case 0xf5: /* pmaddwd */
    for (int i = 0; i < 4; i++)
      elput(&r, i, 4, (u64)(sel(&a, 2 * i, 2) * sel(&b, 2 * i, 2) + sel(&a, 2 * i + 1, 2) * sel(&b, 2 * i + 1, 2)) & 0xffffffffULL);
    break;
  case 0xf6: /* psadbw */
    for (int h = 0; h < 2; h++) {
      u64 s = 0;
      for (int i = 8 * h; i < 8 * h + 8; i++) s += a.b[i] > b.b[i] ? a.b[i] - b.b[i] : b.b[i] - a.b[i];
      elput(&r, h, 8, s);
    }
    break;
  default:
    return X_UNIMPL;
  }
  xput(m, d->reg, r);
  return X_OK;
}


/* ---------------- AVX / AVX2 (U23) ----------------
 * VEX-encoded forms of the same subset at 128 and 256 bits (three operands:
 * dst = reg, first source = vvvv, second = r/m; lane-wise per 128 bits),
 * vzeroupper / vzeroall, vpshufb, vptest, vpbroadcastb/w/d/q. VEX.128 zeroes
 * bits 255:128 of the destination. #UD for a legacy 66/f2/f3/REX before VEX,
 * CR4.OSXSAVE = 0, XCR0[2:1] != 11, vvvv != 1111 in two-operand forms, L = 1
 * where only 128 bits exist, and register-only / memory-only violations; #NM
 * if CR0.TS; #GP(0) when an aligned move (vmovaps/apd/dqa/ntdq/ntps/ntpd) is
 * not aligned to its size. */
typedef struct { x128 l, h; } y256;

static y256 yreg(orc_machine *m, u32 r) {
  y256 v;
  memcpy(v.l.b, m->r.xmm[r & 15], 16);
  memcpy(v.h.b, m->r.ymmh[r & 15], 16);
  return v;
}
/* a VEX destination: bits 255:128 zeroed by VEX.128, bits 511:256 by every
 * VEX write (MAXVL 512, U47) */
static void yput(orc_machine *m, u32 r, y256 v, int l256) {
  memcpy(m->r.xmm[r & 15], v.l.b, 16);
  if (l256) memcpy(m->r.ymmh[r & 15], v.h.b, 16);
  else memset(m->r.ymmh[r & 15], 0, 16);
  memset(m->r.zmmh[r & 15], 0, 32);
}

#include "x86_oracle_fp.inc" /* SSE / AVX floating point (U39 / U40) */
#include "x86_oracle_sse4.inc" /* SSSE3 / SSE4.1 integer, AVX2 lane crossing (U41) */
#include "x86_oracle_ext.inc"  /* BMI1 / BMI2 / ADX / MOVBE / CRC32, SSE4.2, AES, PCLMULQDQ (U45) */
#include "x86_oracle_avx2x.inc" /* FMA3, F16C, AVX2 gathers (U46) */
#include "x86_oracle_avx512.inc" /* the AVX-512 subset and the opmask instructions (U47) */

/* two-source ops of one 128-bit lane (the legacy semantics); 0 = not one */
static int vlane(u32 op, int pc, const x128 *a, const x128 *b, u8 imm, u64 cnt, x128 *r) {
  const u32 lo = op & 0xf7;
  memset(r->b, 0, 16);
  switch (op) {
  case 0x14: case 0x15: *r = unpack(pc ? 8 : 4, op == 0x15, a, b); return 1;
  case 0x54: case 0x55: case 0x56: case 0x57: case 0xdb: case 0xdf: case 0xeb: case 0xef:
    for (int i = 0; i < 16; i++) {
      const u8 x = a->b[i], y = b->b[i];
      r->b[i] = (op == 0x54 || op == 0xdb) ? (u8)(x & y) : (op == 0x55 || op == 0xdf) ? (u8)(~x & y)
              : (op == 0x56 || op == 0xeb) ? (u8)(x | y) : (u8)(x ^ y);
    }
    return 1;
  case 0x60: case 0x61: case 0x62: case 0x6c: case 0x68: case 0x69: case 0x6a: case 0x6d:
    *r = unpack(lo == 0x60 ? 1 : lo == 0x61 ? 2 : lo == 0x62 ? 4 : 8, op == 0x68 || op == 0x69 || op == 0x6a || op == 0x6d, a, b);
    return 1;
  case 0x63: case 0x67: case 0x6b: {
    const int w = op == 0x6b ? 4 : 2, n = 16 / w;
    for (int i = 0; i < 2 * n; i++) {
      const i64 x = i < n ? sel(a, i, w) : sel(b, i - n, w);
      elput(r, i, w / 2, op == 0x67 ? satu(x, 1) : sats(x, w / 2));
    }
    return 1;
  }
  case 0x64: case 0x65: case 0x66: case 0x74: case 0x75: case 0x76:
    *r = ewise(op >= 0x74 ? EW_EQ : EW_GT, 1 << ((op & 0xf) % 4), a, b);
    return 1;
  case 0x70:
    *r = *b;
    if (pc == 1)
      for (int i = 0; i < 4; i++) elput(r, i, 4, el(b, (imm >> (2 * i)) & 3, 4));
    else
      for (int i = 0; i < 4; i++) elput(r, i + (pc == 2 ? 4 : 0), 2, el(b, ((imm >> (2 * i)) & 3) + (pc == 2 ? 4 : 0), 2));
    return 1;
  case 0xc6:
    if (pc == 0) {
      elput(r, 0, 4, el(a, imm & 3, 4));
      elput(r, 1, 4, el(a, (imm >> 2) & 3, 4));
      elput(r, 2, 4, el(b, (imm >> 4) & 3, 4));
      elput(r, 3, 4, el(b, (imm >> 6) & 3, 4));
    } else {
      elput(r, 0, 8, el(a, imm & 1, 8));
      elput(r, 1, 8, el(b, (imm >> 1) & 1, 8));
    }
    return 1;
  case 0xd1: case 0xd2: case 0xd3: *r = shift_el(0, op == 0xd1 ? 2 : op == 0xd2 ? 4 : 8, a, cnt); return 1;
  case 0xe1: case 0xe2: *r = shift_el(1, op == 0xe1 ? 2 : 4, a, cnt); return 1;
  case 0xf1: case 0xf2: case 0xf3: *r = shift_el(2, op == 0xf1 ? 2 : op == 0xf2 ? 4 : 8, a, cnt); return 1;
  case 0xd4: *r = ewise(EW_ADD, 8, a, b); return 1;
  case 0xfb: *r = ewise(EW_SUB, 8, a, b); return 1;
  case 0xfc: case 0xfd: case 0xfe: *r = ewise(EW_ADD, 1 << (op - 0xfc), a, b); return 1;
  case 0xf8: case 0xf9: case 0xfa: *r = ewise(EW_SUB, 1 << (op - 0xf8), a, b); return 1;
  case 0xd5: *r = ewise(EW_MULLO, 2, a, b); return 1;
  case 0xe5: *r = ewise(EW_MULHS, 2, a, b); return 1;
  case 0xe4: *r = ewise(EW_MULHU, 2, a, b); return 1;
  case 0xd8: case 0xd9: *r = ewise(EW_SUBUS, op - 0xd7, a, b); return 1;
  case 0xdc: case 0xdd: *r = ewise(EW_ADDUS, op - 0xdb, a, b); return 1;
  case 0xe8: case 0xe9: *r = ewise(EW_SUBS, op - 0xe7, a, b); return 1;
  case 0xec: case 0xed: *r = ewise(EW_ADDS, op - 0xeb, a, b); return 1;
  case 0xda: *r = ewise(EW_MINU, 1, a, b); return 1;
  case 0xde: *r = ewise(EW_MAXU, 1, a, b); return 1;
  case 0xea: *r = ewise(EW_MINS, 2, a, b); return 1;
  case 0xee: *r = ewise(EW_MAXS, 2, a, b); return 1;
  case 0xe0: *r = ewise(EW_AVG, 1, a, b); return 1;
  case 0xe3: *r = ewise(EW_AVG, 2, a, b); return 1;
  case 0xf4:
    elput(r, 0, 8, el(a, 0, 4) * el(b, 0, 4));
    elput(r, 1, 8, el(a, 2, 4) * el(b, 2, 4));
    return 1;
  case 0xf5:
    for (int i = 0; i < 4; i++)
      elput(r, i, 4, (u64)(sel(a, 2 * i, 2) * sel(b, 2 * i, 2) + sel(a, 2 * i + 1, 2) * sel(b, 2 * i + 1, 2)) & 0xffffffffULL);
    return 1;
  case 0xf6:
    for (int h = 0; h < 2; h++) {
      u64 sum = 0;
      for (int i = 8 * h; i < 8 * h + 8; i++) sum += a->b[i] > b->b[i] ? a->b[i] - b->b[i] : b->b[i] - a->b[i];
      elput(r, h, 8, sum);
    }
    return 1;
  default: return 0;
  }
}

static x128 vshift_imm(u32 op, u32 r3, const x128 *b, u8 imm) {
  x128 r;
  if (op == 0x73 && (r3 == 3 || r3 == 7)) {
    memset(r.b, 0, 16);
    for (int i = 0; i < 16; i++) {
      const int src = r3 == 3 ? i + imm : i - imm;
      if (src >= 0 && src < 16) r.b[i] = b->b[src];
    }
    return r;
  }
  return shift_el(r3 == 2 ? 0 : r3 == 4 ? 1 : 2, op == 0x71 ? 2 : op == 0x72 ? 4 : 8, b, imm);
}

static int vex_valid(u32 map, u32 op, int pp, int mem, u32 r3) {
  if (map == 2) return pp == 1 && (op == 0x00 || op == 0x17 || op == 0x58 || op == 0x59 || op == 0x78 || op == 0x79);
  if (map != 1) return 0;
  if (op == 0x77) return pp == 0;
  if (op >= 0x10 && op <= 0x17) return op <= 0x11 || pp <= 1;
  if (op == 0x28 || op == 0x29 || op == 0x2b || op == 0x50 || op == 0xc6 || (op >= 0x54 && op <= 0x57)) return pp <= 1;
  if ((op >= 0x60 && op <= 0x6e) && op != 0x6f) return pp == 1;
  if (op == 0x6f || op == 0x7f || op == 0x7e) return pp == 1 || pp == 2;
  if (op == 0x70) return pp != 0;
  if (op >= 0x71 && op <= 0x73) {
    if (pp != 1) return 0;
    if (mem) return 1;
    return op == 0x73 ? (r3 == 2 || r3 == 3 || r3 == 6 || r3 == 7) : (r3 == 2 || r3 == 4 || r3 == 6);
  }
  if (op == 0x74 || op == 0x75 || op == 0x76 || op == 0xc4 || op == 0xc5) return pp == 1;
  if (op >= 0xd0) return pp == 1 && op != 0xd0 && op != 0xe6 && op != 0xf0 && op != 0xf7 && op != 0xff;
  return 0;
}

/* U36 / U45: which encodings some x86-64 CPU defines (SDM vol. 2 appendix A
 * and the extension references). The emulated CPU enumerates and executes
 * SSE .. SSE4.2, SSSE3, AVX, AVX2, AES, PCLMULQDQ, BMI1 / BMI2, ADX and MOVBE;
 * the other defined forms (AVX-VNNI / -IFMA / -NE-CONVERT /
 * -VNNI-INT8 / -INT16, GFNI, the 256-bit VAES / VPCLMULQDQ, SHA, CET shadow
 * stack writes, MOVDIRI / MOVDIR64B, ENQCMD, Key Locker, INVEPT / INVVPID /
 * INVPCID, EVEX) are UNIMPLEMENTED: a guest chooses its code from the capture
 * host's CPUID, so such a form is an engine gap, never a crash. An opcode no
 * CPU assigns, or a VEX map other than 0f / 0f 38 / 0f 3a, is #UD, decided
 * from the opcode byte (no ModRM / immediate fetched). pp / pfx: 0 none, 1 66,
 * 2 f3, 3 f2. */
static int vex_defined(u32 map, u32 op, int pp) {
  if (map == 1) {
    switch (op) {
    case 0x10: case 0x11: case 0x12: case 0x51: case 0x58: case 0x59: case 0x5a: case 0x5c: case 0x5d:
    case 0x5e: case 0x5f: case 0xc2: case 0xae:
      return 1;
    case 0x13: case 0x14: case 0x15: case 0x17: case 0x28: case 0x29: case 0x2b: case 0x2e: case 0x2f:
    case 0x50: case 0x54: case 0x55: case 0x56: case 0x57: case 0xc6:
      return pp <= 1;
    case 0x16: case 0x5b: return pp <= 2;
    case 0x2a: case 0x2c: case 0x2d: return pp >= 2;
    case 0x52: case 0x53: return pp == 0 || pp == 2;
    case 0x6f: case 0x7e: case 0x7f: return pp == 1 || pp == 2;
    case 0x70: case 0xe6: return pp >= 1;
    case 0x77: return pp == 0;
    case 0x7c: case 0x7d: case 0xd0: return pp == 1 || pp == 3;
    case 0xf0: return pp == 3;
    case 0x41: case 0x42: case 0x44: case 0x45: case 0x46: case 0x47: case 0x4a: case 0x4b: case 0x90: case 0x91:
    case 0x98: case 0x99: /* the opmask instructions */
      return pp <= 1;
    case 0x92: case 0x93: return pp != 2;
    default:
      return pp == 1 && ((op >= 0x60 && op <= 0x6e) || (op >= 0x71 && op <= 0x76) || op == 0xc4 || op == 0xc5 ||
                         (op >= 0xd1 && op <= 0xfe));
    }
  }
  if (map == 2) {
    switch (op) { /* every prefix: BMI2 / BEXTR (f5 f7), AVX-VNNI-INT8 (50 51), NE-CONVERT (b0), VNNI-INT16 (d2 d3) */
    case 0xf5: case 0xf7: case 0x50: case 0x51: case 0xb0: case 0xd2: case 0xd3: return 1;
    case 0xf2: case 0xf3: return pp == 0;             /* andn, group 17 */
    case 0x72: return pp == 2;                        /* vcvtneps2bf16 */
    case 0xb1: return pp == 1 || pp == 2;             /* vbcstnesh2ps / vbcstnebf162ps */
    case 0xf6: return pp == 3;                        /* mulx */
    default: break;
    }
    if (pp != 1) return 0;
    return op <= 0x0f || op == 0x13 || (op >= 0x16 && op <= 0x1a) || (op >= 0x1c && op <= 0x1e) ||
           (op >= 0x20 && op <= 0x25) || (op >= 0x28 && op <= 0x41) || (op >= 0x45 && op <= 0x47) || op == 0x52 ||
           op == 0x53 || (op >= 0x58 && op <= 0x5a) || op == 0x78 || op == 0x79 || op == 0x8c || op == 0x8e ||
           (op >= 0x90 && op <= 0x93) || (op >= 0x96 && op <= 0x9f) || (op >= 0xa6 && op <= 0xaf) ||
           (op >= 0xb4 && op <= 0xbf) || op == 0xcf || (op >= 0xdb && op <= 0xdf);
  }
  if (map == 3) {
    if (pp == 3) return op == 0xf0; /* rorx */
    if (pp != 1) return 0;
    return op == 0x00 || op == 0x01 || op == 0x02 || op == 0x04 || op == 0x05 || op == 0x06 ||
           (op >= 0x08 && op <= 0x0f) || (op >= 0x14 && op <= 0x19) || op == 0x1d || (op >= 0x20 && op <= 0x22) ||
           (op >= 0x30 && op <= 0x33) || op == 0x38 || op == 0x39 || (op >= 0x40 && op <= 0x42) || op == 0x44 ||
           op == 0x46 || (op >= 0x4a && op <= 0x4c) || (op >= 0x60 && op <= 0x63) || op == 0xce || op == 0xcf || op == 0xdf;
  }
  return 0;
}

/* the legacy (non-VEX) 0f 38 / 0f 3a maps, same rule */
static int legacy_3byte_defined(u32 map, u32 op, int pfx) {
  if (map == 2) {
    switch (pfx) {
    case 0: /* sha1 / sha256 (c8-cd), movbe, wrss, movdiri */
      if ((op >= 0xc8 && op <= 0xcd) || op == 0xf0 || op == 0xf1 || op == 0xf6 || op == 0xf9) return 1;
      break;
    case 1: /* pcmpgtq, invept / invvpid / invpcid, gf2p8mulb, aes, movbe r16, wruss, adcx, movdir64b */
      if (op == 0x37 || (op >= 0x80 && op <= 0x82) || op == 0xcf || (op >= 0xdb && op <= 0xdf) || op == 0xf0 ||
          op == 0xf1 || op == 0xf5 || op == 0xf6 || op == 0xf8)
        return 1;
      break;
    case 2: /* Key Locker (d8 dc-df), adox, enqcmds */
      return op == 0xd8 || (op >= 0xdc && op <= 0xdf) || op == 0xf6 || op == 0xf8;
    default: /* crc32, enqcmd */
      return op == 0xf0 || op == 0xf1 || op == 0xf8;
    }
    return ((op <= 0x0b || (op >= 0x1c && op <= 0x1e)) && pfx <= 1) ||
           (pfx == 1 && (op == 0x10 || op == 0x14 || op == 0x15 || op == 0x17 || (op >= 0x20 && op <= 0x25) ||
                         (op >= 0x28 && op <= 0x2b) || (op >= 0x30 && op <= 0x35) || (op >= 0x38 && op <= 0x41)));
  }
  if (op == 0xcc) return pfx == 0; /* sha1rnds4 */
  return (op == 0x0f && pfx <= 1) ||
         (pfx == 1 && ((op >= 0x08 && op <= 0x0e) || (op >= 0x14 && op <= 0x17) || (op >= 0x20 && op <= 0x22) ||
                       (op >= 0x40 && op <= 0x42) || op == 0x44 || (op >= 0x60 && op <= 0x63) || op == 0xce ||
                       op == 0xcf || op == 0xdf));
}

static int exec_vex(orc_machine *m, insn *d) {
  const u32 op = d->op, r3 = d->reg & 7, map = d->opmap, vv = d->vvvv;
  const int pp = (int)d->vpp, l256 = (int)d->vl, mem = d->is_mem;
  const u8 imm = d->bytes[d->len - 1];
  if (d->evex) return exec_evex(m, d);                 /* U47 */
  if (kop_any(map, op, pp)) return exec_kop(m, d);
  if (fp_form_o(map, op, pp, 1)) return exec_fp(m, d); /* U39 / U40 */
  if (s4_form_o(map, op, pp, 1)) return exec_s4(m, d); /* U41 */
  if (gx_form_o(map, op, pp, 1)) return exec_gext(m, d); /* U45 */
  if (x42_form_o(map, op, pp, 1)) return exec_x42(m, d);
  if (ax_form_o(map, op, pp, 1)) return exec_ax(m, d); /* U46 */
  if (map == 1 && op == 0xae && !(pp == 0 && mem && (r3 == 2 || r3 == 3))) { /* U36: vldmxcsr / vstmxcsr only */
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (!vex_valid(map, op, pp, mem, r3)) return X_UNIMPL;
  int ud = d->vbad || !((m->r.cr4 >> 18) & 1) || (m->r.xcr0 & 6) != 6;
  int two = 0, no256 = 0, reg_only = 0, mem_only = 0;
  if (map == 1) {
    two = ((op == 0x10 || op == 0x11) && (pp <= 1 || mem)) || op == 0x13 || op == 0x17 || op == 0x28 || op == 0x29 ||
          op == 0x2b || op == 0x50 || op == 0x6e || op == 0x6f || op == 0x70 || op == 0x7e || op == 0x7f || op == 0xc5 ||
          op == 0xd6 || op == 0xd7 || op == 0xe7 || op == 0x77;
    no256 = op == 0x12 || op == 0x13 || op == 0x16 || op == 0x17 || op == 0x6e || op == 0x7e || op == 0xc4 ||
            op == 0xc5 || op == 0xd6;
    reg_only = (op >= 0x71 && op <= 0x73) || op == 0x50 || op == 0xd7 || op == 0xc5;
    mem_only = op == 0x13 || op == 0x17 || op == 0x2b || op == 0xe7 || ((op == 0x12 || op == 0x16) && pp == 1);
  } else {
    two = op != 0x00;
  }
  if ((two && vv != 0) || (no256 && l256) || (reg_only && mem) || (mem_only && !mem)) ud = 1;
  if (ud) {
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  if (m->r.cr0 & 8) {
    fault(m, 7, 0);
    return X_FAULT;
  }
  if (map == 1 && op == 0x77) { /* vzeroupper / vzeroall */
    for (int i = 0; i < 16; i++) { /* zmm0..15 bits 511:128; zmm16..31 kept */
      memset(m->r.ymmh[i], 0, 16);
      memset(m->r.zmmh[i], 0, 32);
      if (l256) memset(m->r.xmm[i], 0, 16);
    }
    return X_OK;
  }
  const int vl = l256 ? 32 : 16;
  int n = vl, align = 0;
  if (map == 1) {
    switch (op) {
    case 0x10: case 0x11: n = pp <= 1 ? vl : pp == 2 ? 4 : 8; break;
    case 0x12: case 0x13: case 0x16: case 0x17: case 0xd6: n = 8; break;
    case 0x6e: case 0x7e: n = (pp == 2 || d->rexw) ? 8 : 4; break;
    case 0xc4: n = 2; break;
    case 0x28: case 0x29: case 0x2b: case 0xe7: align = 1; break;
    case 0x6f: case 0x7f: align = pp == 1; break;
    case 0xd1: case 0xd2: case 0xd3: case 0xe1: case 0xe2: case 0xf1: case 0xf2: case 0xf3: n = 16; break;
    default: break;
    }
  } else if (op == 0x58 || op == 0x59 || op == 0x78 || op == 0x79) {
    n = op == 0x78 ? 1 : op == 0x79 ? 2 : op == 0x58 ? 4 : 8;
  }
  if (mem && align && (d->ea & (u64)(vl - 1))) {
    fault(m, WTFGPU_VEC_GP, 0);
    return X_FAULT;
  }
  const int store = map == 1 && (op == 0x11 || op == 0x13 || op == 0x17 || op == 0x29 || op == 0x2b || op == 0x7f ||
                                 op == 0xe7 || op == 0xd6 || (op == 0x7e && pp == 1));
  const y256 s = yreg(m, d->reg), a = yreg(m, vv);
  y256 b, r;
  memset(&b, 0, sizeof(b));
  memset(&r, 0, sizeof(r));
  if (!store) {
    if (mem) {
      if (vread_n(m, d->ea, (u32)n, b.l.b)) return X_FAULT;
    } else if (map == 1 && (op == 0x6e || op == 0xc4)) {
      const u64 g = m->r.gpr[d->rm];
      memcpy(b.l.b, &g, 8);
    } else {
      b = yreg(m, d->rm);
    }
  }
  u32 dst = d->reg;
  if (map == 2) {
    if (op == 0x17) { /* vptest */
      u8 sa[32], sb[32];
      memcpy(sa, s.l.b, 16);
      memcpy(sa + 16, s.h.b, 16);
      memcpy(sb, b.l.b, 16);
      memcpy(sb + 16, b.h.b, 16);
      ptest(m, sa, sb, vl);
      return X_OK;
    }
    if (op == 0x00) { /* vpshufb */
      r.l = pshufb(&a.l, &b.l);
      r.h = pshufb(&a.h, &b.h);
    } else { /* vpbroadcastb / w / d / q */
      const int ew = op == 0x78 ? 1 : op == 0x79 ? 2 : op == 0x58 ? 4 : 8;
      const u64 e = el(&b.l, 0, ew);
      for (int i = 0; i < 16 / ew; i++) elput(&r.l, i, ew, e);
      r.h = r.l;
    }
    yput(m, dst, r, l256);
    return X_OK;
  }
  switch (op) {
  case 0x10:
    if (pp <= 1 || mem) r = b;
    else {
      r.l = a.l;
      memcpy(r.l.b, b.l.b, pp == 2 ? 4 : 8);
    }
    break;
  case 0x11: case 0x29: case 0x2b: case 0x7f: case 0xe7:
    if (mem) {
      u8 buf[32];
      memcpy(buf, s.l.b, 16);
      memcpy(buf + 16, s.h.b, 16);
      return vwrite_n(m, d->ea, (u32)(op == 0x11 ? n : vl), buf) ? X_FAULT : X_OK;
    }
    if (op == 0x11 && pp >= 2) {
      r.l = a.l;
      memcpy(r.l.b, s.l.b, pp == 2 ? 4 : 8);
      yput(m, d->rm, r, 0);
    } else {
      yput(m, d->rm, s, l256);
    }
    return X_OK;
  case 0x12:
    memcpy(r.l.b, mem ? b.l.b : b.l.b + 8, 8);
    memcpy(r.l.b + 8, a.l.b + 8, 8);
    break;
  case 0x16:
    memcpy(r.l.b, a.l.b, 8);
    memcpy(r.l.b + 8, b.l.b, 8);
    break;
  case 0x13: return vwrite(m, d->ea, 8, s.l.b) ? X_FAULT : X_OK;
  case 0x17: return vwrite(m, d->ea, 8, s.l.b + 8) ? X_FAULT : X_OK;
  case 0x28: case 0x6f: r = b; break;
  case 0x50: {
    const int ew = pp ? 8 : 4;
    u64 v = 0;
    for (int i = 0; i < 16 / ew; i++) v |= (el(&b.l, i, ew) >> (8 * ew - 1)) << i;
    if (l256)
      for (int i = 0; i < 16 / ew; i++) v |= (el(&b.h, i, ew) >> (8 * ew - 1)) << (i + 16 / ew);
    m->r.gpr[d->reg] = v;
    return X_OK;
  }
  case 0xd7: {
    u64 v = 0;
    for (int i = 0; i < 16; i++) v |= (u64)(b.l.b[i] >> 7) << i;
    if (l256)
      for (int i = 0; i < 16; i++) v |= (u64)(b.h.b[i] >> 7) << (i + 16);
    m->r.gpr[d->reg] = v;
    return X_OK;
  }
  case 0x6e:
    memset(b.l.b + n, 0, (size_t)(16 - n));
    r.l = b.l;
    break;
  case 0x7e:
    if (pp == 2) {
      memcpy(r.l.b, b.l.b, 8);
      break;
    }
    if (mem) return vwrite(m, d->ea, (u32)n, s.l.b) ? X_FAULT : X_OK;
    m->r.gpr[d->rm] = el(&s.l, 0, n);
    return X_OK;
  case 0x70:
    vlane(0x70, pp, &a.l, &b.l, imm, 0, &r.l);
    vlane(0x70, pp, &a.h, &b.h, imm, 0, &r.h);
    break;
  case 0x71: case 0x72: case 0x73:
    r.l = vshift_imm(op, r3, &b.l, imm);
    r.h = vshift_imm(op, r3, &b.h, imm);
    dst = vv;
    break;
  case 0xc4:
    r.l = a.l;
    elput(&r.l, imm & 7, 2, el(&b.l, 0, 2));
    break;
  case 0xc5:
    m->r.gpr[d->reg] = el(&b.l, imm & 7, 2);
    return X_OK;
  case 0xd6:
    if (mem) return vwrite(m, d->ea, 8, s.l.b) ? X_FAULT : X_OK;
    memcpy(r.l.b, s.l.b, 8);
    yput(m, d->rm, r, 0);
    return X_OK;
  default: {
    const u64 cnt = el(&b.l, 0, 8);
    if (!vlane(op, pp, &a.l, &b.l, imm, cnt, &r.l)) return X_UNIMPL;
    vlane(op, pp, &a.h, &b.h, (u8)(op == 0xc6 && pp == 1 ? imm >> 2 : imm), cnt, &r.h);
    break;
  }
  }
  yput(m, dst, r, l256);
  return X_OK;
}

#include "x86_oracle_sys.inc"

static int exec_insn(orc_machine *m, insn *d, memref *mr, u64 *next_rip) {
  (void)mr;
  const u32 op = d->op;
  const int osz = d->rexw ? 8 : (d->pfx66 ? 2 : 4);
  u64 nrip = d->start + d->len;
  u64 a = 0, b = 0, res = 0;
  *next_rip = nrip;
  if ((d->lock && !lockable(d)) || d->undef) { /* U34, U36 */
    fault(m, WTFGPU_VEC_UD, 0);
    return X_FAULT;
  }
  /* 32-bit code (U29): stack slots and near branch targets are 32-bit; 16-bit
   * addresses (67) and 16-bit instruction pointers (66 on a near branch) are outside */
  const int stk = d->pfx66 ? 2 : (d->m32 ? 4 : 8), nsz = d->m32 ? 4 : 8;
  const u64 sm = d->m32 ? 0xffffffffULL : ~0ULL;
  if (d->m32 && (d->a16 || (d->pfx66 && ((d->opmap == 0 && ((op >= 0x70 && op <= 0x7f) || (op >= 0xe0 && op <= 0xe3) ||
                                                         op == 0xe8 || op == 0xe9 || op == 0xeb || op == 0xc2 ||
                                                         op == 0xc3 || (op == 0xff && ((d->reg & 7) == 2 || (d->reg & 7) == 4)))) ||
                                        (d->opmap == 1 && op >= 0x80 && op <= 0x8f)))))
    return X_UNIMPL;
  if (d->m32 && d->opmap == 0 && !d->vex) {
    if (op >= 0x40 && op <= 0x4f) { /* inc / dec r32 */
      const u32 r = op & 7;
      a = getreg(m, d, r, osz);
      const u64 cf = m->r.rflags & RF_CF;
      res = alu2(m, op < 0x48 ? 0 : 5, a, 1, osz);
      m->r.rflags = (m->r.rflags & ~RF_CF) | cf;
      setreg(m, d, r, osz, res);
      return X_OK;
    }
    switch (op) {
    case 0x06: case 0x07: case 0x0e: case 0x16: case 0x17: case 0x1e: case 0x1f: case 0x27: case 0x2f:
    case 0x37: case 0x3f: case 0x60: case 0x61: case 0x9a: case 0xce: case 0xd4: case 0xd5: case 0xea:
      return exec_sys32(m, d, next_rip);
    case 0x62: { /* bound r, m16&16 / m32&32: #BR (vector 5) unless lower <= index <= upper, signed */
      if (!d->is_mem) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      u64 lo = 0, hi = 0;
      CHK(vread(m, d->ea, (u32)osz, &lo));
      CHK(vread(m, d->ea + (u64)osz, (u32)osz, &hi));
      const i64 ix = (i64)sxn(getreg(m, d, d->reg, osz), osz);
      if (ix < (i64)sxn(lo, osz) || ix > (i64)sxn(hi, osz)) {
        fault(m, 5, 0);
        return X_FAULT;
      }
      return X_OK;
    }
    case 0x63: { /* arpl r/m16, r16: SDM ARPL */
      u64 dv = 0;
      CHK(d->is_mem ? rd_rm_rmw(m, d, 2, &dv) : rd_rm(m, d, 2, &dv));
      const u64 rpl = m->r.gpr[d->reg & 15] & 3;
      const int adj = (dv & 3) < rpl;
      if (adj) CHK(wr_rm(m, d, 2, (dv & ~3ULL) | rpl));
      m->r.rflags = (m->r.rflags & ~RF_ZF) | (adj ? RF_ZF : 0);
      return X_OK;
    }
    case 0xc4: case 0xc5: { /* les / lds r, m16:osz (U30) */
      if (!d->is_mem) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      u64 off = 0, sel = 0;
      CHK(vread(m, d->ea, (u32)osz, &off));
      CHK(vread(m, d->ea + (u64)osz, 2, &sel));
      if (load_sreg(m, op == 0xc4 ? WTFGPU_ES : WTFGPU_DS, (u16)sel)) return X_FAULT;
      setreg(m, d, d->reg, osz, off);
      return X_OK;
    }
    case 0xd6: /* salc */
      m->r.gpr[0] = (m->r.gpr[0] & ~0xffULL) | ((m->r.rflags & RF_CF) ? 0xffULL : 0);
      return X_OK;
    default:
      break;
    }
  }

  if (d->opmap == 0) {
    /* ALU ops 00-3f */
    if (op < 0x40 && (op & 7) < 6) {
      const int aluop = (int)(op >> 3);
      const int form = op & 7;
      const int sz = (form & 1) ? osz : 1;
      if (form <= 1) { /* Ex, Gx */
        if (aluop == 7) {
          CHK(rd_rm(m, d, sz, &a));
          alu2(m, 7, a, getreg(m, d, d->reg, sz), sz);
        } else {
          CHK(rd_rm_rmw(m, d, sz, &a));
          res = alu2(m, aluop, a, getreg(m, d, d->reg, sz), sz);
          CHK(wr_rm(m, d, sz, res));
        }
      } else if (form <= 3) { /* Gx, Ex */
        CHK(rd_rm(m, d, sz, &b));
        res = alu2(m, aluop, getreg(m, d, d->reg, sz), b, sz);
        if (aluop != 7) setreg(m, d, d->reg, sz, res);
      } else { /* AL/eAX, imm */
        b = form == 4 ? d->bytes[d->len - 1] : sxn(0, 1);
        if (form == 5) {
          int isz = osz == 2 ? 2 : 4;
          b = 0;
          memcpy(&b, d->bytes + d->len - isz, (size_t)isz);
          b = sxn(b, isz);
        }
        res = alu2(m, aluop, getreg(m, d, 0, sz), b, sz);
        if (aluop != 7) setreg(m, d, 0, sz, res);
      }
      return X_OK;
    }
    switch (op) {
    case 0x50: case 0x51: case 0x52: case 0x53: case 0x54: case 0x55: case 0x56: case 0x57: {
      const int sz = stk;
      const u32 r = (op & 7) | (d->rexb << 3);
      CHK(push64(m, m->r.gpr[r] & szmask(sz), sz));
      return X_OK;
    }
    case 0x58: case 0x59: case 0x5a: case 0x5b: case 0x5c: case 0x5d: case 0x5e: case 0x5f: {
      const int sz = stk;
      const u32 r = (op & 7) | (d->rexb << 3);
      CHK(pop64(m, &a, sz));
      setreg(m, d, r, sz, a);
      return X_OK;
    }
    case 0x63: /* movsxd */
      CHK(rd_rm(m, d, 4, &a));
      setreg(m, d, d->reg, osz, osz == 8 ? sxn(a, 4) : a);
      return X_OK;
    case 0x68:
    case 0x6a: {
      const int sz = stk;
      int isz = op == 0x6a ? 1 : (d->pfx66 ? 2 : 4);
      memcpy(&a, d->bytes + d->len - isz, (size_t)isz);
      a = sxn(a, isz) & szmask(sz);
      CHK(push64(m, a, sz));
      return X_OK;
    }
    case 0x69:
    case 0x6b: {
      int isz = op == 0x6b ? 1 : (osz == 2 ? 2 : 4);
      b = 0;
      memcpy(&b, d->bytes + d->len - isz, (size_t)isz);
      b = sxn(b, isz);
      CHK(rd_rm(m, d, osz, &a));
      {
      __int128 p = (__int128)(i64)sxn(a & szmask(osz), osz) * (__int128)(i64)sxn(b & szmask(osz), osz);
      u64 lo = (u64)p & szmask(osz);
      int ovf = (__int128)(i64)sxn(lo, osz) != p;
      setreg(m, d, d->reg, osz, lo);
      set_flags(m, RF_STATUS, szp(lo, osz) | (ovf ? (RF_CF | RF_OF) : 0));
      return X_OK;
    }
    }
    case 0x70: case 0x71: case 0x72: case 0x73: case 0x74: case 0x75: case 0x76: case 0x77:
    case 0x78: case 0x79: case 0x7a: case 0x7b: case 0x7c: case 0x7d: case 0x7e: case 0x7f:
      if (cond(m, op & 0xf)) *next_rip = nrip + sxn(d->bytes[d->len - 1], 1);
      return X_OK;
    case 0x80:
    case 0x81:
    case 0x83: {
      const int sz = op == 0x80 ? 1 : osz;
      int isz = op == 0x81 ? (osz == 2 ? 2 : 4) : 1;
      b = 0;
      memcpy(&b, d->bytes + d->len - isz, (size_t)isz);
      b = sxn(b, isz);
      const int aluop = (int)(d->reg & 7);
      if (aluop == 7) {
        CHK(rd_rm(m, d, sz, &a));
        alu2(m, 7, a, b, sz);
      } else {
        CHK(rd_rm_rmw(m, d, sz, &a));
        res = alu2(m, aluop, a, b, sz);
        CHK(wr_rm(m, d, sz, res));
      }
      return X_OK;
    }
    case 0x84:
    case 0x85: {
      const int sz = op == 0x84 ? 1 : osz;
      CHK(rd_rm(m, d, sz, &a));
      alu2(m, 4, a, getreg(m, d, d->reg, sz), sz);
      return X_OK;
    }
    case 0x86:
    case 0x87: {
      const int sz = op == 0x86 ? 1 : osz;
      CHK(rd_rm_rmw(m, d, sz, &a));
      b = getreg(m, d, d->reg, sz);
      CHK(wr_rm(m, d, sz, b));
      setreg(m, d, d->reg, sz, a);
      return X_OK;
    }
    case 0x88:
    case 0x89: {
      const int sz = op == 0x88 ? 1 : osz;
      CHK(wr_rm(m, d, sz, getreg(m, d, d->reg, sz)));
      return X_OK;
    }
    case 0x8a:
    case 0x8b: {
      const int sz = op == 0x8a ? 1 : osz;
      CHK(rd_rm(m, d, sz, &a));
      setreg(m, d, d->reg, sz, a);
      return X_OK;
    }
    case 0x8d:
      if (!d->is_mem) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      /* lea: effective address without segment base */
      setreg(m, d, d->reg, osz, d->ea - seg_base(m, d->seg));
      return X_OK;
    case 0x8f: {
      if ((d->reg & 7) != 0) { /* XOP on AMD; #UD here */
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      const int sz = stk;
      /* pop r/m: the address is computed with rsp already incremented */
      u64 rsp0 = m->r.gpr[WTFGPU_RSP];
      CHK(vread(m, rsp0 & sm, (u32)sz, &a) ? 1 : 0);
      m->r.gpr[WTFGPU_RSP] = ((rsp0 & sm) + (u64)sz) & sm;
      if (d->is_mem) finish_ea(m, d, mr);
      if (wr_rm(m, d, sz, a)) {
        m->r.gpr[WTFGPU_RSP] = rsp0;
        return X_FAULT;
      }
      return X_OK;
    }
    case 0x90:
      if (d->rexb) { /* xchg r8, rax */
        a = getreg(m, d, 8, osz);
        setreg(m, d, 8, osz, getreg(m, d, 0, osz));
        setreg(m, d, 0, osz, a);
      }
      return X_OK; /* nop / pause */
    case 0x91: case 0x92: case 0x93: case 0x94: case 0x95: case 0x96: case 0x97: {
      const u32 r = (op & 7) | (d->rexb << 3);
      a = getreg(m, d, r, osz);
      setreg(m, d, r, osz, getreg(m, d, 0, osz));
      setreg(m, d, 0, osz, a);
      return X_OK;
    }
    case 0x98: /* cbw/cwde/cdqe */
      if (osz == 2) setreg(m, d, 0, 2, sxn(m->r.gpr[0], 1));
      else if (osz == 4) setreg(m, d, 0, 4, sxn(m->r.gpr[0], 2));
      else m->r.gpr[0] = sxn(m->r.gpr[0], 4);
      return X_OK;
    case 0x99: /* cwd/cdq/cqo */
      setreg(m, d, WTFGPU_RDX, osz, msb(m->r.gpr[0], osz) ? ~0ULL : 0);
      return X_OK;
    case 0x9c: { /* pushf */
      const int sz = stk;
      CHK(push64(m, m->r.rflags & 0xfcffffULL & szmask(sz), sz));
      return X_OK;
    }
    case 0x9d: { /* popf */
      const int sz = stk;
      CHK(pop64(m, &a, sz));
      u64 mask = RF_STATUS | RF_TF | RF_DF | 0x4000ULL /*NT*/ | 0x40000ULL /*AC*/ | 0x200000ULL /*ID*/;
      if (cpl(m) == 0) mask |= RF_IF | 0x3000ULL;
      if (sz == 2) mask &= 0xffff;
      m->r.rflags = ((m->r.rflags & ~mask) | (a & mask) | 2) & ~0x10000ULL;
      return X_OK;
    }
    case 0x9e: /* sahf */
      set_flags(m, RF_SF | RF_ZF | RF_AF | RF_PF | RF_CF, (m->r.gpr[0] >> 8) & 0xff);
      return X_OK;
    case 0x9f: /* lahf */
      m->r.gpr[0] = (m->r.gpr[0] & ~0xff00ULL) | (((m->r.rflags & 0xd5) | 2) << 8);
      return X_OK;
    case 0xa0: case 0xa1: case 0xa2: case 0xa3: { /* mov moffs */
      const int sz = (op & 1) ? osz : 1;
      const int asz = d->pfx67 ? 4 : 8;
      u64 addr = 0;
      memcpy(&addr, d->bytes + d->len - asz, (size_t)asz);
      addr += seg_base(m, d->seg);
      if (op <= 0xa1) {
        a = 0;
        CHK(vread(m, addr, (u32)sz, &a));
        setreg(m, d, 0, sz, a);
      } else {
        a = getreg(m, d, 0, sz);
        CHK(vwrite(m, addr, (u32)sz, &a));
      }
      return X_OK;
    }
    case 0xa4: case 0xa5: case 0xa6: case 0xa7: case 0xaa: case 0xab: case 0xac: case 0xad:
    case 0xae: case 0xaf: {
      const int sz = (op & 1) ? osz : 1;
      /* a fault inside rep keeps the completed iterations (rcx/rsi/rdi), rip stays */
      if (string_op(m, d, op & ~1u, sz)) return X_FAULT_KEEP;
      return X_OK;
    }
    case 0xa8:
    case 0xa9: {
      const int sz = op == 0xa8 ? 1 : osz;
      int isz = op == 0xa8 ? 1 : (osz == 2 ? 2 : 4);
      b = 0;
      memcpy(&b, d->bytes + d->len - isz, (size_t)isz);
      alu2(m, 4, getreg(m, d, 0, sz), sxn(b, isz), sz);
      return X_OK;
    }
    case 0xb0: case 0xb1: case 0xb2: case 0xb3: case 0xb4: case 0xb5: case 0xb6: case 0xb7:
      setreg(m, d, (op & 7) | (d->rexb << 3), 1, d->bytes[d->len - 1]);
      return X_OK;
    case 0xb8: case 0xb9: case 0xba: case 0xbb: case 0xbc: case 0xbd: case 0xbe: case 0xbf: {
      int isz = osz;
      a = 0;
      memcpy(&a, d->bytes + d->len - isz, (size_t)isz);
      setreg(m, d, (op & 7) | (d->rexb << 3), osz, a);
      return X_OK;
    }
    case 0xc0: case 0xc1: case 0xd0: case 0xd1: case 0xd2: case 0xd3: {
      const int sz = (op & 1) ? osz : 1;
      u32 cnt = (op <= 0xc1) ? d->bytes[d->len - 1] : (op <= 0xd1 ? 1 : (u32)(m->r.gpr[1] & 0xff));
      CHK(rd_rm_rmw(m, d, sz, &a));
      u64 saved = m->r.rflags;
      res = shift_op(m, (int)(d->reg & 7), a, cnt, sz);
      if (wr_rm(m, d, sz, res)) {
        m->r.rflags = saved;
        return X_FAULT;
      }
      return X_OK;
    }
    case 0xc2:
    case 0xc3: {
      a = 0;
      CHK(vread(m, m->r.gpr[WTFGPU_RSP] & sm, (u32)nsz, &a));
      u64 extra = 0;
      if (op == 0xc2) extra = (u64)d->bytes[d->len - 2] | ((u64)d->bytes[d->len - 1] << 8);
      m->r.gpr[WTFGPU_RSP] = ((m->r.gpr[WTFGPU_RSP] & sm) + (u64)nsz + extra) & sm;
      *next_rip = a;
      return X_OK;
    }
    case 0xc6:
    case 0xc7: {
      if ((d->reg & 7) != 0) { /* the reserved forms; xabort / xbegin: RTM (U48) */
        if ((d->reg & 7) == 7 && !d->is_mem && (d->rm & 7) == 0) {
          if (op == 0xc6) return X_OK; /* xabort imm8: no transaction is ever active, a no-op */
          if (osz == 2) return X_UNIMPL; /* xbegin rel16 */
          /* xbegin rel32: the transaction aborts at once (RTM_ALWAYS_ABORT): EAX = 0 (no
           * abort cause), execution continues at the fallback address */
          u64 rel = 0;
          memcpy(&rel, d->bytes + d->len - 4, 4);
          const u64 target = (nrip + sxn(rel, 4)) & sm;
          if (!d->m32 && !is_canonical(target)) {
            fault(m, WTFGPU_VEC_GP, 0);
            return X_FAULT;
          }
          m->r.gpr[0] = 0;
          *next_rip = target;
          return X_OK;
        }
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      const int sz = op == 0xc6 ? 1 : osz;
      int isz = op == 0xc6 ? 1 : (osz == 2 ? 2 : 4);
      b = 0;
      memcpy(&b, d->bytes + d->len - isz, (size_t)isz);
      CHK(wr_rm(m, d, sz, sxn(b, isz)));
      return X_OK;
    }
    case 0xc9: { /* leave */
      u64 rbp = m->r.gpr[WTFGPU_RBP] & sm;
      a = 0;
      CHK(vread(m, rbp, (u32)nsz, &a));
      m->r.gpr[WTFGPU_RSP] = (rbp + (u64)nsz) & sm;
      m->r.gpr[WTFGPU_RBP] = a;
      return X_OK;
    }
    case 0xcc:
      return X_INT3;
    case 0xcf: { /* iretq (U19); iret / iretd with 16- / 32-bit slots (U29) */
      if (!d->rexw) return far_pop(m, osz, 0, next_rip, 1, (int)d->m32);
      u64 f[5]; /* rip, cs, rflags, rsp, ss: every read before any change */
      for (int i = 0; i < 5; i++) CHK(vread(m, m->r.gpr[WTFGPU_RSP] + 8 * (u64)i, 8, &f[i]));
      const u32 ocpl = (u32)cpl(m), ncpl = (u32)f[1] & 3;
      if ((f[1] & 0xfffc) == 0 || ncpl < ocpl) {
        fault(m, WTFGPU_VEC_GP, (u32)f[1] & 0xfffc);
        return X_FAULT;
      }
      if (!is_canonical(f[0])) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      /* SDM IRET: status, TF, DF, NT, RF, AC, ID always; IF if CPL <= IOPL;
       * IOPL, VIF, VIP at CPL 0 only; VM never in 64-bit mode */
      u64 mask = 0x254dd5ULL;
      const u32 iopl = (u32)(m->r.rflags >> 12) & 3;
      if (ocpl == 0) mask |= 0x200ULL | 0x3000ULL | 0x80000ULL | 0x100000ULL;
      else if (ocpl <= iopl) mask |= 0x200ULL;
      m->r.rflags = (m->r.rflags & ~mask) | (f[2] & mask) | 2;
      m->r.seg[WTFGPU_CS].selector = (u16)f[1];
      m->r.seg[WTFGPU_SS].selector = (u16)f[4];
      m->r.gpr[WTFGPU_RSP] = f[3];
      *next_rip = f[0];
      return X_OK;
    }
    case 0xd7: { /* xlat */
      u64 addr = (m->r.gpr[WTFGPU_RBX] + (m->r.gpr[0] & 0xff));
      if (d->pfx67) addr &= 0xffffffffULL;
      a = 0;
      CHK(vread(m, addr + seg_base(m, d->seg), 1, &a));
      setreg(m, d, 0, 1, a);
      return X_OK;
    }
    case 0xe8: {
      u64 rel = 0;
      memcpy(&rel, d->bytes + d->len - 4, 4);
      CHK(push64(m, nrip, nsz));
      *next_rip = nrip + sxn(rel, 4);
      return X_OK;
    }
    case 0xe9: {
      u64 rel = 0;
      memcpy(&rel, d->bytes + d->len - 4, 4);
      *next_rip = nrip + sxn(rel, 4);
      return X_OK;
    }
    case 0xeb:
      *next_rip = nrip + sxn(d->bytes[d->len - 1], 1);
      return X_OK;
    case 0xf4:
      return X_HLT;
    /* invalid in 64-bit mode: push / pop es cs ss ds, daa das aaa aas, pusha
     * popa, 82 (alias of 80), far call / jmp, aam aad salc (SDM opcode map, i64) */
    case 0x06: case 0x07: case 0x0e: case 0x16: case 0x17: case 0x1e: case 0x1f: case 0x27:
    case 0x2f: case 0x37: case 0x3f: case 0x60: case 0x61: case 0x9a: case 0xd4:
    case 0xd5: case 0xd6: case 0xea:
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    case 0x82: /* 80's alias in 32-bit code */
      if (!d->m32) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      {
        b = sxn(d->bytes[d->len - 1], 1);
        const int aluop = (int)(d->reg & 7);
        if (aluop == 7) {
          CHK(rd_rm(m, d, 1, &a));
          alu2(m, 7, a, b, 1);
        } else {
          CHK(rd_rm_rmw(m, d, 1, &a));
          const u64 saved = m->r.rflags;
          res = alu2(m, aluop, a, b, 1);
          if (wr_rm(m, d, 1, res)) {
            m->r.rflags = saved;
            return X_FAULT;
          }
        }
      }
      return X_OK;
    case 0x62: /* EVEX: AVX-512, defined, not executed (U45) */
      return X_UNIMPL;
    case 0xce: /* into: invalid in 64-bit mode */
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    case 0x6c: case 0x6d: case 0x6e: case 0x6f: { /* ins / outs (U31) */
      const int sz = (op & 1) ? (osz == 2 ? 2 : 4) : 1;
      if (io_string(m, d, sz)) return X_FAULT_KEEP;
      return X_OK;
    }
    case 0xe4: case 0xe5: case 0xec: case 0xed: /* in: all ones (U31) */
      if (!io_allowed(m)) return X_FAULT;
      setreg(m, d, 0, (op & 1) ? (osz == 2 ? 2 : 4) : 1, ~0ULL);
      return X_OK;
    case 0xe6: case 0xe7: case 0xee: case 0xef: /* out */
      if (!io_allowed(m)) return X_FAULT;
      return X_OK;
    case 0x8c: { /* mov r/m, Sreg (U30) */
      const u32 sr = d->reg & 7;
      if (sr > 5) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      a = m->r.seg[sr].selector;
      if (d->is_mem) {
        CHK(vwrite(m, d->ea, 2, &a));
      } else {
        setreg(m, d, d->rm, osz, a);
      }
      return X_OK;
    }
    case 0x8e: { /* mov Sreg, r/m16 */
      const u32 sr = d->reg & 7;
      if (sr == WTFGPU_CS || sr > 5) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      CHK(rd_rm(m, d, 2, &a));
      if (load_sreg(m, sr, (u16)a)) return X_FAULT;
      return X_OK;
    }
    case 0x9b: /* fwait (U32) */
      if ((m->r.cr0 & 0xa) == 0xa) { /* TS and MP */
        fault(m, VEC_NM, 0);
        return X_FAULT;
      }
      if (m->r.fpsw & ~m->r.fpcw & 0x3f) { /* a pending unmasked exception */
        fault(m, VEC_MF, 0);
        return X_FAULT;
      }
      return X_OK;
    case 0xc8: { /* enter (U29): bochs' ENTER64 order (32-bit slots in 32-bit code) */
      if (d->pfx66) return X_UNIMPL;
      const u64 size = (u64)d->bytes[d->len - 3] | ((u64)d->bytes[d->len - 2] << 8);
      const u32 level = d->bytes[d->len - 1] & 31;
      const u32 w = (u32)nsz;
      u64 rsp = m->r.gpr[WTFGPU_RSP] & sm, rbp = m->r.gpr[WTFGPU_RBP] & sm;
      CHK(span_check(m, (rsp - w * (level + 1)) & sm, w * (level + 1), ACC_W));
      rsp = (rsp - w) & sm;
      CHK(vwrite(m, rsp, w, &rbp));
      const u64 frame = rsp;
      if (level > 0) {
        for (u32 i = 1; i < level; i++) {
          rbp = (rbp - w) & sm;
          u64 t = 0;
          CHK(vread(m, rbp, w, &t));
          rsp = (rsp - w) & sm;
          CHK(vwrite(m, rsp, w, &t));
        }
        rsp = (rsp - w) & sm;
        CHK(vwrite(m, rsp, w, &frame));
      }
      m->r.gpr[WTFGPU_RBP] = frame;
      m->r.gpr[WTFGPU_RSP] = (rsp - size) & sm;
      return X_OK;
    }
    case 0xca: case 0xcb: { /* far ret (U29): 32-bit operand size unless REX.W / 66 */
      const u64 imm = op == 0xca ? ((u64)d->bytes[d->len - 2] | ((u64)d->bytes[d->len - 1] << 8)) : 0;
      return far_pop(m, osz, imm, next_rip, 0, (int)d->m32);
    }
    case 0xcd: { /* int n (U24) */
      const u32 vec = d->bytes[d->len - 1];
      if (vec == 3) return X_INT3;
      return soft_int(m, vec, 1, nrip, next_rip);
    }
    case 0xf1: /* int1 (icebp): #DB through the IDT, no DPL check */
      return soft_int(m, VEC_DB, 0, nrip, next_rip);
    case 0xfa: case 0xfb: /* cli / sti (U25) */
      if ((u32)cpl(m) > iopl(m)) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      if (op == 0xfa) m->r.rflags &= ~RF_IF;
      else m->r.rflags |= RF_IF;
      return X_OK;
    case 0xe0: case 0xe1: case 0xe2: case 0xe3: { /* loopne / loope / loop / jrcxz (U26) */
      const u64 amask = d->pfx67 ? 0xffffffffULL : ~0ULL;
      const u64 rel = sxn(d->bytes[d->len - 1], 1);
      int taken;
      if (op == 0xe3) {
        taken = (m->r.gpr[WTFGPU_RCX] & amask) == 0;
      } else {
        const u64 cnt = (m->r.gpr[WTFGPU_RCX] - 1) & amask;
        m->r.gpr[WTFGPU_RCX] = cnt;
        const int zf = (m->r.rflags & RF_ZF) != 0;
        taken = cnt != 0 && (op == 0xe2 || (op == 0xe1 ? zf : !zf));
      }
      if (taken) *next_rip = nrip + rel;
      return X_OK;
    }
    case 0xd8: case 0xd9: case 0xda: case 0xdb: case 0xdc: case 0xdd: case 0xde: case 0xdf:
      return exec_x87(m, d);
    case 0xf5:
      m->r.rflags ^= RF_CF;
      return X_OK;
    case 0xf6:
    case 0xf7: {
      const int sz = op == 0xf6 ? 1 : osz;
      const int sub = (int)(d->reg & 7);
      if (sub <= 1) { /* test */
        int isz = op == 0xf6 ? 1 : (osz == 2 ? 2 : 4);
        b = 0;
        memcpy(&b, d->bytes + d->len - isz, (size_t)isz);
        CHK(rd_rm(m, d, sz, &a));
        alu2(m, 4, a, sxn(b, isz), sz);
      } else if (sub == 2) { /* not */
        CHK(rd_rm_rmw(m, d, sz, &a));
        CHK(wr_rm(m, d, sz, ~a));
      } else if (sub == 3) { /* neg */
        CHK(rd_rm_rmw(m, d, sz, &a));
        u64 saved = m->r.rflags;
        res = alu2(m, 5, 0, a, sz);
        if (wr_rm(m, d, sz, res)) {
          m->r.rflags = saved;
          return X_FAULT;
        }
      } else {
        CHK(rd_rm(m, d, sz, &a));
        if (muldiv(m, d, sub, sz, a)) return X_FAULT;
      }
      return X_OK;
    }
    case 0xf8: m->r.rflags &= ~RF_CF; return X_OK;
    case 0xf9: m->r.rflags |= RF_CF; return X_OK;
    case 0xfc: m->r.rflags &= ~RF_DF; return X_OK;
    case 0xfd: m->r.rflags |= RF_DF; return X_OK;
    case 0xfe:
    case 0xff: {
      const int sz = op == 0xfe ? 1 : osz;
      const int sub = (int)(d->reg & 7);
      if (sub <= 1) { /* inc/dec */
        CHK(rd_rm_rmw(m, d, sz, &a));
        u64 cf = m->r.rflags & RF_CF;
        u64 saved = m->r.rflags;
        res = alu2(m, sub ? 5 : 0, a, 1, sz);
        m->r.rflags = (m->r.rflags & ~RF_CF) | cf;
        if (wr_rm(m, d, sz, res)) {
          m->r.rflags = saved;
          return X_FAULT;
        }
        return X_OK;
      }
      if (op == 0xfe || sub == 7) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      if (sub == 3 || sub == 5) { /* far call / jmp m16:osz (U29): the CPL is kept */
        if (!d->is_mem) {
          fault(m, WTFGPU_VEC_UD, 0);
          return X_FAULT;
        }
        u64 off = 0, sel = 0;
        CHK(vread(m, d->ea, (u32)osz, &off));
        CHK(vread(m, d->ea + (u64)osz, 2, &sel));
        if ((sel & 0xfffc) == 0) {
          fault(m, WTFGPU_VEC_GP, 0);
          return X_FAULT;
        }
        if (osz == 2) off &= 0xffff;
        if (!is_canonical(off)) {
          fault(m, WTFGPU_VEC_GP, 0);
          return X_FAULT;
        }
        const u16 ncs = (u16)((sel & 0xfffc) | (u32)cpl(m));
        if (sub == 3) {
          const u64 rsp = m->r.gpr[WTFGPU_RSP] & sm;
          const u64 ocs = m->r.seg[WTFGPU_CS].selector;
          CHK(span_check(m, (rsp - 2 * (u64)osz) & sm, 2 * (u32)osz, ACC_W));
          CHK(vwrite(m, (rsp - (u64)osz) & sm, (u32)osz, &ocs));
          CHK(vwrite(m, (rsp - 2 * (u64)osz) & sm, (u32)osz, &nrip));
          m->r.gpr[WTFGPU_RSP] = (rsp - 2 * (u64)osz) & sm;
        }
        m->r.seg[WTFGPU_CS].selector = ncs;
        *next_rip = off;
        return X_OK;
      }
      if (sub == 2 || sub == 4) { /* call / jmp near indirect (64-bit; 32-bit in 32-bit code) */
        CHK(rd_rm(m, d, nsz, &a));
        if (sub == 2) CHK(push64(m, nrip, nsz));
        *next_rip = a;
        return X_OK;
      }
      if (sub == 6) { /* push r/m */
        const int psz = stk;
        CHK(rd_rm(m, d, psz, &a));
        CHK(push64(m, a, psz));
        return X_OK;
      }
      return X_UNIMPL;
    }
    default:
      return X_UNIMPL;
    }
  }

  if (d->vex) return exec_vex(m, d);
  if (d->opmap == 2 || d->opmap == 3) return exec_sse(m, d);
  if (d->opmap == 1) {
    if (op == 0xae && !(!d->pfx66 && !d->rep && (d->is_mem ? ((d->reg & 7) == 2 || (d->reg & 7) == 3) : (d->reg & 7) >= 5)))
      return exec_sys0f(m, d, next_rip);
    if (op == 0xff) { /* ud0 */
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    }
    if (sse_opcode(op)) return exec_sse(m, d);
    switch (op) {
    case 0x00: case 0x02: case 0x03: case 0x06: case 0x08: case 0x09: case 0x21: case 0x23: case 0x33:
    case 0x34: case 0x35: case 0xa0: case 0xa1: case 0xa2: case 0xa8: case 0xa9: case 0xb2: case 0xb4:
    case 0xb5: case 0xc7:
      return exec_sys0f(m, d, next_rip);
    /* #UD: 3DNow! / femms, mov to / from test registers, GETSEC (no SMX), RSM
     * outside SMM, UD0 / UD1, the undefined 0f opcodes */
    case 0x04: case 0x0a: case 0x0c: case 0x0e: case 0x0f: case 0x24: case 0x25: case 0x26: case 0x27:
    case 0x36: case 0x37: case 0x39: case 0x3b: case 0x3c: case 0x3d: case 0x3e: case 0x3f: case 0xa6:
    case 0xa7: case 0xaa: case 0xb9: case 0xff:
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    case 0x05: /* syscall (64-bit; SDM vol. 2B; U16) */
    case 0x07: /* sysretq */
      if (!(m->r.efer & 1)) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      if (op == 0x05) {
        m->r.gpr[1] = nrip;
        m->r.gpr[11] = m->r.rflags & ~0x10000ULL;
        m->r.rflags = ((m->r.rflags & ~m->r.sfmask) & ~0x10000ULL) | 2;
        *next_rip = d->m32 ? m->r.cstar : m->r.lstar; /* from 32-bit code: CSTAR (U29) */
        m->r.seg[WTFGPU_CS].selector = (u16)((m->r.star >> 32) & 0xfffc);
        m->r.seg[WTFGPU_SS].selector = (u16)(m->r.seg[WTFGPU_CS].selector + 8);
      } else {
        if (cpl(m) == 0 && !d->rexw) { /* to compatibility mode at ecx (U29) */
          const u64 t32 = m->r.gpr[1] & 0xffffffffULL;
          *next_rip = t32;
          m->r.rflags = (m->r.gpr[11] & 0x3c7fd7ULL) | 2;
          m->r.seg[WTFGPU_CS].selector = (u16)(((m->r.star >> 48) & 0xffff) | 3);
          m->r.seg[WTFGPU_SS].selector = (u16)((((m->r.star >> 48) & 0xffff) + 8) | 3);
          return X_OK;
        }
        if (cpl(m) != 0 || !is_canonical(m->r.gpr[1])) {
          fault(m, WTFGPU_VEC_GP, 0);
          return X_FAULT;
        }
        *next_rip = m->r.gpr[1];
        m->r.rflags = (m->r.gpr[11] & 0x3c7fd7ULL) | 2;
        m->r.seg[WTFGPU_CS].selector = (u16)((((m->r.star >> 48) & 0xffff) + 16) | 3);
        m->r.seg[WTFGPU_SS].selector = (u16)((((m->r.star >> 48) & 0xffff) + 8) | 3);
      }
      return X_OK;
    case 0x01: /* swapgs (0f 01 f8), rdtscp (0f 01 f9); the rest of group 7: exec_sys0f */
      if (d->is_mem || (d->reg & 7) != 7 || (d->rm & 7) > 1) return exec_sys0f(m, d, next_rip);
      if ((d->rm & 7) == 1) {
        if ((m->r.cr4 & 4) && cpl(m) != 0) {
          fault(m, WTFGPU_VEC_GP, 0);
          return X_FAULT;
        }
        a = m->r.tsc + m->icount;
        m->r.gpr[0] = a & 0xffffffffULL;
        m->r.gpr[2] = a >> 32;
        m->r.gpr[1] = m->r.tsc_aux & 0xffffffffULL;
        return X_OK;
      }
      if (cpl(m) != 0) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      a = m->r.seg[WTFGPU_GS].base;
      m->r.seg[WTFGPU_GS].base = m->r.kernel_gs_base;
      m->r.kernel_gs_base = a;
      return X_OK;
    case 0x20: { /* mov r64, crN (ring 0) */
      if (d->is_mem) return X_UNIMPL;
      if (cpl(m) != 0) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      const u32 n = d->reg & 15;
      u64 v;
      if (n == 0) v = m->r.cr0;
      else if (n == 2) v = m->r.cr2;
      else if (n == 3) v = m->r.cr3;
      else if (n == 4) v = m->r.cr4;
      else if (n == 8) v = 0;
      else {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      setreg(m, d, d->rm, 8, v);
      return X_OK;
    }
    case 0x22: { /* mov crN, r64 (ring 0); a cr3 other than the testcase's
                  * initial one ends it with Cr3Change_t after retiring
                  * (bochscpu_backend.cc:628-657; U20) */
      if (cpl(m) != 0) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      const u32 n = d->reg & 15;
      const u64 v = m->r.gpr[d->rm & 15];
      if (n == 0) m->r.cr0 = v;
      else if (n == 2) m->r.cr2 = v;
      else if (n == 3) {
        m->r.cr3 = v;
        if (v != m->initial_cr3) return X_CR3;
      } else if (n == 4) m->r.cr4 = v;
      else if (n == 8) m->r.cr8 = v & 15;
      else {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      return X_OK;
    }
    case 0x31: /* rdtsc: TSC = the snapshot's Tsc + instructions retired (U21) */
      if ((m->r.cr4 & 4) && cpl(m) != 0) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      a = m->r.tsc + m->icount;
      m->r.gpr[0] = a & 0xffffffffULL;
      m->r.gpr[2] = a >> 32;
      return X_OK;
    case 0x30: /* wrmsr */
    case 0x32: { /* rdmsr (the MSRs of CpuState_t; others #GP, U21) */
      if (cpl(m) != 0) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      const u32 idx = (u32)m->r.gpr[1];
      u64 *slot = NULL;
      u64 tsc = m->r.tsc + m->icount, aux = m->r.tsc_aux, sfm = m->r.sfmask;
      int canon = 0, lo32 = 0;
      switch (idx) {
      case 0x10: slot = &tsc; break;
      case 0x1b: slot = &m->r.apic_base; break;
      case 0x174: slot = &m->r.sysenter_cs; break;
      case 0x175: slot = &m->r.sysenter_esp; canon = 1; break;
      case 0x176: slot = &m->r.sysenter_eip; canon = 1; break;
      case 0x277: slot = &m->r.pat; break;
      case 0xc0000080: slot = &m->r.efer; break;
      case 0xc0000081: slot = &m->r.star; break;
      case 0xc0000082: slot = &m->r.lstar; canon = 1; break;
      case 0xc0000083: slot = &m->r.cstar; canon = 1; break;
      case 0xc0000084: slot = &sfm; lo32 = 1; break;
      case 0xc0000100: slot = &m->r.seg[WTFGPU_FS].base; canon = 1; break;
      case 0xc0000101: slot = &m->r.seg[WTFGPU_GS].base; canon = 1; break;
      case 0xc0000102: slot = &m->r.kernel_gs_base; canon = 1; break;
      case 0xc0000103: slot = &aux; lo32 = 1; break;
      default: break;
      }
      if (!slot) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      if (op == 0x32) {
        m->r.gpr[0] = *slot & 0xffffffffULL;
        m->r.gpr[2] = *slot >> 32;
        return X_OK;
      }
      const u64 v = (m->r.gpr[0] & 0xffffffffULL) | (m->r.gpr[2] << 32);
      if ((canon && !is_canonical(v)) || (lo32 && (v >> 32))) {
        fault(m, WTFGPU_VEC_GP, 0);
        return X_FAULT;
      }
      if (idx == 0xc0000080) *slot = (v & ~0x400ULL) | (m->r.efer & 0x400ULL); /* LMA is read-only */
      else *slot = v;
      if (idx == 0x10) m->r.tsc = v - m->icount;
      if (idx == 0xc0000084) m->r.sfmask = v;
      if (idx == 0xc0000103) m->r.tsc_aux = v;
      return X_OK;
    }
    case 0x0b:
      fault(m, WTFGPU_VEC_UD, 0);
      return X_FAULT;
    case 0x0d: /* prefetchw */
    case 0x18: case 0x19: case 0x1a: case 0x1b: case 0x1c: case 0x1d: case 0x1e: case 0x1f:
      return X_OK; /* hint nops, endbr64 */
    case 0x40: case 0x41: case 0x42: case 0x43: case 0x44: case 0x45: case 0x46: case 0x47:
    case 0x48: case 0x49: case 0x4a: case 0x4b: case 0x4c: case 0x4d: case 0x4e: case 0x4f:
      CHK(rd_rm(m, d, osz, &a)); /* source always read */
      if (cond(m, op & 0xf))
        setreg(m, d, d->reg, osz, a);
      else if (osz == 4)
        setreg(m, d, d->reg, 4, m->r.gpr[d->reg]); /* zero upper half */
      return X_OK;
    case 0x80: case 0x81: case 0x82: case 0x83: case 0x84: case 0x85: case 0x86: case 0x87:
    case 0x88: case 0x89: case 0x8a: case 0x8b: case 0x8c: case 0x8d: case 0x8e: case 0x8f: {
      u64 rel = 0;
      memcpy(&rel, d->bytes + d->len - 4, 4);
      if (cond(m, op & 0xf)) *next_rip = nrip + sxn(rel, 4);
      return X_OK;
    }
    case 0x90: case 0x91: case 0x92: case 0x93: case 0x94: case 0x95: case 0x96: case 0x97:
    case 0x98: case 0x99: case 0x9a: case 0x9b: case 0x9c: case 0x9d: case 0x9e: case 0x9f:
      CHK(wr_rm(m, d, 1, (u64)cond(m, op & 0xf)));
      return X_OK;
    case 0xa3: case 0xab: case 0xb3: case 0xbb: case 0xba: {
      /* bt/bts/btr/btc */
      int sub = op == 0xa3 ? 4 : op == 0xab ? 5 : op == 0xb3 ? 6 : op == 0xbb ? 7 : (int)(d->reg & 7);
      if (sub < 4) return X_UNIMPL;
      const int bits = 8 * osz;
      u64 bitoff;
      u64 addr = d->ea;
      if (op == 0xba) {
        bitoff = d->bytes[d->len - 1] & (u64)(bits - 1);
      } else {
        u64 r = getreg(m, d, d->reg, osz);
        if (d->is_mem) {
          i64 s = (i64)sxn(r, osz);
          i64 word = s >> (osz == 8 ? 6 : osz == 4 ? 5 : 4);
          addr = d->ea + (u64)(word * osz);
          bitoff = (u64)s & (u64)(bits - 1);
        } else {
          bitoff = r & (u64)(bits - 1);
        }
      }
      if (d->is_mem) {
        if (sub == 4)
          CHK(vread(m, addr, (u32)osz, &a) ? 1 : 0);
        else
          CHK(vread_rmw(m, addr, (u32)osz, &a) ? 1 : 0);
      } else {
        a = getreg(m, d, d->rm, osz);
      }
      int bit = (int)((a >> bitoff) & 1);
      if (sub == 5) res = a | (1ULL << bitoff);
      else if (sub == 6) res = a & ~(1ULL << bitoff);
      else if (sub == 7) res = a ^ (1ULL << bitoff);
      if (sub != 4) {
        if (d->is_mem) {
          CHK(vwrite(m, addr, (u32)osz, &res));
        } else {
          setreg(m, d, d->rm, osz, res);
        }
      }
      set_flags(m, RF_CF, bit ? RF_CF : 0);
      return X_OK;
    }
    case 0xa4: case 0xa5: case 0xac: case 0xad: { /* shld / shrd */
      const int bits = 8 * osz;
      u32 cnt = (op & 1) ? (u32)(m->r.gpr[1] & 0xff) : d->bytes[d->len - 1];
      cnt &= (osz == 8) ? 0x3f : 0x1f;
      CHK(rd_rm_rmw(m, d, osz, &a));
      /* count 0: flags untouched, but the destination is still written (a
       * 32-bit register is zero-extended, as measured on hardware) */
      if (cnt == 0) return wr_rm(m, d, osz, a) ? X_FAULT : X_OK;
      b = getreg(m, d, d->reg, osz);
      const u64 mk = szmask(osz);
      int cf;
      if (osz == 2) {
        /* 32-bit concatenation, count modulo 32 (U7) */
        if (op <= 0xa5) { /* shift the 48-bit pattern a:b:a */
          u64 pat = ((a & 0xffff) << 32) | ((b & 0xffff) << 16) | (a & 0xffff);
          res = ((pat << cnt) >> 32) & 0xffff;
          cf = (int)(((pat << (cnt - 1)) >> 47) & 1);
        } else {
          u64 pat = ((a & 0xffff)) | ((b & 0xffff) << 16) | ((a & 0xffff) << 32);
          res = (pat >> cnt) & 0xffff;
          cf = (int)((pat >> (cnt - 1)) & 1);
        }
      } else if (op <= 0xa5) {
        res = ((a << cnt) | (b >> (bits - cnt))) & mk;
        cf = (int)((a >> (bits - cnt)) & 1);
      } else {
        res = ((a >> cnt) | (b << (bits - cnt))) & mk;
        cf = (int)((a >> (cnt - 1)) & 1);
      }
      u64 saved = m->r.rflags;
      set_flags(m, RF_STATUS, szp(res, osz) | (cf ? RF_CF : 0) | ((msb(res, osz) ^ msb(a, osz)) ? RF_OF : 0));
      if (wr_rm(m, d, osz, res)) {
        m->r.rflags = saved;
        return X_FAULT;
      }
      return X_OK;
    }
    case 0xaf:
      CHK(rd_rm(m, d, osz, &a));
      b = getreg(m, d, d->reg, osz);
      {
        __int128 p = (__int128)(i64)sxn(a & szmask(osz), osz) * (__int128)(i64)sxn(b & szmask(osz), osz);
        u64 lo = (u64)p & szmask(osz);
        int ovf = (__int128)(i64)sxn(lo, osz) != p;
        setreg(m, d, d->reg, osz, lo);
        set_flags(m, RF_STATUS, szp(lo, osz) | (ovf ? (RF_CF | RF_OF) : 0));
      }
      return X_OK;
    case 0xb0:
    case 0xb1: { /* cmpxchg: destination always written (SDM) */
      const int sz = op == 0xb0 ? 1 : osz;
      CHK(rd_rm_rmw(m, d, sz, &a));
      u64 acc = getreg(m, d, 0, sz);
      u64 saved = m->r.rflags;
      alu2(m, 7, acc, a, sz);
      if ((acc & szmask(sz)) == (a & szmask(sz))) {
        if (wr_rm(m, d, sz, getreg(m, d, d->reg, sz))) {
          m->r.rflags = saved;
          return X_FAULT;
        }
      } else {
        /* memory destinations are written back with the old value (locked cycle);
         * a register destination is left untouched (its upper half survives) */
        if (d->is_mem && wr_rm(m, d, sz, a)) {
          m->r.rflags = saved;
          return X_FAULT;
        }
        setreg(m, d, 0, sz, a);
      }
      return X_OK;
    }
    case 0xb6: case 0xb7: case 0xbe: case 0xbf: {
      const int ssz = (op & 1) ? 2 : 1;
      CHK(rd_rm(m, d, ssz, &a));
      if (op >= 0xbe) a = sxn(a, ssz);
      setreg(m, d, d->reg, osz, a & szmask(osz));
      return X_OK;
    }
    case 0xb8: /* popcnt (f3); without f3 JMPE: #UD */
      if (d->rep != 0xf3) {
        fault(m, WTFGPU_VEC_UD, 0);
        return X_FAULT;
      }
      CHK(rd_rm(m, d, osz, &a));
      res = (u64)__builtin_popcountll(a & szmask(osz));
      setreg(m, d, d->reg, osz, res);
      set_flags(m, RF_STATUS, a & szmask(osz) ? 0 : RF_ZF);
      return X_OK;
    case 0xbc:
    case 0xbd: {
      const int bits = 8 * osz;
      CHK(rd_rm(m, d, osz, &a));
      a &= szmask(osz);
      if (d->rep == 0xf3) { /* tzcnt / lzcnt */
        if (op == 0xbc) res = a ? (u64)__builtin_ctzll(a) : (u64)bits;
        else res = a ? (u64)(__builtin_clzll(a) - (64 - bits)) : (u64)bits;
        setreg(m, d, d->reg, osz, res);
        set_flags(m, RF_CF | RF_ZF, (a == 0 ? RF_CF : 0) | (res == 0 ? RF_ZF : 0));
        return X_OK;
      }
      if (a == 0) {
        set_flags(m, RF_ZF, RF_ZF);
        return X_OK;
      }
      res = op == 0xbc ? (u64)__builtin_ctzll(a) : (u64)(63 - __builtin_clzll(a));
      setreg(m, d, d->reg, osz, res);
      set_flags(m, RF_ZF, 0);
      return X_OK;
    }
    case 0xc0:
    case 0xc1: { /* xadd */
      const int sz = op == 0xc0 ? 1 : osz;
      CHK(rd_rm_rmw(m, d, sz, &a));
      b = getreg(m, d, d->reg, sz);
      res = alu2(m, 0, a, b, sz);
      /* SDM: TEMP := SRC + DEST; SRC := DEST; DEST := TEMP (xadd r,r keeps the sum) */
      setreg(m, d, d->reg, sz, a);
      if (wr_rm(m, d, sz, res)) return X_FAULT; /* registers are rolled back by the caller */
      return X_OK;
    }
    case 0xc8: case 0xc9: case 0xca: case 0xcb: case 0xcc: case 0xcd: case 0xce: case 0xcf: {
      const u32 r = (op & 7) | (d->rexb << 3);
      if (osz == 8) m->r.gpr[r] = __builtin_bswap64(m->r.gpr[r]);
      else if (osz == 4) setreg(m, d, r, 4, __builtin_bswap32((u32)m->r.gpr[r]));
      else setreg(m, d, r, 2, 0);
      return X_OK;
    }
    default:
      return X_UNIMPL;
    }
  }
  return X_UNIMPL;
}

/* Decode at rip. Returns 0 ok, -1 fetch fault (exit filled), 1 unimplemented encoding. */
static int decode(orc_machine *m, insn *d, memref *mr) {
  memset(d, 0, sizeof(*d));
  memset(mr, 0, sizeof(*mr));
  d->start = m->r.rip;
  d->m32 = (u32)is_m32(m);
  u8 b;
  /* legacy prefixes and REX; a REX not immediately before the opcode is ignored */
  for (;;) {
    b = fetch8(m, d);
    if (d->fetch_fail) return -1;
    if ((b & 0xf0) == 0x40 && !d->m32) {
      d->rex = b;
      continue;
    }
    if (b == 0x66) d->pfx66 = 1;
    else if (b == 0x67) d->pfx67 = 1;
    else if (b == 0xf2 || b == 0xf3) d->rep = b;
    else if (b == 0xf0) d->lock = 1;
    else if (b == 0x64) d->seg = 4;
    else if (b == 0x65) d->seg = 5;
    else if (b == 0x26 || b == 0x2e || b == 0x36 || b == 0x3e) { /* null segments in 64-bit */ }
    else break;
    d->rex = 0;
  }
  if (d->rex) {
    d->rexw = (d->rex >> 3) & 1;
    d->rexr = (d->rex >> 2) & 1;
    d->rexx = (d->rex >> 1) & 1;
    d->rexb = d->rex & 1;
  }
  if (d->m32) { /* 32-bit addresses; 67 would make them 16-bit (outside) */
    d->a16 = d->pfx67;
    d->pfx67 = 1;
  }
  int les = 0; /* 32-bit code: c4 / c5 are les / lds unless the next byte's mod is 11 */
  if (d->m32 && (b == 0xc4 || b == 0xc5)) {
    const u64 save = d->pos;
    const u8 nb = fetch8(m, d);
    if (d->fetch_fail) return -1;
    les = (nb & 0xc0) != 0xc0;
    d->pos = (u32)save;
  }
  zform ezf = {ZK_NONE, 0, 0, 0, 0, 0};
  if (b == 0x62 && !d->m32) { /* EVEX (U47; 32-bit code's bound stays outside) */
    const u8 p0 = fetch8(m, d), p1 = fetch8(m, d), p2 = fetch8(m, d);
    b = fetch8(m, d);
    if (d->fetch_fail) return -1;
    d->vex = d->evex = 1;
    d->vbad = d->pfx66 || d->rep || d->rex || (p0 & 8) || !(p1 & 4);
    d->rexr = !((p0 >> 7) & 1);
    d->rexx = !((p0 >> 6) & 1);
    d->rexb = !((p0 >> 5) & 1);
    d->er2 = !((p0 >> 4) & 1);
    d->opmap = p0 & 7u;
    d->vw = d->rexw = (p1 >> 7) & 1u;
    d->rex = 0x40 | (d->rexw << 3) | (d->rexr << 2) | (d->rexx << 1) | d->rexb;
    d->vvvv = ((~p1 >> 3) & 15u) | ((((u32)~p2 >> 3) & 1u) << 4);
    d->vpp = p1 & 3u;
    d->ez = (p2 >> 7) & 1u;
    d->ell = (p2 >> 5) & 3u;
    d->eb = (p2 >> 4) & 1u;
    d->eaaa = p2 & 7u;
    d->op = b;
    ezf = zform_of(d->opmap, b, (int)d->vpp, d->vw);
    /* maps 1-3 and 5-6 (AVX512-FP16) are defined: outside the subset is UNIMPLEMENTED */
    d->undef = d->vbad || d->opmap == 0 || d->opmap == 4 || d->opmap == 7;
    if (d->undef || d->opmap > 3 || ezf.kind == ZK_NONE) {
      d->len = d->pos;
      return 1;
    }
  } else if ((b == 0xc4 || b == 0xc5) && !les) { /* VEX (always VEX in 64-bit mode) */
    d->vex = 1;
    d->vbad = d->pfx66 || d->rep || d->rex;
    const u8 b1 = fetch8(m, d);
    const u8 b2 = b == 0xc4 ? fetch8(m, d) : b1;
    if (d->fetch_fail) return -1;
    d->rexr = !((b1 >> 7) & 1);
    d->rexx = b == 0xc4 ? !((b1 >> 6) & 1) : 0;
    d->rexb = (b == 0xc4 && !d->m32) ? !((b1 >> 5) & 1) : 0;
    d->opmap = b == 0xc4 ? (b1 & 31u) : 1;
    d->vw = b == 0xc4 ? (b2 >> 7) & 1u : 0;
    d->rexw = d->m32 ? 0 : d->vw; /* a 64-bit GPR operand in 64-bit mode only (32-bit code ignores VEX.W1) */
    d->rex = 0x40 | (d->rexw << 3) | (d->rexr << 2) | (d->rexx << 1) | d->rexb;
    d->vvvv = (~b2 >> 3) & (d->m32 ? 7u : 15u);
    d->vl = (b2 >> 2) & 1u;
    d->vpp = b2 & 3u;
    b = fetch8(m, d);
    if (d->fetch_fail) return -1;
    d->undef = d->vbad || d->opmap < 1 || d->opmap > 3 || !vex_defined(d->opmap, b, (int)d->vpp);
    if (d->opmap != 1 && d->opmap != 2 &&
        !(d->opmap == 3 && !d->undef && (fp_form_o(3, b, (int)d->vpp, 1) || s4_form_o(3, b, (int)d->vpp, 1) ||
                                         x42_form_o(3, b, (int)d->vpp, 1) || gx_form_o(3, b, (int)d->vpp, 1) ||
                                         ax_form_o(3, b, (int)d->vpp, 1) || kop_any(3, b, (int)d->vpp)))) {
      d->op = b;
      d->len = d->pos;
      return 1;
    }
    if (d->undef) {
      d->op = b;
      d->len = d->pos;
      return 1;
    }
  } else if (b == 0x0f) {
    d->opmap = 1;
    b = fetch8(m, d);
    if (d->fetch_fail) return -1;
    if (b == 0x38 || b == 0x3a) {
      d->opmap = b == 0x38 ? 2 : 3;
      d->op = fetch8(m, d);
      if (d->fetch_fail) return -1;
      const int pfx = d->rep == 0xf3 ? 2 : d->rep == 0xf2 ? 3 : d->pfx66 ? 1 : 0;
      /* 0f 38 00 pshufb, 0f 38 17 ptest, the floating-point forms; the rest: outside */
      if ((d->opmap == 3 || (d->op != 0x00 && d->op != 0x17)) && !fp_form_o(d->opmap, d->op, pfx, 0) &&
          !s4_form_o(d->opmap, d->op, pfx, 0) && !x42_form_o(d->opmap, d->op, pfx, 0) &&
          !gx_form_o(d->opmap, d->op, pfx, 0) && !(pfx == 0 && ssse3_mm(d->opmap, d->op))) {
        d->undef = !legacy_3byte_defined(d->opmap, d->op, pfx);
        d->len = d->pos;
        return 1;
      }
      b = d->op;
    }
  }
  d->op = b;
  const int osz = d->rexw ? 8 : (d->pfx66 ? 2 : 4);
  const int izsz = osz == 2 ? 2 : 4;
  int has_modrm = 0, imm = 0;
  if (d->opmap == 0) {
    switch (b) {
    case 0x00: case 0x01: case 0x02: case 0x03: case 0x08: case 0x09: case 0x0a: case 0x0b:
    case 0x10: case 0x11: case 0x12: case 0x13: case 0x18: case 0x19: case 0x1a: case 0x1b:
    case 0x20: case 0x21: case 0x22: case 0x23: case 0x28: case 0x29: case 0x2a: case 0x2b:
    case 0x30: case 0x31: case 0x32: case 0x33: case 0x38: case 0x39: case 0x3a: case 0x3b:
    case 0x63: case 0x84: case 0x85: case 0x86: case 0x87: case 0x88: case 0x89: case 0x8a:
    case 0x8b: case 0x8d: case 0x8f: case 0xd0: case 0xd1: case 0xd2: case 0xd3: case 0xfe:
    case 0xff: case 0x8c: case 0x8e: case 0xd8: case 0xd9: case 0xda: case 0xdb: case 0xdc: case 0xdd:
    case 0xde: case 0xdf:
      has_modrm = 1;
      break;
    case 0xc8:
      imm = 3;
      break;
    case 0xca:
      imm = 2;
      break;
    case 0xcd: case 0xe0: case 0xe1: case 0xe2: case 0xe3: case 0xe4: case 0xe5: case 0xe6: case 0xe7:
      imm = 1;
      break;
    case 0x04: case 0x0c: case 0x14: case 0x1c: case 0x24: case 0x2c: case 0x34: case 0x3c:
    case 0x6a: case 0xa8: case 0xb0: case 0xb1: case 0xb2: case 0xb3: case 0xb4: case 0xb5:
    case 0xb6: case 0xb7: case 0xeb:
    case 0x70: case 0x71: case 0x72: case 0x73: case 0x74: case 0x75: case 0x76: case 0x77:
    case 0x78: case 0x79: case 0x7a: case 0x7b: case 0x7c: case 0x7d: case 0x7e: case 0x7f:
      imm = 1;
      break;
    case 0x05: case 0x0d: case 0x15: case 0x1d: case 0x25: case 0x2d: case 0x35: case 0x3d:
    case 0xa9:
      imm = izsz;
      break;
    case 0x68:
      imm = d->pfx66 ? 2 : 4;
      break;
    case 0xe8: case 0xe9:
      imm = 4;
      break;
    case 0xc2:
      imm = 2;
      break;
    case 0xb8: case 0xb9: case 0xba: case 0xbb: case 0xbc: case 0xbd: case 0xbe: case 0xbf:
      imm = osz;
      break;
    case 0xa0: case 0xa1: case 0xa2: case 0xa3:
      imm = d->pfx67 ? 4 : 8;
      break;
    case 0x69:
      has_modrm = 1;
      imm = izsz;
      break;
    case 0x6b: case 0x80: case 0x83: case 0xc0: case 0xc1: case 0xc6:
      has_modrm = 1;
      imm = 1;
      break;
    case 0x82: /* 32-bit code: 80's alias */
      if (d->m32) has_modrm = imm = 1;
      break;
    case 0x62: case 0xc4: case 0xc5: /* 32-bit code: bound, les / lds (c4 / c5 with mod != 11) */
      if (d->m32) has_modrm = 1;
      break;
    case 0x9a: case 0xea: /* 32-bit code: far call / jmp ptr16:32 */
      if (d->m32) imm = osz + 2;
      break;
    case 0xd4: case 0xd5: /* 32-bit code: aam / aad imm8 */
      if (d->m32) imm = 1;
      break;
    case 0x81: case 0xc7:
      has_modrm = 1;
      imm = izsz;
      break;
    case 0xf6: case 0xf7:
      has_modrm = 1;
      break;
    default:
      break;
    }
  } else {
    if ((b >= 0x40 && b <= 0x4f) || (b >= 0x90 && b <= 0x9f) || b == 0xa3 || b == 0xab ||
        b == 0xb3 || b == 0xbb || b == 0xaf || b == 0xb0 || b == 0xb1 || b == 0xb6 ||
        b == 0xb7 || b == 0xbe || b == 0xbf || b == 0xbc || b == 0xbd || b == 0xb8 ||
        b == 0xc0 || b == 0xc1 || b == 0xa5 || b == 0xad || b == 0x0d || b == 0x01 || b == 0xc7 || b == 0x20 ||
        b == 0x22 || b == 0x00 || b == 0x02 || b == 0x03 || b == 0x21 || b == 0x23 || b == 0xb2 || b == 0xb4 ||
        b == 0xb5 || (b >= 0x18 && b <= 0x1f))
      has_modrm = 1;
    if (d->opmap == 1 && (b == 0xa4 || b == 0xac || b == 0xba)) { /* shld / shrd imm8, group 8 (not 0f 38 ac / ba: FMA3) */
      has_modrm = 1;
      imm = 1;
    }
    if (d->opmap == 1 && b >= 0x80 && b <= 0x8f) imm = 4; /* jcc rel32 (0f 38 8x has none) */
    if (d->opmap == 2) has_modrm = 1;
    else if (d->opmap == 3) has_modrm = imm = 1;
    else {
      if (sse_opcode(b) && b != 0x77) has_modrm = 1;
      if ((b >= 0x70 && b <= 0x73) || b == 0xc2 || (b >= 0xc4 && b <= 0xc6)) imm = 1;
    }
  }
  if (d->evex) {
    has_modrm = 1;
    imm = d->opmap == 3;
  }
  if (has_modrm) {
    decode_modrm(m, d, mr);
    if (d->fetch_fail) return -1;
    if (d->evex) { /* 5-bit registers; disp8 * N */
      d->reg |= d->er2 << 4;
      if (d->mod == 3) d->rm |= d->rexx << 4;
      if (d->mod == 1) mr->disp *= zdisp_n(ezf, 16u << d->ell, d->eb);
    }
  }
  if (d->opmap == 0 && (b == 0xf6 || b == 0xf7) && ((d->reg & 7) <= 1)) imm = b == 0xf6 ? 1 : izsz;
  for (int i = 0; i < imm; i++) {
    fetch8(m, d);
    if (d->fetch_fail) return -1;
  }
  d->len = d->pos;
  finish_ea(m, d, mr);
  return 0;
}

static void fill_exit(orc_machine *m, wtfgpu_exit_t *ex, u32 status) {
  ex->status = status;
  if (status == WTFGPU_EXIT_FAULT) ex->opcode = (u32)cpl(m); /* the privilege level it was raised at */
  ex->rip = m->r.rip;
  ex->icount = m->icount;
}

/* One instruction: fetch, decode, coverage, breakpoint, execute, retire. */
/* ---------------- exception delivery (U18) ----------------
 * A fault is delivered through the guest IDT when the snapshot has a present
 * 64-bit interrupt / trap gate for it (SDM vol. 3 6.12-6.14); otherwise, or
 * for a fault before any instruction retired since the last delivery (a
 * double fault), the machine stops with the fault. Implicit supervisor
 * accesses: no permission checks. Frame words are written lowest first. */
static int has_error_code(u32 v) { return v == 8 || (v >= 10 && v <= 14) || v == 17 || v == 21 || v == 29 || v == 30; }
static int sup_read(orc_machine *m, u64 va, void *out, u32 n) {
  u64 pa;
  if (walk(m, va, ACC_R, 0, &pa)) return -1;
  if ((pa & 0xfff) + n > 4096) return -1;
  memcpy(out, phys_ro(m, pa >> 12) + (pa & 0xfff), n);
  return 0;
}
static int sup_write8(orc_machine *m, u64 va, u64 v) {
  u64 pa;
  if (walk(m, va, ACC_W, 0, &pa)) return -1;
  if ((pa & 0xfff) + 8 > 4096) return -1;
  memcpy(phys_rw(m, pa >> 12) + (pa & 0xfff), &v, 8);
  return 0;
}
static int deliver(orc_machine *m, u32 vec, u32 err, u64 cr2) {
  wtfgpu_exit_t keep = *m->ex;
  const int fk = m->faulted;
  int ok = 0;
  do {
    if (m->deliv_valid && m->deliv_icount == m->icount) break;
    if (!m->r.idtr_base || vec > 31 || (u64)vec * 16 + 15 > m->r.idtr_limit) break;
    u64 g[2];
    if (sup_read(m, m->r.idtr_base + (u64)vec * 16, g, 16)) break;
    const u32 attr = (u32)(g[0] >> 40) & 0xff, type = attr & 0xf, ist = (u32)(g[0] >> 32) & 7;
    if (!(attr & 0x80) || (type != 0xe && type != 0xf)) break;
    const u64 target = (g[0] & 0xffff) | ((g[0] >> 32) & 0xffff0000ULL) | (g[1] << 32);
    const u16 sel = (u16)((g[0] >> 16) & 0xffff);
    const u32 ncpl = sel & 3, ocpl = (u32)cpl(m);
    if (!is_canonical(target) || ncpl > ocpl) break;
    u64 rsp = m->r.gpr[WTFGPU_RSP];
    if (ist || ncpl < ocpl) {
      const u64 off = ist ? 0x24 + (u64)(ist - 1) * 8 : 4 + (u64)ncpl * 8;
      if (sup_read(m, m->r.seg[WTFGPU_TR].base + off, &rsp, 8)) break;
    }
    rsp &= ~0xfULL;
    u64 frame[6];
    u32 n = 0;
    if (has_error_code(vec)) frame[n++] = err;
    frame[n++] = m->r.rip;
    frame[n++] = m->r.seg[WTFGPU_CS].selector;
    frame[n++] = m->r.rflags;
    frame[n++] = m->r.gpr[WTFGPU_RSP];
    frame[n++] = m->r.seg[WTFGPU_SS].selector;
    int wr = 1;
    for (u32 i = 0; i < n && wr; i++) wr = sup_write8(m, rsp - 8 * n + 8 * i, frame[i]) == 0;
    if (!wr) break;
    if (ncpl < ocpl) m->r.seg[WTFGPU_SS].selector = (u16)ncpl;
    m->r.seg[WTFGPU_CS].selector = sel;
    if (vec == WTFGPU_VEC_PF) m->r.cr2 = cr2;
    m->deliv_valid = 1;
    m->deliv_icount = m->icount;
    m->r.gpr[WTFGPU_RSP] = rsp - 8 * n;
    m->r.rflags &= ~(0x100ULL | 0x4000ULL | 0x10000ULL | 0x20000ULL | (type == 0xe ? 0x200ULL : 0));
    m->r.rip = target;
    ok = 1;
  } while (0);
  *m->ex = keep;
  m->faulted = fk;
  return ok;
}

/* Diagnostic: executed instructions by (opcode map, opcode, ModRM reg,
 * memory operand), for the engine's fast-path coverage study
 * (scripts/op_mix.py via WTF_OPHIST on the twin). Process-wide, not thread-safe. */
static u64 g_ophist[4 * 256 * 8 * 2];
static int g_ophist_on = -1;
void orc_ophist(u64 *out, int reset) {
  memcpy(out, g_ophist, sizeof(g_ophist));
  if (reset) memset(g_ophist, 0, sizeof(g_ophist));
}

static void ophist_dump(void) { /* "map opcode reg mem count" lines to $WTF_OPHIST */
  FILE *f = fopen(getenv("WTF_OPHIST"), "w");
  if (!f) return;
  for (size_t i = 0; i < sizeof(g_ophist) / 8; i++)
    if (g_ophist[i]) fprintf(f, "%zu %zu %zu %zu %llu\n", i / 4096, (i / 16) % 256, (i / 2) % 8, i % 2,
                             (unsigned long long)g_ophist[i]);
  fclose(f);
}

static int one(orc_machine *m, int check_bp, wtfgpu_exit_t *ex) {
  insn d;
  memref mr;
  memset(ex, 0, sizeof(*ex));
  m->ex = ex;
  m->faulted = 0;
  int rc = decode(m, &d, &mr);
  if (g_ophist_on < 0) {
    g_ophist_on = getenv("WTF_OPHIST") != NULL;
    if (g_ophist_on) atexit(ophist_dump);
  }
  if (g_ophist_on && rc >= 0)
    g_ophist[(((d.opmap & 3) * 256 + (d.op & 0xff)) * 8 + (d.has_modrm ? (d.reg & 7) : 0)) * 2 + (d.is_mem ? 1 : 0)]++;
  if (rc < 0) {
    if (d.fetch_fail == 2) {
      ex->status = WTFGPU_EXIT_FAULT;
      ex->vector = WTFGPU_VEC_GP;
      ex->error = 0;
      ex->addr = 0;
    }
    fill_exit(m, ex, WTFGPU_EXIT_FAULT);
    if (deliver(m, ex->vector, ex->error, ex->addr)) {
      tn_regs(m);
      return ex->status = WTFGPU_RUNNING;
    }
    return ex->status;
  }
  /* coverage (bochscpu_backend.cc:501-504) then breakpoint lookup (:545-547) */
  if (!hm_has(&m->cov, m->r.rip)) {
    *hm_slot(&m->cov, m->r.rip, 1) = (void *)1;
    vec_push(&m->covlist, m->r.rip);
  }
  if (m->trace && !m->resumed) vec_push(&m->tracelist, m->r.rip); /* bochscpu_backend.cc:506-520 */
  m->resumed = 0;
  if (check_bp && hm_has(&m->bps, m->r.rip)) {
    fill_exit(m, ex, WTFGPU_EXIT_BREAKPOINT);
    return ex->status;
  }
  if (rc == 1 && !d.lock && !d.undef) {
    memcpy(&ex->opcode, d.bytes, 4);
    fill_exit(m, ex, WTFGPU_EXIT_UNIMPLEMENTED);
    return ex->status;
  }
  wtfgpu_regs_t saved = m->r;
  u64 saved_bytes = m->bytes;
  u64 next = 0;
  m->tn_ipos = m->tnlist.n; /* Tenet: this instruction's accesses */
  m->tn_last = ~0ULL;
  m->tn_mute = 0;
  int x = exec_insn(m, &d, &mr, &next);
  if (d.m32 && x == X_OK && is_m32(m)) next &= 0xffffffffULL; /* 32-bit code stays below 4 GiB (U29) */
  /* RecordEdge (bochscpu_backend.cc:699-728, hooks :235-257, :308-312): jcc
   * taken or not, indirect near jmp / call; before the retire hook */
  if (m->edges && x == X_OK &&
      ((d.opmap == 0 && d.op >= 0x70 && d.op <= 0x7f) || (d.opmap == 1 && d.op >= 0x80 && d.op <= 0x8f) ||
       (d.opmap == 0 && !d.vex && d.op >= 0xe0 && d.op <= 0xe3) ||
       (d.opmap == 0 && d.op == 0xff && ((d.reg & 7) == 2 || (d.reg & 7) == 4)))) {
    u64 e = d.start;
    e ^= e >> 30;
    e *= 0xbf58476d1ce4e5b9ULL;
    e ^= e >> 27;
    e *= 0x94d049bb133111ebULL;
    e ^= e >> 31;
    e ^= next;
    m->edges_run++;
    if (!hm_has(&m->cov, e)) {
      *hm_slot(&m->cov, e, 1) = (void *)1;
      vec_push(&m->covlist, e);
      m->edges_new++;
    }
  }
  if (x == X_OK || x == X_CR3) {
    m->r.rip = next;
    m->bytes += d.len;
    m->icount++;
    tn_regs(m);
    /* the limit check of the retire hook runs after the cr3 hook and wins */
    if (m->limit > 0 && m->icount > m->limit) {
      fill_exit(m, ex, WTFGPU_EXIT_TIMEOUT);
      return ex->status;
    }
    if (x == X_CR3) {
      fill_exit(m, ex, WTFGPU_EXIT_CR3);
      return ex->status;
    }
    ex->status = WTFGPU_RUNNING;
    return WTFGPU_RUNNING;
  }
  /* not retired: registers rolled back (memory writes precede register updates),
   * except rep string progress which is architecturally committed */
  if (x == X_FAULT_KEEP) {
    m->r.rip = saved.rip;
    x = X_FAULT;
  } else if (x == X_FAULT_PARTIAL) {
    m->r.rip = saved.rip;
    m->bytes = saved_bytes;
    x = X_FAULT;
  } else {
    m->r = saved;
    m->bytes = saved_bytes;
  }
  m->r.mxcsr |= m->xm_flags; /* a SIMD FP exception keeps the flags it set (U40) */
  m->xm_flags = 0;
  switch (x) {
  case X_FAULT: {
    wtfgpu_exit_t keep = *ex;
    fill_exit(m, ex, WTFGPU_EXIT_FAULT);
    ex->vector = keep.vector;
    ex->error = keep.error;
    ex->addr = keep.addr;
    if (deliver(m, ex->vector, ex->error, ex->addr)) {
      tn_regs(m);
      return ex->status = WTFGPU_RUNNING;
    }
    break;
  }
  case X_UNIMPL:
    memcpy(&ex->opcode, d.bytes, 4);
    fill_exit(m, ex, WTFGPU_EXIT_UNIMPLEMENTED);
    break;
  case X_INT3: fill_exit(m, ex, WTFGPU_EXIT_INT3); break;
  case X_HLT: fill_exit(m, ex, WTFGPU_EXIT_HLT); break;
  default: fill_exit(m, ex, WTFGPU_EXIT_UNIMPLEMENTED); break;
  }
  return ex->status;
}

/* Host-injected exception (PageFaultsMemoryIfNeeded, bochscpu_backend.cc:917-999):
 * delivered through the guest IDT before the next instruction. 1 = delivered. */
int orc_inject_fault(orc_machine *m, uint32_t vector, uint32_t error, uint64_t addr) {
  wtfgpu_exit_t ex;
  memset(&ex, 0, sizeof(ex));
  m->ex = &ex;
  const int d = deliver(m, vector, error, addr);
  if (d) {
    m->tn_ipos = m->tnlist.n;
    tn_regs(m);
  }
  return d;
}

int orc_run(orc_machine *m, int skip_bp, wtfgpu_exit_t *ex) {
  int first = 1;
  if (m->tn && m->tnlist.n == 0) tn_regs(m); /* Tenet: the registers at the start */
  for (;;) {
    m->resumed = first && skip_bp; /* its before-execution hook ran at the hit */
    int st = one(m, !(first && skip_bp), ex);
    first = 0;
    if (st != WTFGPU_RUNNING) {
      if (st != WTFGPU_EXIT_BREAKPOINT && m->tn && m->tnlist.n > m->tn_ipos) tn_regs(m); /* open accesses */
      return st;
    }
  }
}

int orc_step(orc_machine *m, wtfgpu_exit_t *ex) {
  m->resumed = 0;
  return one(m, 0, ex);
}
void orc_set_tenet(orc_machine *m, int on) {
  m->tn = on;
  m->tnlist.n = 0;
  m->tn_ipos = 0;
  m->tn_last = ~0ULL;
}
void orc_tenet_event(orc_machine *m) {
  if (!m->tn) return;
  m->tn_ipos = m->tnlist.n;
  tn_regs(m);
}
uint64_t orc_tenet(orc_machine *m, uint64_t *out, uint64_t cap_words) {
  for (u64 i = 0; i < m->tnlist.n && i < cap_words; i++) out[i] = m->tnlist.v[i];
  return m->tnlist.n;
}
void orc_set_trace(orc_machine *m, int on) {
  m->trace = on;
  m->tracelist.n = 0;
}
uint64_t orc_trace(orc_machine *m, uint64_t *out, uint64_t cap) {
  for (u64 i = 0; i < m->tracelist.n && i < cap; i++) out[i] = m->tracelist.v[i];
  return m->tracelist.n;
}
