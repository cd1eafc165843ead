/*
 * wtfgpu.h — C ABI of the MI355X (gfx950) execution backend for wtf.
 *
 * This is the thin `extern "C"` launch layer that the C++ `GpuBackend_t`
 * (wtf_amd/host/gpu_backend.*) drives, and that a maintainer of upstream wtf
 * would bind from `src/wtf/gpu_backend.cc`. No torch,
 * no fmt, no C++ types cross this boundary: plain pointers, sizes and int
 * status codes (0 = ok, < 0 = error), never exceptions.
 *
 * Each entry point replaces one piece of the reference bochscpu backend
 * (paths relative to the reference tree, m4drat/wtf @ 2025-02-17):
 *
 *   wtfgpu_load_pool          <- BochscpuBackend_t::Initialize + StaticGpaMissingHandler
 *                                (src/wtf/bochscpu_backend.cc:269-335, :36-138): the
 *                                kdmp physical pages become a read-only HBM page pool,
 *                                missing GPAs read as zeros (:124-131).
 *   wtfgpu_set_initial_state  <- BochscpuBackend_t::LoadState (bochscpu_backend.cc:1026-1122)
 *   wtfgpu_restore            <- BochscpuBackend_t::Restore (bochscpu_backend.cc:730-797):
 *                                dirty-list reset of per-lane copy-on-write overlays.
 *   wtfgpu_set_limit          <- BochscpuBackend_t::SetLimit (bochscpu_backend.cc:347-350)
 *   wtfgpu_set_breakpoints    <- BochscpuBackend_t::SetBreakpoint (bochscpu_backend.cc:337-345)
 *   wtfgpu_run                <- BochscpuBackend_t::Run / bochscpu_cpu_run
 *                                (bochscpu_backend.cc:352-410) + the before/after execution,
 *                                lin_access, interrupt, hlt hooks (:445-697).
 *   wtfgpu_read_regs/write_regs, wtfgpu_lane_get_cr/set_cr
 *                             <- Get/SetReg (bochscpu_backend.cc:1124-1190)
 *   wtfgpu_lane_translate     <- VirtTranslate (bochscpu_backend.cc:891-896)
 *   wtfgpu_lane_read_phys/write_phys <- PhysTranslate + memcpy / DirtyGpa
 *                                (bochscpu_backend.cc:887-900, backend.cc:16-127)
 *   wtfgpu_read_dirty         <- DirtyGpas_ (bochscpu_backend.h, RunStats_.DirtyGpas)
 *   wtfgpu_read_coverage      <- AggregatedCodeCoverage_/LastNewCoverage_
 *                                (bochscpu_backend.cc:501-504, :1001-1016)
 *   wtfgpu_commit_coverage    <- AggregatedCodeCoverage_.emplace (bochscpu_backend.cc:501)
 *   wtfgpu_coverage_device_map, wtfgpu_coverage_absorb
 *                             <- the per-GPU coverage bitmap merged with RCCL MAX (new).
 */
#ifndef WTFGPU_H
#define WTFGPU_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WTFGPU_ABI_VERSION 4
#define WTFGPU_PAGE_SIZE 4096u

/* Status codes. */
#define WTFGPU_OK 0
#define WTFGPU_ERR_INVALID (-1)
#define WTFGPU_ERR_NODEV (-2)
#define WTFGPU_ERR_OOM (-3)
#define WTFGPU_ERR_HIP (-4)
#define WTFGPU_ERR_STATE (-5)
#define WTFGPU_ERR_TRANSLATE (-6)

/* Per-lane status / exit reasons. A lane with status RUNNING is runnable. */
enum wtfgpu_status {
  WTFGPU_RUNNING = 0,
  WTFGPU_EXIT_BREAKPOINT = 1, /* before executing the instruction at rip; host services it */
  WTFGPU_EXIT_TIMEOUT = 2,    /* retired count > limit (bochscpu_backend.cc:458-469) */
  WTFGPU_EXIT_INT3 = 3,       /* int3 -> Crash_t() (bochscpu_backend.cc:595-619) */
  WTFGPU_EXIT_HLT = 4,        /* hlt -> Crash_t() (bochscpu_backend.cc:690-697) */
  WTFGPU_EXIT_FAULT = 5,      /* architectural exception raised; vector/error/addr in exit */
  WTFGPU_EXIT_UNIMPLEMENTED = 6, /* opcode outside the engine's ISA subset */
  WTFGPU_EXIT_CR3 = 7,        /* cr3 write != initial cr3 (bochscpu_backend.cc:628-657) */
  WTFGPU_EXIT_OVERLAY_FULL = 8, /* lane ran out of copy-on-write pages */
  WTFGPU_EXIT_STOPPED = 9,    /* host called Stop(); result kept on the host */
  WTFGPU_EXIT_IDLE = 10,      /* lane holds no testcase */
  WTFGPU_EXIT_STOP_OK = 11,   /* a device action stopped the lane with Ok_t() (feed drained, STOP_OK) */
  WTFGPU_EXIT_FEED_FAULT = 12, /* a device FEED action could not write its chunk (engine error) */
  WTFGPU_EXIT_STOP_ARGS = 13   /* a STOP_ARGS action stopped the lane; its arguments: wtfgpu_read_stop_args */
};

/* x86 exception vectors reported in wtfgpu_exit_t.vector. */
#define WTFGPU_VEC_DE 0
#define WTFGPU_VEC_UD 6
#define WTFGPU_VEC_GP 13
#define WTFGPU_VEC_PF 14

/* General purpose register indices (x86 encoding order). */
enum wtfgpu_gpr {
  WTFGPU_RAX = 0, WTFGPU_RCX, WTFGPU_RDX, WTFGPU_RBX, WTFGPU_RSP, WTFGPU_RBP,
  WTFGPU_RSI, WTFGPU_RDI, WTFGPU_R8, WTFGPU_R9, WTFGPU_R10, WTFGPU_R11,
  WTFGPU_R12, WTFGPU_R13, WTFGPU_R14, WTFGPU_R15
};

/* Segment register indices in wtfgpu_regs_t.seg. */
enum wtfgpu_segidx { WTFGPU_ES = 0, WTFGPU_CS, WTFGPU_SS, WTFGPU_DS, WTFGPU_FS, WTFGPU_GS,
                  WTFGPU_TR, WTFGPU_LDTR };

typedef struct wtfgpu_seg {
  uint64_t base;
  uint32_t limit;
  uint16_t selector;
  uint16_t attr;
  uint8_t present;
  uint8_t pad[7];
} wtfgpu_seg_t;

/*
 * Architectural state of one lane (= one testcase). Mirrors CpuState_t
 * (src/wtf/globals.h:1020-1082) for the fields the engine models.
 */
typedef struct wtfgpu_regs {
  uint64_t gpr[16];
  uint64_t rip;
  uint64_t rflags;
  uint64_t cr0, cr2, cr3, cr4, cr8;
  uint64_t efer;
  uint64_t xcr0;
  uint64_t kernel_gs_base;
  uint64_t star, lstar, cstar, sfmask;
  uint64_t tsc, tsc_aux, apic_base, pat;
  uint64_t sysenter_cs, sysenter_eip, sysenter_esp;
  wtfgpu_seg_t seg[8]; /* es cs ss ds fs gs tr ldtr; fs/gs .base are the 64-bit bases */
  uint64_t gdtr_base, idtr_base;
  uint32_t gdtr_limit, idtr_limit;
  uint32_t mxcsr, mxcsr_mask;
  uint16_t fpcw, fpsw, fptw, fpop;
  uint32_t pad0;
  uint64_t fpst[8];
  uint64_t xmm[16][2];  /* bits 127:0 of ymm0..15 */
  uint64_t ymmh[16][2]; /* bits 255:128 (CpuState_t::Zmm[i].Q[2..3]) */
  uint16_t fpse[8];     /* sign / exponent words of ST(0..7) (ABI 3): CpuState_t::Fpst
                           carries the 64-bit significands only (globals.h:1067), so a
                           snapshot loads these as 0 */
  /* AVX-512 state (ABI 4; CpuState_t::Zmm[32], globals.h:1061-1062, bochscpu.hpp
   * State::zmm): bits 511:256 of zmm0..15, zmm16..31 whole, and the opmask
   * registers k0..k7 (bochs keeps these in its CPU; CpuState_t has none, so a
   * restore zeroes them). */
  uint64_t zmmh[16][4];   /* bits 511:256 of zmm0..15 (CpuState_t::Zmm[i].Q[4..7]) */
  uint64_t zmm_hi[16][8]; /* zmm16..31 (CpuState_t::Zmm[16..31]) */
  uint64_t k[8];          /* k0..k7 */
} wtfgpu_regs_t;

/* Why a lane stopped. */
typedef struct wtfgpu_exit {
  uint32_t status;   /* enum wtfgpu_status */
  uint32_t vector;   /* FAULT: exception vector */
  uint32_t error;    /* FAULT: error code (#PF bits as in backend.h PfError_t) */
  uint32_t opcode;   /* UNIMPLEMENTED: first opcode bytes, little endian; FAULT: CPL at the fault */
  uint64_t addr;     /* FAULT #PF: faulting linear address (cr2) */
  uint64_t rip;      /* rip at exit */
  uint64_t icount;   /* instructions retired by this testcase so far */
} wtfgpu_exit_t;

typedef struct wtfgpu_run_stats {
  uint64_t kernel_launches;
  uint64_t group_steps;    /* wave-level decode+execute iterations */
  uint64_t lane_retired;   /* instructions retired by all lanes */
  double kernel_ms;        /* device time measured with HIP events */
} wtfgpu_run_stats_t;

typedef struct wtfgpu_ctx wtfgpu_ctx;

/* Device / context. */
int wtfgpu_abi_version(void);
int wtfgpu_device_count(void);
int wtfgpu_create(int device, wtfgpu_ctx **out);
int wtfgpu_destroy(wtfgpu_ctx *ctx);
/* The HIP stream the context launches on (hipStream_t, as void*): the
 * current queue's. */
void *wtfgpu_stream(wtfgpu_ctx *ctx);
/* Queues (no bochscpu counterpart: host/GPU overlap). Every later call is
 * issued on queue `queue` (0 or 1) until the next selection: its own stream
 * and staging scratch, so a slice queued with wtfgpu_run_async on one queue
 * runs while the host services lanes on the other. Lane sets driven through
 * different queues must be disjoint. */
int wtfgpu_select_queue(wtfgpu_ctx *ctx, uint32_t queue);

/* Snapshot physical memory: npages pages of 4096 bytes, page i backs gpfns[i]. */
int wtfgpu_load_pool(wtfgpu_ctx *ctx, const uint64_t *gpfns, const uint8_t *pages,
                     uint64_t npages);

/* Allocate lane storage. overlay_pages: copy-on-write pages per lane;
 * cov_entries: per-lane new-coverage set capacity (power of two; 3/4 usable). */
int wtfgpu_alloc_lanes(wtfgpu_ctx *ctx, uint32_t nlanes, uint32_t overlay_pages,
                       uint32_t cov_entries);
uint32_t wtfgpu_lane_count(wtfgpu_ctx *ctx);

int wtfgpu_set_initial_state(wtfgpu_ctx *ctx, const wtfgpu_regs_t *regs);
int wtfgpu_set_limit(wtfgpu_ctx *ctx, uint64_t limit);
/* Cross-wave regrouping (no bochscpu counterpart: the SIMT schedule only):
 * wtfgpu_run splits its wave-steps into k_run launches of `steps`, and before
 * each one the running lanes are sorted by rip so that lanes at one rip share
 * a wave. 0 = fixed lane order. Results are identical either way. Unless
 * WTFGPU_REGROUP_AUTO=0, each run picks regrouping or the fixed order from
 * measurements of both (probing the other every 32nd run): sliced runs by
 * lanes retired per wave-step (counts only: fixed-seed campaigns reproduce),
 * runs to completion (max_steps >= 2^32) by kernel time per retired
 * instruction. */
int wtfgpu_set_regroup(wtfgpu_ctx *ctx, uint64_t steps);
int wtfgpu_set_breakpoints(wtfgpu_ctx *ctx, const uint64_t *gvas, uint32_t n);

/* Device-side breakpoint actions (new; no bochscpu counterpart). A breakpoint
 * whose handler only moves registers — a Backend_t handler that is
 * SimulateReturnFromFunction(value) (backend.cc:129-146), or one that loads a
 * fixed GPR set + rip (fuzzer_tlv_server.cc:171-179) — can be declared as
 * data; the lane then applies it inside wtfgpu_run and keeps running instead
 * of exiting to the host. The hooked instruction is cancelled as for a host
 * handler that moves rip (U10); a lane whose action fails (the return address
 * does not translate) exits with WTFGPU_EXIT_BREAKPOINT and the host handler
 * runs. Actions apply only at gvas also passed to wtfgpu_set_breakpoints. */
enum wtfgpu_bp_action_kind {
  WTFGPU_BPACT_HOST = 0,           /* exit to the host (default) */
  /* rax = value; rip = [rsp]; rsp += 8. gprs[0] != 0: the handler first reads
   * a C string at gpr[gprs[0] - 1] (at most gprs[1] bytes, VirtReadString):
   * a byte before its terminator that does not translate leaves the hit to
   * the host handler. */
  WTFGPU_BPACT_RETURN = 1,
  WTFGPU_BPACT_SET_GPRS = 2,       /* gprs[0..15] (WTFGPU_RAX order), rip = gprs[16] */
  /* Pop the lane's next feed chunk (wtfgpu_set_feed): none left, or a chunk of
   * `value` bytes or more -> the lane stops with WTFGPU_EXIT_STOP_OK; else the
   * chunk is written (dirty) so that it ends at gpr[b] + value, then gpr[b] =
   * its address and gpr[n] = its size, b = gprs[0], n = gprs[1]; rip is kept
   * and the hooked instruction runs (fuzzer_tlv_server.cc:83-166). A lane
   * without a feed exits to the host handler. */
  WTFGPU_BPACT_FEED = 3,
  /* gpr[gprs[0]] = Rdrand(): the lane's BLAKE3 chain (h = blake3(le64(seed))
   * [0..16), seed = h[0..8), value = h[8..16); bochscpu_backend.cc:874-885),
   * seed reset to the initial state's at restore; rip is kept and the hooked
   * instruction runs (fuzzer_hevd.cc:96-108). */
  WTFGPU_BPACT_RDRAND = 4,
  /* Stop(Ok_t()): the lane exits with WTFGPU_EXIT_STOP_OK (a handler that
   * only ends the testcase, fuzzer_hevd.cc:64-73) */
  WTFGPU_BPACT_STOP_OK = 5,
  /* A handler that ends the testcase with a result computed from the hooked
   * function's arguments (nt!KeBugCheck2 -> Crash_t("crash-<code>-<p0>..."),
   * fuzzer_hevd.cc:114-128): the lane's first `value` (<= 6) Win64 arguments
   * (rcx, rdx, r8, r9, [rsp+0x28], [rsp+0x30]; GetArg, backend.cc:168-192)
   * are kept for wtfgpu_read_stop_args and the lane exits with
   * WTFGPU_EXIT_STOP_ARGS at the breakpoint's rip; a stack argument that does
   * not translate leaves the hit to the host handler. */
  WTFGPU_BPACT_STOP_ARGS = 6,
};
typedef struct wtfgpu_bp_action {
  uint64_t gva;
  uint32_t kind;
  uint32_t pad;
  uint64_t value;
  uint64_t gprs[17];
} wtfgpu_bp_action_t;
int wtfgpu_set_breakpoint_actions(wtfgpu_ctx *ctx, const wtfgpu_bp_action_t *acts, uint32_t n);
/* The Rdrand seeds of a lane list (BochscpuBackend_t::Seed_): read into
 * seeds[i], or written from it (write != 0), so host handlers and the device
 * action share one chain. Restore resets them to the initial seed. */
int wtfgpu_lane_seeds(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, uint64_t *seeds, int write);
/* The arguments a STOP_ARGS action kept: 6 u64 per lane of the list (lanes
 * whose last exit is WTFGPU_EXIT_STOP_ARGS). */
int wtfgpu_read_stop_args(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, uint64_t *out6);
/* Per-lane input feed of lanes [first, first+count): lane first+i owns
 * bytes[offsets[i] .. offsets[i+1]) (count+1 non-decreasing offsets), a
 * sequence of chunks each stored as a little-endian u32 size and that many
 * bytes. has_feed[i] == 0 means "no feed" for that lane: its FEED hits go to
 * the host (has_feed NULL = every lane has one). The bytes replace any earlier
 * feed of the context; wtfgpu_restore leaves the feed in place. */
int wtfgpu_set_feed(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, const uint64_t *offsets,
                    const uint8_t *has_feed, const uint8_t *bytes, uint64_t nbytes);

/* Declared insert (no bochscpu counterpart; the data form of an
 * InsertTestcase that only moves the testcase into registers and guest memory,
 * fuzzer_hevd.cc:20-59). Once set (NULL: none), every feed upload
 * (wtfgpu_set_feed, wtfgpu_set_feed_lanes) also inserts the feed of each lane
 * that has one and is RUNNING, before it runs: the feed's first chunk is the
 * testcase; its first 4 bytes (u32, zero-extended) go to gpr[head_reg], the
 * rest (the payload) is written at gpr[ptr_reg] (dirty; as Backend_t::
 * VirtWriteDirty: supervisor stores, only a missing translation fails), its
 * size goes to gpr[len_reg] and, when len_arg != 0, as a u64 to
 * rsp + 8 + 8 * len_arg (GetArgAddress(len_arg), backend.cc:160-168). A write
 * that fails ends the lane with WTFGPU_EXIT_FEED_FAULT (an engine error, as
 * the module's failed VirtWrite). The feed is consumed. Chunks shorter than 4
 * bytes are left alone. */
typedef struct wtfgpu_insert {
  uint32_t head_reg;
  uint32_t ptr_reg;
  uint32_t len_reg;
  uint32_t len_arg;
} wtfgpu_insert_t;
int wtfgpu_set_insert(wtfgpu_ctx *ctx, const wtfgpu_insert_t *ins);

/* Coverage index space: code pages (gva >> 12) that get a 4096-byte slot in
 * the per-GPU coverage map. Pages outside it are still logged per lane. */
int wtfgpu_set_code_pages(wtfgpu_ctx *ctx, const uint64_t *vpns, uint32_t n);

/* Reset lanes [first, first+count) to the initial state: registers, dirty
 * overlays dropped, retired count 0, coverage logs cleared, status RUNNING. */
int wtfgpu_restore(wtfgpu_ctx *ctx, uint32_t first, uint32_t count);

/* Streaming (continuous batching: lanes are slots refilled as their
 * testcases finish; the same reset as wtfgpu_restore for a lane list). The
 * lanes' coverage-log bits must have been collected with
 * wtfgpu_collect_coverage_lanes first. */
int wtfgpu_restore_lanes(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n);
/* Feeds of a lane list, each in a fixed per-lane region (running lanes keep
 * theirs): lane lanes[i] gets bytes[offsets[i] .. offsets[i+1]); has_feed[i]
 * == 0, or a feed larger than the region, sends that lane's FEED hits to the
 * host handler. Asynchronous on the current queue: `bytes` (pinned memory,
 * wtfgpu_host_alloc, for a DMA) must stay unchanged until the queue's next
 * synchronising call (wtfgpu_run_wait, or any call that returns data). */
int wtfgpu_set_feed_lanes(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, const uint64_t *offsets,
                          const uint8_t *has_feed, const uint8_t *bytes, uint64_t nbytes);
/* New-coverage sets of a lane list (as wtfgpu_read_coverage); a call whose
 * cap covers the count also empties those lanes' sets (cap = 0 with an empty
 * result included). */
int wtfgpu_collect_coverage_lanes(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, uint32_t *out_lanes,
                                  uint64_t *out_rips, uint64_t cap, uint64_t *total, uint32_t *overflow);

/* Bulk register I/O for lanes [first, first+count). */
int wtfgpu_read_regs(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, wtfgpu_regs_t *out);
int wtfgpu_write_regs(wtfgpu_ctx *ctx, uint32_t first, uint32_t count,
                      const wtfgpu_regs_t *in);
/* Only the 16 GPRs + rip + rflags (18 u64 per lane, that order). */
int wtfgpu_read_gprs(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint64_t *out18);
int wtfgpu_write_gprs(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, const uint64_t *in18);

int wtfgpu_read_exits(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, wtfgpu_exit_t *out);
/* Set lanes back to RUNNING. skip_bp != 0: the breakpoint at the current rip
 * is not re-triggered (the handler returned without moving rip). */
int wtfgpu_resume(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, const uint8_t *skip_bp);
/* Mark lanes stopped (host-side Stop()). */
int wtfgpu_stop(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, uint32_t status);

/* Run every RUNNING lane in [first, first+count) until it exits or
 * max_steps wave-steps elapse. Blocking. */
int wtfgpu_run(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint64_t max_steps,
               wtfgpu_run_stats_t *stats);
/* The same for exactly max_steps wave-steps (<= 2^32), queued on the current
 * queue and returning at once; wtfgpu_run_wait blocks until it is done and
 * returns its statistics. One run in flight per queue. */
int wtfgpu_run_async(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint64_t max_steps);
int wtfgpu_run_wait(wtfgpu_ctx *ctx, wtfgpu_run_stats_t *stats);

/* Asynchronous plumbing. The calls that only change lane state
 * (wtfgpu_restore_lanes, wtfgpu_stop, wtfgpu_resume, wtfgpu_set_feed_lanes,
 * wtfgpu_clear_coverage_lanes) are queued on the current queue and return at
 * once: they are ordered before the queue's later work, and
 * wtfgpu_select_queue orders the next queue's work after them. (A
 * synchronous call would wait until the other queue's k_run left a compute
 * unit free, which is at its next launch boundary.)
 *
 * A slice's read-back, queued right after wtfgpu_run_async and complete when
 * wtfgpu_run_wait returns (replaces wtfgpu_read_exits / _read_bytes /
 * _read_dirty_counts / _read_stop_args for the range; every host pointer
 * pinned, wtfgpu_host_alloc): exits[count] as wtfgpu_read_exits; optional
 * bytes[count], dirty[count], stop_args[6 * count] (every lane's six kept
 * arguments, meaningful for WTFGPU_EXIT_STOP_ARGS). Replaces the
 * bochscpu_cpu_run return path's per-testcase state reads
 * (bochscpu_backend.cc:388-410). */
int wtfgpu_prefetch_results(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, wtfgpu_exit_t *exits,
                            uint64_t *bytes, uint32_t *dirty, uint64_t *stop_args);
/* The new-coverage sets of the range's stopped lanes (status neither RUNNING
 * nor IDLE), gathered after the slice: hdr[0] = entries, hdr[1] & 1 = a set
 * overflowed (pinned hdr[2], valid after wtfgpu_run_wait);
 * wtfgpu_prefetched_coverage then copies the first n <= 2^22 (lane, rip)
 * entries (more entries than that: read the sets with
 * wtfgpu_collect_coverage_lanes). WTFGPU_ERR_STATE when coverage is off.
 * The sets are not emptied (wtfgpu_clear_coverage_lanes, or the restore). */
int wtfgpu_prefetch_coverage(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint64_t *hdr);
int wtfgpu_prefetched_coverage(wtfgpu_ctx *ctx, uint32_t *out_lanes, uint64_t *out_rips, uint64_t n);
int wtfgpu_clear_coverage_lanes(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n);

/* Per-lane memory. gva translation uses the lane's cr3 and its overlays. */
int wtfgpu_lane_translate(wtfgpu_ctx *ctx, uint32_t lane, uint64_t gva, uint64_t *gpa);
int wtfgpu_lane_read_phys(wtfgpu_ctx *ctx, uint32_t lane, uint64_t gpa, void *buf, uint64_t len);
/* Writes are copy-on-write into the lane overlay and dirty the page. */
int wtfgpu_lane_write_phys(wtfgpu_ctx *ctx, uint32_t lane, uint64_t gpa, const void *buf,
                           uint64_t len);
int wtfgpu_lane_read_virt(wtfgpu_ctx *ctx, uint32_t lane, uint64_t gva, void *buf, uint64_t len);
int wtfgpu_lane_write_virt(wtfgpu_ctx *ctx, uint32_t lane, uint64_t gva, const void *buf,
                           uint64_t len);

/* Batched guest-memory writes, one record per (lane, gva, len); data packed
 * back to back in `data` at `data_off`. Copy-on-write + dirty per lane. */
typedef struct wtfgpu_write {
  uint32_t lane;
  uint32_t len;
  uint64_t gva;
  uint64_t data_off;
} wtfgpu_write_t;
int wtfgpu_apply_writes(wtfgpu_ctx *ctx, const wtfgpu_write_t *writes, uint32_t n,
                        const uint8_t *data, uint64_t data_len, int32_t *status_out);

/* Same, with gva read as a guest physical address (PhysWrite, backend.cc:16-28). */
int wtfgpu_apply_phys_writes(wtfgpu_ctx *ctx, const wtfgpu_write_t *writes, uint32_t n, const uint8_t *data,
                             uint64_t data_len, int32_t *status_out);

/* Bulk services for breakpoint handling of many lanes per round trip
 * (the batched form of Get/SetReg and of the dirty-page and PhysTranslate views,
 * bochscpu_backend.cc:1124-1190, :887-900):
 * gprs + rip + rflags (18 u64 per lane) of a lane list, read / written;
 * dirty lists: out[i * (overlay_pages + 1)] = count, then the gpfns;
 * pages: the lane's current view of each (lane, gpa) page, 4096 bytes each. */
int wtfgpu_read_gprs_list(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, uint64_t *out18);
int wtfgpu_write_gprs_list(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, const uint64_t *in18);
int wtfgpu_read_dirty_list(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, uint32_t *out);
uint32_t wtfgpu_overlay_pages(wtfgpu_ctx *ctx);
int wtfgpu_gather_pages(wtfgpu_ctx *ctx, const uint32_t *lanes, const uint64_t *gpas, uint32_t n, uint8_t *out);

/* `len` bytes (<= 256) at each (lane, gpa) of the lanes' current views; each
 * range stays within one page. Sub-page prefetch of what handlers read (the
 * return address / stack arguments), instead of whole pages. */
int wtfgpu_gather_bytes(wtfgpu_ctx *ctx, const uint32_t *lanes, const uint64_t *gpas, uint32_t n, uint32_t len,
                        uint8_t *out);

/* Inject an exception into each lane (PageFaultsMemoryIfNeeded,
 * bochscpu_backend.cc:917-999): delivered through the guest IDT now (cr2 :=
 * addrs[i] for #PF); the lane resumes at the handler. delivered[i] = 0 when the
 * snapshot has no usable gate (the lane is left as it was). */
int wtfgpu_inject_fault(wtfgpu_ctx *ctx, const uint32_t *lanes, uint32_t n, uint32_t vector, uint32_t error,
                        const uint64_t *addrs, int32_t *delivered);

/* A lane's cr2 / cr3 (cr = 2 or 3): GetReg / SetReg(Registers_t::Cr2 / Cr3)
 * (bochscpu_backend.cc:1124-1190). cr2 is the lane's, as last written by an
 * exception delivered through the guest IDT; a cr3 written here is the lane's
 * page-table root from its next run on. */
int wtfgpu_lane_get_cr(wtfgpu_ctx *ctx, uint32_t lane, uint32_t cr, uint64_t *value);
int wtfgpu_lane_set_cr(wtfgpu_ctx *ctx, uint32_t lane, uint32_t cr, uint64_t value);

/* Page-locked host memory (for gather/scatter staging buffers). */
int wtfgpu_host_alloc(wtfgpu_ctx *ctx, uint64_t bytes, void **out);
int wtfgpu_host_free(wtfgpu_ctx *ctx, void *p);

/* Dirty GPAs (page aligned) of one lane; *n gets the count (may exceed cap). */
int wtfgpu_read_dirty(wtfgpu_ctx *ctx, uint32_t lane, uint64_t *gpas, uint32_t cap, uint32_t *n);

/* New-coverage sets: RIPs executed by lanes [first, first+count) that were
 * absent from the coverage map when executed. Writes up to cap (lane, rip)
 * pairs; *n gets the total. *overflow != 0 if a lane's set filled up. */
int wtfgpu_read_coverage(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint32_t *lanes,
                         uint64_t *rips, uint64_t cap, uint64_t *n, uint32_t *overflow);
/* Add RIPs to the coverage map (aggregate coverage). */
int wtfgpu_commit_coverage(wtfgpu_ctx *ctx, const uint64_t *rips, uint64_t n);
int wtfgpu_reset_coverage(wtfgpu_ctx *ctx);
/* Edge coverage (--edges; RecordEdge, bochscpu_backend.cc:699-728): every
 * conditional near branch (taken or not) and indirect near jmp / call adds
 * splitmix64_finaliser(rip) ^ next_rip to the coverage values, next to the
 * rips. Values outside code pages (edges, rips elsewhere) live in a per-GPU
 * set that wtfgpu_commit_coverage grows; they are not part of the RCCL map. */
int wtfgpu_set_edges(wtfgpu_ctx *ctx, int on);
/* Rip traces (`wtf run --trace-type rip`, BochscpuBackend_t::SetTraceFile /
 * BeforeExecutionHook, bochscpu_backend.cc:506-520, :799-815): every lane logs
 * the rips it is about to execute, up to per_lane of them (0 = off), reset by
 * restore. wtfgpu_read_trace copies min(count, per_lane, cap) rips of a lane;
 * *n gets the count (larger than per_lane: the trace was truncated). */
int wtfgpu_set_trace(wtfgpu_ctx *ctx, uint32_t per_lane);
int wtfgpu_read_trace(wtfgpu_ctx *ctx, uint32_t lane, uint64_t *rips, uint64_t cap, uint64_t *n);

/* Tenet traces (`wtf run --trace-type tenet`, BochscpuBackend_t::DumpTenetDelta,
 * bochscpu_backend.cc:1215-1323): per lane a stream of bytes_per_lane bytes of
 * 8-byte-aligned entries (0 turns tracing off):
 *   ACC  {u64 va; u64 meta = 1 << 56 | type << 32 | len; data (len bytes,
 *        rounded up to 8)}: one data access of an instruction, type 1 read,
 *        2 write, 3 read-modify-write; data = the memory after the instruction;
 *   REGS {u64 meta = 2 << 56; u64 gpr[16] (rax, rcx, ... r15); u64 rip}: the
 *        registers at the start, after each retired instruction, delivered
 *        exception, breakpoint action or handler that moved rip, and when the
 *        lane stops with accesses open.
 * The stream restarts at restore. wtfgpu_read_tenet copies min(bytes, per_lane,
 * cap) bytes of a lane; *n gets the bytes written (past per_lane: truncated). */
int wtfgpu_set_tenet(wtfgpu_ctx *ctx, uint64_t bytes_per_lane);
int wtfgpu_read_tenet(wtfgpu_ctx *ctx, uint32_t lane, uint8_t *buf, uint64_t cap, uint64_t *n);
/* Device pointer + size of the uint8 coverage map (for an RCCL MAX all-reduce). */
int wtfgpu_coverage_device_map(wtfgpu_ctx *ctx, void **dev_ptr, uint64_t *bytes);
/* After a MAX all-reduce of the map (other shards' coverage merged in): the
 * RIPs set in the map since the last absorb, excluding this context's own
 * wtfgpu_commit_coverage calls, sorted; *n gets the count. cap = 0 only
 * counts; a call with cap >= that count also marks them seen. */
int wtfgpu_coverage_absorb(wtfgpu_ctx *ctx, uint64_t *rips, uint64_t cap, uint64_t *n);
/* MAX a device buffer of the map's size (another shard set's merged map,
 * RCCL all-reduce result) into the coverage map; wtfgpu_coverage_absorb then
 * reports what it added. Returns when done. */
int wtfgpu_coverage_merge_in(wtfgpu_ctx *ctx, const void *dev_src, uint64_t bytes);
/* Host copy of the coverage map's set bytes as RIPs. */
int wtfgpu_coverage_rips(wtfgpu_ctx *ctx, uint64_t *rips, uint64_t cap, uint64_t *n);

/* Per-lane algorithmic byte counters (ilen + data bytes read/written),
 * for the roofline numerator. */
int wtfgpu_read_bytes(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint64_t *out);
/* Per-lane dirty (copy-on-write) page counts: the 2 x 4096 bytes per dirty
 * page of the reference's restore memcpy in B_exec. */
int wtfgpu_read_dirty_counts(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint32_t *out);
/* With edges on (wtfgpu_set_edges): per lane of [first, first+count) two
 * counts, RecordEdge calls of its testcase and those whose edge was new to its
 * coverage set (BochscpuRunStats_t::NumberEdges / NumberUniqueEdges,
 * bochscpu_backend.h:17-45); zeros with edges off. Reset by restore. */
int wtfgpu_read_edge_counts(wtfgpu_ctx *ctx, uint32_t first, uint32_t count, uint32_t *out2);

#ifdef __cplusplus
}
#endif
#endif /* WTFGPU_H */
