/*
 * x86_oracle.h — CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle / "C++ twin" of SURVEY.md §7 step 2: a plain, scalar
 * x86-64 interpreter plus the wtf hook semantics that the reference bochscpu
 * backend layers on top of the (absent) bochscpu core:
 *   - coverage = every unique rip seen before execution   (bochscpu_backend.cc:476-504)
 *   - breakpoints looked up after the coverage insert      (bochscpu_backend.cc:545-547)
 *   - retired count, timeout when count > limit            (bochscpu_backend.cc:445-470)
 *   - write / read-modify-write accesses dirty 4K GPAs     (bochscpu_backend.cc:550-593)
 *   - missing physical pages read as zero                  (bochscpu_backend.cc:124-131)
 *   - restore = drop dirty pages, reload registers         (bochscpu_backend.cc:730-797)
 *   - int3 / hlt -> crash, cr3 change -> cr3               (bochscpu_backend.cc:595-697)
 * x86 semantics follow the Intel SDM; the page walk follows kdmp-parser.h:269-345
 * and kvm_backend.cc:1937-1998 plus the SDM's permission rules.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (wtf_amd/) never links or calls this code.
 *
 * Parity pin: bochscpu itself is unbuildable here, so this oracle is
 * pinned by native-execution golden vectors generated on the x86-64 host
 * (tests/golden/gen_native_vectors.py) — "parity vs bochscpu unpinned" (SURVEY H1).
 */
#ifndef X86_ORACLE_H
#define X86_ORACLE_H
#include "../include/wtfgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_machine orc_machine;

orc_machine *orc_create(void);
void orc_destroy(orc_machine *m);
/* Snapshot page (copied). */
int orc_add_page(orc_machine *m, uint64_t gpfn, const uint8_t *page);
void orc_set_regs(orc_machine *m, const wtfgpu_regs_t *r);
void orc_get_regs(orc_machine *m, wtfgpu_regs_t *r);
void orc_set_limit(orc_machine *m, uint64_t limit);
/* Edge coverage (--edges): jcc and indirect jmp / call add
 * splitmix64_finaliser(rip) ^ next_rip to the coverage (RecordEdge,
 * bochscpu_backend.cc:699-728). */
void orc_set_edges(orc_machine *m, int on);
/* Rip trace (--trace-type rip, bochscpu_backend.cc:506-520): the rips about to
 * execute, in order, since the last restore (a resumed breakpoint is logged
 * once). orc_trace copies up to cap of them and returns the count. */
/* Tenet trace (U38): the stream wtfgpu_set_tenet documents, as u64 words;
 * orc_tenet_event appends a REGS entry (a handler moved rip); orc_tenet copies
 * up to cap words and returns the count. Restarts at orc_restore. */
void orc_set_tenet(orc_machine *m, int on);
void orc_tenet_event(orc_machine *m);
uint64_t orc_tenet(orc_machine *m, uint64_t *out, uint64_t cap_words);
void orc_set_trace(orc_machine *m, int on);
uint64_t orc_trace(orc_machine *m, uint64_t *out, uint64_t cap);
int orc_set_breakpoints(orc_machine *m, const uint64_t *gvas, uint32_t n);
/* Restore: drop overlays, reload registers, zero counters and coverage. */
void orc_restore(orc_machine *m, const wtfgpu_regs_t *r);
/* Run until an exit. skip_bp: do not trigger the breakpoint at the current rip once. */
int orc_inject_fault(orc_machine *m, uint32_t vector, uint32_t error, uint64_t addr);
int orc_run(orc_machine *m, int skip_bp, wtfgpu_exit_t *exit);
/* Execute exactly one instruction (no breakpoint check); returns status. */
int orc_step(orc_machine *m, wtfgpu_exit_t *exit);
/* Diagnostic (WTF_OPHIST set): executed instructions counted by
 * ((map * 256 + opcode) * 8 + ModRM.reg) * 2 + memory operand; out holds 16384
 * counters. */
void orc_ophist(uint64_t *out, int reset);
uint64_t orc_icount(orc_machine *m);
uint64_t orc_bytes(orc_machine *m);
/* RecordEdge calls of the current testcase; *unique: those whose edge was new to its coverage set */
uint64_t orc_edges(orc_machine *m, uint64_t *unique);
/* Unique rips executed since the last restore, in first-execution order. */
uint64_t orc_coverage(orc_machine *m, uint64_t *out, uint64_t cap);
/* Dirty (copy-on-write) GPAs since the last restore, in first-write order. */
uint64_t orc_dirty(orc_machine *m, uint64_t *out, uint64_t cap);
/* Memory helpers for host-side handlers (no permission checks, like
 * bochscpu_mem_virt_translate). Return 0 on success. */
int orc_translate(orc_machine *m, uint64_t gva, uint64_t *gpa);
int orc_read_phys(orc_machine *m, uint64_t gpa, void *buf, uint64_t len);
int orc_write_phys(orc_machine *m, uint64_t gpa, const void *buf, uint64_t len);
int orc_read_virt(orc_machine *m, uint64_t gva, void *buf, uint64_t len);
int orc_write_virt(orc_machine *m, uint64_t gva, const void *buf, uint64_t len);

#ifdef __cplusplus
}
#endif
#endif
