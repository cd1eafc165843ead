/*
 * wtfnode.h — C ABI of one wtf fuzzing node on one MI355X (libwtfnode.so).
 *
 * A node is the batched form of the reference's client loop with its master
 * in process: src/wtf/client.cc:187-258 (receive -> RunTestcaseAndRestore ->
 * send) fed by src/wtf/server.h:629-886 (corpus, mutator, new-coverage and
 * crash bookkeeping), N testcases per step instead of one, over the gpu
 * Backend_t (include/wtfgpu.h). One step = one batch: mutate (overlapped with
 * the previous batch), InsertTestcase per lane, run on the GPU with
 * breakpoints serviced, coverage attributed in lane order, Target.Restore,
 * and, for world > 1, the RCCL MAX merge of every shard's coverage map
 * (SURVEY 8(e)). Shard r of n mutates with seed + r.
 *
 * Plain C: a host in any language drives it (bench.py uses ctypes). Status
 * codes: 0 = ok, < 0 = error.
 */
#ifndef WTFNODE_H
#define WTFNODE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WTFNODE_RCCL_ID_BYTES 128

typedef struct wtfnode wtfnode;

typedef struct wtfnode_opts {
  const char *name;         /* fuzzer module: "tlv_server", "hevd" (targets.h registry) */
  const char *target;       /* target dir: state/{mem.dmp,regs.json,symbol-store.json}, inputs/, outputs/, crashes/ */
  uint32_t lanes;           /* testcases per batch */
  uint32_t overlay_pages;   /* copy-on-write pages per lane */
  uint64_t limit;           /* instruction limit per testcase (--limit) */
  uint64_t seed;            /* master seed (--seed); shard r uses seed + r */
  uint64_t max_len;         /* testcase size cap (--max_len) */
  int32_t device;           /* HIP device */
  int32_t rank, world;      /* shard rank of world; world 1 = alone */
  const uint8_t *rccl_id;   /* world > 1: WTFNODE_RCCL_ID_BYTES from wtfnode_rccl_unique_id on rank 0 */
  uint64_t slice_steps;     /* wave-steps per streaming slice (0 = 4096) */
  uint64_t regroup_steps;   /* k_run launch length with rip regrouping (0 = off, ~0 = engine default) */
} wtfnode_opts_t;

typedef struct wtfnode_stats {
  uint64_t execs, retired, batches, crashes, unique_crashes, timeouts, cr3, errors;
  uint64_t coverage, corpus, merged_rips;
  uint64_t kernel_launches, group_steps, alg_bytes; /* k_run launches, wave-steps, algorithmic bytes */
  uint64_t breakpoint_hits, rounds;
  uint64_t error_retired;   /* instructions of testcases the engine could not finish (engine errors) */
  double run_s, kernel_ms, merge_ms, insert_ms, coverage_ms, service_ms, total_ms;
} wtfnode_stats_t;

/* A fresh RCCL communicator id (rank 0 makes it, every rank passes it to open). */
int wtfnode_rccl_unique_id(uint8_t out[WTFNODE_RCCL_ID_BYTES]);
/* Load the snapshot, initialise the backend and the module (Target.Init), the
 * communicator (world > 1; collective) and the first batch. */
int wtfnode_open(const wtfnode_opts_t *opts, wtfnode **out);
/* One batch (collective when world > 1). */
int wtfnode_step(wtfnode *node);
int wtfnode_stats(wtfnode *node, wtfnode_stats_t *out);
/* The node's summary line (as `wtfgpu fuzz` prints it); returns the length. */
int wtfnode_summary_json(wtfnode *node, char *buf, uint64_t cap);
int wtfnode_close(wtfnode *node);

#ifdef __cplusplus
}
#endif
#endif /* WTFNODE_H */
