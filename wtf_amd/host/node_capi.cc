// node_capi.cc — libwtfnode.so: the C ABI of include/wtfnode.h over
// FuzzSession (runner.h) + GpuBackend_t (gpu_backend.h) + RcclExchange_t.
// One node per process (wtf's g_Backend / g_Dbg / target registry are process
// globals, as in the reference).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "../../include/wtfnode.h"
#include "gpu_backend.h"
#include "rccl_exchange.h"
#include "runner.h"

using namespace wtfgpu_host;

struct wtfnode {
  RunnerOptions O;
  Options_t Opts;
  CpuState_t State;
  GpuBackend_t *B = nullptr;  // lives for the process, like g_Backend
  std::unique_ptr<RcclExchange_t> X;
  std::unique_ptr<ModuleSlots> Slots;
  std::unique_ptr<FuzzSession> F;
};

extern "C" {

int wtfnode_rccl_unique_id(uint8_t out[WTFNODE_RCCL_ID_BYTES]) {
  return out && RcclUniqueId(out) ? 0 : -1;
}

int wtfnode_open(const wtfnode_opts_t *o, wtfnode **out) {
  if (!o || !out || !o->name || !o->target || o->world < 1 || o->rank < 0 || o->rank >= o->world) return -1;
  if (o->world > 1 && !o->rccl_id) return -1;
  *out = nullptr;
  auto N = std::make_unique<wtfnode>();
  RunnerOptions &O = N->O;
  O.mode = "fuzz";
  O.name = o->name;
  O.target = o->target;
  O.lanes = o->lanes ? o->lanes : 1;
  if (o->overlay_pages) O.overlay_pages = o->overlay_pages;
  O.limit = o->limit;
  O.seed = o->seed;
  O.max_len = o->max_len ? o->max_len : 0x1000;
  O.device = o->device;
  O.rank = o->rank;
  O.world = o->world;
  if (o->slice_steps) O.slice = o->slice_steps;
  O.regroup = o->regroup_steps;
  if (!LoadTarget(O, N->Opts, N->State)) return -2;
  N->B = new GpuBackend_t();
  g_Backend = N->B;
  if (!N->B->Initialize(N->Opts, N->State)) return -3;
  if (O.regroup != ~0ull) wtfgpu_set_regroup(N->B->Engine(), O.regroup);
  if (const char *e = getenv("WTF_RCCL_FORCE")) O.rccl_force = atoi(e) != 0;
  if (O.world > 1 || O.rccl_force) {
    uint8_t Own[kRcclIdBytes];
    const uint8_t *Id = o->rccl_id;
    if (!Id) {  // forced at world 1 without an id: this process is the only rank
      if (!RcclUniqueId(Own)) return -4;
      Id = Own;
    }
    N->X = std::make_unique<RcclExchange_t>(O.rank, O.world, O.rccl_force);
    if (!N->X->Init(Id, wtfgpu_stream(N->B->Engine()))) return -4;
  }
  Target_t *T = Targets_t::Instance().Get(O.name);
  if (!T) return -5;
  if (!T->Init(N->Opts, N->State)) return -6;
  N->Slots = std::make_unique<ModuleSlots>();
  N->Slots->Capture(N->B->Lanes());
  N->F = std::make_unique<FuzzSession>(O, *N->B, *T, *N->Slots, N->X.get());
  if (!N->F->Start()) return -7;
  *out = N.release();
  return 0;
}

int wtfnode_step(wtfnode *n) {
  if (!n || !n->F) return -1;
  return n->F->Step() ? 0 : -2;
}

int wtfnode_stats(wtfnode *n, wtfnode_stats_t *out) {
  if (!n || !out) return -1;
  memset(out, 0, sizeof(*out));
  const FuzzStats &S = n->F->Stats();
  const BatchStats &G = n->B->Stats();
  out->execs = S.execs, out->retired = S.retired, out->batches = S.batches, out->crashes = S.crashes;
  out->timeouts = S.timeouts, out->cr3 = S.cr3, out->errors = S.errors, out->merged_rips = S.merged_rips;
  out->unique_crashes = 0;
  out->coverage = n->B->CoverageSize();
  out->corpus = n->F->CorpusSize();
  out->kernel_launches = G.kernel_launches, out->group_steps = G.group_steps, out->alg_bytes = G.alg_bytes;
  out->breakpoint_hits = G.breakpoint_hits, out->rounds = G.rounds;
  out->error_retired = S.error_retired;
  out->run_s = S.run_s, out->kernel_ms = G.kernel_ms, out->merge_ms = S.merge_ms, out->insert_ms = G.insert_ms;
  out->coverage_ms = G.coverage_ms, out->service_ms = G.service_ms, out->total_ms = G.total_ms;
  return 0;
}

int wtfnode_summary_json(wtfnode *n, char *buf, uint64_t cap) {
  if (!n || !buf || !cap) return -1;
  const std::string s = n->F->SummaryJson();
  snprintf(buf, cap, "%s", s.c_str());
  return (int)s.size();
}

int wtfnode_close(wtfnode *n) {
  if (!n) return 0;
  if (n->F && n->X && n->X->Exchanging()) n->F->FinishMerge();  // the merge the last step started (collective)
  n->F.reset();
  n->X.reset();
  delete n;  // the backend stays (process lifetime, as g_Backend in the reference)
  return 0;
}

}  // extern "C"
