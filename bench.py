"""bench.py — execs/s + emulated instr/s of the MI355X `gpu` execution backend
(BASELINE.json metric: "execs/sec + emulated instr/s per node (tlv_server,
HEVD) at 1/2/4/8 GPUs").

Headline (`value`): fuzzer_tlv_server on the gpu backend (BASELINE.json
configs[2] at N=1, configs[3] at N>1): the synthetic tlv_server snapshot
(wtf_amd/tools/tlv.py; the real one cannot be fetched), the tlv
module and its custom mutator, seed 1337, 131,072 lanes per GPU (two waves per
SIMD: the most the k_run register budget keeps resident; configs[2] names no
batch), --limit 100000.
One step = one fuzz batch of the node (include/wtfnode.h, libwtfnode.so, the
same C++ as `wtfgpu fuzz`): mutate (overlapped with the previous batch) ->
InsertTestcase x N -> k_run with breakpoints serviced -> lane-order coverage
attribution -> Target.Restore, and for N > 1 the RCCL MAX merge of the
per-GPU coverage maps (the only collective; every GPU is otherwise an
independent shard with seed + rank). One process per GPU; `value` = testcases
all ranks executed / max-over-ranks wall time of the K timed steps.

Also on the line (N=1, rank 0):
  roofline      k_run (the dominant kernel) on the headline workload:
                algorithmic bytes per launch (instruction bytes + data bytes
                read + written, counted per lane by the kernel) /
                average launch duration (HIP events on the engine's stream);
                `traffic` and VALU utilisation from the committed rocprofv3 PMC
                summary of the same workload (profiles/pmc_tlv_k_run.json).
  cpu_baseline  the oracle twin (`oracle/wtf_twin`: the C restatement behind
                Backend_t, "port" — bochscpu is unbuildable) as one
                `wtf_twin fuzz` process per host core, same module, mutator
                and seed scheme, over a bounded wall window.
  hevd          BASELINE.json configs[4] on one GPU: the synthetic ring-0 HEVD
                snapshot with the I/O manager's IRP path and benign-majority
                seeds (wtf_amd/tools/hevd_io.py), the hevd module, libFuzzer's
                mutator (bit-exact restatement), --limit 10000000, --max_len
                1028, >= 10 s of node wall time, with its own roofline, crash
                share and twin baseline.
  hevd_bare     the same on the bare look-alike (wtf_amd/tools/hevd.py: the
                handlers called from the system-call entry, ~300 instructions
                per exec, mostly crashing traffic), the round-5 HEVD leg.
  syn           BASELINE.json configs[1]: the ring-3 ALU/branch/load-store
                interpreter microbench, 65,536 lanes, with its roofline and the
                C oracle's rate on the host cores.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "execs/sec + emulated instr/s per node (tlv_server, HEVD) at 1/2/4/8 GPUs"
PROFILES = os.path.join(ROOT, "profiles")
WTFGPU = os.path.join(ROOT, "wtf_amd", "host", "wtfgpu")
TWIN = os.path.join(ROOT, "oracle", "wtf_twin")

TARGETS = {
    # name: (snapshot builder module, workload text, --max_len)
    "tlv_server": ("wtf_amd.tools.tlv", "fuzzer_tlv_server on the synthetic tlv_server snapshot "
                                        "(BASELINE.json configs[2]/[3]), tlv CustomMutator_t, seed 1337", 0x1000),
    "hevd": ("wtf_amd.tools.hevd_io", "fuzzer_hevd on the synthetic ring-0 HEVD snapshot with the I/O manager's "
                                      "IRP path (BASELINE.json configs[4] on one GPU), libFuzzer "
                                      "MutationDispatcher, seed 1337", 1028),
    "hevd_bare": ("wtf_amd.tools.hevd", "fuzzer_hevd on the bare HEVD look-alike (IOCTL handlers called from the "
                                        "system-call entry, no I/O manager), libFuzzer MutationDispatcher, seed 1337",
                  1028),
}
# the module a workload's snapshot runs (both HEVD snapshots run fuzzer_hevd)
MODULE = {"tlv_server": "tlv_server", "hevd": "hevd", "hevd_bare": "hevd"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--lanes", type=int, default=262144, help="lanes per GPU of the tlv headline (two waves per SIMD "
                    "per pipelined half)")
    ap.add_argument("--hevd-lanes", type=int, default=131072, help="lanes per GPU of the hevd leg")
    ap.add_argument("--syn-lanes", type=int, default=65536, help="BASELINE.json configs[1]: 64K lanes")
    ap.add_argument("--slice-steps", type=int, default=0, help="wave-steps per streaming slice (0: the node's 4096)")
    ap.add_argument("--regroup-steps", type=int, default=-1,
                    help="k_run launch length with lanes regrouped by rip (0: off; -1: engine default)")
    ap.add_argument("--limit", type=int, default=100000)
    ap.add_argument("--hevd-limit", type=int, default=10_000_000, help="BASELINE.md: HEVD runs --limit 10000000")
    ap.add_argument("--leg-seconds", type=float, default=10.0, help="GPU wall window of the hevd leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="wall window of each CPU baseline")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host CPU share (see cpu_cores)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-legs", action="store_true", help="headline only (skip hevd / syn)")
    return ap.parse_args()


GPUS_PER_NODE = 8  # an MI355X node (BASELINE.json: 1/2/4/8 GPUs)
MUTATION = ("batches of >= 8192 testcases are mutated in parallel chunks of 2048, each chunk with its own "
            "mutator and a generator seeded from the node's seed-1337 stream in chunk order (runner.cc "
            "kParMutateMin / kMutateChunk): deterministic, but not server.h's single-mutator stream "
            "(--serial-mutation restores that)")


def node_extrapolation(value: float, cpu: dict, core_info: dict) -> dict | None:
    """The reference runs one wtf client per core of the node; the box gives
    this job a 16-core share (OMP_NUM_THREADS) of a 256-CPU, 8-GPU machine, so
    the whole-node CPU figure is extrapolated linearly from the measured
    per-core rate (labelled as such), and set against 8 GPUs at this line's
    per-GPU rate (also linear: weak scaling, the driver's SCALE run measures
    the real one)."""
    node_cores = core_info.get("os_cpu_count") or 0
    if not cpu or not node_cores or cpu["cores"] >= node_cores:
        return None
    per_core = cpu["value"] / cpu["cores"]
    return {"kind": "extrapolated", "cores": node_cores, "value": per_core * node_cores,
            "per_core": per_core, "gpus": GPUS_PER_NODE,
            "vs_cpu_node": value * GPUS_PER_NODE / (per_core * node_cores),
            "basis": f"linear in cores from {cpu['cores']} measured cores (the job's CPU share; a process per "
                     f"machine core would exceed it) and linear in GPUs from this 1-GPU value"}


def cpu_cores() -> tuple[int, dict]:
    """Host threads the CPU baselines use: the CPU share the job may use
    (OMP_NUM_THREADS when the environment sets it, as the GPU box does, else
    the affinity mask), recorded with the machine's counts."""
    aff = len(os.sched_getaffinity(0))
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    use = min(aff, env) if env > 0 else aff
    return use, {"os_cpu_count": os.cpu_count(), "affinity": aff, "omp_num_threads": env or None, "used": use}


def build_target(name: str, d: str) -> str:
    import importlib

    mod = importlib.import_module(TARGETS[name][0])
    mod.build(os.path.join(d, "state"), os.path.join(d, "work"))
    mod.seed_inputs(os.path.join(d, "inputs"))
    return d


def engine_sha16() -> str:
    """The engine build (libwtfgpu.so) this run uses: PMC summaries carry the
    hash of the build they were measured on."""
    import hashlib

    with open(os.path.join(ROOT, "wtf_amd", "csrc", "libwtfgpu.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_pmc(name: str, lanes: int, limit: int) -> dict | None:
    """The committed rocprofv3 PMC summary of k_run on this workload (made by
    scripts/pmc_summary.py), if its config matches and it was measured on this
    very engine build (engine_sha16); else None (traffic / valu / wait null)."""
    p = os.path.join(PROFILES, f"pmc_{name}_k_run.json")
    try:
        pmc = json.load(open(p))
    except (OSError, ValueError):
        return None
    if pmc.get("lanes") != lanes or pmc.get("limit") != limit or pmc.get("engine_sha16") != engine_sha16():
        return None
    return pmc


SIMDS = 256 * 4        # MI355X_MICROARCH.md: 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9       # MI355X_MICROARCH.md: max clock 2400 MHz


def issue_roofline(pmc: dict | None, avg_s: float, steps_per_launch: float, retired_per_launch: float) -> dict | None:
    """The bound that binds k_run (latency and issue, not HBM): wave
    instructions issued per launch (the PMC summary's SQ_INSTS_* mix) against
    the sequencer's ceiling of one instruction per SIMD per cycle, plus the
    same count per wave-step and per lane-retired guest instruction."""
    mix = (pmc or {}).get("instruction_mix_per_launch")
    if not mix or avg_s <= 0:
        return None
    insts = sum(v for k, v in mix.items() if k.startswith("SQ_INSTS_"))
    achieved = insts / (SIMDS * CLOCK_HZ * avg_s)
    return {"unit": "wave instructions / SIMD-cycle", "achieved": achieved, "peak": 1.0, "frac": achieved,
            "insts_per_launch": insts,
            "per_wave_step": insts / steps_per_launch if steps_per_launch else None,
            "per_retired_instr": insts / retired_per_launch if retired_per_launch else None,
            "salu_valu_branch": [mix.get("SQ_INSTS_SALU"), mix.get("SQ_INSTS_VALU"), mix.get("SQ_INSTS_BRANCH")]}


def roofline(alg_bytes: float, launches: float, kernel_ms: float, pmc: dict | None, steps: float = 0,
             retired: float = 0) -> dict:
    avg_s = kernel_ms / 1e3 / max(1.0, launches)
    per_launch = alg_bytes / max(1.0, launches)
    achieved = per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
            "kernel": "k_run", "alg_bytes_per_launch": per_launch, "avg_launch_ms": avg_s * 1e3,
            "valu_util": pmc.get("valu_util") if pmc else None,
            "wait_frac": pmc.get("wait_frac") if pmc else None,
            "issue": issue_roofline(pmc, avg_s, steps / max(1.0, launches), retired / max(1.0, launches))}


# ----------------------------------------------------------------- CPU baselines
def twin_baseline(name: str, base: str, seconds: float, cores: int, limit: int) -> dict:
    """One `wtf_twin fuzz` client per host core (the reference's one node per
    core), seeds 1337 + i, for `seconds` of wall time."""
    max_len = TARGETS[name][2]
    module = MODULE[name]
    tmp = tempfile.mkdtemp(prefix=f"twin_{name}_")
    try:
        procs = []
        for i in range(cores):
            d = os.path.join(tmp, f"c{i}")
            shutil.copytree(base, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
            procs.append(subprocess.Popen([TWIN, "fuzz", "--name", module, "--target", d, "--lanes", "1024",
                                           "--seconds", str(seconds), "--seed", str(1337 + i), "--limit", str(limit),
                                           "--max_len", str(max_len)], stdout=subprocess.PIPE, text=True,
                                          env={**os.environ, "OMP_NUM_THREADS": "1"}))
        execs = instr = wall = 0.0
        for p in procs:
            o, _ = p.communicate(timeout=seconds * 4 + 300)
            t = json.loads([x for x in o.splitlines() if x.startswith("{")][-1])
            execs += t["execs"]
            instr += t["retired"]
            wall = max(wall, t["wall_s"])
        return {"value": execs / wall, "unit": "execs/s", "instr_per_s": instr / wall, "cores": cores, "kind": "port",
                "sample": f"{int(execs)} {name} testcases over {wall:.1f}s: {cores} wtf_twin fuzz processes, one per "
                          f"host core (the C oracle behind Backend_t; bochscpu is unbuildable, SURVEY F2)"}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def syn_cpu_baseline(seconds: float, threads: int, limit: int) -> dict:
    """The C oracle (tests/oracle_lib, TEST INFRASTRUCTURE) on the SYN
    workload: each thread owns one oracle machine and runs testcases
    restore -> insert -> run back to back until the time budget is spent."""
    import threading

    from tests.oracle_lib import Oracle
    from wtf_amd.abi import EXIT_BREAKPOINT, regs_from_state
    from wtf_amd.tools import syn

    sp, st, _ = syn.build()
    pfns, blob = sp.phys()
    base = regs_from_state(st)
    inp = syn.inputs(1 << 14, seed=syn.SEED ^ 0xC0FFEE)
    g = np.tile(np.array(list(base.gpr) + [base.rip, base.rflags], dtype=np.uint64), (len(inp), 1))
    syn.insert(g, inp)
    counts = [[0, 0] for _ in range(threads)]
    bad = []
    stop_at = [0.0]

    def worker(t):
        o = Oracle(pfns=pfns, blob=blob)
        o.set_limit(limit)
        o.set_breakpoints([syn.EXIT_VA])
        i = t
        while time.perf_counter() < stop_at[0]:
            o.restore(base)
            r = o.regs()
            for k in range(16):
                r.gpr[k] = int(g[i % len(g), k])
            o.set_regs(r)
            ex = o.run()
            if ex.status != EXIT_BREAKPOINT:
                bad.append(ex.status)
            counts[t][0] += 1
            counts[t][1] += ex.icount
            i += threads

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    stop_at[0] = t0 + seconds
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    execs = sum(c[0] for c in counts)
    instr = sum(c[1] for c in counts)
    assert not bad, f"oracle exits {set(bad)}"
    return {"value": execs / dt, "unit": "execs/s", "instr_per_s": instr / dt, "cores": threads, "kind": "port",
            "sample": f"{execs} SYN testcases ({instr} instructions) over {dt:.1f}s, {threads} threads, "
                      f"one C-oracle machine per thread (bochscpu unbuildable: SURVEY F2)"}


# ----------------------------------------------------------------- GPU legs
def node_fields(s0: dict, s1: dict) -> dict:
    """Kernel-efficiency evidence of a node over [s0, s1]."""
    d = {k: s1[k] - s0[k] for k in s1}
    return {
        "lanes_per_wave_step": d["retired"] / max(1, d["group_steps"]),
        "gpu_retired_fraction": (d["retired"] - d["error_retired"]) / max(1, d["retired"]),
        "kernel_ms": d["kernel_ms"], "kernel_launches": d["kernel_launches"], "group_steps": d["group_steps"],
        "breakpoint_hits": d["breakpoint_hits"], "rounds": d["rounds"], "insert_ms": d["insert_ms"],
        "coverage_ms": d["coverage_ms"], "service_ms": d["service_ms"], "node_ms": d["total_ms"],
        "merge_ms": d["merge_ms"], "errors": d["errors"], "alg_bytes": d["alg_bytes"],
    }


def sched_flags(a) -> list[str]:
    """The node's scheduling flags from bench's (--slice-steps / --regroup-steps)."""
    f = []
    if a.slice_steps:
        f += ["--slice-steps", str(a.slice_steps)]
    if a.regroup_steps >= 0:
        f += ["--regroup-steps", str(a.regroup_steps)]
    return f


def hevd_leg(base: str, lanes: int, limit: int, seconds: float, flags=(), name: str = "hevd") -> dict:
    """`wtfgpu fuzz` (the product node binary) on an HEVD snapshot for
    `seconds` of wall time: `hevd` (the I/O manager's IRP path) or
    `hevd_bare` (the handlers called straight from the system-call entry)."""
    out = subprocess.run([WTFGPU, "fuzz", "--name", "hevd", "--target", base, "--lanes", str(lanes),
                          "--seconds", str(seconds), "--seed", "1337", "--limit", str(limit), "--max_len", "1028",
                          *flags],
                         check=True, capture_output=True, text=True, timeout=seconds * 6 + 300).stdout
    g = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    b = g["backend"]
    pmc = load_pmc(name, lanes, limit)
    return {"workload": TARGETS[name][1], "lanes": lanes, "limit": limit, "execs": g["execs"],
            "wall_s": g["wall_s"], "value": g["execs"] / g["wall_s"], "unit": "execs/s",
            "instr_per_s": g["retired"] / g["wall_s"], "instr_per_exec": g["retired"] / max(1, g["execs"]),
            "crash_share": g["crashes"] / max(1, g["execs"]),
            "unique_crashes": g["unique_crashes"], "coverage": g["coverage"], "errors": g["errors"],
            "gpu_retired_fraction": (g["retired"] - g["error_retired"]) / max(1, g["retired"]),
            "lanes_per_wave_step": g["retired"] / max(1, b["group_steps"]),
            "roofline": roofline(b["alg_bytes"], b["kernel_launches"], b["kernel_ms"], pmc, b["group_steps"],
                                 g["retired"]), "backend": b,
            "kernel_busy_frac": b["kernel_ms"] / (g["wall_s"] * 1e3),
            "note": ("the I/O manager's METHOD_NEITHER path (trap frame, handle table, IRP lookaside, a filter "
                     "device, IofCompleteRequest) and benign-majority traffic; a real Windows + HEVD dump cannot be "
                     "fetched (SURVEY F3)" if name == "hevd" else
                     "the bare look-alike's IOCTL path is ~300 instructions per exec: no I/O manager, mostly "
                     "crashing traffic"),
            "node": {k: g.get(k) for k in ("step_ms", "account_ms", "newcov_ms", "crashsave_ms", "produce_wait_ms",
                                           "make_ms", "fill_ms", "run_s", "batches", "crashes")}}


def syn_leg(lanes: int, limit: int, steps: int, device: int) -> dict:
    from tests.syn_harness import make_engine
    from wtf_amd.abi import EXIT_BREAKPOINT
    from wtf_amd.tools import syn

    eng, sp, st = make_engine(lanes, limit=limit, device=device)
    eng.restore()
    base = eng.read_gprs(0, 1)[0].copy()
    pool = syn.inputs(lanes * 4, seed=syn.SEED)
    acc = {"execs": 0, "retired": 0, "kernel_ms": 0.0, "launches": 0, "bytes": 0, "steps": 0, "bad": 0}

    def step(i, record):
        off = (i * 7919) % (3 * lanes)
        inp = pool[off:off + lanes]
        eng.restore()
        g = np.tile(base, (lanes, 1))
        syn.insert(g, inp)
        eng.write_gprs(g)
        rs = eng.run()
        ex = eng.exits_np()
        cov, _ = eng.coverage()
        new = set().union(*cov.values()) if cov else set()
        if new:
            eng.commit_coverage(new)
        if record:
            acc["execs"] += lanes
            acc["retired"] += rs.lane_retired
            acc["kernel_ms"] += rs.kernel_ms
            acc["launches"] += rs.kernel_launches
            acc["steps"] += rs.group_steps
            # B_exec: instruction + data bytes, the 64-byte input, 2 x 4096 per dirty page
            acc["bytes"] += int(eng.nbytes().sum()) + 64 * lanes + 2 * 4096 * int(eng.dirty_counts().sum())
            acc["bad"] += int(np.count_nonzero(ex["status"] != EXIT_BREAKPOINT))

    step(0, False)
    t0 = time.perf_counter()
    for i in range(steps):
        step(1 + i, True)
    dt = time.perf_counter() - t0
    eng.close()
    if acc["bad"]:
        raise SystemExit(f"SYN: {acc['bad']} testcases did not reach the exit breakpoint")
    return {"workload": "SYN: synthetic ring-3 ALU/branch/load-store loop snapshot (BASELINE.json configs[1]), "
                        "uniform random 64-byte inputs",
            "lanes": lanes, "limit": limit, "steps": steps, "value": acc["execs"] / dt, "unit": "execs/s",
            "instr_per_s": acc["retired"] / dt, "instr_per_exec": acc["retired"] / max(1, acc["execs"]),
            "ms_per_step": dt * 1e3 / steps, "lanes_per_wave_step": acc["retired"] / max(1, acc["steps"]),
            "gpu_retired_fraction": 1.0,
            "roofline": roofline(acc["bytes"], acc["launches"], acc["kernel_ms"], load_pmc("syn", lanes, limit),
                                 acc["steps"], acc["retired"])}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    a.gpus = world
    tmp = tempfile.mkdtemp(prefix=f"wtfbench_r{rank}_")
    try:
        run(a, rank, world, local, tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def run(a, rank, world, local, tmp):
    # snapshots + CPU baselines first (rank 0, N = 1), before anything touches the GPU
    tlv_dir = build_target("tlv_server", os.path.join(tmp, "tlv"))
    legs = rank == 0 and world == 1 and not a.no_legs
    hevd_dir = build_target("hevd", os.path.join(tmp, "hevd")) if legs else None
    bare_dir = build_target("hevd_bare", os.path.join(tmp, "hevd_bare")) if legs else None
    cores, core_info = cpu_cores()
    if a.cpu_threads:
        cores = a.cpu_threads
    cpu = {}
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu["tlv_server"] = twin_baseline("tlv_server", tlv_dir, a.cpu_seconds, cores, a.limit)
        if legs:
            cpu["hevd"] = twin_baseline("hevd", hevd_dir, a.cpu_seconds, cores, a.hevd_limit)
            cpu["hevd_bare"] = twin_baseline("hevd_bare", bare_dir, a.cpu_seconds, cores, a.hevd_limit)
            cpu["syn"] = syn_cpu_baseline(a.cpu_seconds, cores, a.limit)

    import torch

    from wtf_amd import node as wn
    from wtf_amd import shard

    torch.cuda.set_device(local)
    dist = None
    rccl_id = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)  # control plane only
        rccl_id = shard.share_bytes(wn.rccl_unique_id() if rank == 0 else None, dist)

    node = wn.Node("tlv_server", tlv_dir, a.lanes, a.limit, seed=1337, max_len=TARGETS["tlv_server"][2],
                   device=local, rank=rank, world=world, rccl_id=rccl_id, slice_steps=a.slice_steps,
                   regroup_steps=None if a.regroup_steps < 0 else a.regroup_steps)
    for _ in range(a.warmup):
        node.step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    s0 = node.stats()
    sum0 = node.summary()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        node.step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    s1 = node.stats()
    execs, retired = s1["execs"] - s0["execs"], s1["retired"] - s0["retired"]
    dt, execs, retired = shard.job_totals(dt, float(execs), float(retired), dist)
    fields = node_fields(s0, s1)
    summary = node.summary()
    # the timed steps' share of every node / backend counter (summary - summary before)
    # (counters only: a difference of two rates means nothing)
    timed = {k: round(v - sum0[k], 3) for k, v in summary.items()
             if isinstance(v, (int, float)) and k in sum0 and not k.endswith("_per_s")}
    timed["backend"] = {k: round(v - sum0["backend"][k], 3) for k, v in summary["backend"].items()
                        if isinstance(v, (int, float)) and k in sum0["backend"]}
    node.close()

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": execs / dt,
            "unit": "execs/s",
            "instr_per_s": retired / dt,
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (tlv_server look-alike snapshot built in-process; the tlv module's CustomMutator_t "
                    "over its seed corpus)",
            "config": {"workload": TARGETS["tlv_server"][1], "lanes_per_gpu": a.lanes, "limit": a.limit,
                       "max_len": TARGETS["tlv_server"][2], "slice_steps": a.slice_steps or 4096,
                       "regroup_steps": a.regroup_steps if a.regroup_steps >= 0 else 1024,  # engine default
                       "regroup_auto": "the schedule (regrouped or fixed lane order) that retires more lanes per wave-step, measured; the other probed every 32nd run",
                       "mutation": MUTATION,
                       "parallelism": f"shard{world}: one node per GPU (seed + rank), RCCL MAX coverage-map "
                                      f"merge started every step, absorbed the next"},
            "build": {"engine_sha16": engine_sha16()},
            "instr_per_exec": retired / max(1.0, execs),
            "roofline": roofline(fields["alg_bytes"], fields["kernel_launches"], fields["kernel_ms"],
                                 load_pmc("tlv", a.lanes, a.limit), fields["group_steps"], retired),
            **{k: fields[k] for k in ("lanes_per_wave_step", "gpu_retired_fraction")},
            "node": {k: v for k, v in fields.items() if k not in ("lanes_per_wave_step", "gpu_retired_fraction")},
            "coverage": summary["coverage"], "unique_crashes": summary["unique_crashes"],
            "node_summary": summary,
            "node_timed": timed,
            "cpu_baseline": cpu.get("tlv_server"),
            "host_cpus": core_info,
        }
        out["kernel_busy_frac"] = fields["kernel_ms"] / (dt * 1e3)  # sum of k_run time / wall
        if timed.get("cpu_s") is not None and timed.get("wall_s"):  # host cores busy over the timed steps
            out["host_cpu_frac"] = timed["cpu_s"] / (timed["wall_s"] * cores)
        if out["cpu_baseline"]:
            out["vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            out["cpu_node"] = node_extrapolation(out["value"], out["cpu_baseline"], core_info)
            if out["cpu_node"]:
                out["vs_cpu_node"] = out["cpu_node"]["vs_cpu_node"]
        if legs:
            for leg, d in (("hevd", hevd_dir), ("hevd_bare", bare_dir)):
                h = hevd_leg(d, a.hevd_lanes, a.hevd_limit, a.leg_seconds, sched_flags(a), leg)
                if leg in cpu:
                    h["cpu_baseline"] = cpu[leg]
                    h["vs_cpu"] = h["value"] / cpu[leg]["value"]
                    h["cpu_node"] = node_extrapolation(h["value"], cpu[leg], core_info)
                    if h["cpu_node"]:
                        h["vs_cpu_node"] = h["cpu_node"]["vs_cpu_node"]
                out[leg] = h
            s = syn_leg(a.syn_lanes, a.limit, 10, local)
            if "syn" in cpu:
                s["cpu_baseline"] = cpu["syn"]
            out["syn"] = s
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
