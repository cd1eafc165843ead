"""bench.py — execs/s + emulated instr/s of the MI355X `gpu` execution backend.

Workload (BASELINE.json configs[1], SURVEY.md §8(d) "SYN"): the synthetic
ring-3 ALU/branch/load-store loop snapshot (wtf_amd/tools/syn.py), 65,536 lanes
(= testcases) per GPU, `--limit 100000`, 64-byte uniform-random inputs.

One step = one batch through the hot path of wtf's client loop
(`RunTestcaseAndRestore`, reference src/wtf/client.cc:88-180):
    Backend.Restore (dirty-list reset, bochscpu_backend.cc:730-797)
    -> Target.InsertTestcase (64-byte input -> registers)
    -> Backend.Run (HIP kernel k_run until every lane hits the exit breakpoint)
    -> per-lane results + new-coverage log -> aggregate coverage commit
    -> (N > 1) RCCL MAX all-reduce of the per-GPU coverage map.

Multi-GPU: one process per GPU, each an independent shard of the testcase
stream (seed + rank); the only collective is the coverage-map merge. `value` =
testcases all ranks executed / max-over-ranks wall time ("weak" scaling).

The JSON line carries:
  roofline      k_run's algorithmic bytes per launch (Σ ilen + data bytes read +
                written, counted per lane by the kernel itself)
                / its average launch duration (HIP events on the engine stream);
                `traffic` from the committed rocprofv3 PMC summary when present.
  cpu_baseline  the C oracle ("port": the build's scalar restatement, since
                bochscpu is unbuildable) timed on host cores over a
                bounded sample of the same SYN workload, one lane per thread.
  tlv, hevd     (N=1, rank 0) BASELINE.json configs[2] and [4]: the synthetic
                tlv_server / HEVD snapshots fuzzed by the `wtfgpu` node (C++
                GpuBackend_t, tlv / hevd modules, breakpoints serviced on host
                threads), next to the oracle twin `wtf_twin fuzz` run as one
                process per host core (the reference's one-client-per-core
                layout). Both rates are execs / wall time,
                mutation included.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "execs/sec + emulated instr/s per node (tlv_server, HEVD) at 1/2/4/8 GPUs"
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_k_run.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--lanes", type=int, default=65536)
    ap.add_argument("--limit", type=int, default=100000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget (wall)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tlv", action="store_true", help="skip the tlv_server and hevd legs")
    ap.add_argument("--tlv-batches", type=int, default=6)
    ap.add_argument("--tlv-cpu-seconds", type=float, default=10.0)
    return ap.parse_args()


# ----------------------------------------------------------------- tlv_server / hevd legs
FUZZ_TARGETS = {
    # name: (snapshot builder module, workload text, --max_len)
    "tlv_server": ("wtf_amd.tools.tlv", "synthetic tlv_server snapshot (BASELINE.json configs[2]), tlv mutator", 0x1000),
    "hevd": ("wtf_amd.tools.hevd", "synthetic HEVD ring-0 snapshot (BASELINE.json configs[4] on one GPU), "
                                   "default libFuzzer-style mutator", 1028),
}


def fuzz_leg(name: str, lanes: int, batches: int, cpu_seconds: float, cores: int, limit: int, run_cpu: bool,
             gpu_exe: str | None = None):
    """wtfgpu fuzz on a synthetic snapshot (one GPU), and the oracle twin on
    `cores` host processes (one wtf_twin fuzz client per core) over a bounded
    wall window."""
    import importlib
    import shutil
    import subprocess
    import tempfile

    modname, workload, max_len = FUZZ_TARGETS[name]
    mod = importlib.import_module(modname)
    wtfgpu = gpu_exe or os.path.join(ROOT, "wtf_amd", "host", "wtfgpu")
    twin = os.path.join(ROOT, "oracle", "wtf_twin")
    tmp = tempfile.mkdtemp(prefix=f"wtf_{name}_")
    try:
        base = os.path.join(tmp, "t0")
        mod.build(os.path.join(base, "state"), os.path.join(base, "work"))
        mod.seed_inputs(os.path.join(base, "inputs"))
        out = subprocess.run([wtfgpu, "fuzz", "--name", name, "--target", base, "--lanes", str(lanes),
                              "--runs", str(lanes * batches), "--seed", "1337", "--limit", str(limit),
                              "--max_len", str(max_len)],
                             check=True, capture_output=True, text=True, timeout=600).stdout
        g = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
        res = {"workload": workload + ", seed 1337", "lanes": lanes, "execs": g["execs"], "wall_s": g["wall_s"],
               "value": g["execs"] / g["wall_s"], "unit": "execs/s",
               "instr_per_s": g["retired"] / g["wall_s"], "instr_per_exec": g["retired"] / max(1, g["execs"]),
               "unique_crashes": g["unique_crashes"], "coverage": g["coverage"], "errors": g["errors"],
               "gpu_retired_fraction": 1.0 - g["errors"] / max(1, g["execs"]), "backend": g["backend"]}
        if run_cpu:
            procs = []
            for i in range(cores):
                d = os.path.join(tmp, f"c{i}")
                shutil.copytree(base, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
                procs.append(subprocess.Popen([twin, "fuzz", "--name", name, "--target", d, "--lanes", "1024",
                                               "--seconds", str(cpu_seconds), "--seed", str(1337 + i),
                                               "--limit", str(limit), "--max_len", str(max_len)],
                                              stdout=subprocess.PIPE, text=True))
            execs = instr = 0.0
            wall = 0.0
            for p in procs:
                o, _ = p.communicate(timeout=cpu_seconds * 4 + 120)
                t = json.loads([x for x in o.splitlines() if x.startswith("{")][-1])
                execs += t["execs"]
                instr += t["retired"]
                wall = max(wall, t["wall_s"])
            res["cpu_baseline"] = {"value": execs / wall, "unit": "execs/s", "instr_per_s": instr / wall,
                                   "cores": cores, "kind": "port",
                                   "sample": f"{int(execs)} {name} testcases over {wall:.1f}s, {cores} wtf_twin fuzz "
                                             f"processes (oracle behind Backend_t, one per core)"}
            res["vs_cpu"] = res["value"] / res["cpu_baseline"]["value"]
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


# ----------------------------------------------------------------- CPU baseline
def cpu_baseline(seconds: float, threads: int, limit: int):
    """The C oracle (tests/oracle_lib, TEST INFRASTRUCTURE) on the same SYN
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
    return {"value": execs / dt, "unit": "execs/s", "instr_per_s": instr / dt, "cores": threads,
            "kind": "port",
            "sample": f"{execs} SYN testcases ({instr} instructions) over {dt:.1f}s, {threads} threads, "
                      f"one C-oracle machine per thread (bochscpu unbuildable: SURVEY F2)"}


# ----------------------------------------------------------------- coverage merge
class _DevBuf:
    """__cuda_array_interface__ view of an engine device buffer (for RCCL)."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2, "strides": None}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        a.gpus = world

    # CPU baseline first (rank 0, N=1), before anything touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        threads = a.cpu_threads or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(a.cpu_seconds, threads, a.limit)

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)

    from tests.syn_harness import make_engine
    from wtf_amd.abi import EXIT_BREAKPOINT
    from wtf_amd import shard
    from wtf_amd.tools import syn

    n = a.lanes
    eng, sp, st = make_engine(n, limit=a.limit, device=local)
    eng.restore()
    base = eng.read_gprs(0, 1)[0].copy()

    cov_t = None
    if dist is not None:
        import ctypes as C

        p, nb = C.c_void_p(), C.c_uint64()
        eng.L.wtfgpu_coverage_device_map(eng.ctx, C.byref(p), C.byref(nb))
        cov_t = torch.as_tensor(_DevBuf(p.value, nb.value), device=f"cuda:{local}")

    rng_seed = shard.rank_seed(syn.SEED, rank)
    pool = syn.inputs(n * 4, seed=rng_seed)  # input pool; each step takes a rotating window

    stats = {"execs": 0, "retired": 0, "kernel_ms": 0.0, "launches": 0, "bytes_alg": 0, "dirty": 0,
             "input_bytes": 0, "newcov": 0, "bad": 0}

    def step(i, record):
        off = (i * 7919) % (3 * n)
        inp = pool[off:off + n]
        eng.restore()
        g = np.tile(base, (n, 1))
        syn.insert(g, inp)
        eng.write_gprs(g)
        rs = eng.run()
        ex = eng.exits_np()
        ok = int(np.count_nonzero(ex["status"] == EXIT_BREAKPOINT))
        cov, _ovf = eng.coverage()
        new = set()
        for s in cov.values():
            new |= s
        if new:
            eng.commit_coverage(new)
        if cov_t is not None:
            torch.cuda.synchronize()
            shard.merge_coverage_map(cov_t, dist)
            torch.cuda.synchronize()
        if record:
            nb = eng.nbytes()
            stats["execs"] += n
            stats["retired"] += rs.lane_retired
            stats["kernel_ms"] += rs.kernel_ms
            stats["launches"] += rs.kernel_launches
            stats["bytes_alg"] += int(nb.sum())
            stats["dirty"] += n  # SYN: every testcase dirties exactly its scratch page
            stats["input_bytes"] += n * syn.INPUT_SIZE
            stats["newcov"] += len(new)
            stats["bad"] += n - ok

    for i in range(a.warmup):
        step(i, False)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(a.warmup + i, True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0

    dt, execs, retired = shard.job_totals(dt, float(stats["execs"]), float(stats["retired"]), dist,
                                          device=f"cuda:{local}")

    if stats["bad"]:
        raise SystemExit(f"{stats['bad']} testcases did not reach the exit breakpoint")

    if rank == 0:
        avg_launch_s = stats["kernel_ms"] / 1e3 / max(1, stats["launches"])
        bytes_per_launch = stats["bytes_alg"] / max(1, stats["launches"])
        achieved = bytes_per_launch / avg_launch_s / 1e9
        traffic = None
        if os.path.exists(PMC_SUMMARY):
            try:
                pmc = json.load(open(PMC_SUMMARY))
                if pmc.get("lanes") == n and pmc.get("limit") == a.limit:
                    traffic = pmc.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        b_exec = stats["bytes_alg"] + stats["input_bytes"] + 2 * 4096 * stats["dirty"]
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
            "data": "synthetic (SYN ring-3 snapshot built in-process; uniform random 64-byte inputs)",
            "config": {"workload": "SYN: synthetic ring-3 ALU/branch/load-store loop snapshot "
                                   "(BASELINE.json configs[1])",
                       "lanes_per_gpu": n, "limit": a.limit, "input_bytes": syn.INPUT_SIZE,
                       "parallelism": f"shard{world} (independent testcases) + RCCL MAX coverage merge"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_run", "alg_bytes_per_launch": bytes_per_launch,
                         "avg_launch_ms": avg_launch_s * 1e3},
            "gpu_kernel_ms_per_step": stats["kernel_ms"] / a.steps,
            "instr_per_exec": stats["retired"] / max(1, stats["execs"]),
            "b_exec_gbs_wall": b_exec / (dt if world == 1 else dt) / 1e9,
            "gpu_retired_fraction": 1.0,
            "cpu_baseline": cpu,
        }
        if world == 1 and not a.no_tlv:
            eng.close()
            eng = None
            cores = a.cpu_threads or min(16, os.cpu_count() or 1)
            out["tlv"] = fuzz_leg("tlv_server", a.lanes, a.tlv_batches, a.tlv_cpu_seconds, cores, a.limit,
                                  not a.no_cpu)
            out["hevd"] = fuzz_leg("hevd", a.lanes, a.tlv_batches, a.tlv_cpu_seconds, cores, a.limit, not a.no_cpu)
        print(json.dumps(out), flush=True)
    if eng is not None:
        eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
