"""Summarise the rocprofv3 CSV output of scripts/gpu_pmc.sh for k_run on one
workload: python3 scripts/pmc_summary.py <dir> <leg> <lanes> <limit>.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled (k_run's reads are not all wide streams: the
corrected read side is an upper bound, the raw one a lower bound).
valu_util = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, wait_frac = SQ_WAIT_ANY /
SQ_WAVE_CYCLES (both summed over k_run dispatches). The launches of the
workload's warm-up (prof_leg.py prints how many) are left out of the counters,
as bench.py's timed window leaves them out; kernel_trace keeps rocprof's
all-launch statistics and adds the after-warm-up average. engine_sha16 binds
the summary to the libwtfgpu.so it was measured on."""
import csv
import glob
import hashlib
import json
import os
import sys

d, leg, lanes, limit = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])


def warm_launches(sub):
    """k_run launches of the workload's warm-up in this pass (prof_leg.py
    prints them; 0 for a run without one): left out, as bench.py's timed
    window leaves its warm-up steps out."""
    try:
        for line in reversed(open(os.path.join(d, sub + ".log")).read().splitlines()):
            if line.startswith("{") and "warm_launches" in line:
                return int(json.loads(line)["warm_launches"])
    except (OSError, ValueError):
        pass
    return 0


def per_kernel(sub):
    rows = {}
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_run" not in r["Kernel_Name"]:
                continue
            rows.setdefault(int(r["Dispatch_Id"]), []).append((r["Counter_Name"], float(r["Counter_Value"])))
    keep = sorted(rows)[warm_launches(sub):]
    out = {}
    for i in keep:
        for k, v in rows[i]:
            out[k] = out.get(k, 0.0) + v
    return out, max(1, len(keep))


fetch, nf = per_kernel("fetch")
write, nw = per_kernel("write")
mix, nm = per_kernel("mix")
wait, nwt = per_kernel("wait")
stats = {}
for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_run" in r["Name"]:
            stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "pct": float(r["Percentage"])}
# the same average over the launches after the warm-up (the kernel trace)
durs = {}
for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_run" in r["Kernel_Name"]:
            durs[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
if durs:
    kept = [durs[i] for i in sorted(durs)[warm_launches("stats"):]]
    if kept:
        stats["after_warmup"] = {"calls": len(kept), "avg_ns": sum(kept) / len(kept),
                                 "warm_launches": warm_launches("stats")}
fetch_b = fetch.get("FETCH_SIZE", 0) * 1024 / nf
write_b = write.get("WRITE_SIZE", 0) * 1024 / nw
cyc = wait.get("SQ_WAVE_CYCLES", 0)
ENGINE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "wtf_amd", "csrc", "libwtfgpu.so")
summary = {
    "kernel": "k_run",
    # the engine build these counters were taken on (bench.py drops a summary of another build)
    "engine_sha16": hashlib.sha256(open(ENGINE, "rb").read()).hexdigest()[:16],
    "leg": leg,
    "lanes": lanes,
    "limit": limit,
    "hbm_read_bytes_raw": fetch_b,
    "hbm_read_bytes_corrected": 2 * fetch_b,
    "hbm_write_bytes": write_b,
    "hbm_bytes_per_launch": 2 * fetch_b + write_b,
    "valu_util": wait.get("SQ_ACTIVE_INST_VALU", 0) / cyc if cyc else None,
    "wait_frac": wait.get("SQ_WAIT_ANY", 0) / cyc if cyc else None,
    "kernel_trace": stats,
    "dispatches": {"fetch": nf, "write": nw, "mix": nm, "wait": nwt},
    "instruction_mix_per_launch": {k: v / nm for k, v in mix.items()},
    "wave_cycles_per_launch": {k: v / nwt for k, v in wait.items()},
}
print(json.dumps(summary, indent=1))
