"""Summarise the rocprofv3 CSV output of scripts/gpu_pmc.sh for k_run on one
workload: python3 scripts/pmc_summary.py <dir> <leg> <lanes> <limit>.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled (k_run's reads are not all wide streams: the
corrected read side is an upper bound, the raw one a lower bound).
valu_util = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, wait_frac = SQ_WAIT_ANY /
SQ_WAVE_CYCLES (both summed over k_run dispatches). engine_sha16 binds the
summary to the libwtfgpu.so it was measured on."""
import csv
import glob
import hashlib
import json
import os
import sys

d, leg, lanes, limit = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])


def per_kernel(sub):
    out, disp = {}, set()
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_run" not in r["Kernel_Name"]:
                continue
            disp.add((f, r["Dispatch_Id"]))
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out, max(1, len(disp))


fetch, nf = per_kernel("fetch")
write, nw = per_kernel("write")
mix, nm = per_kernel("mix")
wait, nwt = per_kernel("wait")
stats = {}
for f in glob.glob(os.path.join(d, "stats", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_run" in r["Name"]:
            stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "pct": float(r["Percentage"])}
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
