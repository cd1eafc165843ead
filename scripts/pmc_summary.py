"""Summarise rocprofv3 CSV output of scripts/gpu_profile_round.sh for k_run.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled (k_run's reads are not all wide streams: the
corrected read side is an upper bound, the raw one a lower bound)."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]


def per_kernel(sub):
    out, disp = {}, set()
    for f in glob.glob(os.path.join(d, sub, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "k_run" not in r["Kernel_Name"]:
                continue
            disp.add(r["Dispatch_Id"])
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out, max(1, len(disp))


fetch, nf = per_kernel("pmc_fetch")
write, nw = per_kernel("pmc_write")
mix, nm = per_kernel("pmc_mix")
wait, nwt = per_kernel("pmc_wait")
stats = {}
for f in glob.glob(os.path.join(d, "stats", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "k_run" in r["Name"]:
            stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "pct": float(r["Percentage"])}
bench = {}
for line in open(os.path.join(d, "bench.json.log")):
    if line.startswith("{"):
        bench = json.loads(line)
fetch_b = fetch.get("FETCH_SIZE", 0) * 1024 / nf
write_b = write.get("WRITE_SIZE", 0) * 1024 / nw
steps = None
summary = {
    "kernel": "k_run",
    "lanes": bench.get("config", {}).get("lanes_per_gpu"),
    "limit": bench.get("config", {}).get("limit"),
    "hbm_read_bytes_raw": fetch_b,
    "hbm_read_bytes_corrected": 2 * fetch_b,
    "hbm_write_bytes": write_b,
    "hbm_bytes_per_launch": 2 * fetch_b + write_b,
    "kernel_trace": stats,
    "instruction_mix_per_launch": {k: v / nm for k, v in mix.items()},
    "wave_cycles_per_launch": {k: v / nwt for k, v in wait.items()},
}
print(json.dumps(summary, indent=1))
