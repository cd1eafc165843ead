"""scripts/pmc_summary.py on synthetic rocprofv3 CSVs (no GPU): counters and
the kernel-trace average leave the workload's warm-up launches out (the count
prof_leg.py prints), other kernels never count, the summary names the engine
build, and bench.load_pmc accepts only a summary of this very build."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINE = os.path.join(ROOT, "wtf_amd", "csrc", "libwtfgpu.so")
K = "(anonymous namespace)::k_run(wtfgpu_dev::Dev, unsigned int, unsigned int, unsigned long)"


def _counters(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for r in rows:
            w.writerow(r)


def _pass(d, name, counters, warm):
    # dispatches 1..6 of k_run (the first `warm` are the warm-up), one other kernel
    rows = []
    for i in range(1, 7):
        for c, v in counters.items():
            rows.append({"Dispatch_Id": i * 2, "Kernel_Name": K, "Counter_Name": c, "Counter_Value": v * i})
        rows.append({"Dispatch_Id": i * 2 + 1, "Kernel_Name": "k_restore_list", "Counter_Name": next(iter(counters)),
                     "Counter_Value": 1e9})
    _counters(os.path.join(d, name, "run", "run_counter_collection.csv"), rows)
    with open(os.path.join(d, name + ".log"), "w") as f:
        f.write("noise\n" + json.dumps({"leg": "tlv", "warm_launches": warm}) + "\n")


@pytest.mark.skipif(not os.path.exists(ENGINE), reason="engine not built (__graft_entry__.build)")
def test_pmc_summary_leaves_warmup_out(tmp_path):
    d = str(tmp_path)
    warm = 2
    _pass(d, "fetch", {"FETCH_SIZE": 1.0}, warm)
    _pass(d, "write", {"WRITE_SIZE": 2.0}, warm)
    _pass(d, "mix", {"SQ_WAVES": 1.0, "SQ_INSTS_VALU": 10.0}, warm)
    _pass(d, "wait", {"SQ_WAVE_CYCLES": 100.0, "SQ_WAIT_ANY": 50.0, "SQ_ACTIVE_INST_VALU": 20.0}, warm)
    st = os.path.join(d, "stats", "run")
    os.makedirs(st)
    with open(os.path.join(st, "run_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        w.writerow([K, 6, 2100, 350.0, 90.0, 100, 600, 0])
    with open(os.path.join(st, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Dispatch_Id", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for i in range(1, 7):  # durations 100, 200, ..., 600 ns
            w.writerow({"Kernel_Name": K, "Dispatch_Id": i, "Start_Timestamp": 1000 * i,
                        "End_Timestamp": 1000 * i + 100 * i})
    with open(os.path.join(d, "stats.log"), "w") as f:
        f.write(json.dumps({"warm_launches": warm}) + "\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), d, "tlv", "262144",
                          "100000"], check=True, capture_output=True, text=True).stdout
    s = json.loads(out)
    # launches 3..6 only: FETCH_SIZE (3+4+5+6) KB / 4, doubled for gfx950
    assert s["dispatches"] == {"fetch": 4, "write": 4, "mix": 4, "wait": 4}
    assert s["hbm_read_bytes_raw"] == pytest.approx(18 * 1024 / 4)
    assert s["hbm_read_bytes_corrected"] == pytest.approx(2 * 18 * 1024 / 4)
    assert s["hbm_write_bytes"] == pytest.approx(2 * 18 * 1024 / 4)
    assert s["instruction_mix_per_launch"]["SQ_INSTS_VALU"] == pytest.approx(10 * 18 / 4)
    assert s["wait_frac"] == pytest.approx(0.5) and s["valu_util"] == pytest.approx(0.2)
    kt = s["kernel_trace"]
    assert kt["calls"] == 6 and kt["avg_ns"] == 350.0
    assert kt["after_warmup"] == {"calls": 4, "avg_ns": 450.0, "warm_launches": 2}
    assert len(s["engine_sha16"]) == 16

    # bench.load_pmc: accepted for this build, dropped for another
    sys.path.insert(0, ROOT)
    import bench

    assert s["engine_sha16"] == bench.engine_sha16()
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_tlv_k_run.json").write_text(json.dumps(s))
    old = bench.PROFILES
    try:
        bench.PROFILES = str(prof)
        assert bench.load_pmc("tlv", 262144, 100000)["hbm_bytes_per_launch"] == s["hbm_bytes_per_launch"]
        assert bench.load_pmc("tlv", 131072, 100000) is None
        (prof / "pmc_tlv_k_run.json").write_text(json.dumps(dict(s, engine_sha16="0" * 16)))
        assert bench.load_pmc("tlv", 262144, 100000) is None
    finally:
        bench.PROFILES = old
