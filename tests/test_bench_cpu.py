"""bench.py's plumbing on the CPU: snapshot builds, the one-process-per-core
twin baselines, and the JSON field arithmetic (roofline, node fields)."""
import os

import pytest

import bench

from tests.cpu_bins import TWIN  # noqa: E402


@pytest.mark.skipif(not os.path.exists(TWIN), reason="oracle/wtf_twin not built")
@pytest.mark.parametrize("name", ["tlv_server", "hevd", "hevd_bare"])
def test_twin_baseline_fields(name, tmp_path):
    d = bench.build_target(name, str(tmp_path / name))
    cb = bench.twin_baseline(name, d, seconds=1.0, cores=2, limit=100000)
    assert cb["cores"] == 2 and cb["kind"] == "port" and cb["value"] > 0 and cb["instr_per_s"] > 0


def test_roofline_and_node_fields():
    r = bench.roofline(alg_bytes=8e9, launches=4, kernel_ms=100.0, pmc=None)
    assert r["achieved"] == pytest.approx(2e9 / 0.025 / 1e9)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0) and r["traffic"] is None
    keys = ("execs retired batches crashes unique_crashes timeouts cr3 errors coverage corpus merged_rips "
            "kernel_launches group_steps alg_bytes breakpoint_hits rounds error_retired run_s kernel_ms "
            "merge_ms insert_ms coverage_ms service_ms total_ms").split()
    s0 = {k: 0 for k in keys}
    s1 = dict(s0, retired=6400, group_steps=200, error_retired=64, kernel_launches=2, kernel_ms=5.0)
    f = bench.node_fields(s0, s1)
    assert f["lanes_per_wave_step"] == 32 and f["gpu_retired_fraction"] == pytest.approx(0.99)


def test_cpu_cores_reports_share():
    used, info = bench.cpu_cores()
    assert used >= 1 and info["used"] == used and info["os_cpu_count"] >= 1


@pytest.mark.skipif(not os.path.exists(TWIN), reason="oracle/wtf_twin not built")
def test_hevd_io_seeds_return_a_status(tmp_path):
    """The hevd leg's snapshot (wtf_amd/tools/hevd_io.py): every seed takes the
    I/O manager's IRP path to a status (Ok, no bugcheck), the benign requests
    run thousands of instructions, and the bare path is far shorter."""
    from tests import tlv_harness as H

    d = bench.build_target("hevd", str(tmp_path / "io"))
    res = {r["input"]: r for r in H.run(H.TWIN, d, os.path.join(d, "inputs"), str(tmp_path / "r.jsonl"), lanes=64,
                                         limit=10_000_000, name="hevd")}
    assert all(r["result"] == "ok" and not r["error"] for r in res.values()), res
    assert res["crc_1024"]["icount"] > 10000 and res["records_types"]["icount"] > 1500
    assert 400 < res["invalid"]["icount"] < 1000  # the IRP path alone, around an unknown IOCTL
    b = bench.build_target("hevd_bare", str(tmp_path / "bare"))
    bare = {r["input"]: r for r in H.run(H.TWIN, b, os.path.join(b, "inputs"), str(tmp_path / "b.jsonl"), lanes=64,
                                          limit=10_000_000, name="hevd")}
    assert bare["invalid"]["icount"] < res["invalid"]["icount"] // 2
