"""bench.py's fuzz legs on the CPU: the plumbing (snapshot build, node run,
per-core twin clients, JSON fields) with the oracle twin standing in for the
gpu node."""
import os

import pytest

import bench

TWIN = os.path.join(bench.ROOT, "oracle", "wtf_twin")


@pytest.mark.skipif(not os.path.exists(TWIN), reason="oracle/wtf_twin not built")
@pytest.mark.parametrize("name", ["tlv_server", "hevd"])
def test_fuzz_leg_fields(name):
    r = bench.fuzz_leg(name, lanes=256, batches=2, cpu_seconds=1.0, cores=2, limit=100000, run_cpu=True,
                       gpu_exe=TWIN)
    assert r["execs"] == 512 and r["value"] > 0 and r["errors"] == 0
    cb = r["cpu_baseline"]
    assert cb["cores"] == 2 and cb["kind"] == "port" and cb["value"] > 0
    assert r["vs_cpu"] == pytest.approx(r["value"] / cb["value"])
