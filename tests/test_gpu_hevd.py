"""HEVD parity on the GPU: `wtfgpu` (ring-0 paths on the HIP engine: SYSCALL,
SWAPGS, SYSRETQ, RDRAND, supervisor pages; breakpoints serviced on the host)
against the oracle twin, testcase by testcase: result, crash name, retired
count, final registers and coverage set — bit-exact."""
import os

import pytest

from tests import tlv_harness as H
from tests.hevd_inputs import write_inputs

pytestmark = pytest.mark.gpu

FIELDS = ("result", "crash", "error", "icount", "gprs", "coverage")
LIMIT = 10_000_000  # BASELINE.md / README.md:58: HEVD runs --limit 10000000


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("hevd"))
    H.build_hevd_target(d)
    write_inputs(os.path.join(d, "parity"), 1000)
    return d


def test_hevd_full_coverage_parity(target, tmp_path):
    inp = os.path.join(target, "parity")
    g = H.run(H.WTFGPU, target, inp, str(tmp_path / "g.jsonl"), lanes=512, name="hevd", limit=LIMIT)
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=512, name="hevd", limit=LIMIT)
    assert len(g) == len(t) == len(os.listdir(inp))
    bad = []
    for x, y in zip(g, t):
        assert x["input"] == y["input"]
        for k in FIELDS:
            if x[k] != y[k]:
                bad.append((x["input"], k, x[k] if k != "coverage" else len(x[k]),
                            y[k] if k != "coverage" else len(y[k])))
    assert not bad, bad[:10]
    kinds = {r["crash"].split("-")[1] for r in g if r["crash"].startswith("crash-0x")}
    assert {"0xf7", "0x19"} <= kinds
    assert any(r["result"] == "cr3" for r in g)
    assert not any(r["error"] for r in g)


def test_hevd_parity_host_handlers_only(target, tmp_path):
    """nt!DbgPrintEx carries a device-side SimulateReturn action; with device
    actions off every hit is a host handler. Both must match the twin."""
    inp = os.path.join(target, "parity")
    h = H.run(H.WTFGPU, target, inp, str(tmp_path / "h.jsonl"), lanes=512, name="hevd", limit=LIMIT,
              env={"WTFGPU_DEVICE_BP_ACTIONS": "0"})
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=512, name="hevd", limit=LIMIT)
    bad = [(x["input"], k) for x, y in zip(h, t) for k in FIELDS if x[k] != y[k]]
    assert len(h) == len(t) and not bad, bad[:10]


@pytest.mark.parametrize("slice_steps,regroup", [(128, 0), (4096, 0), (4096, 256), (2048, 1024)])
def test_hevd_streaming_parity(target, tmp_path, slice_steps, regroup):
    """Continuous batching (two pipelined halves) with device actions (Rdrand,
    Stop, DbgPrintEx), host-serviced breakpoints (KeBugCheck2, SwapContext) and
    ring-0 paths, with and without cross-wave regrouping: every input as the twin."""
    inp = os.path.join(target, "parity")
    g = H.run(H.WTFGPU, target, inp, str(tmp_path / "g.jsonl"), lanes=256, name="hevd", limit=LIMIT,
              extra=("--stream-run", "--slice-steps", str(slice_steps), "--regroup-steps", str(regroup)))
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=512, name="hevd", limit=LIMIT)
    bad = [(x["input"], k) for x, y in zip(g, t) for k in FIELDS if x[k] != y[k]]
    assert len(g) == len(t) and not bad, bad[:10]


def test_hevd_fuzz_smoke(target):
    st = H.fuzz(H.WTFGPU, target, runs=8192, lanes=4096, name="hevd", max_len=1028, limit=LIMIT)
    assert st["execs"] == 8192 and st["errors"] == 0
