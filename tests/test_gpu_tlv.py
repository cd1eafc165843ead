"""TLV parity on the GPU: `wtfgpu` (GpuBackend_t over the HIP engine, batched
lanes, breakpoints serviced on the host with per-lane module state) against
the oracle twin (one testcase after the other, the reference client loop),
testcase by testcase: result, crash name, retired count, final registers and
coverage set — bit-exact."""
import os

import pytest

from tests import tlv_harness as H
from tests.tlv_inputs import write_inputs

pytestmark = pytest.mark.gpu

FIELDS = ("result", "crash", "error", "icount", "gprs", "coverage")


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("tlv"))
    H.build_target(d)
    write_inputs(os.path.join(d, "parity"), 1500)
    return d


def _diff(a, b):
    bad = []
    for x, y in zip(a, b):
        assert x["input"] == y["input"]
        for k in FIELDS:
            if x[k] != y[k]:
                bad.append((x["input"], k, x[k] if k != "coverage" else len(x[k]),
                            y[k] if k != "coverage" else len(y[k])))
    return bad


def test_tlv_full_coverage_parity(target, tmp_path):
    inp = os.path.join(target, "parity")
    g = H.run(H.WTFGPU, target, inp, str(tmp_path / "g.jsonl"), lanes=512)
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=512)
    assert len(g) == len(t) == len(os.listdir(inp))
    bad = _diff(g, t)
    assert not bad, bad[:10]
    assert sum(r["result"] == "crash" for r in g) > 10
    assert not any(r["error"] for r in g)
    # __fastfail: int 0x29 through the snapshot's IDT gate (DPL 3, stack switch to
    # RSP0) to nt!KiRaiseSecurityCheckFailure, named from the address at [rsp]
    # (crash_detection_umode.cc:131-152), identical on both backends
    ff = [r for r in g if r["input"] == "edge_fastfail"]
    assert ff and ff[0]["crash"].startswith("crash-EXCEPTION_STACK_BUFFER_OVERRUN-0x"), ff


def test_tlv_parity_host_handlers_only(target, tmp_path):
    """ProcessPacket (Feed), the return address (SetGprs) and printf
    (SimulateReturn) carry device-side actions (BreakpointAction_t); with them
    switched off every hit goes through the host handler. Both paths must
    match the twin."""
    inp = os.path.join(target, "parity")
    h = H.run(H.WTFGPU, target, inp, str(tmp_path / "h.jsonl"), lanes=512,
              env={"WTFGPU_DEVICE_BP_ACTIONS": "0"})
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=512)
    assert not _diff(h, t)


def test_tlv_lane_order_coverage_attribution(target, tmp_path):
    """Without --full-coverage each lane reports only coverage no earlier lane
    (or batch) found: the order-dependent LastNewCoverage of the serial client."""
    inp = os.path.join(target, "parity")
    g = H.run(H.WTFGPU, target, inp, str(tmp_path / "g.jsonl"), lanes=256, full_coverage=False)
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=256, full_coverage=False)
    assert not _diff(g, t)


@pytest.mark.parametrize("slice_steps,regroup", [(64, 0), (2048, 0), (2048, 256), (4096, 1024)])
def test_tlv_streaming_parity(target, tmp_path, slice_steps, regroup):
    """Continuous batching (lanes refilled as their testcases finish: per-lane
    restore, feed regions, per-lane coverage collection) replays every input
    exactly as the twin does; short slices force many refills and lanes that
    straddle slices."""
    inp = os.path.join(target, "parity")
    g = H.run(H.WTFGPU, target, inp, str(tmp_path / "g.jsonl"), lanes=256,
              extra=("--stream-run", "--slice-steps", str(slice_steps), "--regroup-steps", str(regroup)))
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=512)
    assert len(g) == len(t)
    assert not _diff(g, t)


@pytest.mark.parametrize("slice_steps", [0, 4096])
def test_tlv_fuzz_smoke(target, slice_steps):
    st = H.fuzz(H.WTFGPU, target, runs=8192, lanes=4096, extra=("--slice-steps", str(slice_steps)))
    assert st["execs"] == 8192 and st["errors"] == 0
    assert st["unique_crashes"] >= 2 and st["coverage"] >= 150
