"""The Backend_t boundary one testcase at a time: `run --serial` drives the
backend through a restatement of the reference client's
RunTestcaseAndRestore (/root/reference/src/wtf/client.cc:88-180; contract
backend.h:178): Target.InsertTestcase -> Backend.Run -> RevokeLastNewCoverage
on a timeout -> Target.Restore -> Backend.Restore(State), and reads the final
registers through GetReg and the new coverage through LastNewCoverage. Its
results must equal the batched path's (RunBatch) for the same inputs:

  * the twin (CPU): serial == batch, field by field, with and without
    --full-coverage (the twin's batch runs in lane order, so even new-coverage
    attribution matches);
  * the GPU backend (gpu): serial == its own RunBatch and == the twin's
    serial run, result / crash / error / icount / GPRs / coverage.
"""
import os

import pytest

from tests import tlv_harness as H
from tests.tlv_inputs import write_inputs

LIMIT = 1500
FIELDS = ("result", "crash", "error", "icount", "gprs", "coverage")


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    d = H.build_target(str(tmp_path_factory.mktemp("serial")))
    write_inputs(os.path.join(d, "parity"), 400)
    return d


def _diff(a, b, fields=FIELDS):
    assert len(a) == len(b)
    bad = []
    for x, y in zip(a, b):
        assert x["input"] == y["input"]
        for k in fields:
            if x[k] != y[k]:
                bad.append((x["input"], k, x[k], y[k]))
    return bad


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
@pytest.mark.parametrize("full", [True, False])
def test_twin_serial_equals_batch(target, tmp_path, full):
    inp = os.path.join(target, "parity")
    # a limit some inputs exceed: timeouts are in the set
    ser = H.run(H.TWIN, target, inp, str(tmp_path / "s.jsonl"), lanes=1, limit=LIMIT, full_coverage=full,
                extra=("--serial",))
    bat = H.run(H.TWIN, target, inp, str(tmp_path / "b.jsonl"), lanes=256, limit=LIMIT, full_coverage=full)
    bad = _diff(ser, bat)
    assert not bad, bad[:5]
    assert {r["result"] for r in ser} >= {"ok", "crash"}
    # timeouts are in the set: their coverage is printed, then revoked
    assert any(r["result"] == "timedout" for r in ser)


@pytest.mark.gpu
def test_gpu_serial_equals_batch_and_twin(target, tmp_path):
    inp = os.path.join(target, "parity")
    ser = H.run(H.WTFGPU, target, inp, str(tmp_path / "gs.jsonl"), lanes=512, limit=LIMIT, extra=("--serial",),
                timeout=600)
    bat = H.run(H.WTFGPU, target, inp, str(tmp_path / "gb.jsonl"), lanes=512, limit=LIMIT)
    tw = H.run(H.TWIN, target, inp, str(tmp_path / "ts.jsonl"), lanes=1, limit=LIMIT, extra=("--serial",))
    bad = _diff(ser, bat) + _diff(ser, tw)
    assert not bad, bad[:5]


@pytest.mark.gpu
def test_gpu_serial_aggregate_coverage(target, tmp_path):
    """Without --full-coverage each serial testcase reports what it adds to the
    aggregate (bochscpu_backend.cc:501-504): equal to the twin's serial run."""
    inp = os.path.join(target, "parity")
    ser = H.run(H.WTFGPU, target, inp, str(tmp_path / "gs.jsonl"), lanes=512, limit=LIMIT, full_coverage=False,
                extra=("--serial",), timeout=600)
    tw = H.run(H.TWIN, target, inp, str(tmp_path / "ts.jsonl"), lanes=1, limit=LIMIT, full_coverage=False,
               extra=("--serial",))
    bad = _diff(ser, tw)
    assert not bad, bad[:5]
