"""U43: a handler's (or InsertTestcase's) guest access whose translation
fails ends that testcase as an engine error, on the twin and on the GPU node.

The reference stops the whole node at such an access: Backend_t::VirtRead /
VirtWrite print the GVA and run `int3` (__debugbreak, backend.cc:39-42,
58-72, 101-104; platform.h:35), as do VirtRead4 / VirtRead8 and the string
readers (backend.h:352-356). Batched, one testcase must not take its lanes'
neighbours with it: the helper abandons the handler at the access (where the
reference stops), the testcase is an engine error (an unnamed crash with
`error` set, kept under errors/ by the fuzz loop), every other testcase of the
batch ends as it would alone.

The probe module (tests/native/fault_probe_module.cc, --module-so) picks the
access from the testcase's first byte."""
import os

import pytest

from tests import tlv_harness as H
from tests.cpu_bins import ensure

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "native", "libfaultprobe.so")

# mode -> (result, crash name, engine error)
EXPECT = {
    0: ("ok", "", 0),
    1: ("crash", "", 1),   # VirtRead8(0)
    2: ("crash", "", 1),   # VirtReadString into an unmapped page
    3: ("crash", "", 1),   # VirtWriteDirty(0x10)
    4: ("crash", "", 1),   # InsertTestcase's VirtWrite(0x10)
    5: ("crash", "probe-done", 0),  # SimulateReturnFromFunction on a good stack
    6: ("crash", "probe-arg", 0),   # GetArg(4)
}


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    ensure(PROBE, os.path.join(ROOT, "tests", "native"), "libfaultprobe.so")
    d = str(tmp_path_factory.mktemp("probe"))
    H.build_target(d)
    inp = os.path.join(d, "probe")
    os.makedirs(inp)
    # each mode several times, interleaved, so that faulting lanes sit
    # between lanes that must finish normally
    for i in range(35):
        with open(os.path.join(inp, f"p{i:03d}"), "wb") as f:
            f.write(bytes([i % 7, i]))
    return d


def _check(rows):
    assert len(rows) == 35
    for r in rows:
        mode = int(r["input"][1:]) % 7
        assert (r["result"], r["crash"], r["error"]) == EXPECT[mode], (r["input"], r)


def test_twin_handler_fault_is_engine_error(target, tmp_path):
    rows = H.run(H.TWIN, target, os.path.join(target, "probe"), str(tmp_path / "t.jsonl"), lanes=35,
                 name="fault_probe", extra=("--module-so", PROBE))
    _check(rows)


def test_twin_serial_client_handler_fault(target, tmp_path):
    """The reference client loop shape (--serial: InsertTestcase, Run, Restore)."""
    rows = H.run(H.TWIN, target, os.path.join(target, "probe"), str(tmp_path / "t.jsonl"), lanes=1,
                 name="fault_probe", extra=("--module-so", PROBE, "--serial"))
    _check(rows)


@pytest.mark.gpu
def test_gpu_handler_fault_is_engine_error(target, tmp_path):
    rows = H.run(H.WTFGPU, target, os.path.join(target, "probe"), str(tmp_path / "g.jsonl"), lanes=64,
                 name="fault_probe", extra=("--module-so", PROBE))
    _check(rows)
    twin = H.run(H.TWIN, target, os.path.join(target, "probe"), str(tmp_path / "t.jsonl"), lanes=35,
                 name="fault_probe", extra=("--module-so", PROBE))
    for g, t in zip(rows, twin):
        for k in ("result", "crash", "error", "icount", "gprs"):
            assert g[k] == t[k], (g["input"], k)
