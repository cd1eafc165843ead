"""TLV on the CPU: the synthetic snapshot, the tlv module and the batched
runner driven through the oracle twin (no GPU)."""
import os

import pytest

from tests import tlv_harness as H
from tests.tlv_inputs import write_inputs
from wtf_amd.tools.snapshot import read_kdmp

pytestmark = pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    return H.build_target(str(tmp_path_factory.mktemp("tlv")))


def test_snapshot_layout(target):
    index, _, cr3 = read_kdmp(os.path.join(target, "state", "mem.dmp"))
    assert cr3 and len(index) > 64  # code, data, 64 heap slots, packet page, stack, tables


def test_seeds_run_ok(target, tmp_path):
    res = H.run(H.TWIN, target, os.path.join(target, "inputs"), str(tmp_path / "r.jsonl"), lanes=8)
    assert [r["result"] for r in res] == ["ok"] * 4
    assert all(r["icount"] > 50 and r["coverage"] for r in res)
    # every testcase ends at the ProcessPacket breakpoint with no packet left
    assert len({r["gprs"][16] for r in res}) == 1


def test_edge_cases(target, tmp_path):
    d = str(tmp_path / "in")
    write_inputs(d, 0)
    res = {r["input"]: r for r in H.run(H.TWIN, target, d, str(tmp_path / "r.jsonl"), lanes=8)}
    assert res["edge_no_packets"]["result"] == "ok" and res["edge_no_packets"]["icount"] == 0
    assert res["edge_too_big"]["result"] == "ok"
    assert res["edge_bad_json"]["crash"] == "insert-testcase-failed"
    # the fifth Allocate lands past the 4-entry table, on LastFreed: nothing was
    # deleted yet, so the pointer it overwrote is null and nothing is freed
    assert res["edge_five_allocs"]["result"] == "ok"
    assert res["edge_big_edit"]["crash"].startswith("crash-EXCEPTION_ACCESS_VIOLATION")
    # a free the heap rejects: __fastfail = int 0x29 through the IDT gate to
    # nt!KiRaiseSecurityCheckFailure, named from the return address at [rsp]
    ff = res["edge_fastfail"]
    assert ff["crash"].startswith("crash-EXCEPTION_STACK_BUFFER_OVERRUN-0x140"), ff["crash"]


def test_batch_size_does_not_change_results(target, tmp_path):
    d = str(tmp_path / "in")
    write_inputs(d, 200)
    a = H.run(H.TWIN, target, d, str(tmp_path / "a.jsonl"), lanes=1)
    b = H.run(H.TWIN, target, d, str(tmp_path / "b.jsonl"), lanes=64)
    assert a == b


def test_fuzz_finds_crashes(target):
    st = H.fuzz(H.TWIN, target, runs=3000, lanes=512)
    assert st["execs"] == 3000 and st["errors"] == 0
    assert st["unique_crashes"] >= 2 and st["coverage"] > 100
    assert os.listdir(os.path.join(target, "crashes"))
