"""The tlv module's packet writes when the packet buffer is not a plain
read-write page (fuzzer_tlv_server.cc:130-158 writes each packet with
VirtWriteStructDirty / VirtWriteDirty and std::abort()s when one fails):

  * read-only page: Backend_t::VirtWrite translates with ValidateRead only
    (backend.cc:91-121), so the writes land and every testcase ends as with a
    read-write page: on the twin (host handler) and on the GPU (device Feed
    action, whose stores skip the U/S and R/W checks the same way);
  * no page at all: the write fails. The reference node stops there
    (VirtWrite's __debugbreak, backend.cc:101-104); here the handler is
    abandoned and the testcase ends as an engine error (U43): on the twin
    (host handler, HandlerFault_t) and on the GPU (the device Feed action exits
    WTFGPU_EXIT_FEED_FAULT), testcase by testcase the same; a testcase with no
    packet to write ends Ok on both.
"""
import os
import subprocess

import pytest

from tests import tlv_harness as H
from tests.tlv_inputs import write_inputs


def _target(d, packet):
    from wtf_amd.tools.tlv import build, seed_inputs
    build(os.path.join(d, "state"), os.path.join(d, "work"), packet=packet)
    seed_inputs(os.path.join(d, "inputs"))
    write_inputs(os.path.join(d, "parity"), 300)
    return d


@pytest.fixture(scope="module")
def targets(tmp_path_factory):
    base = tmp_path_factory.mktemp("feed")
    return {p: _target(str(base / p), p) for p in ("rw", "ro", "none")}


def _cmp(a, b, keys=("result", "crash", "icount", "gprs", "coverage")):
    assert len(a) == len(b)
    bad = [(x["input"], k) for x, y in zip(a, b) for k in keys if x[k] != y[k]]
    assert not bad, bad[:5]


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_twin_read_only_packet_page(targets, tmp_path):
    rw, ro = targets["rw"], targets["ro"]
    a = H.run(H.TWIN, rw, os.path.join(rw, "parity"), str(tmp_path / "rw.jsonl"), lanes=64)
    b = H.run(H.TWIN, ro, os.path.join(ro, "parity"), str(tmp_path / "ro.jsonl"), lanes=64)
    _cmp(a, b)


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_twin_missing_packet_page_is_engine_error(targets, tmp_path):
    t = targets["none"]
    rows = H.run(H.TWIN, t, os.path.join(t, "parity"), str(tmp_path / "n.jsonl"), lanes=64)
    errs = [r for r in rows if r["error"]]
    assert len(errs) > len(rows) // 2
    assert all(r["result"] == "crash" and r["crash"] == "" for r in errs)
    # the rest never write a packet: no packet at all, or JSON the module rejects
    assert {(r["result"], r["crash"]) for r in rows if not r["error"]} <= {("ok", ""),
                                                                          ("crash", "insert-testcase-failed")}


@pytest.mark.gpu
def test_gpu_read_only_packet_page(targets, tmp_path):
    rw, ro = targets["rw"], targets["ro"]
    a = H.run(H.TWIN, rw, os.path.join(rw, "parity"), str(tmp_path / "rw.jsonl"), lanes=64)
    b = H.run(H.WTFGPU, ro, os.path.join(ro, "parity"), str(tmp_path / "ro.jsonl"), lanes=512)
    _cmp(a, b)


@pytest.mark.gpu
def test_gpu_missing_packet_page_is_engine_error(targets, tmp_path):
    t = targets["none"]
    a = H.run(H.TWIN, t, os.path.join(t, "parity"), str(tmp_path / "t.jsonl"), lanes=64)
    b = H.run(H.WTFGPU, t, os.path.join(t, "parity"), str(tmp_path / "g.jsonl"), lanes=512)
    _cmp(a, b, ("result", "crash", "error", "icount"))
    # the registers of a testcase abandoned mid-handler are the handler's
    # partial work (the reference node stops there): compared where it finished
    _cmp([r for r in a if not r["error"]], [r for r in b if not r["error"]], ("gprs",))
    # the node finishes the batch and keeps the testcases under errors/; then
    # it stops where the reference's mutator does ("The corpus is empty,
    # exiting", mutator.cc:27-31): every testcase errored, none joined the corpus
    st = H.fuzz(H.WTFGPU, t, runs=4096, lanes=512, timeout=120)
    assert st["execs"] >= 512 and st["errors"] > 0 and st["backend"]["err_handler"] == st["errors"]
    assert os.listdir(os.path.join(t, "errors"))
