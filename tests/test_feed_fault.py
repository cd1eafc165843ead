"""The tlv module's packet writes when the packet buffer is not a plain
read-write page (fuzzer_tlv_server.cc:130-158 writes each packet with
VirtWriteStructDirty / VirtWriteDirty and std::abort()s when one fails):

  * read-only page: Backend_t::VirtWrite translates with ValidateRead only
    (backend.cc:91-121), so the writes land and every testcase ends as with a
    read-write page: on the twin (host handler) and on the GPU (device Feed
    action, whose stores skip the U/S and R/W checks the same way);
  * no page at all: the write fails; the twin's handler aborts the process,
    the GPU backend's device Feed action exits WTFGPU_EXIT_FEED_FAULT and the
    run fails with an error (never a testcase result).
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


def _cmp(a, b):
    assert len(a) == len(b)
    bad = [(x["input"], k) for x, y in zip(a, b) for k in ("result", "crash", "icount", "gprs", "coverage")
           if x[k] != y[k]]
    assert not bad, bad[:5]


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_twin_read_only_packet_page(targets, tmp_path):
    rw, ro = targets["rw"], targets["ro"]
    a = H.run(H.TWIN, rw, os.path.join(rw, "parity"), str(tmp_path / "rw.jsonl"), lanes=64)
    b = H.run(H.TWIN, ro, os.path.join(ro, "parity"), str(tmp_path / "ro.jsonl"), lanes=64)
    _cmp(a, b)


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_twin_missing_packet_page_aborts(targets, tmp_path):
    t = targets["none"]
    with pytest.raises(subprocess.CalledProcessError) as e:
        H.run(H.TWIN, t, os.path.join(t, "inputs"), str(tmp_path / "n.jsonl"), lanes=4)
    assert e.value.returncode in (-6, 134)


@pytest.mark.gpu
def test_gpu_read_only_packet_page(targets, tmp_path):
    rw, ro = targets["rw"], targets["ro"]
    a = H.run(H.TWIN, rw, os.path.join(rw, "parity"), str(tmp_path / "rw.jsonl"), lanes=64)
    b = H.run(H.WTFGPU, ro, os.path.join(ro, "parity"), str(tmp_path / "ro.jsonl"), lanes=512)
    _cmp(a, b)


@pytest.mark.gpu
def test_gpu_missing_packet_page_is_a_run_error(targets, tmp_path):
    t = targets["none"]
    cmd = [H.WTFGPU, "run", "--name", "tlv_server", "--target", t, "--input", os.path.join(t, "inputs"),
           "--results", str(tmp_path / "n.jsonl"), "--lanes", "64", "--limit", "100000"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and p.returncode > 0
    assert "VirtWriteDirty failed" in p.stderr and "RunBatch failed" in p.stdout
    # the fuzz loop stops the same way
    p = subprocess.run([H.WTFGPU, "fuzz", "--name", "tlv_server", "--target", t, "--runs", "256", "--lanes", "64",
                        "--limit", "100000"], capture_output=True, text=True, timeout=120)
    assert p.returncode > 0 and "VirtWriteDirty failed" in p.stderr
