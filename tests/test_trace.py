"""Rip traces (`run --trace-path --trace-type rip|cov`; SURVEY §8(f) rank 4,
BochscpuBackend_t::SetTraceFile / BeforeExecutionHook, bochscpu_backend.cc:
506-520, subcommands.cc:52-74): one `<input>.trace` per input, one "%#x" rip
per line, every rip about to execute (rip) or only those new to the aggregate
(cov), which the Restore after a traced run empties (bochscpu_backend.cc:
778-789): a cov trace holds the rips unique within its run. Under --runs only
an input's first run is traced (the same Restore closes the file). The GPU records them on the device (wtfgpu_set_trace); the twin from
the oracle; their files must be identical. Tenet traces (`--trace-type
tenet`, bochscpu_backend.cc:1215-1323; the format is checked in
tests/test_tenet.py) likewise, byte for byte.
"""
import os

import pytest

from tests import tlv_harness as H

pytestmark = pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")


def read_trace(path):
    with open(path) as f:
        return [int(x, 16) for x in f.read().split()]


def traces(exe, target, out, kind="rip", name="tlv_server", lanes=16, runs=1):
    res = H.run(exe, target, os.path.join(target, "inputs"), str(out) + ".jsonl", lanes=lanes, name=name,
                extra=["--trace-path", str(out), "--trace-type", kind] + (["--runs", str(runs)] if runs > 1 else []))
    return res, {f[:-6]: read_trace(os.path.join(out, f)) for f in os.listdir(out)}


@pytest.fixture(scope="module")
def tlv(tmp_path_factory):
    return H.build_target(str(tmp_path_factory.mktemp("tlvt")))


@pytest.fixture(scope="module")
def hevd(tmp_path_factory):
    return H.build_hevd_target(str(tmp_path_factory.mktemp("hevdt")))


def test_twin_rip_trace_is_the_executed_rips(tlv, tmp_path):
    res, tr = traces(H.TWIN, tlv, tmp_path / "t")
    assert set(tr) == {r["input"] for r in res}
    for r in res:
        t = tr[r["input"]]
        assert t[0] == 0x140001000 or len(t) > 0
        assert set(t) == set(r["coverage"])  # full coverage = every rip the hook saw
        assert len(t) >= r["icount"]


def _first_occurrences(rips, seen):
    want = []
    for v in rips:
        if v not in seen:
            seen.add(v)
            want.append(v)
    return want


def test_cov_trace_is_the_run_s_unique_rips(tlv, tmp_path):
    _, rip = traces(H.TWIN, tlv, tmp_path / "r", "rip")
    _, cov = traces(H.TWIN, tlv, tmp_path / "c", "cov")
    for name in sorted(rip):
        assert cov[name] == _first_occurrences(rip[name], set()), name


def test_runs_trace_the_first_run_only(tlv, tmp_path):
    """--runs 3: each input's first run is traced; its other two runs add
    their rips to the aggregate the next input's cov trace starts from (the
    reference empties it only after a traced run)."""
    _, rip = traces(H.TWIN, tlv, tmp_path / "r", "rip")
    res3, rip3 = traces(H.TWIN, tlv, tmp_path / "r3", "rip", runs=3)
    assert rip3 == rip and len(res3) == 3 * len(rip)
    _, cov3 = traces(H.TWIN, tlv, tmp_path / "c3", "cov", runs=3)
    prev = set()
    for name in sorted(rip):
        assert cov3[name] == _first_occurrences(rip[name], set(prev)), name
        prev = set(rip[name])


def test_existing_traces_are_skipped(tlv, tmp_path):
    out = tmp_path / "s"
    traces(H.TWIN, tlv, out)
    first = sorted(os.listdir(out))
    victim = os.path.join(out, first[0])
    with open(victim, "w") as f:
        f.write("0x1\n")
    traces(H.TWIN, tlv, out)
    assert read_trace(victim) == [1]


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["tlv", "hevd"])
def test_gpu_traces_equal_twin(which, tlv, hevd, tmp_path):
    target, name = (tlv, "tlv_server") if which == "tlv" else (hevd, "hevd")
    for kind, runs in (("rip", 1), ("cov", 1), ("cov", 2)):
        ra, a = traces(H.TWIN, target, tmp_path / f"twin_{kind}{runs}", kind, name=name, runs=runs)
        rb, b = traces(H.WTFGPU, target, tmp_path / f"gpu_{kind}{runs}", kind, name=name, runs=runs)
        assert a == b, kind
        assert sum(len(t) for t in a.values()) > 100


def tenet_files(exe, target, out, name):
    H.run(exe, target, os.path.join(target, "inputs"), str(out) + ".jsonl", lanes=16, name=name,
          extra=["--trace-path", str(out), "--trace-type", "tenet"])
    files = {}
    for f in os.listdir(out):
        with open(os.path.join(out, f), "rb") as fh:
            files[f] = fh.read()
    return files


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["tlv", "hevd"])
def test_gpu_tenet_traces_equal_twin(which, tlv, hevd, tmp_path):
    target, name = (tlv, "tlv_server") if which == "tlv" else (hevd, "hevd")
    a = tenet_files(H.TWIN, target, tmp_path / "twin", name)
    b = tenet_files(H.WTFGPU, target, tmp_path / "gpu", name)
    assert sorted(a) == sorted(b)
    for f in sorted(a):
        if a[f] != b[f]:
            la, lb = a[f].split(b"\n"), b[f].split(b"\n")
            k = next((i for i, (x, y) in enumerate(zip(la, lb)) if x != y), min(len(la), len(lb)))
            pytest.fail(f"{f}: line {k}: twin {la[k:k + 2]} gpu {lb[k:k + 2]}")
    assert sum(x.count(b"\n") for x in a.values()) > 200
    assert sum(x.count(b",mw=") for x in a.values()) > 20
