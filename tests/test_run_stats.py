"""The `run` subcommand's surface (subcommands.cc:30-96): `--runs R` runs each
input R times in a row, and a single input run once prints the backend's run
stats in the reference's format (BochscpuRunStats_t::Print,
bochscpu_backend.h:17-45; NumberToHuman / BytesToHuman, human.cc:38-72):
instructions executed (the aggregate coverage as the unique count), dirty
pages, memory-access bytes and edges executed (unique: new to the testcase's
coverage set). The per-testcase counters are also printed with every result
("bytes", "dirty", "edges", "edges_new") and must be the same on the GPU node
and on the twin. Memory accesses count the engine's B_insn (instruction and
data bytes); bochscpu's count of linear + physical accesses is unpinned
(no bochscpu build)."""
import os
import re
import subprocess

import pytest

from tests import tlv_harness as H
from tests.tlv_inputs import write_inputs


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("runstats"))
    H.build_target(d)
    write_inputs(os.path.join(d, "parity"), 200)
    os.makedirs(os.path.join(d, "one"))
    name = sorted(os.listdir(os.path.join(d, "inputs")))[0]
    with open(os.path.join(d, "inputs", name), "rb") as f, open(os.path.join(d, "one", name), "wb") as g:
        g.write(f.read())
    return d


def _run(exe, target, inp, extra=(), results=None):
    cmd = [exe, "run", "--name", "tlv_server", "--target", target, "--input", inp, "--lanes", "64", "--limit",
           "100000", *extra]
    if results:
        cmd += ["--results", results]
    return subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300).stdout


STATS = re.compile(r"Run stats:\nInstructions executed: [0-9.]+[km]? \([0-9.]+[km]? unique\)\n"
                   r" +Dirty pages: [0-9.]+(b|kb|mb|gb)\n +Memory accesses: [0-9.]+(b|kb|mb|gb)\n"
                   r" +Edges executed: [0-9.]+[km]? \([0-9.]+[km]? unique\)\n")


def test_twin_single_input_prints_run_stats(target, tmp_path):
    out = _run(H.TWIN, target, os.path.join(target, "one"), results=str(tmp_path / "r.jsonl"))
    assert STATS.search(out), out
    out = _run(H.TWIN, target, os.path.join(target, "one"), ("--edges",), results=str(tmp_path / "r.jsonl"))
    m = re.search(r"Edges executed: ([0-9.]+)", out)
    assert m and float(m.group(1)) > 0, out


def test_twin_runs_repeats_each_input(target, tmp_path):
    out = _run(H.TWIN, target, os.path.join(target, "one"), ("--runs", "3"), results=str(tmp_path / "r.jsonl"))
    assert "Run stats" not in out
    import json
    rows = [json.loads(x) for x in open(tmp_path / "r.jsonl")]
    assert len(rows) == 3 and len({(r["result"], r["icount"], tuple(r["gprs"])) for r in rows}) == 1
    assert rows[0]["dirty"] > 0 and rows[0]["bytes"] > rows[0]["icount"]


@pytest.mark.gpu
def test_gpu_run_stats_equal_twin(target, tmp_path):
    inp = os.path.join(target, "parity")
    g = H.run(H.WTFGPU, target, inp, str(tmp_path / "g.jsonl"), lanes=256, extra=("--edges",))
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=256, extra=("--edges",))
    bad = [(a["input"], k) for a, b in zip(g, t) for k in ("bytes", "dirty", "edges", "edges_new", "icount")
           if a[k] != b[k]]
    assert len(g) == len(t) and not bad, bad[:5]
    assert sum(r["edges"] for r in g) > 0
    out = _run(H.WTFGPU, target, os.path.join(target, "one"), results=str(tmp_path / "r.jsonl"))
    assert STATS.search(out), out
