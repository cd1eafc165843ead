"""Multi-shard fuzzing on the CPU (the GPU node does the same with
RCCL, rccl_exchange.cc): two `wtf_twin fuzz` ranks, each an independent shard
(seed + rank, its own corpus), merge their coverage maps after every batch
through the node's CoverageExchange_t (TCP on the CPU, net_exchange.cc).

  * both ranks end with the same aggregate coverage: the union;
  * rips one rank found reached the other (merged_rips > 0 somewhere; merges
    are absorbed one step after they start), and each kept only its own
    testcases in its corpus;
  * the union is at least what either shard alone covers.
"""
import json
import os
import shutil
import socket
import subprocess

import pytest

from tests import tlv_harness as H

pytestmark = pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fuzz_cmd(d, rank, world, port, runs=3072, lanes=512):
    return [H.TWIN, "fuzz", "--name", "tlv_server", "--target", d, "--runs", str(runs), "--lanes", str(lanes),
            "--seed", "1337", "--limit", "100000", "--rank", str(rank), "--world", str(world),
            "--exchange", f"127.0.0.1:{port}"]


def _last_json(out):
    return json.loads([x for x in out.splitlines() if x.startswith("{")][-1])


@pytest.fixture(scope="module")
def base(tmp_path_factory):
    return H.build_target(str(tmp_path_factory.mktemp("tlv_shards")))


def test_two_twin_shards_merge_coverage(base, tmp_path):
    # the shards start from different seed inputs, so each finds code the
    # other has not run yet
    seeds = sorted(os.listdir(os.path.join(base, "inputs")))
    dirs = []
    for r in range(2):
        d = str(tmp_path / f"r{r}")
        shutil.copytree(base, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
        for i, name in enumerate(seeds):
            if i % 2 != r:
                os.remove(os.path.join(d, "inputs", name))
        dirs.append(d)
    port = _free_port()
    procs = [subprocess.Popen(_fuzz_cmd(dirs[r], r, 2, port), stdout=subprocess.PIPE, text=True) for r in range(2)]
    res = [_last_json(p.communicate(timeout=300)[0]) for p in procs]
    assert all(p.returncode == 0 for p in procs)
    assert [r["rank"] for r in res] == [0, 1] and all(r["world"] == 2 for r in res)
    assert res[0]["coverage"] == res[1]["coverage"]
    # merges are absorbed one step after they start: a shard may find what the
    # other found in the meantime itself, but the two cannot both miss out
    assert sum(r["merged_rips"] for r in res) > 0
    # corpora stay per shard: rank 1's seed differs, so its corpus differs
    c0, c1 = (set(os.listdir(os.path.join(d, "outputs"))) for d in dirs)
    assert c0 != c1
    # one shard alone (same seed as rank 0) covers no more than the union
    solo = str(tmp_path / "solo")
    shutil.copytree(base, solo, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
    one = subprocess.run(_fuzz_cmd(solo, 0, 1, port), capture_output=True, text=True, timeout=300, check=True)
    assert _last_json(one.stdout)["coverage"] <= res[0]["coverage"]


def test_two_twin_shards_merge_edges_outside_the_map(base, tmp_path):
    """--edges: branch edge values live outside the code-page map (SURVEY
    8(e)'s overflow list); every merge all-gathers each shard's new ones
    (CoverageExchange_t::AllGatherV) and both shards end with the same
    aggregate, edges included."""
    dirs = []
    for r in range(2):
        d = str(tmp_path / f"e{r}")
        shutil.copytree(base, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
        dirs.append(d)
    port = _free_port()
    procs = [subprocess.Popen(_fuzz_cmd(dirs[r], r, 2, port, runs=2048) + ["--edges", "--seed", str(1337 + r)],
                              stdout=subprocess.PIPE, text=True) for r in range(2)]
    res = [_last_json(p.communicate(timeout=300)[0]) for p in procs]
    assert all(p.returncode == 0 for p in procs)
    assert res[0]["coverage"] == res[1]["coverage"]
    # edges make the aggregate larger than the rips alone
    solo = str(tmp_path / "solo_noedges")
    shutil.copytree(base, solo, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
    one = subprocess.run(_fuzz_cmd(solo, 0, 1, port, runs=2048), capture_output=True, text=True, timeout=300,
                         check=True)
    assert res[0]["coverage"] > _last_json(one.stdout)["coverage"]


def test_shards_stopping_at_different_times(base, tmp_path):
    """--seconds budgets that end at different moments: a finished shard keeps
    joining the other's merges (Done() is read once per step) until every
    shard is done; neither hangs nor mismatches a collective."""
    dirs = []
    for r in range(2):
        d = str(tmp_path / f"t{r}")
        shutil.copytree(base, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
        dirs.append(d)
    port = _free_port()
    cmds = [_fuzz_cmd(dirs[r], r, 2, port, runs=0, lanes=64) + ["--seconds", str(1.0 + 2.0 * r)] for r in range(2)]
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, text=True) for c in cmds]
    res = [_last_json(p.communicate(timeout=120)[0]) for p in procs]
    assert all(p.returncode == 0 for p in procs)
    assert res[0]["coverage"] == res[1]["coverage"]
