"""The deferred multi-shard coverage merge (runner.cc
FuzzSession::MergeCoverage, rccl_exchange.cc, merge_block.h).

  * MergeBlocks, the per-shard block both exchanges pack and read (RCCL on the
    GPU node, TCP between CPU twins): more than a block's worth of overflow
    values drains over several merges in order, a shard says "done" only in
    the block that empties its queue, and the values come back in rank order;
  * two world-2 twin campaigns with the same seeds agree exactly (execs,
    crashes, coverage, corpus file names): the merge a step starts is
    absorbed at the next step's start on every shard, so fixed-seed
    campaigns reproduce at N > 1 (DESIGN U44);
  * a tiny block (WTF_MERGE_CAP) with --edges, whose values lie outside the
    map: the queued values drain over many merges and both shards still end
    with the same aggregate.
"""
import os
import shutil
import subprocess

import pytest

from tests import tlv_harness as H
from tests.cpu_bins import ALT, HOSTCHECK
from tests.test_shard_twin import _free_port, _fuzz_cmd, _last_json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _hostcheck():
    if not ALT and not os.path.exists(HOSTCHECK):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "hostcheck"])
    return HOSTCHECK


def _merge(cap, world, *steps):
    out = subprocess.run([_hostcheck(), "merge-blocks", str(cap), str(world), *steps], check=True,
                         capture_output=True, text=True).stdout.split("\n")
    res = []
    for ln in out:
        if ln.startswith("S "):
            f = ln.split()
            res.append((f[1] == "1", [int(x, 16) for x in f[2:]]))
    assert len(res) == len(steps)
    return res


def v(rank, i):
    return rank << 32 | i


def test_merge_blocks_drain_in_order_and_hold_done_back():
    r = _merge(3, 2, "5,2", "1d,0", "0,4d", "0d,0d", "0d,0d")
    # step 1: rank 0 sends 3 of its 5 (cap), rank 1 both; rank order
    assert r[0] == (False, [v(0, 0), v(0, 1), v(0, 2), v(1, 0), v(1, 1)])
    # step 2: rank 0's queue empties in this block, so its done counts; rank 1 is not done
    assert r[1] == (False, [v(0, 3), v(0, 4), v(0, 5)])
    # step 3: rank 1 says done with 4 queued: 3 go, done is held back
    assert r[2] == (False, [v(1, 2), v(1, 3), v(1, 4)])
    # step 4: its last value goes with done: every shard done
    assert r[3] == (True, [v(1, 5)])
    assert r[4] == (True, [])


def test_merge_blocks_large_backlog_three_shards():
    steps = ["100,0,7"] + ["0,0,0"] * 40 + ["0d,0d,0d"] * 40
    r = _merge(4, 3, *steps)
    got = [x for _, vals in r for x in vals]
    # nothing lost or duplicated; each shard's values in their own order
    assert sorted(got) == sorted([v(0, i) for i in range(100)] + [v(2, i) for i in range(7)])
    for rank in (0, 2):
        mine = [x for x in got if x >> 32 == rank]
        assert mine == sorted(mine)
    # done only once rank 0's 100 values are through (4 per merge: 25 merges)
    first_done = next(i for i, (d, _) in enumerate(r) if d)
    assert sum(len([x for x in vals if x >> 32 == 0]) for _, vals in r[:first_done + 1]) == 100
    assert all(d for d, _ in r[first_done:])
    assert not any(d for d, _ in r[:first_done])


pytestmark_twin = pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")


@pytest.fixture(scope="module")
def base(tmp_path_factory):
    return H.build_target(str(tmp_path_factory.mktemp("tlv_merge")))


def _campaign(base, tmp, tag, extra=(), env=None, runs=2048, lanes=256, split=False):
    seeds = sorted(os.listdir(os.path.join(base, "inputs")))
    dirs = []
    for r in range(2):
        d = os.path.join(tmp, f"{tag}{r}")
        shutil.copytree(base, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
        if split:  # each shard starts from half the seed inputs: each finds code the other has not run
            for i, name in enumerate(seeds):
                if i % 2 != r:
                    os.remove(os.path.join(d, "inputs", name))
        dirs.append(d)
    port = _free_port()
    procs = [subprocess.Popen(_fuzz_cmd(dirs[r], r, 2, port, runs=runs, lanes=lanes) + list(extra),
                              stdout=subprocess.PIPE, text=True, env={**os.environ, **(env or {})})
             for r in range(2)]
    res = [_last_json(p.communicate(timeout=300)[0]) for p in procs]
    assert all(p.returncode == 0 for p in procs)
    files = [(sorted(os.listdir(os.path.join(d, "outputs"))), sorted(os.listdir(os.path.join(d, "crashes"))))
             for d in dirs]
    return res, files


@pytestmark_twin
def test_world2_fixed_seed_campaign_reproduces(base, tmp_path):
    a, fa = _campaign(base, str(tmp_path), "a")
    b, fb = _campaign(base, str(tmp_path), "b")
    keys = ("execs", "retired", "crashes", "unique_crashes", "timeouts", "coverage", "corpus", "merged_rips")
    for r in range(2):
        assert {k: a[r][k] for k in keys} == {k: b[r][k] for k in keys}, f"rank {r}"
    assert fa == fb
    assert a[0]["coverage"] == a[1]["coverage"]


@pytestmark_twin
def test_world2_small_merge_blocks_drain_edges(base, tmp_path):
    res, _ = _campaign(base, str(tmp_path), "e", extra=["--edges"], env={"WTF_MERGE_CAP": "2"}, runs=1024,
                       split=True)
    assert res[0]["coverage"] == res[1]["coverage"]
    assert sum(r["merged_rips"] for r in res) > 0
