"""The RCCL coverage merge (`wtf_amd/host/rccl_exchange.cc`)
executed on the MI355X at world 1.

A one-GPU box cannot run the 8-GPU configs (BASELINE configs[3] / [4]), but it
can run every RCCL call they make: `--rccl-force` (or WTF_RCCL_FORCE=1) makes
a world-1 node build a one-rank communicator (ncclCommInitRank) and take the
shard path each node step — the frozen D2D copy of the device coverage map,
the fused ncclAllReduce(uint8, ncclMax) + ncclAllGather group on the
exchange's stream, the event, MergeBlocks::Unpack, and the absorb one step
later (k_cov_absorb) — plus the consensus stop on the merged done flags.

With one rank the merged map is this node's own map as it stood a step
earlier and the gathered extras are its own, so the campaign must be exactly
the campaign without the switch: same counts, same crash names, same corpus
(the master's aggregate, server.h:816-854, sees nothing new from a merge).
The summary's `merges` / `merged_map_bytes` show the merges really ran."""
import os
import shutil

import pytest

from tests import tlv_harness as H

pytestmark = pytest.mark.gpu

_SAME = ("execs", "retired", "coverage", "corpus", "crashes", "unique_crashes", "timeouts", "cr3", "errors")


def _campaign(tmp_path, base, tag, extra):
    t = str(tmp_path / tag)
    shutil.copytree(base, t)
    st = H.fuzz(H.WTFGPU, t, runs=4 * 65536, lanes=65536, name="tlv_server", limit=100000, timeout=600,
                extra=extra)
    return st, sorted(os.listdir(os.path.join(t, "crashes"))), sorted(os.listdir(os.path.join(t, "outputs")))


@pytest.mark.parametrize("edges", [False, True], ids=["rips", "edges"])
def test_rccl_forced_world1_campaign_equals_plain(tmp_path, edges):
    """With --edges the all-gather also carries values outside the map
    (the overflow list, MergeBlocks)."""
    base = H.build_target(str(tmp_path / "tlv"))
    ex = ("--edges",) if edges else ()
    plain, cp, op = _campaign(tmp_path, base, "plain", ex)
    forced, cf, of = _campaign(tmp_path, base, "forced", ex + ("--rccl-force",))
    assert plain["execs"] == 4 * 65536
    assert {k: plain[k] for k in _SAME} == {k: forced[k] for k in _SAME}
    assert plain["backend"]["group_steps"] == forced["backend"]["group_steps"]
    assert cp == cf and op == of
    # the merges ran: one per node step, each carrying the whole device map
    assert plain["merges"] == 0
    assert forced["merges"] >= forced["batches"] > 0
    assert forced["merged_map_bytes"] > 0 and forced["merged_map_bytes"] % forced["merges"] == 0
    # a one-rank merge brings nothing this node did not have
    assert forced["merged_rips"] == 0
