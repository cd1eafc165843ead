"""Parity at the configurations as benchmarked (bench.py): `wtfgpu fuzz` at
131,072 lanes per GPU with the bench's scheduling (two pipelined halves,
4096-wave-step slices, regrouping every 1024 wave-steps, mutation in parallel
chunks) records every k-th testcase it accounted (--sample: the testcase
bytes, result, crash name, retired count, final GPRs and the coverage it
reported as new); each sampled testcase is then replayed alone through the
oracle twin (`wtf_twin run`, one testcase after the other like the reference
client) and must end identically: result, crash name, retired count, GPRs,
rip and rflags, and every rip the GPU reported must be in the twin's set.
tlv_server at --limit 100000 and HEVD at --limit 10000000."""
import json
import os

import pytest

from tests import tlv_harness as H

pytestmark = pytest.mark.gpu

LANES = 131072


def _sample_and_replay(tmp, target, name, runs, every, limit, max_len):
    sample = os.path.join(tmp, "sample.jsonl")
    st = H.fuzz(H.WTFGPU, target, runs=runs, lanes=LANES, name=name, limit=limit, max_len=max_len,
                extra=("--sample", sample, "--sample-every", str(every)), timeout=600)
    # engine errors (opcodes outside the engine, e.g. x87 arithmetic in runaway
    # HEVD code) stay rare; a sampled one must be an error on the twin too
    assert st["execs"] == runs and st["errors"] <= runs // 10000, st
    with open(sample) as f:
        got = [json.loads(line) for line in f]
    inp = os.path.join(tmp, "replay")
    os.makedirs(inp)
    for i, g in enumerate(got):
        with open(os.path.join(inp, f"s{i:06d}"), "wb") as f:
            f.write(bytes.fromhex(g["tc"]))
    want = H.run(H.TWIN, target, inp, os.path.join(tmp, "twin.jsonl"), lanes=1024, limit=limit, name=name,
                 timeout=900)
    assert len(want) == len(got)
    bad = []
    for i, (g, w) in enumerate(zip(got, want)):
        assert w["input"] == f"s{i:06d}"
        for k in ("result", "crash", "error", "icount", "gprs"):
            if g[k] != w[k]:
                bad.append((i, k, g[k], w[k]))
        if not set(g["coverage"]) <= set(w["coverage"]):
            bad.append((i, "coverage", sorted(set(g["coverage"]) - set(w["coverage"]))[:4]))
    assert not bad, f"{len(bad)} of {len(got)} differ; first: {bad[:5]}"
    return got


def test_tlv_bench_config_parity(tmp_path):
    target = H.build_target(str(tmp_path / "tlv"))
    got = _sample_and_replay(str(tmp_path), target, "tlv_server", runs=655360, every=128, limit=100000,
                             max_len=0x1000)
    assert len(got) >= 4096
    assert sum(g["result"] == "crash" for g in got) > 10 and sum(g["result"] == "ok" for g in got) > 100


def test_hevd_bench_config_parity(tmp_path):
    target = H.build_hevd_target(str(tmp_path / "hevd"))
    got = _sample_and_replay(str(tmp_path), target, "hevd", runs=655360, every=128, limit=10_000_000,
                             max_len=1028)
    assert len(got) >= 4096
    assert {g["result"] for g in got} >= {"ok", "crash"}
