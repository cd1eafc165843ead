"""Parity at the configurations as benchmarked (bench.py): `wtfgpu fuzz` at
the bench's lane counts (tlv 262,144 lanes per GPU, the headline; HEVD
131,072) with the bench's scheduling (two pipelined halves,
4096-wave-step slices, regrouping every 1024 wave-steps, mutation in parallel
chunks) records every k-th testcase it accounted (--sample: the testcase
bytes, result, crash name, retired count, final GPRs and the coverage it
reported as new); each sampled testcase is then replayed alone through the
oracle twin (`wtf_twin run`, one testcase after the other like the reference
client) and must end identically: result, crash name, retired count, GPRs,
rip and rflags, and every rip the GPU reported as new must be in the twin's
set. The samples are then run again on the GPU node at the same lane count
through the streaming path (`wtfgpu run --stream-run --full-coverage`, two
copies of each: two pipelined halves, regrouping), and each testcase's FULL
coverage set must equal the twin's. tlv_server at --limit 100000 and HEVD at
--limit 10000000; the bench's HEVD leg runs the snapshot with
the I/O manager's IRP path (wtf_amd/tools/hevd_io.py), checked the same way.

Engine errors: the only ones allowed are handler faults (U43: a handler's
guest access that does not translate, e.g. HEVD's nt!DbgPrintEx handler
reading a format pointer the runaway guest left in r8, which the reference
would __debugbreak on, backend.cc:39-42), none an opcode outside the engine, a
full overlay or anything else, whatever the campaign's length; every testcase
the node kept under errors/ must be a handler fault on the twin as well.

Reproducibility (U44): the same fixed-seed `--runs` campaign twice at the
headline lane count gives the same summary, the same crash names and the same
corpus."""
import json
import os
import shutil

import pytest

from tests import tlv_harness as H

pytestmark = pytest.mark.gpu

TLV_LANES = 262144  # bench.py's headline leg
HEVD_LANES = 131072  # bench.py's hevd leg


def _replay_errors(tmp, target, name, limit):
    """Every testcase kept under errors/ is a handler fault (U43) on the twin too."""
    err = os.path.join(target, "errors")
    if not os.path.isdir(err) or not os.listdir(err):
        return 0
    want = H.run(H.TWIN, target, err, os.path.join(tmp, "twin_errors.jsonl"), lanes=1024, limit=limit, name=name,
                 timeout=900)
    bad = [w["input"] for w in want if not (w["error"] and w["handler_fault"])]
    assert not bad, f"{len(bad)} of {len(want)} GPU engine errors are not handler faults on the twin: {bad[:5]}"
    return len(want)


def _full_coverage_replay(tmp, target, name, limit, lanes, inp, want):
    """The samples again on the GPU node at the bench's lane count, streaming
    (two copies of each), full coverage: every testcase's rip set equals the twin's."""
    res = os.path.join(tmp, "gpu_full.jsonl")
    H.run(H.WTFGPU, target, inp, res, lanes=lanes, limit=limit, name=name, timeout=900,
          extra=["--stream-run", "--runs", "2"])
    full = {w["input"]: set(w["coverage"]) for w in want}
    seen = bad = 0
    first = []
    with open(res) as f:
        for line in f:
            g = json.loads(line)
            seen += 1
            if set(g["coverage"]) != full[g["input"]]:
                bad += 1
                if len(first) < 4:
                    first.append((g["input"], sorted(full[g["input"]] ^ set(g["coverage"]))[:4]))
    assert seen == 2 * len(want)
    assert bad == 0, f"{bad} of {seen} full coverage sets differ; first: {first}"


def _sample_and_replay(tmp, target, name, runs, every, limit, max_len, lanes):
    sample = os.path.join(tmp, "sample.jsonl")
    st = H.fuzz(H.WTFGPU, target, runs=runs, lanes=lanes, name=name, limit=limit, max_len=max_len,
                extra=("--sample", sample, "--sample-every", str(every)), timeout=600)
    # engine errors stay rare, and none is an opcode outside the engine or a
    # full overlay; a sampled one must be an error on the twin too
    b = st["backend"]
    assert st["execs"] == runs, st
    assert b["err_unimpl"] == 0 and b["err_overlay"] == 0 and b["err_other"] == 0, b
    assert st["errors"] == b["err_handler"], st
    _replay_errors(tmp, target, name, limit)
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
    _full_coverage_replay(tmp, target, name, limit, lanes, inp, want)
    return got


def test_tlv_bench_config_parity(tmp_path):
    target = H.build_target(str(tmp_path / "tlv"))
    got = _sample_and_replay(str(tmp_path), target, "tlv_server", runs=5 * TLV_LANES, every=256, limit=100000,
                             max_len=0x1000, lanes=TLV_LANES)
    assert len(got) >= 4096
    assert sum(g["result"] == "crash" for g in got) > 10 and sum(g["result"] == "ok" for g in got) > 100


def test_hevd_bench_config_parity(tmp_path):
    target = H.build_hevd_target(str(tmp_path / "hevd"))
    got = _sample_and_replay(str(tmp_path), target, "hevd", runs=655360, every=128, limit=10_000_000,
                             max_len=1028, lanes=HEVD_LANES)
    assert len(got) >= 4096
    assert {g["result"] for g in got} >= {"ok", "crash"}


def test_hevd_io_bench_config_parity(tmp_path):
    """The hevd leg as benchmarked (the I/O manager's IRP path, benign-majority
    seeds): mostly statuses, thousands of instructions per testcase."""
    target = H.build_hevd_io_target(str(tmp_path / "hevd_io"))
    got = _sample_and_replay(str(tmp_path), target, "hevd", runs=655360, every=128, limit=10_000_000,
                             max_len=1028, lanes=HEVD_LANES)
    assert len(got) >= 4096
    ok = sum(g["result"] == "ok" for g in got)
    assert ok > 0.8 * len(got) and {g["result"] for g in got} >= {"ok", "crash"}
    assert sum(g["icount"] for g in got) / len(got) > 1500


_SAME = ("execs", "retired", "coverage", "corpus", "crashes", "unique_crashes", "timeouts", "cr3", "errors")


def test_tlv_fixed_seed_campaign_reproduces(tmp_path):
    """U44: two runs of the same `wtfgpu fuzz --seed 1337 --runs N` at the
    headline lane count agree on every count, every crash name and every
    corpus entry (slices end after a fixed number of wave-steps whichever
    path ran each group; coverage is attributed in lane order on the host)."""
    base = H.build_target(str(tmp_path / "tlv"))
    runs = 6 * TLV_LANES
    out = []
    for k in (1, 2):
        t = str(tmp_path / f"tlv{k}")
        shutil.copytree(base, t)
        st = H.fuzz(H.WTFGPU, t, runs=runs, lanes=TLV_LANES, name="tlv_server", limit=100000, timeout=600)
        out.append((st, sorted(os.listdir(os.path.join(t, "crashes"))), sorted(os.listdir(os.path.join(t, "outputs")))))
    (a, ca, oa), (b, cb, ob) = out
    assert a["execs"] == runs
    assert {k: a[k] for k in _SAME} == {k: b[k] for k in _SAME}
    assert a["backend"]["group_steps"] == b["backend"]["group_steps"]
    assert ca == cb and oa == ob
