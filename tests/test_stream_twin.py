"""The fuzz loop's streaming bookkeeping on the CPU (runner.cc
FuzzSession::StreamStep / AccountStep; the gpu node's path): the oracle twin
serves the streaming interface synchronously (WTF_TWIN_STREAM=1, every step's
testcases run to their end), so a streaming campaign must equal the batch
campaign of the same seed count for count, crash name for crash name and
corpus entry for corpus entry:

  * testcases are taken from the ready queue in bulk into free slots, and the
    results are accounted with the order-independent counts summed on all
    host threads and only the order-dependent results (new crash names, new
    coverage, engine errors) handled one by one;
  * --sample makes every result go through the one-by-one path: the same
    campaign again;
  * released testcase arenas are reused by later batches.
"""
import json
import os
import shutil
import subprocess

import pytest

from tests import tlv_harness as H

pytestmark = pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")

KEYS = ("execs", "retired", "coverage", "corpus", "crashes", "unique_crashes", "timeouts", "cr3", "errors",
        "error_retired")


def _campaign(base, d, name, runs, lanes, stream, extra=(), limit=100000, max_len=0x1000):
    shutil.copytree(base, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work", "errors"))
    env = {**os.environ, "WTF_TWIN_STREAM": "1" if stream else "0"}
    out = subprocess.run([H.TWIN, "fuzz", "--name", name, "--target", d, "--runs", str(runs), "--lanes", str(lanes),
                          "--seed", "1337", "--limit", str(limit), "--max_len", str(max_len), *extra],
                         check=True, capture_output=True, text=True, timeout=600, env=env).stdout
    st = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    files = tuple(sorted(os.listdir(os.path.join(d, sub))) if os.path.isdir(os.path.join(d, sub)) else []
                  for sub in ("outputs", "crashes", "errors"))
    return {k: st[k] for k in KEYS}, files


@pytest.mark.parametrize("which", ["tlv", "hevd"])
def test_streaming_campaign_equals_batch(which, tmp_path):
    if which == "tlv":
        base = H.build_target(str(tmp_path / "base"))
        args = ("tlv_server", 12000, 512)
        kw = {}
    else:
        base = H.build_hevd_target(str(tmp_path / "base"))
        args = ("hevd", 12000, 512)
        kw = {"limit": 10_000_000, "max_len": 1028}
    a = _campaign(base, str(tmp_path / "batch"), *args, stream=False, **kw)
    b = _campaign(base, str(tmp_path / "stream"), *args, stream=True, **kw)
    c = _campaign(base, str(tmp_path / "serial"), *args, stream=True, **kw,
                  extra=("--sample", str(tmp_path / "s.jsonl"), "--sample-every", "997"))
    assert a[0]["execs"] == args[1]
    assert a == b
    assert a == c
    assert a[0]["crashes"] > 0
