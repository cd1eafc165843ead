"""CPU-side sanity of the random-program generator and the oracle on it."""
from collections import Counter

from tests import progfuzz
from wtf_amd.abi import STATUS_NAMES


def test_oracle_runs_random_programs():
    sp, st, lanes = progfuzz.build(64, seed=7)
    res = progfuzz.oracle_run(sp, st, lanes)
    c = Counter(STATUS_NAMES[r["status"]] for r in res)
    # most programs reach their final int3; some fault on purpose
    assert c["int3"] >= 20, c
    assert sum(r["icount"] for r in res) > 64 * 20
    assert all(r["cov"] for r in res)
