"""SYN at the headline configuration (BASELINE.json configs[1]; bench.py's SYN
leg): 65,536 lanes, --limit 100000, syn.inputs(seed=syn.SEED), one batch on
the HIP engine, checked

  * for every lane: exit at the exit breakpoint, retired count
    (syn.expected_instructions), final rax/rbx/rcx/rdx/r8/r9/r10, rflags and
    rip against the numpy restatement of the loop (syn.model, itself pinned
    to the C oracle by tests/test_syn_model.py);
  * for 8,192 lanes: the whole scratch page against the model;
  * for 512 lanes spread over the batch: everything against the C oracle
    (GPRs, rflags, rip, retired count, dirty set, scratch page);
  * the batch's coverage set (the loop and the exit) and its byte counter.
"""
import numpy as np
import pytest

from tests.syn_harness import make_engine, oracle_lane, run_batch
from wtf_amd.abi import EXIT_BREAKPOINT
from wtf_amd.tools import syn

pytestmark = pytest.mark.gpu

N = 65536
LIMIT = 100000
GPR = {"rax": 0, "rcx": 1, "rdx": 2, "rbx": 3, "r8": 8, "r9": 9, "r10": 10}


@pytest.fixture(scope="module")
def batch():
    inp = syn.inputs(N, seed=syn.SEED)
    eng, sp, st = make_engine(N, limit=LIMIT)
    rs = run_batch(eng, inp)
    ex = eng.exits_np()
    g = eng.read_gprs()
    yield eng, sp, st, inp, rs, ex, g
    eng.close()


def test_every_lane_matches_model(batch):
    eng, sp, st, inp, rs, ex, g = batch
    want_ic = syn.expected_instructions(inp)
    assert np.all(ex["status"] == EXIT_BREAKPOINT)
    assert np.all(ex["rip"] == syn.EXIT_VA)
    assert np.array_equal(ex["icount"].astype(np.int64), want_ic)
    assert rs.lane_retired == int(want_ic.sum())
    table = bytes(sp.pages[sp.translate(syn.TABLE_VA) >> 12])
    regs, _ = syn.model(inp, table)
    for name, k in GPR.items():
        bad = np.nonzero(g[:, k] != regs[name])[0]
        assert bad.size == 0, (name, bad[:8])
    assert np.all(g[:, 16] == syn.EXIT_VA) and np.all(g[:, 17] == 0x246)
    assert np.all(g[:, 4] == syn.STACK_TOP)


def test_scratch_pages_match_model(batch):
    eng, sp, st, inp, rs, ex, g = batch
    lanes = np.arange(0, N, N // 8192, dtype=np.uint32)
    gpa = sp.translate(syn.SCRATCH_VA)
    pages = eng.gather_pages(lanes, np.full(len(lanes), gpa, dtype=np.uint64)).view(np.uint64)
    table = bytes(sp.pages[sp.translate(syn.TABLE_VA) >> 12])
    _, scratch = syn.model(inp[lanes], table)
    bad = np.nonzero((pages != scratch).any(axis=1))[0]
    assert bad.size == 0, lanes[bad[:8]]


def test_sampled_lanes_match_oracle(batch):
    eng, sp, st, inp, rs, ex, g = batch
    for i in np.linspace(0, N - 1, 512).astype(int).tolist():
        o, oex = oracle_lane(sp, st, inp[i], limit=LIMIT)
        r = o.regs()
        assert oex.status == int(ex["status"][i]) and oex.icount == int(ex["icount"][i]), i
        assert [int(x) for x in g[i, :16]] == list(r.gpr), i
        assert int(g[i, 16]) == r.rip and int(g[i, 17]) == r.rflags, i
        assert set(eng.dirty(i)) == set(o.dirty()), i
        assert eng.read_virt(i, syn.SCRATCH_VA, 4096) == o.read_virt(syn.SCRATCH_VA, 4096), i


def test_coverage_and_bytes(batch):
    eng, sp, st, inp, rs, ex, g = batch
    cov, ovf = eng.coverage()
    rips = set().union(*cov.values())
    insn_starts = {syn.CODE_VA + o for o in (0, 3, 9, 13, 16, 19, 22, 27, 34, 38, 41, 43)} | {syn.EXIT_VA}
    assert not ovf and rips == insn_starts
    # algorithmic bytes: per iteration 47 instruction bytes + 8 loaded + 8 stored
    trips = (syn.expected_instructions(inp) - 1) // syn.INSNS_PER_ITER
    nb = eng.nbytes()
    assert np.array_equal(nb.astype(np.int64), trips * syn.BYTES_PER_ITER + 1 + 8)  # + ret: 1 byte, 8 popped
