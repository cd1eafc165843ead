"""SYN snapshot driver shared by smoke(), tests and bench: one batch =
restore -> insert N testcases -> run -> collect exits (TEST/BENCH HARNESS)."""
from __future__ import annotations

import numpy as np

from wtf_amd.abi import EXIT_BREAKPOINT, regs_from_state
from wtf_amd.tools import syn


def make_engine(nlanes, limit=100000, device=0):
    from wtf_amd.engine import Engine

    sp, st, _ = syn.build()
    eng = Engine(device)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(nlanes, overlay_pages=4, cov_entries=256)
    eng.set_initial_state(regs_from_state(st))
    eng.set_limit(limit)
    eng.set_breakpoints([syn.EXIT_VA])
    eng.set_code_pages([syn.CODE_VA >> 12, syn.EXIT_VA >> 12])
    return eng, sp, st


def run_batch(eng, inp):
    eng.restore()
    g = eng.read_gprs()
    syn.insert(g, inp)
    eng.write_gprs(g)
    return eng.run()


def oracle_lane(sp, st, inp_row, limit=100000):
    from tests.oracle_lib import Oracle

    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    base = regs_from_state(st)
    o.restore(base)
    o.set_limit(limit)
    o.set_breakpoints([syn.EXIT_VA])
    g = np.zeros((1, 18), dtype=np.uint64)
    r = o.regs()
    for k in range(16):
        g[0, k] = r.gpr[k]
    syn.insert(g, inp_row[None, :])
    for k in range(16):
        r.gpr[k] = int(g[0, k])
    o.set_regs(r)
    ex = o.run()
    return o, ex


def run_smoke(n=256, check=16):
    inp = syn.inputs(n, seed=123)
    inp[:, 1] &= 0x03  # short trip counts for a quick check
    eng, sp, st = make_engine(n)
    run_batch(eng, inp)
    ex = eng.exits()
    g = eng.read_gprs()
    want_ic = syn.expected_instructions(inp)
    for i in range(n):
        assert ex[i].status == EXIT_BREAKPOINT and ex[i].rip == syn.EXIT_VA, (i, ex[i].status, hex(ex[i].rip))
        assert ex[i].icount == want_ic[i], (i, ex[i].icount, want_ic[i])
    for i in range(0, n, max(1, n // check)):
        o, oex = oracle_lane(sp, st, inp[i])
        r = o.regs()
        assert oex.status == ex[i].status and oex.icount == ex[i].icount
        assert [int(x) for x in g[i, :16]] == list(r.gpr) and int(g[i, 17]) == r.rflags, i
        assert set(eng.dirty(i)) == set(o.dirty()), i
        assert eng.read_virt(i, syn.SCRATCH_VA, 4096) == o.read_virt(syn.SCRATCH_VA, 4096), i
    eng.close()
    print(f"smoke ok: {n} SYN testcases on cuda:0 match the oracle")
