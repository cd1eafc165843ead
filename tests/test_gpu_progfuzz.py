"""GPU engine vs CPU oracle on random x86-64 programs (tests/progfuzz.py).

Per lane: exit status / vector / error code / fault address, final rip,
retired instruction count, all 16 GPRs, RFLAGS, the coverage set (every rip
executed), the dirty-page set, the algorithmic byte counter and the contents
of the data window and the stack. Bit-exact.
"""
import numpy as np
import pytest

from tests import progfuzz
from wtf_amd.abi import regs_from_state

pytestmark = pytest.mark.gpu


def run_gpu(sp, st, lanes, limit=20000, overlay_pages=8):
    from wtf_amd.engine import Engine

    n = len(lanes)
    eng = Engine(0)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(n, overlay_pages=overlay_pages, cov_entries=4096)
    eng.set_initial_state(regs_from_state(st))
    eng.set_limit(limit)
    eng.restore()
    g = eng.read_gprs()
    for i, (va, regs, flags) in enumerate(lanes):
        g[i, :16] = np.array(regs, dtype=np.uint64)
        g[i, 16] = va
        g[i, 17] = flags
    eng.write_gprs(g)
    stats = eng.run()
    return eng, stats


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_gpu_matches_oracle_on_random_programs(seed):
    n = 512
    sp, st, lanes = progfuzz.build(n, seed=seed)
    want = progfuzz.oracle_run(sp, st, lanes)
    eng, stats = run_gpu(sp, st, lanes)
    ex = eng.exits()
    g = eng.read_gprs()
    cov, ovf = eng.coverage()
    assert not ovf
    nb = eng.nbytes()
    bad = []
    for i, w in enumerate(want):
        e = ex[i]
        got = {"status": e.status, "vector": e.vector if e.status == 5 else 0,
               "error": e.error if e.status == 5 else 0, "addr": e.addr if e.status == 5 else 0,
               "rip": int(g[i, 16]), "icount": e.icount}
        exp = {"status": w["status"], "vector": w["vector"] if w["status"] == 5 else 0,
               "error": w["error"] if w["status"] == 5 else 0, "addr": w["addr"] if w["status"] == 5 else 0,
               "rip": w["rip"], "icount": w["icount"]}
        if got != exp:
            bad.append((i, "exit", got, exp))
            continue
        if [int(x) for x in g[i, :16]] != w["gpr"] or int(g[i, 17]) != w["rflags"]:
            bad.append((i, "regs", [hex(int(x)) for x in g[i, :18]], [hex(x) for x in w["gpr"] + [w["rflags"]]]))
            continue
        if cov.get(i, set()) != w["cov"]:
            bad.append((i, "cov", len(cov.get(i, set())), len(w["cov"])))
            continue
        if set(eng.dirty(i)) != w["dirty"]:
            bad.append((i, "dirty", sorted(eng.dirty(i)), sorted(w["dirty"])))
            continue
        if int(nb[i]) != w["bytes"]:
            bad.append((i, "bytes", int(nb[i]), w["bytes"]))
            continue
        if i % 8 == 0:
            if eng.read_virt(i, progfuzz.WIN_VA, 0x2000) != w["win"] or \
                    eng.read_virt(i, progfuzz.STACK_VA, 0x2000) != w["stack"]:
                bad.append((i, "memory"))
    assert stats.lane_retired == sum(w["icount"] for w in want)
    assert not bad, f"{len(bad)}/{n} lanes differ; first: {bad[:3]}"
