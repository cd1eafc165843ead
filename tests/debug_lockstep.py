"""Find the first instruction where GPU and oracle diverge (debug tool, GPU box).

python -m tests.debug_lockstep SEED [NLANES] [MAXLANES]
For every mismatching lane of the tests/progfuzz.py programs, binary-search the
instruction limit k at which the GPU state (16 GPRs, rip, rflags, byte count)
first differs from the oracle's state after the same number of retired
instructions, and print the instruction there.
"""
import sys

import numpy as np

from tests import progfuzz
from tests.oracle_lib import Oracle
from tests.test_gpu_progfuzz import run_gpu
from wtf_amd.abi import RUNNING, regs_from_state


def oracle_trace(sp, st, lane, maxn=4000):
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    va, regs, flags = lane
    r = regs_from_state(st)
    for k in range(16):
        r.gpr[k] = regs[k]
    r.rip, r.rflags = va, flags
    o.restore(regs_from_state(st))
    o.set_regs(r)
    states = []
    for _ in range(maxn):
        before = o.regs()
        ex = o.step()
        rr = o.regs()
        states.append((list(rr.gpr) + [rr.rip, rr.rflags], o.nbytes(), ex.status, before.rip))
        if ex.status != RUNNING:
            break
    return states


def main():
    seed = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    maxl = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    sp, st, lanes = progfuzz.build(n, seed=seed)
    want = progfuzz.oracle_run(sp, st, lanes)
    eng, _ = run_gpu(sp, st, lanes)
    g = eng.read_gprs()
    nb = eng.nbytes()
    g0 = np.zeros_like(g)
    for i, (va, regs, flags) in enumerate(lanes):
        g0[i, :16] = np.array(regs, dtype=np.uint64)
        g0[i, 16] = va
        g0[i, 17] = flags
    bad = [i for i, w in enumerate(want) if [int(x) for x in g[i, :18]] != w["gpr"] + [w["rip"], w["rflags"]]
           or int(nb[i]) != w["bytes"] or set(eng.dirty(i)) != w["dirty"]]
    print("bad lanes:", bad)
    cache = {}

    def gpu_at(k):
        if k not in cache:
            eng.set_limit(k)
            eng.restore()
            eng.write_gprs(g0)
            eng.run()
            cache[k] = (eng.read_gprs(), eng.nbytes())
        return cache[k]

    for i in bad[:maxl]:
        t = oracle_trace(sp, st, lanes[i])

        def differs(k):
            gg, bb = gpu_at(k)
            idx = min(k, len(t) - 1)
            return [int(x) for x in gg[i, :18]] != t[idx][0] or int(bb[i]) != t[idx][1]

        lo, hi = 0, len(t) - 1
        if not differs(hi):
            print(i, "state matches at every retired count; dirty-set only:", sorted(eng.dirty(i)), sorted(want[i]["dirty"]))
            continue
        while lo < hi:
            mid = (lo + hi) // 2
            if differs(mid):
                hi = mid
            else:
                lo = mid + 1
        k = lo
        gg, bb = gpu_at(k)
        idx = min(k, len(t) - 1)
        rip = t[idx][3]
        pa = sp.translate(rip)
        code = bytes(sp.pages[pa >> 12][pa & 0xFFF:(pa & 0xFFF) + 15]).hex() if pa else ""
        got = [int(x) for x in gg[i, :18]]
        diff = [(r, hex(got[r]), hex(t[idx][0][r])) for r in range(18) if got[r] != t[idx][0][r]]
        print(i, "k", k, "rip", hex(rip), "code", code, "diff", diff, "bytes", int(bb[i]), t[idx][1])


if __name__ == "__main__":
    main()
