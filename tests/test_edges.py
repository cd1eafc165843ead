"""Edge coverage (--edges; SURVEY §8(a) a6, RecordEdge bochscpu_backend.cc:699-728).

Every conditional near branch (taken or not) and every indirect near jmp / call
adds splitmix64_finaliser(rip) ^ next_rip to the coverage set, next to the
rips (hooks :235-257 and :308-312: direct jmp / call and ret are not
recorded). Checked on the oracle by hand, then GPU vs oracle on random
programs and GPU vs twin on the tlv snapshot.
"""
import os

import pytest

from tests import progfuzz
from tests import tlv_harness as H
from tests.oracle_lib import Oracle
from wtf_amd.abi import EXIT_INT3, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

M64 = (1 << 64) - 1


def edge(rip, nxt):
    e = rip
    e ^= e >> 30
    e = (e * 0xBF58476D1CE4E5B9) & M64
    e ^= e >> 27
    e = (e * 0x94D049BB133111EB) & M64
    e ^= e >> 31
    return e ^ nxt


def run_oracle(code, edges=True, **gprs):
    va = 0x140001000
    sp = AddressSpace()
    sp.map(va, code, write=False)
    sp.map(0x7FF000000000 - 0x1000, b"")
    pf, blob = sp.phys()
    o = Oracle(pfns=pf, blob=blob)
    r = regs_from_state(user_state(va, 0x7FF000000000 - 0x100, sp.cr3, **gprs))
    o.set_edges(edges)
    o.restore(r)
    ex = o.run()
    return ex, set(o.coverage())


def test_jcc_taken_and_not_taken():
    # mov ecx, 3 ; l: dec ecx ; jnz l ; int3
    code = bytes([0xB9, 3, 0, 0, 0, 0xFF, 0xC9, 0x75, 0xFC, 0xCC])
    ex, cov = run_oracle(code)
    assert ex.status == EXIT_INT3
    rips = {0x140001000, 0x140001005, 0x140001007, 0x140001009}
    assert cov == rips | {edge(0x140001007, 0x140001005), edge(0x140001007, 0x140001009)}
    _, plain = run_oracle(code, edges=False)
    assert plain == rips


def test_indirect_branches_only():
    # lea rax,[rip+6] ; call rax ; int3 ; (target:) lea rbx,[rip+2] ; jmp rbx ; jmp +0 ; ret ...
    #   0: 48 8d 05 03 00 00 00   lea rax, [rip+3]   -> 0xa
    #   7: ff d0                  call rax           (indirect: edge)
    #   9: cc                     int3
    #   a: 48 8d 1d 02 00 00 00   lea rbx, [rip+2]   -> 0x13
    #  11: ff e3                  jmp rbx            (indirect: edge)
    #  13: eb 00                  jmp +0             (direct: no edge)
    #  15: e8 00 00 00 00         call +0            (direct: no edge)
    #  1a: 58                     pop rax
    #  1b: c3                     ret                (no edge)
    code = bytes([0x48, 0x8D, 0x05, 0x03, 0, 0, 0, 0xFF, 0xD0, 0xCC, 0x48, 0x8D, 0x1D, 0x02, 0, 0, 0, 0xFF, 0xE3,
                  0xEB, 0x00, 0xE8, 0, 0, 0, 0, 0x58, 0xC3])
    b = 0x140001000
    ex, cov = run_oracle(code)
    assert ex.status == EXIT_INT3 and ex.rip == b + 9
    edges = {v for v in cov if not (b <= v < b + 0x1000)}
    assert edges == {edge(b + 7, b + 0xA), edge(b + 0x11, b + 0x13)}


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_twin_edges_add_coverage(tmp_path):
    t = H.build_target(str(tmp_path / "tlv"))
    a = H.run(H.TWIN, t, os.path.join(t, "inputs"), str(tmp_path / "a.jsonl"), lanes=4)
    b = H.run(H.TWIN, t, os.path.join(t, "inputs"), str(tmp_path / "b.jsonl"), lanes=4, extra=["--edges"])
    for x, y in zip(a, b):
        assert x["result"] == y["result"] and x["icount"] == y["icount"]
        assert set(x["coverage"]) < set(y["coverage"])  # the rips, plus edges


@pytest.mark.gpu
def test_gpu_edges_match_oracle_on_random_programs():
    from tests.test_gpu_progfuzz import run_gpu

    n = 512
    sp, st, lanes = progfuzz.build(n, seed=41)
    # the oracle with edges: progfuzz.oracle_run builds its own Oracle, so wrap set_limit to switch edges on
    orig = Oracle.set_limit

    def set_limit(self, v):
        self.set_edges(True)
        orig(self, v)

    Oracle.set_limit = set_limit
    try:
        want = progfuzz.oracle_run(sp, st, lanes)
    finally:
        Oracle.set_limit = orig
    from wtf_amd.engine import Engine

    eng = Engine(0)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(n, overlay_pages=8, cov_entries=4096)
    eng.set_initial_state(regs_from_state(st))
    eng.set_limit(20000)
    eng.set_edges(True)
    eng.restore()
    g = eng.read_gprs()
    import numpy as np

    for i, (va, regs, flags) in enumerate(lanes):
        g[i, :16] = np.array(regs, dtype=np.uint64)
        g[i, 16] = va
        g[i, 17] = flags
    eng.write_gprs(g)
    eng.run()
    cov, ovf = eng.coverage()
    assert not ovf
    bad = [i for i, w in enumerate(want) if cov.get(i, set()) != w["cov"]]
    with_edges = sum(1 for w in want if any(not (progfuzz.CODE_VA <= v < progfuzz.CODE_VA + n * progfuzz.SLOT)
                                            for v in w["cov"]))
    assert with_edges > n // 4
    assert not bad, f"{len(bad)}/{n} lanes differ in coverage; first {bad[:4]}"


@pytest.mark.gpu
def test_gpu_tlv_edges_match_twin(tmp_path):
    t = H.build_target(str(tmp_path / "tlv"))
    a = H.run(H.TWIN, t, os.path.join(t, "inputs"), str(tmp_path / "a.jsonl"), lanes=64, extra=["--edges"])
    b = H.run(H.WTFGPU, t, os.path.join(t, "inputs"), str(tmp_path / "b.jsonl"), lanes=64, extra=["--edges"])
    assert [(x["result"], x["crash"], x["icount"], sorted(x["coverage"])) for x in a] == \
           [(y["result"], y["crash"], y["icount"], sorted(y["coverage"])) for y in b]
