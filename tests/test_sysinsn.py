"""Ring-0 system instructions: the oracle's semantics on
hand-checked cases (CPU), and the GPU engine against the oracle lane by lane on
random operands (-m gpu): exit, rip, retired count, GPRs, RFLAGS, control
registers, MSRs, selectors, coverage and dirty pages."""
import pytest

from tests import sysprog as S
from wtf_amd import abi
from wtf_amd.tools import hevd

HLT, CR3, FAULT = abi.EXIT_HLT, abi.EXIT_CR3, abi.EXIT_FAULT


@pytest.fixture(scope="module")
def space(tmp_path_factory):
    sp, st = S.build_space(str(tmp_path_factory.mktemp("sys")))
    _, _, symbols, _ = hevd.build_space(str(tmp_path_factory.mktemp("sym")))
    return sp, st, symbols


def _one(space, name, **regs):
    sp, st, _ = space
    g = [0] * 16
    g[4] = S.KSP
    for k, v in regs.items():
        g[abi.GPR_ORDER.index(k)] = v
    return S.oracle_run(sp, st, [(S.SLOT[name], g, 0x202)])[0]


def test_rdmsr_wrmsr_roundtrip(space):
    r = _one(space, "msr", r8=0xC0000082, r9=0x00401000, r10=0xFFFFF800)
    assert r["status"] == HLT and r["regs"]["lstar"] == 0xFFFFF80000401000
    assert (r["gpr"][2] << 32 | r["gpr"][0]) == 0xFFFFF80000401000          # rdmsr after wrmsr
    assert (r["gpr"][7] << 32 | r["gpr"][6]) == space[1]["lstar"]           # rdmsr before
    r = _one(space, "msr", r8=0x10, r9=0x5000, r10=0)                       # TSC: reads base + retired
    assert (r["gpr"][2] << 32 | r["gpr"][0]) == 0x5000 + 1                  # one instruction after wrmsr
    r = _one(space, "msr", r8=0xC0000084, r9=0x1, r10=1)                    # SFMASK upper bits: #GP(0)
    assert r["status"] == HLT and r["rip"] == space[2]["nt!KeBugCheck2"] and r["gpr"][1] == 0x1E
    r = _one(space, "msr", r8=0x12345678)                                   # unknown MSR: #GP(0)
    assert r["rip"] == space[2]["nt!KeBugCheck2"]


def test_rdtsc_counts_retired_instructions(space):
    r = _one(space, "tsc")
    tsc = space[1]["tsc"]
    assert (r["gpr"][7] << 32 | r["gpr"][6]) == tsc                         # nothing retired yet
    assert (r["gpr"][2] << 32 | r["gpr"][0]) == tsc + 3 and r["gpr"][1] == space[1]["tsc_aux"]


def test_mov_cr3_other_value_ends_with_cr3_change(space):
    st = space[1]
    same = _one(space, "cr", r8=0x1234, r9=0x7, r10=st["cr3"])
    assert same["status"] == HLT and same["rip"] == space[2]["nt!KeBugCheck2"]  # went on to mov cr5 (#UD)
    assert same["regs"]["cr2"] == 0x1234 and same["regs"]["cr8"] == 7 and same["gpr"][1] == 0x1E  # #UD bugcheck
    other = _one(space, "cr", r8=0x1234, r9=0x17, r10=0x5000)
    assert other["status"] == CR3 and other["icount"] == 11 and other["regs"]["cr3"] == 0x5000
    assert other["regs"]["cr2"] == 0x1234 and other["regs"]["cr8"] == 7


def test_iretq(space):
    st = space[1]
    ring0 = _one(space, "iret", r13=st["cr4"], r8=0x18, r9=S.KSP - 0x100, r10=0x246, r11=0x10, r12=S.HLT_TARGET)
    assert ring0["status"] == HLT and ring0["rip"] == S.HLT_TARGET + 2
    assert ring0["gpr"][4] == S.KSP - 0x100 and ring0["rflags"] == 0x246 and ring0["regs"]["cs"] == 0x10
    ring3 = _one(space, "iret", r13=st["cr4"], r8=0x2B, r9=S.USTACK, r10=0x3202, r11=0x33, r12=S.USER_CODE)
    assert ring3["status"] == HLT and ring3["rip"] == S.USER_CODE + 2 and ring3["regs"]["cs"] == 0x33
    assert ring3["rflags"] == 0x3202                                        # IOPL set from ring 0
    tsd = _one(space, "iret", r13=st["cr4"] | 4, r8=0x2B, r9=S.USTACK, r10=0x202, r11=0x33, r12=S.USER_CODE)
    assert tsd["rip"] == space[2]["nt!SwapContext"]                     # ring-3 #GP ends the thread
    null_cs = _one(space, "iret", r13=st["cr4"], r8=0x18, r9=S.KSP, r10=0x202, r11=0, r12=S.HLT_TARGET)
    assert null_cs["rip"] == space[2]["nt!KeBugCheck2"] and null_cs["gpr"][1] == 0x1E


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_matches_oracle(space, seed):
    import numpy as np
    from wtf_amd.engine import Engine

    sp, st, _ = space
    n = 1024
    ln = S.lanes(n, seed, st)
    want = S.oracle_run(sp, st, ln)
    eng = Engine(0)
    try:
        pfns, blob = sp.phys()
        eng.load_pool(pfns, blob)
        eng.alloc_lanes(n, overlay_pages=8, cov_entries=256)
        eng.set_initial_state(abi.regs_from_state(st))
        eng.set_limit(2000)
        eng.restore()
        g = eng.read_gprs()
        for i, (va, regs, flags) in enumerate(ln):
            g[i, :16] = np.array(regs, dtype=np.uint64)
            g[i, 16], g[i, 17] = va, flags
        eng.write_gprs(g)
        eng.run()
        ex = eng.exits()
        g = eng.read_gprs()
        cov, ovf = eng.coverage()
        assert not ovf
        regs = eng.read_regs(0, n)
        bad = []
        for i, w in enumerate(want):
            e = ex[i]
            f = e.status == FAULT
            got = (e.status, e.vector if f else 0, e.error if f else 0, e.addr if f else 0, int(g[i, 16]), e.icount)
            exp = (w["status"], w["vector"] if f else 0, w["error"] if f else 0, w["addr"] if f else 0, w["rip"],
                   w["icount"])
            if got != exp:
                bad.append((i, "exit", got, exp))
            elif [int(x) for x in g[i, :16]] != w["gpr"] or int(g[i, 17]) != w["rflags"]:
                bad.append((i, "gprs"))
            elif S.reg_view(regs[i]) != w["regs"]:
                a, b = S.reg_view(regs[i]), w["regs"]
                bad.append((i, "regs", {k: (hex(a[k]), hex(b[k])) for k in a if a[k] != b[k]}))
            elif cov.get(i, set()) != w["cov"] or set(eng.dirty(i)) != w["dirty"]:
                bad.append((i, "cov/dirty"))
        assert not bad, f"{len(bad)}/{n} lanes differ; first: {bad[:4]}"
        kinds = {(w["status"], w["rip"]) for w in want}
        assert len(kinds) >= 6
    finally:
        eng.close()
