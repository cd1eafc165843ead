"""FMA3, F16C and the AVX2 gathers (convention U46; engine_avx2x.h,
oracle/x86_oracle_avx2x.inc), which cpuid_leaf now enumerates (FMA, F16C;
the gathers belong to AVX2).

Native-execution vectors (tests/golden/gen_avx2x_vectors.py, run on this
host's CPU, which executes every one of these forms) pin the oracle (which
runs FMA3 / F16C natively itself and restates the gathers) and the engine's
device code built for the host (which computes them in integer arithmetic);
the GPU runs them in tests/test_gpu_sse.py. Hand-checked: the #UD rules, the
CPUID bits, and a gather whose element faults (the earlier elements stay
done, engine and oracle alike).
"""
import gzip
import json
import os

import pytest

from tests.golden.gen_avx2x_vectors import case_inputs
from tests.oracle_lib import Oracle
from tests.test_avx import get_ymm, set_ymm
from tests.test_fp import check
from tests.test_sse import layout, sim_lib, sim_run

from wtf_amd.abi import EXIT_FAULT

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with gzip.open(os.path.join(HERE, "golden", "avx2x_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def inputs(c):
    ymm, win = case_inputs(int(c["seed"], 16), c["ew"], c["kind"])
    for i, v in c.get("yset", []):
        ymm[i // 4][i % 4] = int(v, 16)
    return [v for r in ymm for v in r], b"".join(v.to_bytes(8, "little") for v in win)


def case_regs(c, regs, yin):
    for i in range(16):
        regs.gpr[i] = int(c["in"][i], 16)
    regs.rflags = int(c["fl"], 16) | 0x200
    set_ymm(regs, yin)
    regs.mxcsr = int(c["mx"], 16)
    return regs


def window_after(c, win):
    w = bytearray(win)
    for i, v in c.get("mdiff", []):
        w[i] = v
    return bytes(w)


def oracle_step(code, buf_va, win, setup):
    sp, regs = layout(code, buf_va, win)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(setup(regs))
    ex = o.step()
    return o, ex, o.regs()


@pytest.mark.parametrize("chunk", range(2))
def test_oracle_matches_native_avx2x(chunk):
    buf_va = int(DOC["buf_va"], 16)
    cases = DOC["cases"][chunk::2]
    fails = []
    for c in cases:
        yin, win = inputs(c)
        o, ex, r = oracle_step(bytes.fromhex(c["code"]), buf_va, win, lambda regs: case_regs(c, regs, yin))
        ymm = get_ymm([r.xmm[i][h] for i in range(16) for h in range(2)], [r.ymmh[i][h] for i in range(16) for h in range(2)])
        bad = check(c, ex.status, ex.vector, r.gpr, r.rflags, ymm, r.mxcsr, yin)
        if not bad and o.read_virt(buf_va, 256) != window_after(c, win):
            bad = ("mem",)
        if bad:
            fails.append((c["name"], c["code"], c["mx"]) + bad)
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:5]}"


def test_engine_avx2x_code_matches_native_vectors():
    L = sim_lib()
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    for c in DOC["cases"]:
        yin, win = inputs(c)
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, win)
        out = sim_run(L, sp, case_regs(c, regs, yin), win_va=buf_va)
        bad = check(c, out.status, out.vector, out.gpr, out.rflags, get_ymm(list(out.xmm), list(out.ymmh)),
                    out.mxcsr, yin)
        if not bad and bytes(out.win[:256]) != window_after(c, win):
            bad = ("mem",)
        if bad:
            fails.append((c["name"], c["code"], c["mx"]) + bad)
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:5]}"


def test_avx2x_vector_file_is_substantial():
    names = {c["name"].split(".")[0] for c in DOC["cases"]}
    assert len(DOC["cases"]) > 3000
    for op in ("fmadd", "fmsub", "fnmadd", "fnmsub"):
        for order in ("132", "213", "231"):
            for suf in ("ps", "pd", "ss", "sd"):
                assert f"v{op}{order}{suf}" in names
    for n in ("vfmaddsub132ps", "vfmsubadd231pd", "vcvtph2ps", "vcvtps2ph", "vpgatherdd", "vpgatherdq", "vpgatherqd",
              "vpgatherqq", "vgatherdps", "vgatherdpd", "vgatherqps", "vgatherqpd"):
        assert n in names, n
    # the special values were met: traps (unmasked exceptions), NaN / denormal inputs
    assert sum("trap_mx" in c for c in DOC["cases"]) > 100


# ---- hand-checked rules, engine (host build) and oracle alike
def _both(code, setup, buf_va=0x10000, win=bytes(256)):
    """(status, vector, regs) from the oracle and from the engine's host build."""
    o, ex, r = oracle_step(code, buf_va, win, setup)
    sp, regs = layout(code, buf_va, win)
    out = sim_run(sim_lib(), sp, setup(regs), win_va=buf_va)
    return (ex.status, ex.vector, r), (out.status, out.vector, out)


GATHER_DD_L0 = bytes([0xC4, 0xE2, 0x71, 0x90, 0x04, 0x90])  # vpgatherdd xmm0, [rax + xmm2 * 4], xmm1


@pytest.mark.parametrize("code,why", [
    (bytes([0xC4, 0xE2, 0x71, 0x90, 0xC2]), "register operand"),
    (bytes([0xC4, 0xE2, 0x71, 0x90, 0x00]), "no SIB byte"),
    (bytes([0xC4, 0xE2, 0x71, 0x90, 0x04, 0x80]), "destination = index"),
    (bytes([0xC4, 0xE2, 0x79, 0x90, 0x04, 0x90]), "destination = mask"),
    (bytes([0xC4, 0xE2, 0x69, 0x90, 0x04, 0x90]), "mask = index"),
    (bytes([0xC4, 0xE2, 0xF9, 0x13, 0xC1]), "vcvtph2ps with VEX.W1"),
    (bytes([0xC4, 0xE2, 0x71, 0x13, 0xC1]), "vcvtph2ps with vvvv != 1111"),
    (bytes([0xC4, 0xE3, 0x71, 0x1D, 0xC1, 0x00]), "vcvtps2ph with vvvv != 1111"),
])
def test_ud_rules(code, why):
    def setup(regs):
        regs.gpr[0] = 0x10000
        return regs
    (so, vo, _), (se, ve, _) = _both(code, setup)
    assert (so, vo) == (EXIT_FAULT, 6), why
    assert (se, ve) == (EXIT_FAULT, 6), why


def test_gather_fault_keeps_the_done_elements():
    """vpgatherdd xmm0, [rax + xmm2 * 4], xmm1 with element 2 on an unmapped
    page: elements 0 and 1 are in xmm0 with their mask elements cleared, 2 and 3
    untouched, and the lane takes #PF at element 2's address (no IDT: the exit)."""
    buf_va = 0x10000
    win = bytes(range(256))

    def setup(regs):
        regs.gpr[0] = buf_va
        y = [0] * 64
        y[0], y[1] = 0x1111111122222222, 0x3333333344444444           # xmm0: old destination
        y[4], y[5] = 0x8000000080000000, 0x8000000080000000           # xmm1: all four masked in
        y[8], y[9] = (1 << 32) | 0, (3 << 32) | 0x40000               # xmm2: indices 0, 1, 0x40000, 3
        set_ymm(regs, y)
        return regs
    (so, vo, ro), (se, ve, re) = _both(GATHER_DD_L0, setup, buf_va, win)
    assert so == se == EXIT_FAULT and vo == ve == 14
    eng = get_ymm(list(re.xmm), list(re.ymmh))
    orc = get_ymm([ro.xmm[i][h] for i in range(16) for h in range(2)], [ro.ymmh[i][h] for i in range(16) for h in range(2)])
    assert eng[:12] == orc[:12]
    assert eng[0] == int.from_bytes(win[0:8], "little")               # elements 0 (index 0), 1 (index 1)
    assert eng[1] == 0x3333333344444444                               # elements 2, 3: untouched
    assert eng[4] == 0 and eng[5] == 0x8000000080000000               # mask: 0, 1 cleared; 2, 3 kept


def test_cpuid_enumerates_fma_and_f16c():
    code = bytes([0x0F, 0xA2])  # cpuid

    def setup(regs):
        regs.gpr[0] = 1
        regs.gpr[1] = 0
        return regs
    (_, _, ro), (_, _, re) = _both(code, setup)
    for ecx in (ro.gpr[1], re.gpr[1]):
        assert ecx & (1 << 12) and ecx & (1 << 29)
