"""SSE / AVX floating point (conventions U39 / U40; engine_ssefp.h / engine_fp.h,
oracle/x86_oracle_fp.inc).

Native-execution vectors (tests/golden/gen_fp_vectors.py: legacy and VEX
forms, special values, every rounding mode, DAZ / FTZ, sticky flags, unmasked
exceptions that trap) pin the oracle (which runs the instruction on the host
CPU in register form, around its own decode, checks and memory access) and
the engine's own device code built for the host (tests/native/sim_lane.cc,
the integer arithmetic of engine_fp.h). The GPU runs the same vectors in
tests/test_gpu_sse.py. The #UD / #NM / #GP rules native execution cannot show
are hand-checked below.
"""
import gzip
import json
import os

import pytest

from tests.golden.gen_fp_vectors import case_inputs
from tests.oracle_lib import Oracle
from tests.test_avx import get_ymm, set_ymm
from tests.test_sse import BUF, layout, sim_lib, sim_run
from wtf_amd.abi import EXIT_FAULT, EXIT_UNIMPLEMENTED, RUNNING

HERE = os.path.dirname(os.path.abspath(__file__))
CODE_VA = 0x140001000
VEC_XM = 19


def load():
    with gzip.open(os.path.join(HERE, "golden", "fp_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def inputs(c):
    ymm, win = case_inputs(int(c["seed"], 16), c["ew"], bool(c["ints"]))
    return [v for r in ymm for v in r], b"".join(v.to_bytes(8, "little") for v in win)


def case_regs(c, regs, yin):
    for i in range(16):
        regs.gpr[i] = int(c["in"][i], 16)
    regs.rflags = int(c["fl"], 16) | 0x200
    set_ymm(regs, yin)
    regs.mxcsr = int(c["mx"], 16)
    return regs


def expected(c, yin):
    """(gprs, ymm) after the instruction."""
    g = [int(v, 16) for v in c["in"]]
    for i, v in c["gdiff"]:
        g[i] = int(v, 16)
    y = list(yin)
    for i, v in c["ydiff"]:
        y[i] = int(v, 16)
    return g, y


def check(c, status, vector, gpr, rflags, ymm, mxcsr, yin):
    """A mismatch description, or None."""
    if "trap_mx" in c:
        if status != EXIT_FAULT or vector != VEC_XM:
            return ("trap expected", status, vector)
        if mxcsr != int(c["trap_mx"], 16):
            return ("trap mxcsr", hex(mxcsr), c["trap_mx"])
        return None
    if status != RUNNING and status != 3:
        return ("exit", status, vector)
    g, y = expected(c, yin)
    if list(gpr) != g:
        return ("gprs", [(i, hex(gpr[i]), hex(g[i])) for i in range(16) if gpr[i] != g[i]])
    if (rflags ^ int(c["flo"], 16)) & int(c.get("flm", "8d5"), 16):
        return ("rflags", hex(rflags), c["flo"])
    if ymm != y:
        return ("ymm", [(i // 4, i % 4, hex(ymm[i]), hex(y[i])) for i in range(64) if ymm[i] != y[i]][:4])
    if mxcsr != int(c["mxo"], 16):
        return ("mxcsr", hex(mxcsr), c["mxo"])
    return None


@pytest.mark.parametrize("chunk", range(4))
def test_oracle_matches_native_fp(chunk):
    buf_va = int(DOC["buf_va"], 16)
    cases = DOC["cases"][chunk::4]
    fails = []
    for c in cases:
        yin, win = inputs(c)
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, win)
        pfns, blob = sp.phys()
        o = Oracle(pfns=pfns, blob=blob)
        o.restore(case_regs(c, regs, yin))
        ex = o.step()
        r = o.regs()
        ymm = get_ymm([r.xmm[i][h] for i in range(16) for h in range(2)], [r.ymmh[i][h] for i in range(16) for h in range(2)])
        bad = check(c, ex.status, ex.vector, r.gpr, r.rflags, ymm, r.mxcsr, yin)
        if bad:
            fails.append((c["name"], c["code"], c["mx"]) + bad)
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:5]}"


def test_engine_fp_code_matches_native_vectors():
    L = sim_lib()
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    for c in DOC["cases"]:
        yin, win = inputs(c)
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, win)
        out = sim_run(L, sp, case_regs(c, regs, yin))
        bad = check(c, out.status, out.vector, out.gpr, out.rflags, get_ymm(list(out.xmm), list(out.ymmh)),
                    out.mxcsr, yin)
        if bad:
            fails.append((c["name"], c["code"], c["mx"]) + bad)
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:5]}"


def test_fp_vector_file_is_substantial():
    cases = DOC["cases"]
    assert len(cases) > 5000
    assert sum("trap_mx" in c for c in cases) > 100  # unmasked exceptions
    names = {c["name"].split(".")[0] for c in cases}
    for n in ("addps", "sqrtsd", "divss", "minpd", "cmpps", "comiss", "ucomisd", "cvtsd2ss", "cvttps2dq", "cvtsi2sd",
              "cvtss2si", "haddps", "addsubpd", "movddup", "roundsd", "blendvps", "vaddps", "vcmpsd", "vcvtpd2ps",
              "vroundps", "vblendvpd", "vtcvtsd2si"):
        assert n in names, n


# ---- hand-checked: what native execution cannot show
FP_FAULT_CASES = [
    # legacy packed operands need 16-byte alignment, scalar ones do not
    ([0x0F, 0x58, 0x06], EXIT_FAULT, 13),                    # addps xmm0, [rsi] (misaligned)
    ([0xF3, 0x0F, 0x58, 0x06], RUNNING, None),               # addss xmm0, [rsi]
    ([0x66, 0x0F, 0x5A, 0x06], EXIT_FAULT, 13),              # cvtpd2ps xmm0, [rsi]
    ([0x0F, 0x5A, 0x06], RUNNING, None),                     # cvtps2pd xmm0, [rsi] (m64)
    ([0xF2, 0x0F, 0x12, 0x06], RUNNING, None),               # movddup xmm0, [rsi] (m64)
    ([0xF3, 0x0F, 0x12, 0x06], EXIT_FAULT, 13),              # movsldup xmm0, [rsi] (m128)
    ([0xF2, 0x0F, 0xF0, 0x06], RUNNING, None),               # lddqu xmm0, [rsi]
    ([0xF2, 0x0F, 0xF0, 0xC1], EXIT_FAULT, 6),               # lddqu xmm0, xmm1: memory only
    ([0xC5, 0xFC, 0x58, 0x06], RUNNING, None),               # vaddps ymm0, ymm0, [rsi]: VEX needs no alignment
    ([0xC5, 0xF8, 0x51, 0xC1], RUNNING, None),               # vsqrtps xmm0, xmm1
    ([0xC5, 0xF0, 0x51, 0xC1], EXIT_FAULT, 6),               # vsqrtps with vvvv != 1111
    ([0xC5, 0xF0, 0x2F, 0xC1], EXIT_FAULT, 6),               # vcomiss with vvvv != 1111
    ([0xC5, 0xF2, 0x58, 0xC1], RUNNING, None),               # vaddss xmm0, xmm1, xmm1
    ([0xC4, 0xE3, 0xF1, 0x4A, 0xC2, 0x30], EXIT_FAULT, 6),   # vblendvps with VEX.W = 1
    ([0xC4, 0xE3, 0x71, 0x4A, 0xC2, 0x30], RUNNING, None),   # vblendvps xmm0, xmm1, xmm2, xmm3
    ([0x66, 0xC5, 0xF8, 0x58, 0xC1], EXIT_FAULT, 6),         # 66 before VEX
    ([0x66, 0x0F, 0x3A, 0x40, 0xC1, 0xFF], RUNNING, None),   # dpps
    ([0x66, 0x0F, 0x3A, 0x41, 0x06, 0x33], EXIT_FAULT, 13),  # dppd xmm0, [rsi]: legacy needs alignment
    ([0xC4, 0xE3, 0x7D, 0x40, 0x06, 0xFF], RUNNING, None),   # vdpps ymm0, ymm0, [rsi]
    ([0x0F, 0x53, 0xC1], RUNNING, None),                     # rcpps
    ([0x0F, 0x52, 0x06], EXIT_FAULT, 13),                    # rsqrtps xmm0, [rsi]: legacy needs alignment
    ([0xC5, 0xF0, 0x53, 0xC1], EXIT_FAULT, 6),               # vrcpps with vvvv != 1111
    ([0xC5, 0xF2, 0x52, 0x06], RUNNING, None),               # vrsqrtss xmm0, xmm1, [rsi]
    ([0x0F, 0x2A, 0xC1], RUNNING, None),                     # cvtpi2ps xmm0, mm1 (tests/test_mmx.py)
    ([0x0F, 0x2D, 0xC1], RUNNING, None),                     # cvtps2pi mm0, xmm1
    ([0xC5, 0xF8, 0x2A, 0xC1], EXIT_FAULT, 6),               # no VEX form
]


def fault_regs(regs):
    regs.gpr[6] = BUF + 4  # rsi: misaligned for 16-byte operands
    return regs


def run_case(code, sim=None, cr0=None, cr4=None, mx=0x1F80, xmm=None):
    sp, regs = layout(bytes(code), BUF, b"\0" * 256, cr0, cr4)
    fault_regs(regs)
    regs.mxcsr = mx
    for i, v in (xmm or {}).items():
        regs.xmm[i][0], regs.xmm[i][1] = v
    if sim is not None:
        out = sim_run(sim, sp, regs)
        return out.status, out.vector, out.mxcsr, [(out.xmm[2 * i], out.xmm[2 * i + 1]) for i in range(16)]
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.step()
    r = o.regs()
    return ex.status, ex.vector, r.mxcsr, [(r.xmm[i][0], r.xmm[i][1]) for i in range(16)]


def norm(status):
    return RUNNING if status == 3 else status


@pytest.mark.parametrize("code,status,vector", FP_FAULT_CASES)
def test_fp_faults_oracle_and_engine(code, status, vector):
    L = sim_lib()
    for got in (run_case(code), run_case(code, sim=L)):
        assert norm(got[0]) == status, (bytes(code).hex(), got[:2])
        if vector is not None:
            assert got[1] == vector


def test_fp_gating_and_unmasked_exceptions():
    """#UD (CR0.EM / !CR4.OSFXSR), #NM (CR0.TS), and an unmasked exception:
    #XM with CR4.OSXMMEXCPT, #UD without it; the flags land in MXCSR, the
    destination keeps its value."""
    L = sim_lib()
    divps = [0x0F, 0x5E, 0xC1]  # divps xmm0, xmm1: 1 / 0 raises ZE
    one, zero = (0x3F8000003F800000, 0x3F8000003F800000), (0, 0)
    for sim in (None, L):
        assert run_case(divps, sim, cr0=0x80050037)[:2] == (EXIT_FAULT, 6)   # EM
        assert run_case(divps, sim, cr4=0x370478)[:2] == (EXIT_FAULT, 6)     # !OSFXSR
        assert run_case(divps, sim, cr0=0x8005003B)[:2] == (EXIT_FAULT, 7)   # TS
        st, vec, mx, x = run_case(divps, sim, mx=0x1F80 & ~0x200, xmm={0: one, 1: zero})
        assert (st, vec, mx, x[0]) == (EXIT_FAULT, VEC_XM, 0x1D84, one)
        st, vec, mx, x = run_case(divps, sim, cr4=0x370278, mx=0x1F80 & ~0x200, xmm={0: one, 1: zero})
        assert (st, vec, mx) == (EXIT_FAULT, 6, 0x1D84)
        st, vec, mx, x = run_case(divps, sim, xmm={0: one, 1: zero})  # masked: infinities, ZE set
        assert norm(st) == RUNNING and mx == 0x1F84 and x[0] == (0x7F8000007F800000, 0x7F8000007F800000)
