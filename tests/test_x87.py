"""x87 arithmetic (convention U42; engine_x87.h, oracle/x86_oracle_x87.inc).

The golden vectors (tests/golden/gen_x87_vectors.py) hold random x87 states
under every non-control d8-df form with the host CPU's answer (the oracle
runs each form natively): they pin the oracle's native path (regression) and
the engine's integer extended-precision arithmetic built for the host; the
GPU runs the same vectors in tests/test_gpu_sse.py. Hand-checked here: #UD /
#NM / #MF / UNIMPLEMENTED, stores that fault, FNINIT, the FSW that a loaded
image normalises, and the MMX exponent words.
"""
import gzip
import json
import os

import pytest

from tests.golden.gen_x87_vectors import case_regs, mem_forms, reg_forms, run_oracle
from tests.oracle_lib import Oracle
from tests.test_mmx import sim_lib, sim_run
from tests.test_sse import BUF, layout
from wtf_amd.abi import EXIT_FAULT, EXIT_UNIMPLEMENTED

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with gzip.open(os.path.join(HERE, "golden", "x87_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def norm_st(st):
    return [tuple(x) for x in st]


def mismatch(c, got):
    want = c["out"]
    for k in ("status", "vector", "fcw", "fsw", "ftw", "fl", "mem"):
        if got[k] != want[k]:
            return (k, got[k], want[k])
    if norm_st(got["st"]) != norm_st(want["st"]):
        return ("st",)
    return None


def run_sim(L, c, buf_va):
    sp, regs = layout(bytes.fromhex(c["code"]), buf_va, bytes.fromhex(c["mem"]).ljust(256, b"\0"))
    regs.gpr[6] = buf_va
    case_regs(c, regs)
    out, r = sim_run(L, sp, regs, win_va=buf_va)
    st = 0 if out.status == 3 else out.status
    return dict(status=st, vector=out.vector if st == EXIT_FAULT else 0, fcw=r.fpcw, fsw=r.fpsw, ftw=r.fptw,
                st=[(r.fpst[i], r.fpse[i]) for i in range(8)], fl=r.rflags & 0x8D5, mem=bytes(out.win[:16]).hex())


@pytest.mark.parametrize("chunk", range(2))
def test_oracle_matches_x87_vectors(chunk):
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    for c in DOC["cases"][chunk::2]:
        bad = mismatch(c, run_oracle(c, buf_va))
        if bad:
            fails.append((c["code"],) + bad)
    assert not fails, f"{len(fails)} mismatches, first: {fails[:5]}"


@pytest.mark.parametrize("chunk", range(2))
def test_engine_x87_code_matches_vectors(chunk):
    L = sim_lib()
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    for c in DOC["cases"][chunk::2]:
        bad = mismatch(c, run_sim(L, c, buf_va))
        if bad:
            fails.append((c["code"],) + bad)
    assert not fails, f"{len(fails)} mismatches, first: {fails[:5]}"


def test_x87_vector_file_covers_every_form():
    codes = {c["code"] for c in DOC["cases"]}
    for f in reg_forms():
        assert f.hex() in codes, f.hex()
    for f, _ in mem_forms():
        assert f.hex() in codes, f.hex()
    assert len(DOC["cases"]) > 4000
    # every outcome class appears: faults (#MF), stack faults, unmasked exceptions, stores
    outs = [c["out"] for c in DOC["cases"]]
    assert any(o["status"] == EXIT_FAULT and o["vector"] == 16 for o in outs)
    assert sum(1 for o in outs if o["fsw"] & 0x40) > 200
    assert sum(1 for o in outs if o["fsw"] & 0x8000) > 500


ONE = (0x8000000000000000, 0x3FFF)


def x87_case(code, **kw):
    c = dict(code=bytes(code).hex(), mem="00" * 16, fcw=0x37F, fsw=0, ftw=0xFFFF, st=[(0, 0)] * 8, fl=0)
    c.update(kw)
    return c


X87_FAULT_CASES = [
    ([0xD9, 0xD1], EXIT_FAULT, 6, {}),                        # reserved d9 d1
    ([0xDD, 0xF0], EXIT_FAULT, 6, {}),                        # reserved dd f0
    ([0xD9, 0x0E], EXIT_FAULT, 6, {}),                        # d9 /1 m: reserved
    ([0xDB, 0x26], EXIT_FAULT, 6, {}),                        # db /4 m: reserved
    ([0xD9, 0xFE], EXIT_UNIMPLEMENTED, None, {}),             # fsin: outside
    ([0xD9, 0xFF], EXIT_UNIMPLEMENTED, None, {}),             # fcos: outside
    ([0xDF, 0x26], 0, None, {}),                              # fbld m80bcd (runs)
    ([0xD8, 0xC1], EXIT_FAULT, 16, dict(fcw=0x37E, fsw=0x8081)),  # pending unmasked IE: #MF
    ([0xD8, 0xC1], EXIT_FAULT, 16, dict(fcw=0x37E, fsw=0x0001)),  # pending even with ES clear
    ([0xD8, 0xC1], 0, None, dict(fcw=0x37F, fsw=0x0080)),     # ES alone, every flag masked: runs
    ([0xDB, 0xE0], 0, None, dict(fcw=0x37E, fsw=0x8081)),     # fneni does not wait
    ([0xD9, 0xD0], EXIT_FAULT, 16, dict(fcw=0x37E, fsw=0x8081)),  # fnop waits
]


@pytest.mark.parametrize("code,status,vector,kw", X87_FAULT_CASES)
def test_x87_faults_oracle_and_engine(code, status, vector, kw):
    L = sim_lib()
    c = x87_case(code, **kw)
    for got in (run_oracle(c, BUF), run_sim(L, c, BUF)):
        assert got["status"] == status, (bytes(code).hex(), got["status"], got["vector"])
        if vector is not None:
            assert got["vector"] == vector


def test_x87_nm_when_cr0_ts():
    L = sim_lib()
    sp, regs = layout(bytes([0xD9, 0xE8]), BUF, bytes(256), cr0=0x80050033 | 8)
    out, _ = sim_run(L, sp, regs)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.step()
    assert (out.status, out.vector) == (EXIT_FAULT, 7) and (ex.status, ex.vector) == (EXIT_FAULT, 7)


def prog_state(code, st0=ONE):
    """A short program over a clean x87 state; rsi = BUF, rdi = BUF + 0x40."""
    sp, regs = layout(bytes(code), BUF, bytes(256))
    regs.gpr[6], regs.gpr[7] = BUF, BUF + 0x40
    regs.fpcw, regs.fptw = 0x37F, 0xFFFF
    return sp, regs


def run_both(code):
    L = sim_lib()
    sp, regs = prog_state(code)
    out, fin = sim_run(L, sp, regs, win_va=BUF)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    for _ in range(64):
        ex = o.step()
        if ex.status != 0:
            break
    return out, fin, ex, o


def test_fninit_keeps_register_contents_and_fxsave_shows_exponents():
    # fld1; fldpi; fninit; fxsave [rdi]; int3: the host keeps R7 = 1 and R6 = pi (TOP = 0)
    code = [0xD9, 0xE8, 0xD9, 0xEB, 0xDB, 0xE3, 0x0F, 0xAE, 0x07]
    out, fin, ex, o = run_both(code)
    img = bytes(out.win[0x40:0x40 + 0xA0])
    assert img == o.read_virt(BUF + 0x40, 0xA0)
    assert int.from_bytes(img[32 + 16 * 7:40 + 16 * 7], "little") == 0x8000000000000000
    assert int.from_bytes(img[40 + 16 * 7:42 + 16 * 7], "little") == 0x3FFF
    assert int.from_bytes(img[32 + 16 * 6:40 + 16 * 6], "little") == 0xC90FDAA22168C235
    assert img[4] == 0 and fin.fpsw == 0 and fin.fptw == 0xFFFF


def test_mmx_write_sets_exponent_word():
    # movq mm0, [rsi]; fxsave [rdi]: ST0 / MM0's sign + exponent read all ones
    code = [0x0F, 0x6F, 0x06, 0x0F, 0xAE, 0x07]
    out, fin, ex, o = run_both(code)
    img = bytes(out.win[0x40:0x40 + 0xA0])
    assert img == o.read_virt(BUF + 0x40, 0xA0)
    assert int.from_bytes(img[40:42], "little") == 0xFFFF and fin.fpse[0] == 0xFFFF


def test_fxrstor_normalises_es():
    # fxrstor [rsi] of fcw = 037e / fsw = 0001 -> fsw 8081; then fnstsw ax
    img = bytearray(512)
    img[0:2] = (0x37E).to_bytes(2, "little")
    img[2:4] = (0x0001).to_bytes(2, "little")
    img[24:28] = (0x1F80).to_bytes(4, "little")
    L = sim_lib()
    sp, regs = layout(bytes([0x0F, 0xAE, 0x0E, 0xDF, 0xE0]), BUF, bytes(img[:256]))
    regs.gpr[6] = BUF
    out, fin = sim_run(L, sp, regs)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    o.step()
    o.step()
    assert fin.fpsw == 0x8081 and out.gpr[0] & 0xFFFF == 0x8081
    assert o.regs().gpr[0] & 0xFFFF == 0x8081


def _env_prog(code, data):
    L = sim_lib()
    sp, regs = layout(bytes(code), BUF, bytes(data) + bytes(256 - len(data)))
    regs.gpr[6], regs.gpr[7] = BUF, BUF + 0x80
    regs.fpcw, regs.fptw = 0x37F, 0xFFFF
    out, fin = sim_run(L, sp, regs, win_va=BUF)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    for _ in range(16):
        if o.step().status != 0:
            break
    env = bytes(out.win[0x80:0x80 + 28])
    assert env == o.read_virt(BUF + 0x80, 28)
    return [int.from_bytes(env[i:i + 2], "little") for i in (0, 4, 8)]


def test_fldenv_frstor_normalise_fcw_and_retag():
    """FLDENV / FRSTOR load FCW as FLDCW does and recompute every non-empty
    tag from the register contents; the values are this host's (fnstenv after
    the load): fldz / fld1 / fldpi, fldenv of fcw 0 / ftw 0 -> 0040 / 4155;
    fcw ffff / ftw aaaa -> 1f7f / 4155; frstor of fcw ffff, ST0 = 1.0 -> 1f7f / 5554."""
    ld3 = [0xD9, 0xEE, 0xD9, 0xE8, 0xD9, 0xEB]           # fldz; fld1; fldpi
    fldenv_fnstenv = [0xD9, 0x26, 0xD9, 0x37, 0xCC]     # fldenv [rsi]; fnstenv [rdi]; int3
    assert _env_prog(ld3 + fldenv_fnstenv, bytes(28)) == [0x0040, 0, 0x4155]
    env = bytearray(28)
    env[0:2], env[8:10] = (0xFFFF).to_bytes(2, "little"), (0xAAAA).to_bytes(2, "little")
    assert _env_prog(ld3 + fldenv_fnstenv, env) == [0x1F7F, 0, 0x4155]
    img = bytearray(108)
    img[0:2] = (0xFFFF).to_bytes(2, "little")
    img[28:36], img[36:38] = (1 << 63).to_bytes(8, "little"), (0x3FFF).to_bytes(2, "little")
    assert _env_prog([0xDD, 0x26, 0xD9, 0x37, 0xCC], img) == [0x1F7F, 0, 0x5554]   # frstor [rsi]; fnstenv [rdi]


def test_x87_store_fault_leaves_the_stack():
    # fstp dword [rsi + 0x2000] (unmapped): #PF (write), TOP and ST0 unchanged
    L = sim_lib()
    c = x87_case([0xD9, 0x9E, 0x00, 0x20, 0x00, 0x00], fsw=0x3800, ftw=0x3FFF, st=[ONE] + [(0, 0)] * 7)
    for got in (run_oracle(c, BUF), run_sim(L, c, BUF)):
        assert (got["status"], got["vector"]) == (EXIT_FAULT, 14)
        assert got["fsw"] == 0x3800 and tuple(got["st"][0]) == ONE
