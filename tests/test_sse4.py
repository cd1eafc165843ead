"""SSSE3 / SSE4.1 integer forms and the AVX / AVX2 lane-crossing forms
(convention U41; engine_sse4.h, oracle/x86_oracle_sse4.inc).

Native-execution vectors (tests/golden/gen_sse4_vectors.py) pin the oracle
(the host CPU computes each form in register form around the oracle's decode,
checks and memory access) and the engine's device code built for the host;
the GPU runs them in tests/test_gpu_sse.py. Hand-checked: the #UD rules
(VEX.L, VEX.W, vvvv, memory-only forms) and alignment.
"""
import gzip
import json
import os

import pytest

from tests.golden.gen_sse4_vectors import case_inputs
from tests.oracle_lib import Oracle
from tests.test_avx import get_ymm, set_ymm
from tests.test_fp import check, norm, run_case
from tests.test_sse import layout, sim_lib, sim_run
from wtf_amd.abi import EXIT_FAULT, RUNNING

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with gzip.open(os.path.join(HERE, "golden", "sse4_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def inputs(c):
    ymm, win = case_inputs(int(c["seed"], 16))
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
    for i, v in c["mdiff"]:
        w[i] = v
    return bytes(w)


@pytest.mark.parametrize("chunk", range(2))
def test_oracle_matches_native_sse4(chunk):
    buf_va = int(DOC["buf_va"], 16)
    cases = DOC["cases"][chunk::2]
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
        if not bad and o.read_virt(buf_va, 256) != window_after(c, win):
            bad = ("mem",)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:5]}"


def test_engine_sse4_code_matches_native_vectors():
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
            fails.append((c["name"], c["code"]) + bad)
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:5]}"


def test_sse4_vector_file_is_substantial():
    names = {c["name"].split(".")[0] for c in DOC["cases"]}
    assert len(DOC["cases"]) > 1900
    for n in ("phaddw", "pmaddubsw", "pabsd", "pmovzx30", "pmovsx25", "pminud", "pmulld", "packusdw", "palignr",
              "pextrd", "pinsrb", "insertps", "movntdqa", "vpermq", "vpermd", "vperm2i128", "vinserti128",
              "vextracti128", "vpsllv", "vpsrav", "vpblendvb", "vbroadcastss", "vbroadcasti128", "vtestps",
              "mpsadbw", "vmpsadbw", "vmaskmovps", "vmaskmovpd", "vpmaskmovq", "vpmaskmovd"):
        assert n in names, n


SSE4_FAULT_CASES = [
    ([0x66, 0x0F, 0x38, 0x40, 0x06], EXIT_FAULT, 13),               # pmulld xmm0, [rsi]: misaligned
    ([0x66, 0x0F, 0x38, 0x30, 0x06], RUNNING, None),                # pmovzxbw xmm0, [rsi] (m64)
    ([0x66, 0x0F, 0x38, 0x2A, 0xC1], EXIT_FAULT, 6),                # movntdqa xmm0, xmm1: memory only
    ([0x66, 0x0F, 0x38, 0x2A, 0x06], EXIT_FAULT, 13),               # movntdqa xmm0, [rsi]: aligned
    ([0xC4, 0xE2, 0x7D, 0x2A, 0x06], EXIT_FAULT, 13),               # vmovntdqa ymm0, [rsi]: aligned
    ([0xC4, 0xE2, 0x7D, 0x40, 0x06], RUNNING, None),                # vpmulld ymm0, ymm0, [rsi]
    ([0xC4, 0xE3, 0x7D, 0x00, 0xC1, 0x1B], EXIT_FAULT, 6),          # vpermq with VEX.W = 0
    ([0xC4, 0xE3, 0xF9, 0x00, 0xC1, 0x1B], EXIT_FAULT, 6),          # vpermq with VEX.L = 0
    ([0xC4, 0xE3, 0xFD, 0x00, 0xC1, 0x1B], RUNNING, None),          # vpermq ymm0, ymm1, 0x1b
    ([0xC4, 0xE3, 0x7D, 0x14, 0xC1, 0x01], EXIT_FAULT, 6),          # vpextrb with VEX.L = 1
    ([0xC4, 0xE3, 0x75, 0x19, 0xC1, 0x01], EXIT_FAULT, 6),          # vextractf128 with vvvv != 1111
    ([0xC4, 0xE2, 0x7D, 0x1A, 0xC1], EXIT_FAULT, 6),                # vbroadcastf128 ymm0, xmm1: memory only
    ([0xC4, 0xE2, 0x79, 0x1A, 0x06], EXIT_FAULT, 6),                # vbroadcastf128 with VEX.L = 0
    ([0xC4, 0xE2, 0xF9, 0x46, 0xC1], EXIT_FAULT, 6),                # vpsravq (AVX-512 only): #UD
    ([0x66, 0x0F, 0x3A, 0x42, 0x06, 0x00], EXIT_FAULT, 13),          # mpsadbw xmm0, [rsi]: misaligned
    ([0xC4, 0xE2, 0x79, 0x2C, 0xC1], EXIT_FAULT, 6),                # vmaskmovps xmm0, xmm0, xmm1: memory only
    ([0xC4, 0xE2, 0xF9, 0x2C, 0x06], EXIT_FAULT, 6),                # vmaskmovps with VEX.W = 1
    ([0xC4, 0xE2, 0x79, 0x2C, 0x86, 0x00, 0x40, 0x00, 0x00], RUNNING, None),  # mask 0: no access, no fault
    ([0x0F, 0x38, 0x00, 0xC1], RUNNING, None),                      # pshufb mm0, mm1 (SSSE3 on mm registers)
]


@pytest.mark.parametrize("code,status,vector", SSE4_FAULT_CASES)
def test_sse4_faults_oracle_and_engine(code, status, vector):
    L = sim_lib()
    for got in (run_case(code), run_case(code, sim=L)):
        assert norm(got[0]) == status, (bytes(code).hex(), got[:2])
        if vector is not None:
            assert got[1] == vector
