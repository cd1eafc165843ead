"""AVX / AVX2 (VEX) subset and the legacy pshufb / ptest.

The oracle and the engine's own code built for the host (tests/native/
sim_lane.cc) against native-execution vectors (tests/golden/gen_avx_vectors.py:
16 GPRs, RFLAGS, 16 YMM registers at 256 bits and a 256-byte memory window),
then the #UD / #NM / #GP rules native execution cannot show. The GPU runs the
same vectors in tests/test_gpu_sse.py.
"""
import gzip
import json
import os

import pytest

from tests.golden.gen_native_vectors import splitmix_bytes
from tests.test_sse import BUF, layout, sim_lib, sim_run
from tests.oracle_lib import Oracle
from wtf_amd.abi import EXIT_FAULT, EXIT_TIMEOUT, EXIT_UNIMPLEMENTED, RUNNING

HERE = os.path.dirname(os.path.abspath(__file__))
CODE_VA = 0x140001000


def load():
    with gzip.open(os.path.join(HERE, "golden", "avx_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def set_ymm(regs, ys):
    for i in range(16):
        regs.xmm[i][0], regs.xmm[i][1] = ys[4 * i], ys[4 * i + 1]
        regs.ymmh[i][0], regs.ymmh[i][1] = ys[4 * i + 2], ys[4 * i + 3]


def get_ymm(xmm, ymmh):
    """32 + 32 u64 (xmm / ymmh, reg-major) -> 64 u64 in native ymm order."""
    out = []
    for i in range(16):
        out += [xmm[2 * i], xmm[2 * i + 1], ymmh[2 * i], ymmh[2 * i + 1]]
    return out


def case_regs(c, regs):
    for i in range(16):
        regs.gpr[i] = int(c["in"][i], 16)
    regs.rflags = int(c["fl"], 16) | 0x200
    set_ymm(regs, [int(v, 16) for v in c["yin"]])
    return regs


def window(c):
    return splitmix_bytes(int(c["seed"], 16), 256)


@pytest.mark.parametrize("chunk", range(4))
def test_oracle_matches_native_avx(chunk):
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    cases = DOC["cases"][chunk::4]
    for c in cases:
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, window(c))
        pfns, blob = sp.phys()
        o = Oracle(pfns=pfns, blob=blob)
        o.restore(case_regs(c, regs))
        ex = o.step()
        if ex.status != RUNNING:
            fails.append((c["name"], c["code"], "exit", ex.status, ex.vector))
            continue
        r = o.regs()
        if list(r.gpr) != [int(x, 16) for x in c["out"]] or (r.rflags ^ int(c["flo"], 16)) & 0x8D5:
            fails.append((c["name"], c["code"], "regs"))
            continue
        got = get_ymm([r.xmm[i][h] for i in range(16) for h in range(2)],
                      [r.ymmh[i][h] for i in range(16) for h in range(2)])
        if got != [int(v, 16) for v in c["yout"]]:
            fails.append((c["name"], c["code"], "ymm"))
            continue
        win = bytearray(window(c))
        for i, v in c["diff"]:
            win[i] = v
        if o.read_virt(buf_va, 256) != bytes(win):
            fails.append((c["name"], c["code"], "mem"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def test_engine_avx_code_matches_native_vectors():
    L = sim_lib()
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    for c in DOC["cases"]:
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, window(c))
        out = sim_run(L, sp, case_regs(c, regs))
        if out.status != 3 or out.icount != 1:
            fails.append((c["name"], c["code"], "exit", out.status, out.vector))
        elif list(out.gpr) != [int(x, 16) for x in c["out"]] or (out.rflags ^ int(c["flo"], 16)) & 0x8D5:
            fails.append((c["name"], c["code"], "regs"))
        elif get_ymm(list(out.xmm), list(out.ymmh)) != [int(v, 16) for v in c["yout"]]:
            fails.append((c["name"], c["code"], "ymm"))
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:6]}"


def test_avx_vector_file_is_substantial():
    assert len(DOC["cases"]) > 2000
    names = {c["name"].split(".")[0] for c in DOC["cases"]}
    for n in ("vmovdqu", "vmovdqa", "vpmovmskb", "vzero", "vptest", "vpshufb", "vpbroadcast78", "pshufb", "ptest"):
        assert n in names, n


# ---- hand-checked: VEX #UD rules, alignment, AVX state
AVX_FAULT_CASES = [
    ([0xC5, 0xFE, 0x6F, 0x06], RUNNING, None),             # vmovdqu ymm0, [rsi]: unaligned is fine
    ([0xC5, 0xFD, 0x6F, 0x03], EXIT_FAULT, 13),             # vmovdqa ymm0, [rbx]: rbx 16- but not 32-aligned
    ([0xC5, 0xF9, 0x6F, 0x03], RUNNING, None),             # vmovdqa xmm0, [rbx]: 16-aligned
    ([0xC5, 0xF9, 0x6F, 0x06], EXIT_FAULT, 13),             # vmovdqa xmm0, [rsi]: misaligned
    ([0xC5, 0xF5, 0xEF, 0x06], RUNNING, None),             # vpxor ymm0, ymm1, [rsi]: VEX needs no alignment
    ([0xC5, 0xF6, 0x6F, 0xC1], EXIT_FAULT, 6),              # vmovdqu with vvvv != 1111
    ([0xC5, 0xFD, 0x6E, 0xC0], EXIT_FAULT, 6),              # vmovd with L = 1
    ([0x66, 0xC5, 0xF9, 0xEF, 0xC1], EXIT_FAULT, 6),        # 66 before VEX
    ([0x48, 0xC5, 0xF9, 0xEF, 0xC1], EXIT_FAULT, 6),        # REX before VEX
    ([0xC5, 0xFD, 0xD7, 0x03], EXIT_FAULT, 6),              # vpmovmskb eax, [rbx]: register only
    ([0xC5, 0xFC, 0x58, 0xC1], RUNNING, None),              # vaddps (floating point, U39)
    ([0xC4, 0xE3, 0x79, 0x0F, 0xC1, 0x04], RUNNING, None),  # vpalignr (0f 3a, U41)
    ([0xC4, 0xE2, 0x79, 0x1C, 0xC1], RUNNING, None),        # vpabsb (0f 38 1c, U41)
    ([0x66, 0x0F, 0x38, 0x00, 0x06], EXIT_FAULT, 13),      # pshufb xmm0, [rsi]: legacy needs alignment
    ([0x66, 0x0F, 0x38, 0x1C, 0xC1], RUNNING, None),        # pabsb (U41)
    ([0x66, 0x0F, 0x3A, 0x42, 0xC1, 0x00], RUNNING, None),  # mpsadbw (U41)
    ([0x66, 0x0F, 0x3A, 0x40, 0xC1, 0x00], RUNNING, None),   # dpps
    ([0xC4, 0xE3, 0x7D, 0x41, 0xC1, 0x31], EXIT_FAULT, 6),   # vdppd ymm: no 256-bit form
    # U36 / U45: encodings no CPU defines are #UD; defined ones outside the engine are UNIMPLEMENTED
    ([0xC4, 0x30, 0x02, 0x00], EXIT_FAULT, 6),              # VEX map 0x10 (runaway HEVD bytes)
    ([0xC4, 0xE0, 0x79, 0x58, 0xC1], EXIT_FAULT, 6),        # VEX map 0
    ([0xC4, 0xE4, 0x79, 0x58, 0xC1], EXIT_FAULT, 6),        # VEX map 4
    ([0xC5, 0xF8, 0x00, 0xC1], EXIT_FAULT, 6),              # VEX 0f 00: no AVX form
    ([0xC5, 0xF8, 0x60, 0xC1], EXIT_FAULT, 6),              # VEX.NP 0f 60: MMX only
    ([0xC5, 0xFA, 0x14, 0xC1], EXIT_FAULT, 6),              # VEX.F3 0f 14
    ([0xC4, 0xE2, 0x79, 0x50, 0xC1], EXIT_UNIMPLEMENTED, None),  # vpdpbusd: AVX-VNNI defined, not executed
    ([0xC4, 0xE2, 0x78, 0xF2, 0xC1], RUNNING, None),        # andn (BMI1)
    ([0xC4, 0xE2, 0x79, 0x13, 0xC1], RUNNING, None),        # vcvtph2ps (F16C, U46)
    ([0xC4, 0xE2, 0x79, 0xA8, 0xC1], RUNNING, None),        # vfmadd213ps (FMA3, U46)
    ([0xC4, 0xE2, 0x71, 0x92, 0xC1], EXIT_FAULT, 6),        # vgatherdps with a register operand (U46)
    ([0xC4, 0xE3, 0x79, 0x44, 0xC1, 0x00], RUNNING, None),  # vpclmulqdq xmm (PCLMULQDQ)
    ([0xC4, 0xE3, 0x7D, 0x44, 0xC1, 0x00], EXIT_UNIMPLEMENTED, None),  # vpclmulqdq ymm: VPCLMULQDQ
    ([0xC4, 0xE2, 0x7D, 0xDC, 0xC1], EXIT_UNIMPLEMENTED, None),  # vaesenc ymm: VAES
    ([0xC4, 0xE3, 0x7B, 0xF0, 0xC1, 0x01], RUNNING, None),  # rorx (BMI2)
    ([0xC4, 0xE2, 0x7C, 0xF2, 0xC1], EXIT_FAULT, 6),        # andn with VEX.L = 1
    ([0xC4, 0xE2, 0x78, 0xF3, 0xC1], EXIT_FAULT, 6),        # group 17 /0: undefined
    ([0xC4, 0xE2, 0x70, 0xF3, 0xC9], RUNNING, None),        # blsr ecx, ecx
    ([0xC4, 0xE3, 0x79, 0x63, 0xC1, 0x0C], RUNNING, None),  # vpcmpistri
    ([0xC4, 0xE3, 0x7D, 0x63, 0xC1, 0x0C], EXIT_FAULT, 6),  # vpcmpistri with VEX.L = 1
    ([0xC5, 0xF8, 0xAE, 0x16], EXIT_UNIMPLEMENTED, None),   # vldmxcsr [rsi]: defined, outside the subset
    ([0xC5, 0xF8, 0xAE, 0xC1], EXIT_FAULT, 6),              # VEX 0f ae, register form
    ([0xC5, 0xF8, 0xAE, 0x06], EXIT_FAULT, 6),              # VEX 0f ae /0 (fxsave has no VEX form)
    ([0xC4, 0xE3, 0x79, 0x0F, 0x06, 0x04], RUNNING, None),  # vpalignr xmm, [rsi] (U41)
    ([0x66, 0x0F, 0x38, 0x37, 0xC1], RUNNING, None),        # pcmpgtq (SSE4.2)
    ([0x66, 0x0F, 0x38, 0x37, 0x06], EXIT_FAULT, 13),       # pcmpgtq xmm0, [rsi]: legacy needs alignment
    ([0x66, 0x0F, 0x3A, 0x61, 0x06, 0x00], RUNNING, None),  # pcmpestri xmm0, [rsi]: no alignment
    ([0x0F, 0x38, 0xF0, 0x06], RUNNING, None),              # movbe eax, [rsi]
    ([0x0F, 0x38, 0xF0, 0xC1], EXIT_FAULT, 6),              # movbe eax, ecx: memory only
    ([0xF2, 0x0F, 0x38, 0xF1, 0xC1], RUNNING, None),        # crc32 eax, ecx
    ([0x66, 0x0F, 0x38, 0xF6, 0xC1], RUNNING, None),        # adcx eax, ecx
    ([0xF0, 0x66, 0x0F, 0x38, 0xF6, 0x06], EXIT_FAULT, 6),  # lock adcx: #UD (U34)
    ([0x66, 0x0F, 0x38, 0xDC, 0xC1], RUNNING, None),        # aesenc (AES)
    ([0x66, 0x0F, 0x38, 0x50, 0xC1], EXIT_FAULT, 6),        # 0f 38 50: undefined
    ([0x0F, 0x38, 0xC9, 0xC1], RUNNING, None),              # sha1msg1 (SHA)
    ([0x0F, 0x38, 0xC9, 0x06], EXIT_FAULT, 13),             # sha1msg1 xmm0, [rsi]: legacy needs alignment
    ([0xC4, 0xE2, 0x78, 0xC9, 0xC1], EXIT_FAULT, 6),        # SHA has no VEX form
    ([0x66, 0x0F, 0x3A, 0x44, 0xC1, 0x00], RUNNING, None),  # pclmulqdq
    ([0x62, 0xF1, 0x7C, 0x48, 0x58, 0xC1], EXIT_UNIMPLEMENTED, None),  # EVEX vaddps zmm: AVX-512
    ([0x0F, 0x38, 0x00, 0xC1], RUNNING, None),              # pshufb mm, mm (SSSE3 on mm registers, U41)
    ([0x0F, 0x3A, 0x0F, 0xC1, 0x01], RUNNING, None),        # palignr mm, mm, 1 (U41)
]


def run1(code, cr0=None, cr4=None, xcr0=None, L=None):
    sp, regs = layout(bytes(code), BUF, bytes(range(256)), cr0=cr0, cr4=cr4)
    regs.gpr[3] = BUF + 0x10  # rbx: 16-aligned, not 32-aligned (BUF is 0x...800)
    regs.gpr[6] = BUF + 0x13
    if xcr0 is not None:
        regs.xcr0 = xcr0
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.step()
    sim = sim_run(L, sp, regs) if L is not None else None
    return ex, sim


@pytest.mark.parametrize("code,status,vector", AVX_FAULT_CASES)
def test_avx_faults_oracle_and_engine(code, status, vector):
    L = sim_lib()
    ex, sim = run1(code, L=L)
    assert ex.status == status, (bytes(code).hex(), ex.status, ex.vector)
    if vector is not None:
        assert ex.vector == vector
    want_sim = 3 if status == RUNNING else status
    assert sim.status == want_sim and (vector is None or sim.vector == vector), (sim.status, sim.vector)


def test_avx_state_gating():
    L = sim_lib()
    vpxor = [0xC5, 0xF5, 0xEF, 0xC2]
    for kw, vec in ((dict(cr4=0x370678 & ~0x40000), 6), (dict(xcr0=0x3), 6), (dict(cr0=0x80050031 | 8), 7)):
        ex, sim = run1(vpxor, L=L, **kw)
        assert (ex.status, ex.vector) == (EXIT_FAULT, vec), kw
        assert (sim.status, sim.vector) == (EXIT_FAULT, vec), kw
    ex, sim = run1(vpxor, L=L, cr0=0x80050031 | 4)  # CR0.EM does not gate VEX
    assert ex.status == RUNNING and sim.status == 3


def test_vzeroupper_keeps_low_halves_and_legacy_keeps_high():
    # vzeroupper ; movaps xmm1, xmm2 (legacy: ymm1's upper half stays) ; vmovaps xmm3, xmm2 (VEX.128: zeroed)
    code = [0xC5, 0xF8, 0x77, 0x0F, 0x28, 0xCA, 0xC5, 0xF8, 0x28, 0xDA]
    sp, regs = layout(bytes(code), BUF, bytes(256))
    for i in range(16):
        regs.xmm[i][0], regs.xmm[i][1] = i + 1, i + 2
        regs.ymmh[i][0], regs.ymmh[i][1] = 100 + i, 200 + i
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    assert o.step().status == RUNNING
    r = o.regs()
    assert all(r.ymmh[i][0] == 0 and r.ymmh[i][1] == 0 for i in range(16))
    assert all(r.xmm[i][0] == i + 1 for i in range(16))


def test_encoding_space_oracle_equals_engine():
    """U36 over the whole opcode space of VEX maps 0-4 (each pp) and of the
    legacy 0f 38 / 0f 3a maps (each mandatory prefix): the oracle and the
    engine's decode agree on #UD / UNIMPLEMENTED / executed for every opcode,
    register and memory ModRM forms alike."""
    L = sim_lib()
    codes = []
    for modrm in (0xC1, 0x06):
        for m in range(5):
            for pp in range(4):
                for op in range(256):
                    codes.append([0xC4, 0xE0 | m, 0x78 | pp, op, modrm, 0x01, 0xCC])
        for pfx in ([], [0x66], [0xF3], [0xF2]):
            for esc in (0x38, 0x3A):
                for op in range(256):
                    codes.append(pfx + [0x0F, esc, op, modrm, 0x01, 0xCC])
    bad = []
    for code in codes:
        sp, regs = layout(bytes(code), BUF, bytes(range(256)))
        regs.gpr[3], regs.gpr[6] = BUF + 0x10, BUF + 0x13
        pfns, blob = sp.phys()
        o = Oracle(pfns=pfns, blob=blob)
        o.restore(regs)
        ex = o.step()
        if ex.status == RUNNING:  # the limit stops the lane after its second instruction
            ex = o.step()
        sim = sim_run(L, sp, regs, limit=1)
        want = (EXIT_TIMEOUT, 3) if ex.status == RUNNING else (ex.status,)
        if sim.status not in want or (ex.status == EXIT_FAULT and sim.vector != ex.vector):
            bad.append((bytes(code).hex(), ex.status, ex.vector, sim.status, sim.vector))
    assert not bad, (len(bad), bad[:8])
