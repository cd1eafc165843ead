"""MMX (U37): the oracle and the engine's code built for the host
(tests/native/sim_lane.cc) against native-execution vectors
(tests/golden/gen_mmx_vectors.py: GPRs, RFLAGS, XMM, mm0-7, FSW and the
abridged tag byte after the instruction, the memory window), then the rules
native execution cannot show: #UD / #NM / #MF and the TOS rotation. The GPU
runs the same vectors in tests/test_gpu_sse.py."""
import ctypes as C
import gzip
import json
import os

import pytest

from tests.cpu_bins import SIMLANE_SO, ensure
from tests.golden.gen_native_vectors import splitmix_bytes
from tests.oracle_lib import Oracle
from tests.test_sse import CODE_VA, SimResult, layout
from wtf_amd.abi import EXIT_FAULT, EXIT_UNIMPLEMENTED, RUNNING, Regs

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with gzip.open(os.path.join(HERE, "golden", "mmx_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()
BUF = int(DOC["buf_va"], 16)


def case_regs(c, regs):
    for i in range(16):
        regs.gpr[i] = int(c["in"][i], 16)
    regs.rflags = int(c["fl"], 16) | 0x200
    xs = [int(v, 16) for v in c["xin"]]
    for i in range(16):
        regs.xmm[i][0], regs.xmm[i][1] = xs[2 * i], xs[2 * i + 1]
    for i in range(8):
        regs.fpst[i] = int(c["mmin"][i], 16)
    regs.fpsw = 0       # the stub's movq loads leave TOS = 0
    regs.fptw = 0x0000  # and every tag valid
    return regs


def abridged(ftw):
    return sum(1 << i for i in range(8) if (ftw >> (2 * i)) & 3 != 3)


def check(c, r):
    want = [int(x, 16) for x in c["out"]]
    if list(r.gpr) != want:
        return ("regs", [(i, hex(r.gpr[i]), hex(want[i])) for i in range(16) if r.gpr[i] != want[i]])
    if (r.rflags ^ int(c["flo"], 16)) & 0x8D5:
        return ("flags",)
    if [r.xmm[i][h] for i in range(16) for h in range(2)] != [int(v, 16) for v in c["xout"]]:
        return ("xmm",)
    mm = [int(v, 16) for v in c["mmout"]]
    if list(r.fpst) != mm:
        return ("mm", [(i, hex(r.fpst[i]), hex(mm[i])) for i in range(8) if r.fpst[i] != mm[i]])
    if r.fpsw != int(c["fsw"], 16) or abridged(r.fptw) != int(c["ftw"], 16):
        return ("x87", hex(r.fpsw), hex(r.fptw), c["fsw"], c["ftw"])
    return None


def window_after(c):
    win = bytearray(splitmix_bytes(int(c["seed"], 16), 256))
    for i, v in c["diff"]:
        win[i] = v
    return bytes(win)


@pytest.mark.parametrize("chunk", range(2))
def test_oracle_matches_native_mmx(chunk):
    fails = []
    cases = DOC["cases"][chunk::2]
    for c in cases:
        code = bytes.fromhex(c["code"])
        sp, regs = layout(code, BUF, splitmix_bytes(int(c["seed"], 16), 256))
        pfns, blob = sp.phys()
        o = Oracle(pfns=pfns, blob=blob)
        o.restore(case_regs(c, regs))
        ex = o.step()
        if ex.status != RUNNING:
            fails.append((c["name"], c["code"], "exit", ex.status, ex.vector))
            continue
        r = o.regs()
        bad = check(c, r)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
        elif o.read_virt(BUF, 256) != window_after(c):
            fails.append((c["name"], c["code"], "mem"))
        elif r.rip != CODE_VA + len(code):
            fails.append((c["name"], c["code"], "rip"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def test_mmx_vector_file_is_substantial():
    assert len(DOC["cases"]) > 1500
    names = {c["name"].split(".")[0] for c in DOC["cases"]}
    for n in ("m60", "m6f", "mfe", "pshufw", "shimm", "movq", "movntq", "movd", "pextrw", "pinsrw", "pmovmskb",
              "movq2dq", "movdq2q", "emms"):
        assert n in names, n


def sim_lib():
    L = C.CDLL(ensure(SIMLANE_SO, os.path.join(HERE, "native")))
    L.sim_run_full.argtypes = [C.POINTER(C.c_uint64), C.c_char_p, C.c_uint64, C.POINTER(Regs), C.c_uint64,
                               C.POINTER(SimResult), C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(Regs),
                               C.c_char_p]
    return L


def sim_run(L, sp, regs, limit=0, win_va=0):
    """One lane until it stops; the merged final registers (x87 / MMX state included)."""
    pfns, blob = sp.phys()
    arr = (C.c_uint64 * len(pfns))(*pfns)
    out = SimResult()
    final = Regs()
    cnt = C.c_uint64(0)
    L.sim_run_full(arr, blob, len(pfns), C.byref(regs), limit, C.byref(out), 0, C.byref(cnt), win_va, C.byref(final),
                   None)
    return out, final


def test_engine_mmx_code_matches_native_vectors():
    L = sim_lib()
    fails = []
    for c in DOC["cases"]:
        sp, regs = layout(bytes.fromhex(c["code"]), BUF, splitmix_bytes(int(c["seed"], 16), 256))
        out, r = sim_run(L, sp, case_regs(c, regs), win_va=BUF)
        if out.status != 3 or out.icount != 1:  # the int3 after the instruction
            fails.append((c["name"], c["code"], "exit", out.status, out.vector))
            continue
        bad = check(c, r)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
        elif bytes(out.win[:256]) != window_after(c):
            fails.append((c["name"], c["code"], "mem"))
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:6]}"


# ---- hand-checked: the rules native execution cannot show
FAULT_CASES = [
    ([0x0F, 0xFC, 0xC1], dict(cr0=0x80050031 | 4), EXIT_FAULT, 6),    # CR0.EM: #UD
    ([0x0F, 0xFC, 0xC1], dict(cr0=0x80050031 | 8), EXIT_FAULT, 7),    # CR0.TS: #NM
    ([0x0F, 0xFC, 0xC1], dict(fsw=0x8081, fcw=0x37E), EXIT_FAULT, 16),  # an unmasked flag pending: #MF
    ([0x0F, 0x77], dict(fsw=0x8081, fcw=0x37E), EXIT_FAULT, 16),      # emms too
    ([0x0F, 0x77], dict(fsw=0x0001, fcw=0x37E), EXIT_FAULT, 16),      # the host's rule: ES not needed
    ([0x0F, 0x77], dict(fsw=0x0080, fcw=0x37F), RUNNING, None),       # ES with every flag masked: none
    ([0x0F, 0x73, 0xD9, 0x01], {}, EXIT_FAULT, 6),                    # psrldq has no MMX form
    ([0x0F, 0x71, 0xC1, 0x01], {}, EXIT_FAULT, 6),                    # 71 /0
    ([0x0F, 0x71, 0x16, 0x01], {}, EXIT_FAULT, 6),                    # shift-by-imm of memory
    ([0x0F, 0xD7, 0x06], {}, EXIT_FAULT, 6),                          # pmovmskb of memory
    ([0x0F, 0xE7, 0xC1], {}, EXIT_FAULT, 6),                          # movntq to a register
    ([0x0F, 0xD6, 0xC1], {}, EXIT_FAULT, 6),                          # 0f d6 without a prefix
    ([0x0F, 0xF7, 0xC1], {}, RUNNING, None),                          # maskmovq, no byte selected (U37)
    ([0x0F, 0xF7, 0x06], {}, EXIT_FAULT, 6),                          # maskmovq with a memory operand
    ([0x0F, 0x2A, 0xC1], {}, RUNNING, None),                          # cvtpi2ps xmm0, mm1
    ([0x0F, 0x2A, 0xC1], dict(fsw=0x8081, fcw=0x37E), EXIT_FAULT, 16),  # an mm source: #MF first
    ([0x0F, 0x2A, 0x06], dict(fsw=0x8081, fcw=0x37E), RUNNING, None),   # an m64 source: no x87 state touched
    ([0x0F, 0x2D, 0xC1], dict(fsw=0x8081, fcw=0x37E), EXIT_FAULT, 16),  # cvtps2pi: an mm destination
    ([0x66, 0x0F, 0x2D, 0x06], {}, EXIT_FAULT, 13),                   # cvtpd2pi mm0, [rsi]: m128 needs alignment
    ([0x0F, 0x38, 0x01, 0xC1], {}, RUNNING, None),                    # phaddw mm (SSSE3 on mm registers, U41)
    ([0x0F, 0x38, 0x01, 0xC1], dict(fsw=0x8081, fcw=0x37E), EXIT_FAULT, 16),  # ... #MF first
    ([0x0F, 0x38, 0x0C, 0xC1], {}, EXIT_FAULT, 6),                    # 0f 38 0c without 66: no instruction (U36)
]


def run_one(code, L=None, cr0=None, fsw=0, tos=0, fptw=0xFFFF, mm=None, fcw=0x37F):
    sp, regs = layout(bytes(code), BUF, bytes(range(256)), cr0=cr0)
    regs.gpr[6] = BUF + 0x13
    regs.fpcw = fcw
    regs.fpsw = fsw | (tos << 11)
    regs.fptw = fptw
    for i in range(8):
        regs.fpst[i] = mm[i] if mm else 0x1111111111111111 * (i + 1)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.step()
    sim = sim_run(L, sp, regs, limit=0) if L is not None else None
    return ex, o.regs(), sim


@pytest.mark.parametrize("code,kw,status,vector", FAULT_CASES)
def test_mmx_faults_oracle_and_engine(code, kw, status, vector):
    L = sim_lib()
    ex, _, (out, _) = run_one(code, L, **kw)
    assert (ex.status, ex.vector if vector else None) == (status, vector), bytes(code).hex()
    want = 3 if status == RUNNING else status
    assert (out.status, out.vector if vector else None) == (want, vector)


def test_tos_rotation_and_tags():
    """paddb mm1, mm2 with TOS = 3: mm i is ST((i - 3) & 7) = fpst[(i - 3) & 7]
    before; after, TOS = 0, fpst is in R order and every tag valid; emms
    then empties the tags and keeps the values."""
    L = sim_lib()
    mm = [0x0101010101010101 * (i + 1) for i in range(8)]
    ex, r, (out, f) = run_one([0x0F, 0xFC, 0xCA, 0x0F, 0x77], L, tos=3, fptw=0x5555, mm=mm)
    phys = [mm[(i - 3) & 7] for i in range(8)]
    want = list(phys)
    want[1] = sum((((phys[1] >> (8 * k)) + (phys[2] >> (8 * k))) & 0xFF) << (8 * k) for k in range(8))
    assert ex.status == RUNNING
    assert list(r.fpst) == want and (r.fpsw >> 11) & 7 == 0 and r.fptw == 0
    assert out.status == 3 and list(f.fpst) == want and f.fptw == 0xFFFF and (f.fpsw >> 11) & 7 == 0
