"""SSE / SSE2 subset (convention U22).

The CPU oracle is pinned by native-execution vectors (tests/golden/
gen_sse_vectors.py: 16 GPRs, RFLAGS, 16 XMM registers, MXCSR and a 256-byte
memory window, run natively on the x86-64 host). Behaviour native execution
cannot show without crashing (misaligned 16-byte operands, CR0/CR4 gating,
register-only / memory-only encodings) is checked by hand here; the GPU engine
is compared with the oracle on all of it in test_gpu_sse.py.
"""
import gzip
import json
import os

import pytest

from tests.golden.gen_native_vectors import splitmix_bytes
from tests.golden.gen_sse_vectors import window_in
from tests.oracle_lib import Oracle
from wtf_amd.abi import EXIT_FAULT, EXIT_UNIMPLEMENTED, RUNNING, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

HERE = os.path.dirname(os.path.abspath(__file__))
CODE_VA = 0x140001000


def load():
    with gzip.open(os.path.join(HERE, "golden", "sse_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def case_regs(case, regs):
    for i in range(16):
        regs.gpr[i] = int(case["in"][i], 16)
    regs.rflags = int(case["fl"], 16) | 0x200
    xs = [int(v, 16) for v in case["xin"]]
    for i in range(16):
        regs.xmm[i][0], regs.xmm[i][1] = xs[2 * i], xs[2 * i + 1]
    regs.mxcsr = int(case["mx"], 16)
    return regs


def layout(code: bytes, buf_va, window: bytes, cr0=None, cr4=None):
    """The address space of one case (code page, window page + the next page)
    and its initial registers."""
    page_va = buf_va & ~0xFFF
    sp = AddressSpace()
    sp.map(CODE_VA, code + b"\xcc", write=False)
    first = bytearray(4096)
    off = buf_va - page_va
    first[off:off + len(window)] = window
    sp.map(page_va, bytes(first))
    sp.map(page_va + 0x1000, b"")
    regs = regs_from_state(user_state(CODE_VA, 0, sp.cr3))
    if cr0 is not None:
        regs.cr0 = cr0
    if cr4 is not None:
        regs.cr4 = cr4
    return sp, regs


def build(code: bytes, buf_va, window: bytes, cr0=None, cr4=None):
    sp, regs = layout(code, buf_va, window, cr0, cr4)
    pfns, blob = sp.phys()
    return Oracle(pfns=pfns, blob=blob), regs


def check_case(c, buf_va, o, r):
    """Mismatch description, or None."""
    want = [int(x, 16) for x in c["out"]]
    if list(r.gpr) != want:
        return ("regs", [(i, hex(r.gpr[i]), hex(want[i])) for i in range(16) if r.gpr[i] != want[i]])
    if (r.rflags ^ int(c["flo"], 16)) & 0x8D5:
        return ("flags", hex(r.rflags), c["flo"])
    xo = [int(v, 16) for v in c["xout"]]
    got = [r.xmm[i][h] for i in range(16) for h in range(2)]
    if got != xo:
        return ("xmm", [(i // 2, hex(got[i]), hex(xo[i])) for i in range(32) if got[i] != xo[i]])
    if r.mxcsr != int(c["mxo"], 16):
        return ("mxcsr", hex(r.mxcsr), c["mxo"])
    return None


@pytest.mark.parametrize("chunk", range(4))
def test_oracle_matches_native_sse(chunk):
    buf_va = int(DOC["buf_va"], 16)
    cases = DOC["cases"][chunk::4]
    fails = []
    for c in cases:
        o, regs = build(bytes.fromhex(c["code"]), buf_va, window_in(int(c["seed"], 16), c["ldmx"]))
        o.restore(case_regs(c, regs))
        ex = o.step()
        if ex.status != RUNNING:
            fails.append((c["name"], c["code"], "exit", ex.status, ex.vector))
            continue
        r = o.regs()
        bad = check_case(c, buf_va, o, r)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
            continue
        win = bytearray(window_in(int(c["seed"], 16), c["ldmx"]))
        for i, v in c["diff"]:
            win[i] = v
        if o.read_virt(buf_va, 256) != bytes(win):
            fails.append((c["name"], c["code"], "mem"))
            continue
        if r.rip != CODE_VA + len(bytes.fromhex(c["code"])):
            fails.append((c["name"], c["code"], "rip"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def test_sse_vector_file_is_substantial():
    assert len(DOC["cases"]) > 2500
    names = {c["name"].split(".")[0] for c in DOC["cases"]}
    for n in ("movaps", "movdqu", "pef", "pmovmskb", "pshufd", "movd", "movq", "ldmxcsr", "shimm"):
        assert n in names, n


# ---- hand-checked faults and encodings (what native execution cannot show)
BUF = 0x7FF000100800  # any user address: these cases do not use the native window


def run1(code, regs_fn=None, cr0=None, cr4=None):
    o, regs = build(bytes(code), BUF, bytes(range(256)), cr0=cr0, cr4=cr4)
    regs.gpr[3] = BUF + 0x10  # rbx -> window + 16 (16-byte aligned)
    regs.gpr[6] = BUF + 0x13  # rsi -> misaligned
    if regs_fn:
        regs_fn(regs)
    o.restore(regs)
    return o, o.step()


SSE_FAULT_CASES = [
    # (bytes, expected status, vector)
    ([0x0F, 0x28, 0x06], EXIT_FAULT, 13),             # movaps xmm0, [rsi] misaligned -> #GP(0)
    ([0x66, 0x0F, 0xEF, 0x06], EXIT_FAULT, 13),       # pxor xmm0, [rsi] misaligned
    ([0x66, 0x0F, 0x7F, 0x06], EXIT_FAULT, 13),       # movdqa [rsi], xmm0 misaligned
    ([0xF3, 0x0F, 0x6F, 0x06], RUNNING, None),        # movdqu xmm0, [rsi]: fine
    ([0x0F, 0x11, 0x06], RUNNING, None),              # movups [rsi], xmm0: fine
    ([0x0F, 0x28, 0x03], RUNNING, None),              # movaps xmm0, [rbx] aligned
    ([0x66, 0x0F, 0xD7, 0x03], EXIT_FAULT, 6),        # pmovmskb eax, [rbx]: register-only -> #UD
    ([0x66, 0x0F, 0x73, 0x1B, 0x04], EXIT_FAULT, 6),  # psrldq [rbx], 4: register-only
    ([0x0F, 0x13, 0xC1], EXIT_FAULT, 6),              # movlps xmm1, xmm0 (0f 13 reg): #UD
    ([0x0F, 0x2B, 0xC1], EXIT_FAULT, 6),              # movntps reg form: #UD
    ([0x0F, 0xC3, 0xC1], EXIT_FAULT, 6),              # movnti reg form: #UD
    ([0x0F, 0xEF, 0xC1], RUNNING, None),              # MMX pxor mm0, mm1 (U37)
    ([0x0F, 0xF7, 0xC1], RUNNING, None),              # MMX maskmovq (no byte selected: nothing written)
    ([0x0F, 0x58, 0xC1], RUNNING, None),              # addps (floating point, U39)
    ([0xF2, 0x0F, 0xF0, 0x03], RUNNING, None),        # lddqu (SSE3, U39)
    ([0x0F, 0x53, 0xC1], RUNNING, None),              # rcpps (the host CPU's table, U40)
]


@pytest.mark.parametrize("code,status,vector", SSE_FAULT_CASES)
def test_oracle_sse_faults(code, status, vector):
    _, ex = run1(code)
    assert ex.status == status, (bytes(code).hex(), ex.status, ex.vector)
    if vector is not None:
        assert ex.vector == vector


def test_oracle_sse_control_register_gating():
    # CR4.OSFXSR = 0 -> #UD; CR0.EM -> #UD; CR0.TS -> #NM (7); fences are not gated
    _, ex = run1([0x66, 0x0F, 0xEF, 0xC1], cr4=0x370678 & ~0x200)
    assert (ex.status, ex.vector) == (EXIT_FAULT, 6)
    _, ex = run1([0x66, 0x0F, 0xEF, 0xC1], cr0=0x80050031 | 4)
    assert (ex.status, ex.vector) == (EXIT_FAULT, 6)
    _, ex = run1([0x66, 0x0F, 0xEF, 0xC1], cr0=0x80050031 | 8)
    assert (ex.status, ex.vector) == (EXIT_FAULT, 7)
    _, ex = run1([0x0F, 0xAE, 0xF0], cr0=0x80050031 | 8)
    assert ex.status == RUNNING


def test_oracle_ldmxcsr_reserved_bits_gp():
    o, regs = build(bytes([0x0F, 0xAE, 0x13]), BUF, (0x10000).to_bytes(4, "little") * 64)
    regs.gpr[3] = BUF + 0x10
    o.restore(regs)
    ex = o.step()
    assert (ex.status, ex.vector) == (EXIT_FAULT, 13)
    assert o.regs().mxcsr == 0x1F80


def test_oracle_page_crossing_movdqu_store_faults_whole():
    # movdqu [rsi], xmm0 with rsi 8 bytes before an unmapped page: #PF, nothing written
    def put(regs):
        regs.gpr[6] = (BUF & ~0xFFF) + 0x2000 - 8
        regs.xmm[0][0], regs.xmm[0][1] = 0x1111111111111111, 0x2222222222222222

    o, ex = run1([0xF3, 0x0F, 0x7F, 0x06], put)
    assert (ex.status, ex.vector) == (EXIT_FAULT, 14)
    assert o.read_virt((BUF & ~0xFFF) + 0x2000 - 8, 8) == bytes(8)


# ---- the engine's own SSE code (engine_sse.h), built for the host
# (tests/native/sim_lane.cc: one lane of k_run's decode / exec / retry loop)
# against the native vectors and the oracle, so the device semantics are
# checked on CPU before any GPU run.
import ctypes as C  # noqa: E402

from tests.cpu_bins import SIMLANE_SO, ensure  # noqa: E402
from wtf_amd.abi import Regs  # noqa: E402


class SimResult(C.Structure):
    _fields_ = [("gpr", C.c_uint64 * 16), ("rip", C.c_uint64), ("rflags", C.c_uint64), ("icount", C.c_uint64),
                ("nbytes", C.c_uint64), ("status", C.c_uint32), ("vector", C.c_uint32), ("error", C.c_uint32),
                ("ovn", C.c_uint32), ("addr", C.c_uint64), ("dirty", C.c_uint64 * 64), ("xmm", C.c_uint64 * 32),
                ("mxcsr", C.c_uint32), ("pad", C.c_uint32), ("ymmh", C.c_uint64 * 32), ("win", C.c_uint8 * 512)]


def sim_lib():
    L = C.CDLL(ensure(SIMLANE_SO, os.path.join(HERE, "native")))
    L.sim_run.argtypes = [C.POINTER(C.c_uint64), C.c_char_p, C.c_uint64, C.POINTER(Regs), C.c_uint64,
                          C.POINTER(SimResult)]
    L.sim_run_mode.argtypes = L.sim_run.argtypes + [C.c_int, C.POINTER(C.c_uint64), C.c_uint64]
    return L


def sim_run(L, sp, regs, limit=0, fast=False, counter=None, win_va=0):
    """One lane from `regs` until it stops; fast=True tries the fast loop's
    form of each instruction first (k_run's order). `counter` (a c_uint64)
    counts the instructions the fast form retired; `win_va` selects the 512
    bytes returned in `win`."""
    pfns, blob = sp.phys()
    arr = (C.c_uint64 * len(pfns))(*pfns)
    out = SimResult()
    cnt = counter if counter is not None else C.c_uint64(0)
    L.sim_run_mode(arr, blob, len(pfns), C.byref(regs), limit, C.byref(out), 1 if fast else 0, C.byref(cnt), win_va)
    return out


def test_engine_sse_code_matches_native_vectors():
    L = sim_lib()
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    for c in DOC["cases"]:
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, window_in(int(c["seed"], 16), c["ldmx"]))
        out = sim_run(L, sp, case_regs(c, regs))
        if out.status != 3 or out.icount != 1:  # int3 after the instruction
            fails.append((c["name"], c["code"], "exit", out.status, out.vector))
        elif list(out.gpr) != [int(x, 16) for x in c["out"]] or (out.rflags ^ int(c["flo"], 16)) & 0x8D5:
            fails.append((c["name"], c["code"], "regs"))
        elif list(out.xmm) != [int(v, 16) for v in c["xout"]] or out.mxcsr != int(c["mxo"], 16):
            fails.append((c["name"], c["code"], "xmm"))
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:6]}"


@pytest.mark.parametrize("code,status,vector", SSE_FAULT_CASES)
def test_engine_sse_code_faults(code, status, vector):
    L = sim_lib()
    sp, regs = layout(bytes(code), BUF, bytes(range(256)))
    regs.gpr[3] = BUF + 0x10
    regs.gpr[6] = BUF + 0x13
    out = sim_run(L, sp, regs)
    want = 3 if status == RUNNING else status  # a clean run stops at the int3
    assert out.status == want, (bytes(code).hex(), out.status, out.vector)
    if vector is not None:
        assert out.vector == vector


@pytest.mark.parametrize("fast,fp", [(False, False), (True, False), (True, True)])
def test_engine_sse_code_matches_oracle_on_random_programs(fast, fp):
    """fp: with the floating-point and SSE4 / AVX2 forms and a random MXCSR per lane."""
    from tests import progfuzz

    L = sim_lib()
    n = 160
    seed = 33 if fp else 31
    sp, st, lanes = progfuzz.build(n, seed=seed, sse=True, fp=fp)
    xmm = progfuzz.lane_xmm(n, seed)
    ymmh = progfuzz.lane_xmm(n, seed, 0x4E4)
    mx = progfuzz.lane_mxcsr(n, seed) if fp else None
    want = progfuzz.oracle_run(sp, st, lanes, xmm=xmm, ymmh=ymmh, mxcsr=mx)
    bad = []
    for i, ((va, g, flags), w) in enumerate(zip(lanes, want)):
        regs = regs_from_state(st)
        for k in range(16):
            regs.gpr[k] = g[k]
            regs.xmm[k][0], regs.xmm[k][1] = xmm[i][2 * k], xmm[i][2 * k + 1]
            regs.ymmh[k][0], regs.ymmh[k][1] = ymmh[i][2 * k], ymmh[i][2 * k + 1]
        regs.rip, regs.rflags = va, flags
        if mx is not None:
            regs.mxcsr = mx[i]
        out = sim_run(L, sp, regs, limit=20000, fast=fast)
        got = (out.status, out.vector if out.status == EXIT_FAULT else 0, out.rip, out.icount)
        exp = (w["status"], w["vector"] if w["status"] == EXIT_FAULT else 0, w["rip"], w["icount"])
        if got != exp:
            bad.append((i, "exit", got, exp))
        elif list(out.gpr) != w["gpr"] or out.rflags != w["rflags"]:
            bad.append((i, "regs"))
        elif list(out.xmm) != w["xmm"] or out.mxcsr != w["mxcsr"]:
            bad.append((i, "xmm"))
        elif list(out.ymmh) != w["ymmh"]:
            bad.append((i, "ymm"))
        elif out.nbytes != w["bytes"]:
            bad.append((i, "bytes", out.nbytes, w["bytes"]))
        elif {out.dirty[k] for k in range(min(out.ovn, 64))} != w["dirty"]:
            bad.append((i, "dirty"))
    sse_ran = sum(1 for i, w in enumerate(want) if w["xmm"] != xmm[i])
    assert sse_ran > n // 4, sse_ran
    assert not bad, f"{len(bad)}/{n} lanes differ; first: {bad[:4]}"
