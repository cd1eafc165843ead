"""The AVX-512 subset (convention U47; engine_avx512.h, oracle/x86_oracle_avx512.inc).

Native-execution vectors (tests/golden/gen_avx512_vectors.py, run on an
AVX512F / BW / VL / DQ host) pin the oracle and the engine's device code built
for the host: GPRs, RFLAGS, zmm0-31, k0-7 and a 512-byte window across a page
boundary, and for the faulting cases the vector, the page-fault error code and
CR2 (memory fault suppression: "guard" cases whose second page is absent).
The GPU runs the same vectors in tests/test_gpu_sse.py.
"""
import ctypes as C
import gzip
import json
import os

import pytest

from tests.cpu_bins import SIMLANE_SO, ensure
from tests.golden.gen_avx512_vectors import BOUND, WIN, case_inputs, guard_window
from tests.oracle_lib import Oracle
from tests.test_sse import CODE_VA, SimResult
from wtf_amd.abi import EXIT_FAULT, EXIT_INT3, RUNNING, Regs, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

HERE = os.path.dirname(os.path.abspath(__file__))
XCR0 = 0xE7


def load():
    with gzip.open(os.path.join(HERE, "golden", "avx512_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def set_zmm(r, z):
    """z: 256 u64 (zmm0-31, 8 each) into the state's xmm / ymmh / zmmh / zmm_hi."""
    for i in range(32):
        q = z[8 * i: 8 * i + 8]
        if i < 16:
            r.xmm[i][0], r.xmm[i][1] = q[0], q[1]
            r.ymmh[i][0], r.ymmh[i][1] = q[2], q[3]
            for j in range(4):
                r.zmmh[i][j] = q[4 + j]
        else:
            for j in range(8):
                r.zmm_hi[i - 16][j] = q[j]


def get_zmm(r):
    out = []
    for i in range(32):
        if i < 16:
            out += [r.xmm[i][0], r.xmm[i][1], r.ymmh[i][0], r.ymmh[i][1]] + [r.zmmh[i][j] for j in range(4)]
        else:
            out += [r.zmm_hi[i - 16][j] for j in range(8)]
    return out


def window_in(c):
    _, win = case_inputs(int(c["seed"], 16))
    return guard_window(win, c["guard"])


def inputs(c):
    zmm, _ = case_inputs(int(c["seed"], 16))
    return [v for r in zmm for v in r], window_in(c)


def case_regs(c, regs, zin):
    for i in range(16):
        regs.gpr[i] = int(c["in"][i], 16)
    regs.rflags = int(c["fl"], 16) | 0x200
    set_zmm(regs, zin)
    for i in range(8):
        regs.k[i] = int(c["k"][i], 16)
    regs.xcr0 = XCR0
    return regs


def address_space(code_blob, buf_va, win, guard):
    """Code at CODE_VA; the window's first 256 bytes end one page, the rest start
    the next (guard 1: the second page absent; guard 2: the first)."""
    sp = AddressSpace()
    sp.map_range(CODE_VA, code_blob, write=False)
    page = buf_va & ~0xFFF
    off = buf_va - page
    assert off + BOUND == 0x1000
    first = bytearray(4096)
    first[off:] = win[:BOUND]
    if guard != 2:
        sp.map(page, bytes(first))
    if guard != 1:
        sp.map(page + 0x1000, bytes(win[BOUND:]) + bytes(4096 - (WIN - BOUND)))
    return sp


def expected(c, zin, win):
    """(gprs, zmm, k, window) after the case (no fault)."""
    g = [int(v, 16) for v in c["in"]]
    for i, v in c["gdiff"]:
        g[i] = int(v, 16)
    z = list(zin)
    for i, v in c["zdiff"]:
        z[i] = int(v, 16)
    w = bytearray(win)
    for i, v in c["mdiff"]:
        w[i] = v
    return g, z, [int(v, 16) for v in c["ko"]], bytes(w)


def check(c, status, vector, error, addr, gpr, rflags, zmm, k, mem, zin, win):
    """Mismatch description, or None. status: the exit after one instruction
    (RUNNING / INT3 for a clean step)."""
    if "fault" in c:
        f = c["fault"]
        if status != EXIT_FAULT or vector != f["vec"]:
            return ("fault", status, vector, f)
        if f["vec"] == 14 and (error != f["err"] or addr != int(f["addr"], 16)):
            return ("pf", hex(error), hex(addr), f)
        if list(zmm) != list(zin) or mem != win:
            return ("fault state",)
        return None
    if status not in (RUNNING, EXIT_INT3):
        return ("exit", status, vector)
    g, z, ko, w = expected(c, zin, win)
    if list(gpr) != g:
        return ("gpr", [(i, hex(gpr[i]), hex(g[i])) for i in range(16) if gpr[i] != g[i]])
    if (rflags ^ int(c["flo"], 16)) & 0x8D5:
        return ("flags", hex(rflags), c["flo"])
    if list(zmm) != z:
        return ("zmm", [(i // 8, i % 8, hex(zmm[i]), hex(z[i])) for i in range(256) if zmm[i] != z[i]][:4])
    if list(k) != ko:
        return ("k", [hex(x) for x in k], c["ko"])
    if mem != w:
        return ("mem", [(i, mem[i], w[i]) for i in range(WIN) if mem[i] != w[i]][:6])
    return None


def oracle_case(c):
    buf_va = int(DOC["buf_va"], 16)
    zin, win = inputs(c)
    code = bytes.fromhex(c["code"])
    sp = address_space(code + b"\xcc", buf_va, win, c["guard"])
    regs = regs_from_state(user_state(CODE_VA, 0, sp.cr3))
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(case_regs(c, regs, zin))
    ex = o.step()
    r = o.regs()
    g = c["guard"]
    mem = (bytes(BOUND) if g == 2 else o.read_virt(buf_va, BOUND)) + \
        (bytes(WIN - BOUND) if g == 1 else o.read_virt(buf_va + BOUND, WIN - BOUND))
    return check(c, ex.status, ex.vector, ex.error, ex.addr, list(r.gpr), r.rflags, get_zmm(r), list(r.k), mem,
                 zin, win)


@pytest.mark.parametrize("chunk", range(2))
def test_oracle_matches_native_avx512(chunk):
    cases = DOC["cases"][chunk::2]
    fails = []
    for c in cases:
        bad = oracle_case(c)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:5]}"


def sim_full():
    L = C.CDLL(ensure(SIMLANE_SO, os.path.join(HERE, "native")))
    L.sim_run_full.argtypes = [C.POINTER(C.c_uint64), C.c_char_p, C.c_uint64, C.POINTER(Regs), C.c_uint64,
                               C.POINTER(SimResult), C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(Regs),
                               C.c_void_p]
    return L


def sim_case(L, c, fast=False):
    buf_va = int(DOC["buf_va"], 16)
    zin, win = inputs(c)
    sp = address_space(bytes.fromhex(c["code"]) + b"\xcc", buf_va, win, c["guard"])
    regs = case_regs(c, regs_from_state(user_state(CODE_VA, 0, sp.cr3)), zin)
    pfns, blob = sp.phys()
    arr = (C.c_uint64 * len(pfns))(*pfns)
    out, fin, cnt = SimResult(), Regs(), C.c_uint64(0)
    L.sim_run_full(arr, blob, len(pfns), C.byref(regs), 0, C.byref(out), 1 if fast else 0, C.byref(cnt), buf_va,
                   C.byref(fin), None)
    icount_ok = out.icount == (0 if "fault" in c else 1)
    if not icount_ok:
        return ("icount", out.icount, out.status, out.vector)
    mem = bytes(out.win[:WIN])
    return check(c, out.status, out.vector, out.error, out.addr, list(out.gpr), out.rflags, get_zmm(fin),
                 list(fin.k), mem, zin, win)


@pytest.mark.parametrize("fast", [False, True], ids=["exec", "fast"])
def test_engine_avx512_code_matches_native_vectors(fast):
    """The engine's decode / exec built for the host (tests/native/sim_lane.cc);
    fast=True goes through k_run's fast-loop digest first (EVEX stays generic)."""
    L = sim_full()
    fails = []
    for c in DOC["cases"]:
        bad = sim_case(L, c, fast)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:5]}"


def test_avx512_vector_file_is_substantial():
    cases = DOC["cases"]
    names = {c["name"].split(".")[0] for c in cases}
    assert len(cases) > 2500
    for n in ("vmovdqu8", "vmovdqu16", "vmovdqu32", "vmovdqu64", "vmovdqa32", "vmovdqa64", "vmovups", "vmovapd",
              "vpternlogd", "vpternlogq", "vpcmpub", "vpcmpq", "vptestnmb", "vpbroadcastq", "vpminuw", "vpcmpeqb",
              "kmovq", "kortestd", "ktestb", "kshiftlq", "kxnorw", "knotb"):
        assert n in names, n
    # memory fault suppression was exercised both ways: guard cases that fault and that complete
    guard = [c for c in cases if c["guard"]]
    assert sum("fault" in c for c in guard) > 20 and sum("fault" not in c for c in guard) > 20
    # the #UD rules and the aligned forms' #GP were met natively
    assert sum(c.get("fault", {}).get("vec") == 6 for c in cases) > 100
    assert sum(c.get("fault", {}).get("vec") == 13 for c in cases) > 20
    # every vector length and zmm16-31 appear
    assert {c["name"].split(".")[1] for c in cases if c["name"].startswith("vp")} >= {"L0", "L1", "L2"}


def _cpuid(leaf, sub, xcr0=XCR0):
    sp = AddressSpace()
    sp.map_range(CODE_VA, bytes([0x0F, 0xA2, 0xCC]), write=False)
    regs = regs_from_state(user_state(CODE_VA, 0, sp.cr3))
    regs.gpr[0], regs.gpr[1] = leaf, sub
    regs.xcr0 = xcr0
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    o.step()
    return list(o.regs().gpr)


def test_avx512_disabled_by_xcr0_is_ud():
    """With XCR0[7:5] clear (a guest that never enabled the AVX-512 state) every
    EVEX form and the opmask instructions are #UD, engine and oracle."""
    c = next(c for c in DOC["cases"] if c["name"].startswith("vpaddd") and "fault" not in c)
    k = next(c for c in DOC["cases"] if c["name"].startswith("kandw") and "fault" not in c)
    L = sim_full()
    for case in (c, k):
        for xcr0 in (0x7, 0x1F, 0x67):
            zin, win = inputs(case)
            buf_va = int(DOC["buf_va"], 16)
            sp = address_space(bytes.fromhex(case["code"]) + b"\xcc", buf_va, win, 0)
            regs = case_regs(case, regs_from_state(user_state(CODE_VA, 0, sp.cr3)), zin)
            regs.xcr0 = xcr0
            pfns, blob = sp.phys()
            o = Oracle(pfns=pfns, blob=blob)
            o.restore(regs)
            ex = o.step()
            assert (ex.status, ex.vector) == (EXIT_FAULT, 6), (case["name"], xcr0)
            arr = (C.c_uint64 * len(pfns))(*pfns)
            out, fin, cnt = SimResult(), Regs(), C.c_uint64(0)
            L.sim_run_full(arr, blob, len(pfns), C.byref(regs), 0, C.byref(out), 0, C.byref(cnt), 0, C.byref(fin),
                           None)
            assert (out.status, out.vector) == (EXIT_FAULT, 6), (case["name"], xcr0)


def test_cpuid_enumerates_avx512_f_bw_vl():
    g = _cpuid(7, 0)
    ebx = g[3]
    assert ebx & (1 << 16) and ebx & (1 << 30) and ebx & (1 << 31)
