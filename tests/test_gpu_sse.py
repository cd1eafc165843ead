"""GPU engine on the SSE / SSE2 subset and MMX (U37).

1. Every native SSE vector (tests/golden/sse_vectors.json.gz) as one lane:
   GPRs, RFLAGS, all 16 XMM registers, MXCSR and the memory window; every
   native MMX vector (mmx_vectors.json.gz) likewise, with mm0-7, FSW and the
   tags.
2. The fault / encoding cases of tests/test_sse.py, GPU vs oracle.
3. Random programs mixing SSE and integer forms, GPU vs oracle lane by lane
   (exit, registers, XMM, coverage, dirty pages, bytes, memory).
"""
import gzip
import json
import os

import numpy as np
import pytest

from tests import progfuzz
from tests.golden.gen_sse_vectors import window_in
from tests.oracle_lib import Oracle
from tests.test_sse import BUF, SSE_FAULT_CASES, layout
from wtf_amd.abi import EXIT_INT3, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

HERE = os.path.dirname(os.path.abspath(__file__))
CODE_VA = 0x140000000

pytestmark = pytest.mark.gpu


def set_xmm(r, xs):
    for k in range(16):
        r.xmm[k][0], r.xmm[k][1] = xs[2 * k], xs[2 * k + 1]


def get_xmm(r):
    return [r.xmm[k][h] for k in range(16) for h in range(2)]


def test_gpu_matches_native_sse_vectors():
    from wtf_amd.engine import Engine

    with gzip.open(os.path.join(HERE, "golden", "sse_vectors.json.gz"), "rt") as f:
        doc = json.load(f)
    cases = doc["cases"]
    codes = sorted({c["code"] for c in cases})
    slot = {c: i for i, c in enumerate(codes)}
    blob = bytearray(32 * len(codes))
    for c, i in slot.items():
        b = bytes.fromhex(c) + b"\xcc"
        blob[32 * i: 32 * i + len(b)] = b
    sp = AddressSpace()
    sp.map_range(CODE_VA, bytes(blob), write=False)
    buf_va = int(doc["buf_va"], 16)
    page_va = buf_va & ~0xFFF
    sp.map(page_va, b"", nx=True)
    sp.map(page_va + 0x1000, b"", nx=True)
    n = (len(cases) + 63) // 64 * 64
    eng = Engine(0)
    pfns, pblob = sp.phys()
    eng.load_pool(pfns, pblob)
    eng.alloc_lanes(n, overlay_pages=4, cov_entries=64)
    base = regs_from_state(user_state(CODE_VA, 0, sp.cr3))
    eng.set_initial_state(base)
    eng.set_limit(0)
    eng.restore()
    regs = eng.read_regs(0, n)
    writes = []
    for i, c in enumerate(cases):
        r = regs[i]
        for k in range(16):
            r.gpr[k] = int(c["in"][k], 16)
        r.rip = CODE_VA + 32 * slot[c["code"]]
        r.rflags = int(c["fl"], 16) | 0x200
        set_xmm(r, [int(v, 16) for v in c["xin"]])
        r.mxcsr = int(c["mx"], 16)
        writes.append((i, buf_va, window_in(int(c["seed"], 16), c["ldmx"])))
    for i in range(len(cases), n):  # padding lanes run a lone int3
        regs[i].rip = CODE_VA + 32 * slot[cases[0]["code"]] + len(bytes.fromhex(cases[0]["code"]))
    eng.write_regs(regs)
    eng.apply_writes(writes)
    eng.run()
    ex = eng.exits()
    out = eng.read_regs(0, n)
    fails = []
    for i, c in enumerate(cases):
        r = out[i]
        if ex[i].status != EXIT_INT3 or ex[i].icount != 1:
            fails.append((c["name"], c["code"], "exit", ex[i].status, ex[i].vector))
            continue
        if [r.gpr[k] for k in range(16)] != [int(v, 16) for v in c["out"]]:
            fails.append((c["name"], c["code"], "gpr"))
            continue
        if (r.rflags ^ int(c["flo"], 16)) & 0x8D5:
            fails.append((c["name"], c["code"], "flags"))
            continue
        if get_xmm(r) != [int(v, 16) for v in c["xout"]] or r.mxcsr != int(c["mxo"], 16):
            fails.append((c["name"], c["code"], "xmm"))
            continue
        win = bytearray(window_in(int(c["seed"], 16), c["ldmx"]))
        for k, v in c["diff"]:
            win[k] = v
        if (c["diff"] or i % 5 == 0) and eng.read_virt(i, buf_va, 256) != bytes(win):
            fails.append((c["name"], c["code"], "mem"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def test_gpu_matches_native_mmx_vectors():
    from tests.golden.gen_native_vectors import splitmix_bytes
    from tests.test_mmx import DOC, abridged
    from wtf_amd.engine import Engine

    cases = DOC["cases"]
    codes = sorted({c["code"] for c in cases})
    slot = {c: i for i, c in enumerate(codes)}
    blob = bytearray(32 * len(codes))
    for c, i in slot.items():
        b = bytes.fromhex(c) + b"\xcc"
        blob[32 * i: 32 * i + len(b)] = b
    sp = AddressSpace()
    sp.map_range(CODE_VA, bytes(blob), write=False)
    buf_va = int(DOC["buf_va"], 16)
    page_va = buf_va & ~0xFFF
    sp.map(page_va, b"", nx=True)
    sp.map(page_va + 0x1000, b"", nx=True)
    n = (len(cases) + 63) // 64 * 64
    eng = Engine(0)
    pfns, pblob = sp.phys()
    eng.load_pool(pfns, pblob)
    eng.alloc_lanes(n, overlay_pages=4, cov_entries=64)
    eng.set_initial_state(regs_from_state(user_state(CODE_VA, 0, sp.cr3)))
    eng.set_limit(0)
    eng.restore()
    regs = eng.read_regs(0, n)
    writes = []
    for i, c in enumerate(cases):
        r = regs[i]
        for k in range(16):
            r.gpr[k] = int(c["in"][k], 16)
        r.rip = CODE_VA + 32 * slot[c["code"]]
        r.rflags = int(c["fl"], 16) | 0x200
        set_xmm(r, [int(v, 16) for v in c["xin"]])
        for k in range(8):
            r.fpst[k] = int(c["mmin"][k], 16)
        r.fpsw, r.fptw = 0, 0
        writes.append((i, buf_va, splitmix_bytes(int(c["seed"], 16), 256)))
    for i in range(len(cases), n):  # padding lanes run a lone int3
        regs[i].rip = CODE_VA + 32 * slot[cases[0]["code"]] + len(bytes.fromhex(cases[0]["code"]))
    eng.write_regs(regs)
    eng.apply_writes(writes)
    eng.run()
    ex = eng.exits()
    out = eng.read_regs(0, n)
    fails = []
    for i, c in enumerate(cases):
        r = out[i]
        if ex[i].status != EXIT_INT3 or ex[i].icount != 1:
            fails.append((c["name"], c["code"], "exit", ex[i].status, ex[i].vector))
        elif [r.gpr[k] for k in range(16)] != [int(v, 16) for v in c["out"]] or (r.rflags ^ int(c["flo"], 16)) & 0x8D5:
            fails.append((c["name"], c["code"], "gpr"))
        elif get_xmm(r) != [int(v, 16) for v in c["xout"]]:
            fails.append((c["name"], c["code"], "xmm"))
        elif [r.fpst[k] for k in range(8)] != [int(v, 16) for v in c["mmout"]]:
            fails.append((c["name"], c["code"], "mm"))
        elif r.fpsw != int(c["fsw"], 16) or abridged(r.fptw) != int(c["ftw"], 16):
            fails.append((c["name"], c["code"], "x87"))
        else:
            win = bytearray(splitmix_bytes(int(c["seed"], 16), 256))
            for k, v in c["diff"]:
                win[k] = v
            if c["diff"] and eng.read_virt(i, buf_va, 256) != bytes(win):
                fails.append((c["name"], c["code"], "mem"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def test_gpu_sse_faults_match_oracle():
    """Misaligned operands, register-only / memory-only forms, MMX / FP /
    SSE3 encodings and CR0 / CR4 gating: GPU exits equal the oracle's."""
    from wtf_amd.engine import Engine

    variants = [(code, None, None) for code, _, _ in SSE_FAULT_CASES]
    pxor = [0x66, 0x0F, 0xEF, 0xC1]
    variants += [(pxor, None, 0x370678 & ~0x200), (pxor, 0x80050031 | 4, None), (pxor, 0x80050031 | 8, None),
                 ([0x0F, 0xAE, 0xF0], 0x80050031 | 8, None)]
    for code, cr0, cr4 in variants:
        sp, regs = layout(bytes(code), BUF, bytes(range(256)), cr0=cr0, cr4=cr4)
        regs.gpr[3] = BUF + 0x10
        regs.gpr[6] = BUF + 0x13
        pfns, blob = sp.phys()
        o = Oracle(pfns=pfns, blob=blob)
        o.restore(regs)
        want = o.run()
        eng = Engine(0)
        eng.load_pool(pfns, blob)
        eng.alloc_lanes(64, overlay_pages=4, cov_entries=64)
        eng.set_initial_state(regs)
        eng.set_limit(0)
        eng.restore()
        eng.run()
        e = eng.exits(0, 1)[0]
        got = (e.status, e.vector if e.status == 5 else 0, e.rip, e.icount)
        exp = (want.status, want.vector if want.status == 5 else 0, want.rip, want.icount)
        assert got == exp, (bytes(code).hex(), cr0, cr4, got, exp)
        eng.close()


@pytest.mark.parametrize("seed,fp", [(21, False), (22, False), (23, True), (24, True)])
def test_gpu_matches_oracle_on_random_sse_programs(seed, fp):
    """fp: with the floating-point and SSE4 / AVX2 forms and a random MXCSR per lane."""
    from wtf_amd.engine import Engine

    n = 512
    sp, st, lanes = progfuzz.build(n, seed=seed, sse=True, fp=fp)
    xmm = progfuzz.lane_xmm(n, seed)
    ymmh = progfuzz.lane_xmm(n, seed, 0x4E4)
    mx = progfuzz.lane_mxcsr(n, seed) if fp else None
    want = progfuzz.oracle_run(sp, st, lanes, xmm=xmm, ymmh=ymmh, mxcsr=mx)
    eng = Engine(0)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(n, overlay_pages=8, cov_entries=4096)
    eng.set_initial_state(regs_from_state(st))
    eng.set_limit(20000)
    eng.restore()
    regs = eng.read_regs(0, n)
    for i, (va, g, flags) in enumerate(lanes):
        for k in range(16):
            regs[i].gpr[k] = g[k]
        regs[i].rip = va
        regs[i].rflags = flags
        set_xmm(regs[i], xmm[i])
        for k in range(16):
            regs[i].ymmh[k][0], regs[i].ymmh[k][1] = ymmh[i][2 * k], ymmh[i][2 * k + 1]
        if mx is not None:
            regs[i].mxcsr = mx[i]
    eng.write_regs(regs)
    stats = eng.run()
    ex = eng.exits()
    out = eng.read_regs(0, n)
    cov, ovf = eng.coverage()
    nb = eng.nbytes()
    bad = []
    for i, w in enumerate(want):
        e, r = ex[i], out[i]
        got = (e.status, e.vector if e.status == 5 else 0, e.addr if e.status == 5 else 0, r.rip, e.icount)
        exp = (w["status"], w["vector"] if w["status"] == 5 else 0, w["addr"] if w["status"] == 5 else 0,
               w["rip"], w["icount"])
        if got != exp:
            bad.append((i, "exit", got, exp))
        elif [r.gpr[k] for k in range(16)] != w["gpr"] or r.rflags != w["rflags"]:
            bad.append((i, "regs"))
        elif get_xmm(r) != w["xmm"] or r.mxcsr != w["mxcsr"]:
            bad.append((i, "xmm"))
        elif [r.ymmh[k][h] for k in range(16) for h in range(2)] != w["ymmh"]:
            bad.append((i, "ymm"))
        elif cov.get(i, set()) != w["cov"]:
            bad.append((i, "cov"))
        elif set(eng.dirty(i)) != w["dirty"]:
            bad.append((i, "dirty"))
        elif int(nb[i]) != w["bytes"]:
            bad.append((i, "bytes", int(nb[i]), w["bytes"]))
        elif i % 8 == 0 and (eng.read_virt(i, progfuzz.WIN_VA, 0x2000) != w["win"] or
                             eng.read_virt(i, progfuzz.STACK_VA, 0x2000) != w["stack"]):
            bad.append((i, "memory"))
    assert not ovf
    assert stats.lane_retired == sum(w["icount"] for w in want)
    statuses = np.bincount([w["status"] for w in want], minlength=13)
    assert statuses[EXIT_INT3] > n // 8, statuses  # most programs run to the end
    assert not bad, f"{len(bad)}/{n} lanes differ; first: {bad[:4]}"


def test_gpu_matches_native_avx_vectors():
    """Every AVX / AVX2 vector (tests/golden/avx_vectors.json.gz) as one lane:
    GPRs, RFLAGS, all 16 YMM registers and the memory window."""
    from tests.test_avx import DOC, get_ymm, set_ymm, window
    from wtf_amd.engine import Engine

    cases = DOC["cases"]
    codes = sorted({c["code"] for c in cases})
    slot = {c: i for i, c in enumerate(codes)}
    blob = bytearray(32 * len(codes))
    for c, i in slot.items():
        b = bytes.fromhex(c) + b"\xcc"
        blob[32 * i: 32 * i + len(b)] = b
    sp = AddressSpace()
    sp.map_range(CODE_VA, bytes(blob), write=False)
    buf_va = int(DOC["buf_va"], 16)
    sp.map(buf_va & ~0xFFF, b"", nx=True)
    sp.map((buf_va & ~0xFFF) + 0x1000, b"", nx=True)
    n = (len(cases) + 63) // 64 * 64
    eng = Engine(0)
    pfns, pblob = sp.phys()
    eng.load_pool(pfns, pblob)
    eng.alloc_lanes(n, overlay_pages=4, cov_entries=64)
    eng.set_initial_state(regs_from_state(user_state(CODE_VA, 0, sp.cr3)))
    eng.set_limit(0)
    eng.restore()
    regs = eng.read_regs(0, n)
    writes = []
    for i, c in enumerate(cases):
        r = regs[i]
        for k in range(16):
            r.gpr[k] = int(c["in"][k], 16)
        r.rip = CODE_VA + 32 * slot[c["code"]]
        r.rflags = int(c["fl"], 16) | 0x200
        set_ymm(r, [int(v, 16) for v in c["yin"]])
        writes.append((i, buf_va, window(c)))
    for i in range(len(cases), n):
        regs[i].rip = CODE_VA + 32 * slot[cases[0]["code"]] + len(bytes.fromhex(cases[0]["code"]))
    eng.write_regs(regs)
    eng.apply_writes(writes)
    eng.run()
    ex = eng.exits()
    out = eng.read_regs(0, n)
    fails = []
    for i, c in enumerate(cases):
        r = out[i]
        if ex[i].status != EXIT_INT3 or ex[i].icount != 1:
            fails.append((c["name"], c["code"], "exit", ex[i].status, ex[i].vector))
        elif [r.gpr[k] for k in range(16)] != [int(v, 16) for v in c["out"]] or \
                (r.rflags ^ int(c["flo"], 16)) & 0x8D5:
            fails.append((c["name"], c["code"], "regs"))
        elif get_ymm([r.xmm[k][h] for k in range(16) for h in range(2)],
                     [r.ymmh[k][h] for k in range(16) for h in range(2)]) != [int(v, 16) for v in c["yout"]]:
            fails.append((c["name"], c["code"], "ymm"))
        else:
            win = bytearray(window(c))
            for k, v in c["diff"]:
                win[k] = v
            if (c["diff"] or i % 5 == 0) and eng.read_virt(i, buf_va, 256) != bytes(win):
                fails.append((c["name"], c["code"], "mem"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def _run_vector_doc(DOC, inputs, mem=False):
    """Every case of a native-vector document (gen_fp_vectors.run_native's
    format) as one lane: GPRs, RFLAGS, all 16 YMM registers, MXCSR, the window
    (mem), and for the unmasked-exception cases the #XM exit with the trap's MXCSR."""
    from tests.test_avx import get_ymm, set_ymm
    from tests.test_fp import VEC_XM, expected
    from wtf_amd.abi import EXIT_FAULT
    from wtf_amd.engine import Engine

    cases = DOC["cases"]
    codes = sorted({c["code"] for c in cases})
    slot = {c: i for i, c in enumerate(codes)}
    blob = bytearray(32 * len(codes))
    for c, i in slot.items():
        b = bytes.fromhex(c) + b"\xcc"
        blob[32 * i: 32 * i + len(b)] = b
    sp = AddressSpace()
    sp.map_range(CODE_VA, bytes(blob), write=False)
    buf_va = int(DOC["buf_va"], 16)
    sp.map(buf_va & ~0xFFF, b"", nx=True)
    sp.map((buf_va & ~0xFFF) + 0x1000, b"", nx=True)
    n = (len(cases) + 63) // 64 * 64
    eng = Engine(0)
    pfns, pblob = sp.phys()
    eng.load_pool(pfns, pblob)
    eng.alloc_lanes(n, overlay_pages=4, cov_entries=64)
    eng.set_initial_state(regs_from_state(user_state(CODE_VA, 0, sp.cr3)))
    eng.set_limit(0)
    eng.restore()
    regs = eng.read_regs(0, n)
    writes, ins, wins = [], [], []
    for i, c in enumerate(cases):
        yin, win = inputs(c)
        ins.append(yin)
        wins.append(win)
        r = regs[i]
        for k in range(16):
            r.gpr[k] = int(c["in"][k], 16)
        r.rip = CODE_VA + 32 * slot[c["code"]]
        r.rflags = int(c["fl"], 16) | 0x200
        r.mxcsr = int(c["mx"], 16)
        set_ymm(r, yin)
        writes.append((i, buf_va, win))
    for i in range(len(cases), n):
        regs[i].rip = CODE_VA + 32 * slot[cases[0]["code"]] + len(bytes.fromhex(cases[0]["code"]))
    eng.write_regs(regs)
    eng.apply_writes(writes)
    eng.run()
    ex = eng.exits()
    out = eng.read_regs(0, n)
    fails = []
    for i, c in enumerate(cases):
        r = out[i]
        if "trap_mx" in c:
            if ex[i].status != EXIT_FAULT or ex[i].vector != VEC_XM or r.mxcsr != int(c["trap_mx"], 16):
                fails.append((c["name"], c["code"], "trap", ex[i].status, ex[i].vector, hex(r.mxcsr)))
            continue
        g, y = expected(c, ins[i])
        if ex[i].status != EXIT_INT3 or ex[i].icount != 1:
            fails.append((c["name"], c["code"], "exit", ex[i].status, ex[i].vector))
        elif [r.gpr[k] for k in range(16)] != g or (r.rflags ^ int(c["flo"], 16)) & int(c.get("flm", "8d5"), 16):
            fails.append((c["name"], c["code"], "regs"))
        elif get_ymm([r.xmm[k][h] for k in range(16) for h in range(2)],
                     [r.ymmh[k][h] for k in range(16) for h in range(2)]) != y:
            fails.append((c["name"], c["code"], "ymm"))
        elif r.mxcsr != int(c["mxo"], 16):
            fails.append((c["name"], c["code"], "mxcsr", hex(r.mxcsr), c["mxo"]))
        elif mem and c.get("mdiff"):
            w = bytearray(wins[i])
            for k, v in c["mdiff"]:
                w[k] = v
            if eng.read_virt(i, buf_va, 256) != bytes(w):
                fails.append((c["name"], c["code"], "mem"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def test_gpu_matches_native_fp_vectors():
    """SSE / AVX floating point (tests/golden/fp_vectors.json.gz, U39 / U40)."""
    from tests.test_fp import DOC, inputs
    _run_vector_doc(DOC, inputs)


def test_gpu_matches_native_sse4_vectors():
    """SSSE3 / SSE4.1 integer and AVX2 lane-crossing forms (tests/golden/sse4_vectors.json.gz, U41)."""
    from tests.test_sse4 import DOC, inputs
    _run_vector_doc(DOC, inputs, mem=True)


def test_gpu_matches_x87_vectors():
    """x87 arithmetic (tests/golden/x87_vectors.json.gz, U42): every case one
    lane; its x87 state, status flags and 16-byte memory operand in, the
    host CPU's answer out (registers, sign / exponent words, FCW / FSW / tags,
    RFLAGS, the operand bytes, #MF / #UD / stack-fault outcomes)."""
    from tests.golden.gen_x87_vectors import case_regs
    from tests.test_x87 import DOC
    from wtf_amd.abi import EXIT_FAULT
    from wtf_amd.engine import Engine

    cases = DOC["cases"]
    codes = sorted({c["code"] for c in cases})
    slot = {c: i for i, c in enumerate(codes)}
    blob = bytearray(32 * len(codes))
    for c, i in slot.items():
        b = bytes.fromhex(c) + b"\xcc"
        blob[32 * i: 32 * i + len(b)] = b
    sp = AddressSpace()
    sp.map_range(CODE_VA, bytes(blob), write=False)
    buf_va = int(DOC["buf_va"], 16)
    sp.map(buf_va & ~0xFFF, b"", nx=True)
    sp.map((buf_va & ~0xFFF) + 0x1000, b"", nx=True)
    n = (len(cases) + 63) // 64 * 64
    eng = Engine(0)
    pfns, pblob = sp.phys()
    eng.load_pool(pfns, pblob)
    eng.alloc_lanes(n, overlay_pages=4, cov_entries=64)
    eng.set_initial_state(regs_from_state(user_state(CODE_VA, 0, sp.cr3)))
    eng.set_limit(0)
    eng.restore()
    regs = eng.read_regs(0, n)
    writes = []
    for i, c in enumerate(cases):
        r = regs[i]
        case_regs(c, r)
        r.gpr[6] = buf_va
        r.rip = CODE_VA + 32 * slot[c["code"]]
        writes.append((i, buf_va, bytes.fromhex(c["mem"])))
    for i in range(len(cases), n):
        regs[i].rip = CODE_VA + 32 * slot[cases[0]["code"]] + len(bytes.fromhex(cases[0]["code"]))
    eng.write_regs(regs)
    eng.apply_writes(writes)
    eng.run()
    ex = eng.exits()
    out = eng.read_regs(0, n)
    fails = []
    for i, c in enumerate(cases):
        w, r = c["out"], out[i]
        if w["status"] == EXIT_FAULT:
            if ex[i].status != EXIT_FAULT or ex[i].vector != w["vector"]:
                fails.append((c["code"], "fault", ex[i].status, ex[i].vector))
            continue
        if ex[i].status != EXIT_INT3 or ex[i].icount != 1:
            fails.append((c["code"], "exit", ex[i].status, ex[i].vector))
        elif (r.fpcw, r.fpsw, r.fptw, r.rflags & 0x8D5) != (w["fcw"], w["fsw"], w["ftw"], w["fl"]):
            fails.append((c["code"], "status", hex(r.fpsw), hex(w["fsw"])))
        elif [(r.fpst[k], r.fpse[k]) for k in range(8)] != [tuple(x) for x in w["st"]]:
            fails.append((c["code"], "st"))
        elif eng.read_virt(i, buf_va, 16).hex() != w["mem"]:
            fails.append((c["code"], "mem"))
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:6]}"


def test_gpu_matches_native_ext_vectors():
    """BMI1 / BMI2 / ADX / MOVBE / CRC32, SSE4.2, AES, PCLMULQDQ (tests/golden/ext_vectors.json.gz, U45)."""
    from tests.test_ext import DOC, inputs
    _run_vector_doc(DOC, inputs, mem=True)


def test_gpu_matches_native_avx2x_vectors():
    """FMA3, F16C and the AVX2 gathers (tests/golden/avx2x_vectors.json.gz, U46)."""
    from tests.test_avx2x import DOC, inputs
    _run_vector_doc(DOC, inputs, mem=True)


def test_gpu_matches_native_avx512_vectors():
    """The AVX-512 subset and the opmask instructions (tests/golden/avx512_vectors.json.gz, U47):
    every case one lane with GPRs, RFLAGS, zmm0-31, k0-7 and the 512-byte window
    across a page boundary; the guard cases (one of the two pages absent) in
    their own address spaces, with the #PF error code and CR2 of the faults
    (memory fault suppression)."""
    from tests.test_avx512 import BOUND, DOC, WIN, XCR0, address_space, case_regs, check, get_zmm, inputs
    from tests.test_avx512 import CODE_VA as CVA
    from wtf_amd.abi import EXIT_FAULT
    from wtf_amd.engine import Engine

    buf_va = int(DOC["buf_va"], 16)
    fails = []
    total = 0
    for guard in (0, 1, 2):
        cases = [c for c in DOC["cases"] if c["guard"] == guard]
        total += len(cases)
        codes = sorted({c["code"] for c in cases})
        slot = {c: i for i, c in enumerate(codes)}
        blob = bytearray(32 * len(codes))
        for c, i in slot.items():
            b = bytes.fromhex(c) + b"\xcc"
            blob[32 * i: 32 * i + len(b)] = b
        sp = address_space(bytes(blob), buf_va, bytes(WIN), guard)
        n = (len(cases) + 63) // 64 * 64
        eng = Engine(0)
        pfns, pblob = sp.phys()
        eng.load_pool(pfns, pblob)
        eng.alloc_lanes(n, overlay_pages=4, cov_entries=64)
        init = regs_from_state(user_state(CVA, 0, sp.cr3))
        init.xcr0 = XCR0
        eng.set_initial_state(init)
        eng.set_limit(0)
        eng.restore()
        regs = eng.read_regs(0, n)
        writes, ins, wins = [], [], []
        for i, c in enumerate(cases):
            zin, win = inputs(c)
            ins.append(zin)
            wins.append(win)
            r = case_regs(c, regs[i], zin)
            r.rip = CVA + 32 * slot[c["code"]]
            if guard != 2:
                writes.append((i, buf_va, win[:BOUND]))
            if guard != 1:
                writes.append((i, buf_va + BOUND, win[BOUND:]))
        for i in range(len(cases), n):
            regs[i].rip = CVA + 32 * slot[cases[0]["code"]] + len(bytes.fromhex(cases[0]["code"]))
        eng.write_regs(regs)
        eng.apply_writes(writes)
        eng.run()
        ex = eng.exits()
        out = eng.read_regs(0, n)
        for i, c in enumerate(cases):
            r, e = out[i], ex[i]
            if "fault" not in c and (e.status != EXIT_INT3 or e.icount != 1):
                fails.append((c["name"], c["code"], "exit", e.status, e.vector))
                continue
            if "fault" in c and e.status != EXIT_FAULT:
                fails.append((c["name"], c["code"], "no fault", e.status))
                continue
            lo = bytes(BOUND) if guard == 2 else eng.read_virt(i, buf_va, BOUND)
            hi = bytes(WIN - BOUND) if guard == 1 else eng.read_virt(i, buf_va + BOUND, WIN - BOUND)
            bad = check(c, e.status, e.vector, e.error, e.addr, list(r.gpr), r.rflags, get_zmm(r), list(r.k),
                        lo + hi, ins[i], wins[i])
            if bad:
                fails.append((c["name"], c["code"]) + bad)
    assert total == len(DOC["cases"])
    assert not fails, f"{len(fails)}/{total} mismatches, first: {fails[:6]}"
