"""XSAVE / XSAVEC with the AVX-512 state, byte for byte against native
execution (convention U47; tests/golden/gen_xsave512_vectors.py).

Each native image is the buffer (pre-filled with 0xa5) after one of xsave /
xsave64 / xsavec / xsavec64 with a requested-feature bitmap under
XCR0 = 0xe7 (x87, SSE, AVX, opmask, ZMM_Hi256, Hi16_ZMM), every component in
use: the engine's device code built for the host and the oracle must write
exactly the same bytes (the untouched ones included: a standard-form XSAVE
changes only the RFBM bits of XSTATE_BV and leaves the legacy area's x87
fields alone when RFBM[0] = 0, and XSAVEC writes MXCSR only with RFBM[1]).
XRSTOR of each full image (its header's untouched bytes cleared) restores
the state it came from.
"""
import ctypes as C
import json
import os
import struct

import pytest

from tests.cpu_bins import SIMLANE_SO, ensure
from tests.oracle_lib import Oracle
from tests.test_avx512 import get_zmm, set_zmm
from tests.test_sse import SimResult
from wtf_amd.abi import Regs, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "xsave512_vectors.json")) as _f:
    DOC = json.load(_f)
CODE_VA = 0x140001000
BUF_VA = 0x7FF000200000
SPAN = DOC["span"]


def state_regs(regs, s):
    set_zmm(regs, [int(v, 16) for v in s["zmm"]])
    for i in range(8):
        regs.k[i] = int(s["k"][i], 16)
        regs.fpst[i] = int(s["st"][i][0], 16)
        regs.fpse[i] = s["st"][i][1]
    regs.fpcw, regs.fpsw, regs.fptw, regs.fpop = s["fcw"], s["fsw"], s["ftw_full"], 0
    regs.mxcsr, regs.mxcsr_mask = s["mxcsr"], DOC["mxcsr_mask"]
    regs.xcr0 = 0xE7
    return regs


def space(code, buf=None):
    sp = AddressSpace()
    sp.map_range(CODE_VA, bytes(code) + b"\xcc", write=False)
    data = buf if buf is not None else b"\xa5" * SPAN
    sp.map_range(BUF_VA, data + b"\xa5" * (4096 - len(data) % 4096))
    return sp


def run_oracle(sp, regs):
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.step()
    return ex, o.regs(), o.read_virt(BUF_VA, SPAN)


def run_sim(sp, regs):
    L = C.CDLL(ensure(SIMLANE_SO, os.path.join(HERE, "native")))
    L.sim_run_full.argtypes = [C.POINTER(C.c_uint64), C.c_char_p, C.c_uint64, C.POINTER(Regs), C.c_uint64,
                               C.POINTER(SimResult), C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(Regs),
                               C.c_char_p]
    pfns, blob = sp.phys()
    arr = (C.c_uint64 * len(pfns))(*pfns)
    out, fin, cnt = SimResult(), Regs(), C.c_uint64(0)
    pages = C.create_string_buffer(64 * 4096)
    L.sim_run_full(arr, blob, len(pfns), C.byref(regs), 1, C.byref(out), 0, C.byref(cnt), 0, C.byref(fin), pages)
    dirty = {int(out.dirty[k]): pages.raw[k * 4096:(k + 1) * 4096] for k in range(min(out.ovn, 64))}
    mem = bytearray()
    for off in range(0, SPAN, 4096):
        pa = sp.translate(BUF_VA + off) & ~0xFFF
        page = dirty.get(pa)
        if page is None:
            pfns_list = list(pfns)
            page = blob[pfns_list.index(pa >> 12) * 4096:][:4096]
        mem += page
    return out, fin, bytes(mem[:SPAN])


def _case_regs(sp, c):
    regs = regs_from_state(user_state(CODE_VA, 0, sp.cr3))
    state_regs(regs, DOC["states"][c["state"]])
    regs.gpr[7] = BUF_VA + DOC["area"]
    regs.gpr[0], regs.gpr[2] = c["rfbm"], 0
    return regs


@pytest.mark.parametrize("engine", ["oracle", "sim"])
def test_xsave_images_match_native(engine):
    fails = []
    for c in DOC["cases"]:
        sp = space(bytes.fromhex(c["code"]))
        regs = _case_regs(sp, c)
        if engine == "oracle":
            ex, _, mem = run_oracle(sp, regs)
            status = ex.status
        else:
            out, _, mem = run_sim(sp, regs)
            status = out.status
        want = bytes.fromhex(c["buf"])
        if mem != want:
            bad = [i - DOC["area"] for i in range(SPAN) if mem[i] != want[i]]
            fails.append((c["insn"], hex(c["rfbm"]), c["state"], status, len(bad), bad[:8]))
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} images differ (image offsets): {fails[:6]}"


@pytest.mark.parametrize("engine", ["oracle", "sim"])
def test_xrstor_of_native_images_restores_the_state(engine):
    """xrstor [rdi] (EDX:EAX = 0xe7) of each full native image (standard and
    compacted) from a zeroed state gives back zmm0-31, k0-7, the x87 registers
    and MXCSR the image was made from."""
    n = 0
    for c in DOC["cases"]:
        if c["rfbm"] != 0xE7 or c["insn"] not in ("xsave64", "xsavec64"):
            continue
        s = DOC["states"][c["state"]]
        buf = bytearray.fromhex(c["buf"])
        h = DOC["area"] + 512  # the header's untouched 0xa5 bytes would be #GP: XSTATE_BV & XCR0, the rest zero
        keep = 16 if c["insn"] == "xsavec64" else 8
        buf[h:h + 8] = (int.from_bytes(buf[h:h + 8], "little") & 0xE7).to_bytes(8, "little")
        buf[h + keep:h + 64] = bytes(64 - keep)
        sp = space(bytes([0x48, 0x0F, 0xAE, 0x2F]), bytes(buf))  # xrstor64 [rdi]
        regs = regs_from_state(user_state(CODE_VA, 0, sp.cr3))
        regs.xcr0, regs.mxcsr_mask = 0xE7, DOC["mxcsr_mask"]
        regs.gpr[7], regs.gpr[0], regs.gpr[2] = BUF_VA + DOC["area"], 0xE7, 0
        fin = run_oracle(sp, regs)[1] if engine == "oracle" else run_sim(sp, regs)[1]
        assert get_zmm(fin) == [int(v, 16) for v in s["zmm"]], c["insn"]
        assert list(fin.k) == [int(v, 16) for v in s["k"]], c["insn"]
        assert [(fin.fpst[i], fin.fpse[i]) for i in range(8)] == [(int(a, 16), b) for a, b in s["st"]]
        assert (fin.fpcw, fin.fpsw, fin.mxcsr) == (s["fcw"], s["fsw"], s["mxcsr"])
        assert (fin.fptw == 0xFFFF) == (s["ftw_full"] == 0xFFFF)
        n += 1
    assert n == 4


def test_xsave_vector_file_covers_the_forms():
    insns = {c["insn"] for c in DOC["cases"]}
    assert insns == {"xsave", "xsave64", "xsavec", "xsavec64"}
    hdr = {c["insn"]: struct.unpack_from("<QQ", bytes.fromhex(c["buf"]), DOC["area"] + 512)
           for c in DOC["cases"] if c["rfbm"] == 0xE7 and c["state"] == 0}
    assert hdr["xsavec"] == (0xE7, 0x80000000000000E7)
    assert hdr["xsave"][0] & 0xFF == 0xE7
