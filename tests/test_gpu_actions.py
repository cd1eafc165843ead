"""The register-only device actions k_run applies inline (engine.hip: SetGprs
and StopOk without the lane copy, WTFGPU_INLINE_ACTIONS), both kinds met by
the lanes of one launch.

A build once ran them wrong on MI355X (lanes stopping Ok at their SetGprs
breakpoint, DESIGN.md §3 "inline actions"): here every wave holds lanes of
both paths. Odd lanes hit a SetGprs breakpoint that moves them (every GPR and
rip) to code that adds to rax and then hits a StopOk breakpoint; even lanes
hit a StopOk breakpoint directly. Each lane must end STOP_OK at its own
breakpoint with the registers its path gives and the instruction count of
its path."""
import ctypes as C

import numpy as np
import pytest

from wtf_amd import abi
from wtf_amd.abi import EXIT_STOP_OK, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

pytestmark = pytest.mark.gpu

CODE_VA = 0x140000000
B, A, C_, D = CODE_VA + 0x05, CODE_VA + 0x0F, CODE_VA + 0x20, CODE_VA + 0x24
SET = [0x1000 + 0x111 * i for i in range(16)]
BPACT_STOP_OK = 5  # include/wtfgpu.h WTFGPU_BPACT_STOP_OK


def program():
    code = bytearray(b"\xcc" * 0x40)
    code[0x00:0x03] = b"\xf6\xc1\x01"      # test cl, 1
    code[0x03:0x05] = b"\x74\x0a"          # jz A
    code[0x05:0x06] = b"\x90"              # B: nop   (SetGprs -> C)
    code[0x0F:0x10] = b"\x90"              # A: nop   (StopOk)
    code[0x20:0x24] = b"\x48\x83\xc0\x07"  # C: add rax, 7
    code[0x24:0x25] = b"\x90"              # D: nop   (StopOk)
    return bytes(code)


def actions():
    acts = (abi.BpAction * 3)()
    acts[0].gva, acts[0].kind = B, abi.BPACT_SET_GPRS
    for i in range(16):
        acts[0].gprs[i] = SET[i]
    acts[0].gprs[16] = C_
    acts[1].gva, acts[1].kind = A, BPACT_STOP_OK
    acts[2].gva, acts[2].kind = D, BPACT_STOP_OK
    return acts


@pytest.mark.parametrize("lanes", [256, 4096])
def test_setgprs_and_stopok_in_one_launch(lanes):
    from wtf_amd.engine import Engine

    sp = AddressSpace()
    sp.map_range(CODE_VA, program(), write=False)
    sp.map(0x7FF000000000, b"")
    eng = Engine(0)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(lanes, overlay_pages=4, cov_entries=64)
    eng.set_initial_state(regs_from_state(user_state(CODE_VA, 0x7FF000000800, sp.cr3)))
    eng.set_limit(0)
    eng.set_breakpoints([B, A, D])
    acts = actions()
    assert eng.L.wtfgpu_set_breakpoint_actions(eng.ctx, acts, 3) == 0
    eng.restore()
    rng = np.random.default_rng(7)
    g = eng.read_gprs(0, lanes)
    rcx = rng.integers(0, 1 << 32, size=lanes, dtype=np.uint64)
    g[:, 1] = rcx
    g[:, 0] = np.arange(lanes, dtype=np.uint64) * 3
    eng.write_gprs(g)
    eng.run()
    ex = eng.exits_np(0, lanes)
    out = eng.read_gprs(0, lanes)
    odd = (rcx & 1) == 1
    assert odd.any() and (~odd).any()
    bad = []
    for i in range(lanes):
        st, rip, ic = int(ex["status"][i]), int(ex["rip"][i]), int(ex["icount"][i])
        if odd[i]:
            want = (EXIT_STOP_OK, D, 3)
            regs_ok = int(out[i, 0]) == SET[0] + 7 and all(int(out[i, k]) == SET[k] for k in range(1, 16))
        else:
            want = (EXIT_STOP_OK, A, 2)
            regs_ok = int(out[i, 1]) == int(rcx[i]) and int(out[i, 0]) == 3 * i
        if (st, rip, ic) != want or not regs_ok:
            bad.append((i, bool(odd[i]), st, hex(rip), ic))
    assert not bad, f"{len(bad)}/{lanes} lanes wrong, first: {bad[:6]}"
