"""Guest memory at the edges of a page in the device breakpoint actions
(engine.hip bp_apply_action, host_write, the Feed prefault in k_run):

  * SimulateReturn after reading a C string (VirtReadString, backend.h:333-430)
    reads the string in aligned 32-byte blocks. The string sits at the end of
    a mapped page whose next page is not mapped: the action applies when the
    terminator, or the length limit, comes before the page end (a block never
    crosses a page, so no block of the unmapped page is read), and leaves the
    hit to the host (WTFGPU_EXIT_BREAKPOINT, registers untouched) when a byte
    the scan needs lies on the unmapped page — byte for byte as a read one
    byte at a time decides it.
  * A Feed chunk written across a page boundary (Backend_t::VirtWrite,
    backend.cc:91-121: page by page): with both pages mapped every byte lands
    (the first page copied on write by the whole wave before the action, the
    second inside it); with the second page unmapped the lane ends with
    WTFGPU_EXIT_FEED_FAULT and the first page's part is written, as VirtWrite
    leaves it.
Expected values are written out here by hand from those rules."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from wtf_amd import abi
from wtf_amd.abi import regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

pytestmark = pytest.mark.gpu

CODE_VA = 0x140000000
DATA_VA = 0x150000000  # data pages at DATA_VA + 0x2000 k, the page after each unmapped unless said
STACK_VA = 0x7FF000000000
STACK_TOP = STACK_VA + 0x800
CALL, RET_AT, HOOK = CODE_VA + 0x00, CODE_VA + 0x05, CODE_VA + 0x20
BPACT_STOP_OK = 5
HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "wtfgpu.h")


def _exit_codes():
    codes = {m.group(1): int(m.group(2))
             for m in re.finditer(r"WTFGPU_EXIT_(\w+)\s*=\s*(\d+)", open(HEADER).read())}
    return codes["BREAKPOINT"], codes["STOP_OK"], codes["FEED_FAULT"]


def _code():
    code = bytearray(b"\xcc" * 0x40)
    code[0x00:0x05] = b"\xe8" + (HOOK - RET_AT).to_bytes(4, "little")  # call HOOK
    code[0x05:0x06] = b"\x90"  # RET_AT: nop (StopOk)
    code[0x20:0x21] = b"\x90"  # HOOK: nop (the action's breakpoint)
    code[0x21:0x22] = b"\xc3"  # ret (a Feed keeps rip: the nop runs, then this)
    return bytes(code)


def _engine(sp, lanes):
    from wtf_amd.engine import Engine
    eng = Engine(0)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(lanes, overlay_pages=8, cov_entries=64)
    eng.set_initial_state(regs_from_state(user_state(CALL, STACK_TOP, sp.cr3)))
    eng.set_limit(0)
    eng.set_breakpoints([HOOK, RET_AT])
    return eng


def _actions(first):
    acts = (abi.BpAction * 2)()
    acts[0] = first
    acts[1].gva, acts[1].kind = RET_AT, BPACT_STOP_OK
    return acts


# (string start offset in the data page, bytes written there, limit, applies)
STRING_CASES = [
    (0xFFC, b"abc\x00", 64, True),         # terminator on the page's last byte
    (0xFF0, b"A" * 16, 64, False),         # runs into the unmapped page
    (0xFF8, b"B" * 8, 8, True),            # the limit ends at the page end
    (0x013, b"x\x00", 64, True),           # a block start that is not the string's
    (0xFE1, b"C" * 31, 31, True),          # 31 bytes, limit 31: page 2 never read
    (0xFE1, b"C" * 31, 32, False),         # limit 32: the 32nd byte is on page 2
]


def test_simulate_return_string_at_page_end():
    ex_bp, ex_ok, _ = _exit_codes()
    sp = AddressSpace()
    sp.map_range(CODE_VA, _code(), write=False)
    sp.map(STACK_VA, b"")
    for k, (off, data, _, _) in enumerate(STRING_CASES):  # each case its own page, the next one unmapped
        page = bytearray(0x1000)
        page[off:off + len(data)] = data
        sp.map(DATA_VA + 0x2000 * k, bytes(page))
    lanes = 256
    eng = _engine(sp, lanes)
    results = []
    for limit in sorted({c[2] for c in STRING_CASES}):
        a = abi.BpAction()
        a.gva, a.kind, a.value = HOOK, abi.BPACT_RETURN, 0x77
        a.gprs[0], a.gprs[1] = 1 + 1, limit  # the string at rcx (register 1), at most `limit` bytes
        acts = _actions(a)
        assert eng.L.wtfgpu_set_breakpoint_actions(eng.ctx, acts, 2) == 0
        eng.restore()
        cases = [(k, c) for k, c in enumerate(STRING_CASES) if c[2] == limit]
        g = eng.read_gprs(0, lanes)
        for i in range(lanes):
            k, c = cases[i % len(cases)]
            g[i, 1] = DATA_VA + 0x2000 * k + c[0]
            g[i, 0] = 0x1000 + i
        eng.write_gprs(g)
        eng.run()
        ex = eng.exits_np(0, lanes)
        out = eng.read_gprs(0, lanes)
        for i in range(lanes):
            off, _, _, applies = cases[i % len(cases)][1]
            st, rip = int(ex["status"][i]), int(ex["rip"][i])
            if applies:
                ok = (st, rip) == (ex_ok, RET_AT) and int(out[i, 0]) == 0x77 and int(out[i, 4]) == STACK_TOP
            else:  # left to the host handler at the hook, nothing applied
                ok = (st, rip) == (ex_bp, HOOK) and int(out[i, 0]) == 0x1000 + i and int(out[i, 4]) == STACK_TOP - 8
            results.append((ok, i, hex(off), limit, st, hex(rip)))
    bad = [r for r in results if not r[0]]
    assert not bad, f"{len(bad)} lanes wrong, first: {bad[:6]}"


def _feed_run(second_page_mapped):
    ex_bp, ex_ok, ex_ff = _exit_codes()
    sp = AddressSpace()
    sp.map_range(CODE_VA, _code(), write=False)
    sp.map(STACK_VA, b"")
    sp.map(DATA_VA, bytes(range(256)) * 16)
    if second_page_mapped:
        sp.map(DATA_VA + 0x1000, bytes(0x1000))
    lanes = 128
    eng = _engine(sp, lanes)
    a = abi.BpAction()
    a.gva, a.kind, a.value = HOOK, abi.BPACT_FEED, 0x900  # the chunk ends at rbx + 0x900
    a.gprs[0], a.gprs[1] = 3, 2  # buffer in rbx, size to rdx
    acts = _actions(a)
    assert eng.L.wtfgpu_set_breakpoint_actions(eng.ctx, acts, 2) == 0
    eng.restore()
    rbx = DATA_VA + 0x800  # window [rbx, rbx + 0x900) crosses into the second page
    g = eng.read_gprs(0, lanes)
    g[:, 3] = rbx
    eng.write_gprs(g)
    rng = np.random.default_rng(11)
    chunks, blob, offs = [], b"", [0]
    for i in range(lanes):
        n = int(rng.integers(0x101, 0x8FF))  # every chunk reaches past the page end
        data = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        chunks.append(data)
        blob += n.to_bytes(4, "little") + data
        offs.append(len(blob))
    o = (C.c_uint64 * (lanes + 1))(*offs)
    assert eng.L.wtfgpu_set_feed(eng.ctx, 0, lanes, o, None, blob, len(blob)) == 0
    eng.run()
    return eng, chunks, rbx, (ex_bp, ex_ok, ex_ff)


def test_feed_chunk_across_two_pages():
    eng, chunks, rbx, (_, ex_ok, _) = _feed_run(True)
    lanes = len(chunks)
    ex = eng.exits_np(0, lanes)
    out = eng.read_gprs(0, lanes)
    bad = []
    for i, data in enumerate(chunks):
        n = len(data)
        dst = rbx + 0x900 - n
        got = eng.read_virt(i, dst, n)
        before = eng.read_virt(i, dst - 8, 8)  # untouched: the page's original bytes
        want_before = bytes((dst - 8 - DATA_VA + k) & 0xFF for k in range(8))
        if (int(ex["status"][i]), int(ex["rip"][i])) != (ex_ok, RET_AT) or got != data or before != want_before or \
                int(out[i, 3]) != dst or int(out[i, 2]) != n:
            bad.append((i, n, int(ex["status"][i])))
    assert not bad, f"{len(bad)}/{lanes} lanes wrong, first: {bad[:6]}"


def test_feed_chunk_into_unmapped_page_writes_the_first():
    eng, chunks, rbx, (_, _, ex_ff) = _feed_run(False)
    lanes = len(chunks)
    ex = eng.exits_np(0, lanes)
    bad = []
    for i, data in enumerate(chunks):
        n = len(data)
        dst = rbx + 0x900 - n
        head = DATA_VA + 0x1000 - dst  # the chunk's bytes on the mapped page
        got = eng.read_virt(i, dst, head)
        if (int(ex["status"][i]), int(ex["rip"][i])) != (ex_ff, HOOK) or got != data[:head]:
            bad.append((i, n, int(ex["status"][i]), hex(int(ex["rip"][i]))))
    assert not bad, f"{len(bad)}/{lanes} lanes wrong, first: {bad[:6]}"
