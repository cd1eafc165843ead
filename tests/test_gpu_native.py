"""GPU engine vs native x86-64 execution: every golden vector is one lane.

All 1007 encodings of tests/golden/native_vectors.json.gz live in one code
region (one 32-byte slot each, followed by int3); each lane gets its vector's
registers and its own copy of the 256-byte data window (copy-on-write through
wtfgpu_apply_writes), runs one instruction, and stops at the int3.
"""
import gzip
import json
import os

import numpy as np
import pytest

from tests.golden.gen_native_vectors import splitmix_bytes
from wtf_amd.abi import EXIT_INT3, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

HERE = os.path.dirname(os.path.abspath(__file__))
CODE_VA = 0x140000000

pytestmark = pytest.mark.gpu


def load_vectors():
    with gzip.open(os.path.join(HERE, "golden", "native_vectors.json.gz"), "rt") as f:
        return json.load(f)


def build_native_snapshot(doc):
    codes = sorted({c["code"] for c in doc["cases"]})
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
    return sp, slot, buf_va


def test_gpu_matches_native_vectors():
    from wtf_amd.engine import Engine

    doc = load_vectors()
    cases = doc["cases"]
    sp, slot, buf_va = build_native_snapshot(doc)
    n = (len(cases) + 63) // 64 * 64
    eng = Engine(0)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(n, overlay_pages=4, cov_entries=64)
    st = user_state(CODE_VA, 0, sp.cr3)
    eng.set_initial_state(regs_from_state(st))
    eng.set_limit(0)
    eng.restore()
    g = eng.read_gprs()
    writes = []
    for i, c in enumerate(cases):
        for r in range(16):
            g[i, r] = int(c["in"][r], 16)
        g[i, 16] = CODE_VA + 32 * slot[c["code"]]
        g[i, 17] = int(c["fl"], 16) | 0x200
        writes.append((i, buf_va, splitmix_bytes(int(c["seed"], 16), 256)))
    for i in range(len(cases), n):  # idle padding lanes run a lone int3
        g[i, 16] = CODE_VA + 32 * slot[cases[0]["code"]] + len(bytes.fromhex(cases[0]["code"]))
    eng.write_gprs(g)
    eng.apply_writes(writes)
    eng.run()
    ex = eng.exits()
    out = eng.read_gprs()
    fails = []
    for i, c in enumerate(cases):
        code = bytes.fromhex(c["code"])
        if ex[i].status != EXIT_INT3 or ex[i].icount != 1:
            fails.append((c["name"], c["code"], "exit", ex[i].status, ex[i].vector, hex(ex[i].rip)))
            continue
        want = [int(x, 16) for x in c["out"]]
        got = [int(v) for v in out[i, :16]]
        if c["cls"] == "bsx" and (int(c["flo"], 16) & 0x40):
            got[c["dst"]] = want[c["dst"]]
        if got != want:
            fails.append((c["name"], c["code"], "regs", [(r, hex(got[r]), hex(want[r])) for r in range(16) if got[r] != want[r]]))
            continue
        if (int(out[i, 17]) ^ int(c["flo"], 16)) & int(c["fmask"], 16):
            fails.append((c["name"], c["code"], "flags", hex(int(out[i, 17])), c["flo"], c["fmask"]))
            continue
        if int(out[i, 16]) != CODE_VA + 32 * slot[c["code"]] + len(code):
            fails.append((c["name"], c["code"], "rip"))
            continue
    # memory windows: sample every lane whose instruction wrote memory
    memfails = []
    for i, c in enumerate(cases):
        if not c["diff"] and i % 7:
            continue
        win = bytearray(splitmix_bytes(int(c["seed"], 16), 256))
        for k, v in c["diff"]:
            win[k] = v
        if eng.read_virt(i, buf_va, 256) != bytes(win):
            memfails.append((c["name"], c["code"]))
    if fails:
        import collections
        print("failing classes:", collections.Counter(f[0] for f in fails).most_common())
    assert not fails, f"{len(fails)}/{len(cases)} register mismatches, first: {fails[:6]}"
    assert not memfails, f"{len(memfails)} memory mismatches, first: {memfails[:6]}"
