"""Pin the CPU oracle against native-execution golden vectors (tests/golden).

Each vector executed one instruction natively on an x86-64 host
(tests/golden/gen_native_vectors.py). The oracle executes the same bytes from a
synthetic ring-3 address space whose data window sits at the same virtual
address, and must reproduce every GPR, the defined RFLAGS bits (fmask) and
every byte of the 256-byte memory window.
"""
import gzip
import json
import os

import pytest

from tests.oracle_lib import Oracle
from wtf_amd.abi import EXIT_FAULT, RUNNING, regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state
from tests.golden.gen_native_vectors import splitmix_bytes

HERE = os.path.dirname(os.path.abspath(__file__))
VECS = os.path.join(HERE, "golden", "native_vectors.json.gz")
CODE_VA = 0x140001000


def load():
    with gzip.open(VECS, "rt") as f:
        return json.load(f)


DOC = load()


def build_case(case, buf_va):
    page_va = buf_va & ~0xFFF  # window = g_buf + 0x800
    sp = AddressSpace()
    code = bytes.fromhex(case["code"]) + b"\xcc"
    sp.map(CODE_VA, code, write=False)
    win = splitmix_bytes(int(case["seed"], 16), 256)
    first = bytearray(4096)
    off = buf_va - page_va
    first[off:off + 256] = win
    sp.map(page_va, bytes(first))
    sp.map(page_va + 0x1000, b"")
    st = user_state(CODE_VA, 0, sp.cr3)
    regs = regs_from_state(st)
    for i in range(16):
        regs.gpr[i] = int(case["in"][i], 16)
    regs.rflags = int(case["fl"], 16) | 0x200  # ring 3 cannot clear IF: the native run had IF=1
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    return o


@pytest.mark.parametrize("chunk", range(8))
def test_oracle_matches_native_execution(chunk):
    buf_va = int(DOC["buf_va"], 16)
    cases = DOC["cases"][chunk::8]
    failures = []
    for c in cases:
        o = build_case(c, buf_va)
        ex = o.step()
        if ex.status != RUNNING:
            failures.append((c["name"], c["code"], "exit", ex.status, ex.vector))
            continue
        r = o.regs()
        want = [int(x, 16) for x in c["out"]]
        got = list(r.gpr)
        if c["cls"] == "bsx" and (int(c["flo"], 16) & 0x40):
            got[c["dst"]] = want[c["dst"]]  # BSF/BSR dest undefined for a zero source
        fmask = int(c["fmask"], 16)
        if got != want:
            bad = [(i, hex(got[i]), hex(want[i])) for i in range(16) if got[i] != want[i]]
            failures.append((c["name"], c["code"], "regs", bad))
            continue
        if (r.rflags ^ int(c["flo"], 16)) & fmask:
            failures.append((c["name"], c["code"], "flags", hex(r.rflags), c["flo"], c["fmask"]))
            continue
        win = bytearray(splitmix_bytes(int(c["seed"], 16), 256))
        for i, v in c["diff"]:
            win[i] = v
        mem = o.read_virt(buf_va, 256)
        if mem != bytes(win):
            failures.append((c["name"], c["code"], "mem"))
            continue
        assert r.rip == CODE_VA + len(bytes.fromhex(c["code"])), c["name"]
    assert not failures, f"{len(failures)}/{len(cases)} mismatches, first: {failures[:8]}"


def test_vector_file_is_substantial():
    assert len(DOC["cases"]) > 5000
    assert len({c["code"] for c in DOC["cases"]}) > 900
