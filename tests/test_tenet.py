"""Tenet traces (U38; bochscpu_backend.cc:1215-1323, `--trace-type tenet`).

The stream both engines write (include/wtfgpu.h wtfgpu_set_tenet): REGS
entries at the start and after each instruction, ACC entries for its data
accesses with the memory after it. Here, on the CPU:
  * the engine's lane code built for the host (tests/native/sim_lane.cc)
    writes the same stream as the oracle on random integer / SSE / AVX
    programs, byte for byte;
  * the twin's `run --trace-type tenet` files (runner.cc's formatter) are in
    the reference's text format: the first line sets every register, later
    lines only the changed ones, memory as `,mr=` / `,mw=` / `,mrw=`
    0x<address>:<HEX bytes>.
The GPU's files equal the twin's in tests/test_trace.py.
"""
import ctypes as C
import os
import re
import struct

import pytest

from tests import progfuzz
from tests import tlv_harness as H
from tests.oracle_lib import Oracle
from tests.test_mmx import sim_lib as _sim_lib
from tests.test_sse import SimResult
from wtf_amd.abi import Regs, regs_from_state

CAP = 1 << 22


def sim_lib():
    L = _sim_lib()
    L.sim_set_tenet.argtypes = [C.c_uint64]
    L.sim_tenet.argtypes = [C.c_char_p, C.c_uint64]
    L.sim_tenet.restype = C.c_uint64
    return L


def parse(stream: bytes):
    """[(kind, fields)]: ('acc', va, type, data) / ('regs', gpr16, rip)."""
    out, q = [], 0
    while q < len(stream):
        w0, w1 = struct.unpack_from("<QQ", stream, q)
        if w0 == 2 << 56:
            vals = struct.unpack_from("<17Q", stream, q + 8)
            out.append(("regs", vals[:16], vals[16]))
            q += 8 + 17 * 8
        else:
            assert w1 >> 56 == 1, hex(w1)
            n = w1 & 0xFFFFFFFF
            out.append(("acc", w0, (w1 >> 32) & 0xFF, stream[q + 16:q + 16 + n]))
            q += 16 + (n + 7) // 8 * 8
    return out


@pytest.mark.parametrize("sse", [False, True])
def test_engine_stream_equals_oracle_on_random_programs(sse):
    L = sim_lib()
    n = 120
    sp, st, lanes = progfuzz.build(n, seed=77 if sse else 78, sse=sse)
    xmm = progfuzz.lane_xmm(n, 77)
    ymmh = progfuzz.lane_xmm(n, 77, 0x4E4)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.set_limit(3000)
    base = regs_from_state(st)
    arr = (C.c_uint64 * len(pfns))(*pfns)
    bad, accs = [], 0
    for i, (va, g, flags) in enumerate(lanes):
        r = regs_from_state(st)
        for k in range(16):
            r.gpr[k] = g[k]
            r.xmm[k][0], r.xmm[k][1] = xmm[i][2 * k], xmm[i][2 * k + 1]
            r.ymmh[k][0], r.ymmh[k][1] = ymmh[i][2 * k], ymmh[i][2 * k + 1]
        r.rip, r.rflags = va, flags
        o.restore(base)
        o.set_regs(r)
        o.set_tenet(True)
        o.run()
        want = o.tenet()
        L.sim_set_tenet(CAP)
        out, final = SimResult(), Regs()
        cnt = C.c_uint64(0)
        L.sim_run_full(arr, blob, len(pfns), C.byref(r), 3000, C.byref(out), 0, C.byref(cnt), 0, C.byref(final), None)
        buf = C.create_string_buffer(CAP)
        m = L.sim_tenet(buf, CAP)
        got = buf.raw[:m]
        L.sim_set_tenet(0)
        if got != want:
            a, b = parse(got), parse(want)
            k = next((j for j, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
            bad.append((i, k, a[k] if k < len(a) else None, b[k] if k < len(b) else None))
        accs += sum(1 for e in parse(want) if e[0] == "acc")
    assert accs > n, accs
    assert not bad, f"{len(bad)}/{n} lanes differ; first: {bad[:3]}"


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_twin_tenet_files_are_in_the_reference_format(tmp_path):
    d = H.build_target(str(tmp_path / "tlv"))
    inp = os.path.join(d, "inputs")
    out = tmp_path / "traces"
    H.run(H.TWIN, d, inp, str(tmp_path / "r.jsonl"), lanes=4,
          extra=("--trace-path", str(out), "--trace-type", "tenet"))
    names = sorted(os.listdir(inp))
    assert sorted(os.listdir(out)) == sorted(n + ".trace" for n in names)
    regs = ["rax", "rbx", "rcx", "rdx", "rbp", "rsp", "rsi", "rdi"] + [f"r{i}" for i in range(8, 16)] + ["rip"]
    reg_re = re.compile(r"(r[a-z0-9]+)=0x[0-9a-f]+")
    mem_re = re.compile(r"(mr|mw|mrw)=0x[0-9a-f]+:(?:[0-9A-F]{2})+")
    mems = 0
    for n in names:
        lines = (out / (n + ".trace")).read_text().splitlines()
        assert len(lines) > 50
        first = lines[0]
        assert first == ",".join(f"{r}=" + first.split(f"{r}=")[1].split(",")[0] for r in regs)
        for ln in lines[1:]:
            parts = [p for p in ln.split(",") if p]
            for p in parts:
                assert reg_re.fullmatch(p) or mem_re.fullmatch(p), (n, ln)
            mems += sum(1 for p in parts if mem_re.fullmatch(p))
    assert mems > 100
