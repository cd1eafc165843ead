"""The extensions beyond SSE4.1 / AVX2 (convention U45; engine_ext.h,
oracle/x86_oracle_ext.inc): BMI1 / BMI2, ADX, MOVBE, CRC32, SSE4.2, AES and
PCLMULQDQ, which cpuid_leaf now enumerates.

Native-execution vectors (tests/golden/gen_ext_vectors.py, run on this host's
CPU, which executes every one of these forms) pin the oracle and the engine's
device code built for the host; the GPU runs them in tests/test_gpu_sse.py.
The string compares (which the oracle computes in C, not natively) are covered
under all 128 control bytes each. Hand-checked:
the CPUID bits, and #UD / UNIMPLEMENTED rules (tests/test_avx.py).
"""
import gzip
import json
import os

import pytest

from tests.golden.gen_ext_vectors import case_inputs
from tests.oracle_lib import Oracle
from tests.test_avx import get_ymm, set_ymm
from tests.test_fp import check
from tests.test_sse import layout, sim_lib, sim_run

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with gzip.open(os.path.join(HERE, "golden", "ext_vectors.json.gz"), "rt") as f:
        return json.load(f)


DOC = load()


def inputs(c):
    ymm, win = case_inputs(int(c["seed"], 16), c["ints"])
    return [v for r in ymm for v in r], b"".join(v.to_bytes(8, "little") for v in win)


def case_regs(c, regs, yin):
    for i in range(16):
        regs.gpr[i] = int(c["in"][i], 16)
    regs.rflags = int(c["fl"], 16) | 0x200
    set_ymm(regs, yin)
    regs.mxcsr = int(c["mx"], 16)
    return regs


def window_after(c, win):
    w = bytearray(win)
    for i, v in c.get("mdiff", []):
        w[i] = v
    return bytes(w)


@pytest.mark.parametrize("chunk", range(2))
def test_oracle_matches_native_ext(chunk):
    buf_va = int(DOC["buf_va"], 16)
    cases = DOC["cases"][chunk::2]
    fails = []
    for c in cases:
        yin, win = inputs(c)
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, win)
        pfns, blob = sp.phys()
        o = Oracle(pfns=pfns, blob=blob)
        o.restore(case_regs(c, regs, yin))
        ex = o.step()
        r = o.regs()
        ymm = get_ymm([r.xmm[i][h] for i in range(16) for h in range(2)], [r.ymmh[i][h] for i in range(16) for h in range(2)])
        bad = check(c, ex.status, ex.vector, r.gpr, r.rflags, ymm, r.mxcsr, yin)
        if not bad and o.read_virt(buf_va, 256) != window_after(c, win):
            bad = ("mem",)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
    assert not fails, f"{len(fails)}/{len(cases)} mismatches, first: {fails[:5]}"


def test_engine_ext_code_matches_native_vectors():
    L = sim_lib()
    buf_va = int(DOC["buf_va"], 16)
    fails = []
    for c in DOC["cases"]:
        yin, win = inputs(c)
        sp, regs = layout(bytes.fromhex(c["code"]), buf_va, win)
        out = sim_run(L, sp, case_regs(c, regs, yin), win_va=buf_va)
        bad = check(c, out.status, out.vector, out.gpr, out.rflags, get_ymm(list(out.xmm), list(out.ymmh)),
                    out.mxcsr, yin)
        if not bad and bytes(out.win[:256]) != window_after(c, win):
            bad = ("mem",)
        if bad:
            fails.append((c["name"], c["code"]) + bad)
    assert not fails, f"{len(fails)}/{len(DOC['cases'])} mismatches, first: {fails[:5]}"


def test_ext_vector_file_is_substantial():
    names = {c["name"].split(".")[0] for c in DOC["cases"]}
    assert len(DOC["cases"]) > 4000
    for n in ("andn", "blsr", "blsmsk", "blsi", "bzhi", "bextr", "shlx", "sarx", "shrx", "pdep", "pext", "mulx",
              "rorx", "adcx", "adox", "movbe16", "movbe32", "movbe64", "crc32b", "crc32w", "crc32d", "crc32q",
              "pcmpgtq", "vpcmpgtq", "pcmpestri", "pcmpestrm", "pcmpistri", "pcmpistrm", "vpcmpestri", "vpcmpistrm",
              "aesenc", "aesenclast", "aesdec", "aesdeclast", "aesimc", "aeskeygenassist", "vaesenc",
              "pclmulqdq", "vpclmulqdq", "sha1rnds4", "sha1nexte", "sha1msg1", "sha1msg2", "sha256rnds2",
              "sha256msg1", "sha256msg2"):
        assert n in names, n
