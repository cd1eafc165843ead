#!/usr/bin/env python3
"""Native-execution golden vectors for the SSSE3 / SSE4.1 integer forms and the
AVX / AVX2 lane-crossing forms (convention U41; wtf_amd/csrc/engine_sse4.h,
oracle/x86_oracle_sse4.inc).

Same machinery as gen_fp_vectors.py (16 GPRs, RFLAGS, 16 YMM registers,
MXCSR, a 256-byte window; one stub per encoding), with integer inputs: random
bytes mixed with saturation / sign / shuffle-control edge patterns, and
memory writes recorded (pextr*, extractps, vextract*128 store forms).

Output: tests/golden/sse4_vectors.json.gz. Re-run with
    python tests/golden/gen_sse4_vectors.py
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.gen_avx_vectors import vmem, vrr  # noqa: E402
from tests.golden.gen_fp_vectors import Form, leg_mem, leg_rr, run_native  # noqa: E402
from tests.golden.gen_native_vectors import WIN, rand_val  # noqa: E402

OUT = os.path.join(HERE, "sse4_vectors.json.gz")
RSP = 4

# (map, opcode, name, kind): kind "lane" two-source, "one" r/m only, "pmov" (r/m narrower),
# legacy and VEX unless noted
M2_LANE = [(0x01, "phaddw"), (0x02, "phaddd"), (0x03, "phaddsw"), (0x04, "pmaddubsw"), (0x05, "phsubw"),
           (0x06, "phsubd"), (0x07, "phsubsw"), (0x08, "psignb"), (0x09, "psignw"), (0x0A, "psignd"),
           (0x0B, "pmulhrsw"), (0x28, "pmuldq"), (0x29, "pcmpeqq"), (0x2B, "packusdw"), (0x38, "pminsb"),
           (0x39, "pminsd"), (0x3A, "pminuw"), (0x3B, "pminud"), (0x3C, "pmaxsb"), (0x3D, "pmaxsd"),
           (0x3E, "pmaxuw"), (0x3F, "pmaxud"), (0x40, "pmulld")]
M2_ONE = [(0x1C, "pabsb"), (0x1D, "pabsw"), (0x1E, "pabsd")]
PMOV = [(0x20, 2), (0x21, 4), (0x22, 8), (0x23, 2), (0x24, 4), (0x25, 2), (0x30, 2), (0x31, 4), (0x32, 8),
        (0x33, 2), (0x34, 4), (0x35, 2)]  # (opcode, source bytes per 16 destination bytes divisor)


def gen_forms(rng):
    forms = []
    x = lambda: rng.randrange(16)  # noqa: E731
    g = lambda: rng.choice([r for r in range(16) if r != RSP])  # noqa: E731
    imm = lambda: [rng.randrange(256)]  # noqa: E731

    def add(code, name, p=(), s=()):
        forms.append(Form(code, name, 1, p, s))

    for op, nm in M2_LANE + [(0x10, "pblendvb")]:
        for _ in range(2):
            add(leg_rr(1, op, x(), x(), map3=2), nm + ".rr")
        c, p, s = leg_mem(rng, 1, op, x(), 16, map3=2)
        add(c, nm + ".m", p, s)
    for op, nm in M2_ONE:
        add(leg_rr(1, op, x(), x(), map3=2), nm + ".rr")
        c, p, s = leg_mem(rng, 1, op, x(), 16, map3=2)
        add(c, nm + ".m", p, s)
    for op, _div in PMOV:
        nm = ("pmovsx" if op < 0x30 else "pmovzx") + "%02x" % op
        add(leg_rr(1, op, x(), x(), map3=2), nm + ".rr")
        c, p, s = leg_mem(rng, 1, op, x(), 1, map3=2)
        add(c, nm + ".m", p, s)
    c, p, s = leg_mem(rng, 1, 0x2A, x(), 16, map3=2)
    add(c, "movntdqa.m", p, s)
    add(leg_rr(1, 0x41, x(), x(), map3=2), "phminposuw.rr")
    c, p, s = leg_mem(rng, 1, 0x41, x(), 16, map3=2)
    add(c, "phminposuw.m", p, s)
    # 0f 3a
    for op, nm in ((0x0E, "pblendw"), (0x0F, "palignr"), (0x42, "mpsadbw")):
        for _ in range(3):
            add(leg_rr(1, op, x(), x(), map3=3) + [rng.choice([0, 1, 4, 8, 15, 16, 17, 31, 32, 40, rng.randrange(256)])],
                nm + ".rr")
        c, p, s = leg_mem(rng, 1, op, x(), 16, map3=3)
        add(c + imm(), nm + ".m", p, s)
    for op, nm in ((0x14, "pextrb"), (0x15, "pextrw"), (0x16, "pextrd"), (0x17, "extractps")):
        for w in ((0, 1) if op == 0x16 else (0,)):
            add(leg_rr(1, op, x(), g(), w, map3=3) + imm(), f"{nm}.w{w}.r")
            c, p, s = leg_mem(rng, 1, op, x(), 1, w, map3=3)
            add(c + imm(), f"{nm}.w{w}.m", p, s)
    for op, nm in ((0x20, "pinsrb"), (0x22, "pinsrd")):
        for w in ((0, 1) if op == 0x22 else (0,)):
            add(leg_rr(1, op, x(), g(), w, map3=3) + imm(), f"{nm}.w{w}.r")
            c, p, s = leg_mem(rng, 1, op, x(), 1, w, map3=3)
            add(c + imm(), f"{nm}.w{w}.m", p, s)
    for _ in range(3):
        add(leg_rr(1, 0x21, x(), x(), map3=3) + imm(), "insertps.rr")
    c, p, s = leg_mem(rng, 1, 0x21, x(), 1, map3=3)
    add(c + imm(), "insertps.m", p, s)
    # ---- VEX
    for l in (0, 1):
        for op, nm in M2_LANE:
            add(vrr(rng, op, x(), x(), x(), l, 1, mmmmm=2), f"v{nm}.L{l}.rr")
            c, p, s = vmem(rng, op, x(), x(), l, 1, 1, mmmmm=2)
            add(c, f"v{nm}.L{l}.m", p, s)
        for op, nm in M2_ONE:
            add(vrr(rng, op, x(), 0, x(), l, 1, mmmmm=2), f"v{nm}.L{l}.rr")
        for op, _div in PMOV:
            nm = ("vpmovsx" if op < 0x30 else "vpmovzx") + "%02x" % op
            add(vrr(rng, op, x(), 0, x(), l, 1, mmmmm=2), f"{nm}.L{l}.rr")
            c, p, s = vmem(rng, op, x(), 0, l, 1, 1, mmmmm=2)
            add(c, f"{nm}.L{l}.m", p, s)
        for op, nm in ((0x0C, "vpermilps"), (0x0D, "vpermilpd"), (0x0E, "vtestps"), (0x0F, "vtestpd")):
            vv = 0 if op >= 0x0E else x()
            add(vrr(rng, op, x(), vv, x(), l, 1, mmmmm=2), f"{nm}.L{l}.rr")
        for w in (0, 1):
            for op, nm in ((0x45, "vpsrlv"), (0x47, "vpsllv"), (0x46, "vpsrav")):
                if op == 0x46 and w:
                    continue
                add(vrr(rng, op, x(), x(), x(), l, 1, mmmmm=2, w=w), f"{nm}.w{w}.L{l}.rr")
        add(vrr(rng, 0x18, x(), 0, x(), l, 1, mmmmm=2), f"vbroadcastss.L{l}.rr")
        c, p, s = vmem(rng, 0x18, x(), 0, l, 1, 1, mmmmm=2)
        add(c, f"vbroadcastss.L{l}.m", p, s)
        for op, nm in ((0x0E, "vpblendw"), (0x0F, "vpalignr"), (0x02, "vpblendd"), (0x42, "vmpsadbw")):
            add(vrr(rng, op, x(), x(), x(), l, 1, mmmmm=3) + imm(), f"{nm}.L{l}.rr")
        for op, nm in ((0x04, "vpermilps.i"), (0x05, "vpermilpd.i")):
            add(vrr(rng, op, x(), 0, x(), l, 1, mmmmm=3) + imm(), f"{nm}.L{l}.rr")
        add(vrr(rng, 0x4C, x(), x(), x(), l, 1, mmmmm=3) + [x() << 4], f"vpblendvb.L{l}.rr")
    for op, nm in ((0x16, "vpermps"), (0x36, "vpermd")):
        add(vrr(rng, op, x(), x(), x(), 1, 1, mmmmm=2), nm + ".rr")
    add(vrr(rng, 0x19, x(), 0, x(), 1, 1, mmmmm=2), "vbroadcastsd.rr")
    for l in (0, 1):
        for op, nm, w in ((0x2C, "vmaskmovps", 0), (0x2D, "vmaskmovpd", 0), (0x2E, "vmaskmovps.st", 0),
                          (0x2F, "vmaskmovpd.st", 0), (0x8C, "vpmaskmovd", 0), (0x8C, "vpmaskmovq", 1),
                          (0x8E, "vpmaskmovd.st", 0), (0x8E, "vpmaskmovq.st", 1)):
            for _ in range(2):
                c, p, s = vmem(rng, op, x(), x(), l, 1, 1, mmmmm=2, w=w)
                add(c, f"{nm}.L{l}.m", p, s)
    for op, nm in ((0x1A, "vbroadcastf128"), (0x5A, "vbroadcasti128")):
        c, p, s = vmem(rng, op, x(), 0, 1, 1, 1, mmmmm=2)
        add(c, nm + ".m", p, s)
    for op, nm in ((0x00, "vpermq"), (0x01, "vpermpd")):
        add(vrr(rng, op, x(), 0, x(), 1, 1, mmmmm=3, w=1) + imm(), nm + ".rr")
    for op, nm in ((0x06, "vperm2f128"), (0x46, "vperm2i128"), (0x18, "vinsertf128"), (0x38, "vinserti128")):
        add(vrr(rng, op, x(), x(), x(), 1, 1, mmmmm=3) + imm(), nm + ".rr")
    for op, nm in ((0x19, "vextractf128"), (0x39, "vextracti128")):
        add(vrr(rng, op, x(), 0, x(), 1, 1, mmmmm=3) + imm(), nm + ".rr")
        c, p, s = vmem(rng, op, x(), 0, 1, 1, 1, mmmmm=3)
        add(c + imm(), nm + ".m", p, s)
    for op, nm in ((0x14, "vpextrb"), (0x16, "vpextrd"), (0x17, "vextractps")):
        add(vrr(rng, op, x(), 0, g(), 0, 1, mmmmm=3) + imm(), nm + ".r")
    for op, nm in ((0x20, "vpinsrb"), (0x22, "vpinsrd"), (0x21, "vinsertps")):
        add(vrr(rng, op, x(), x(), g() if op != 0x21 else x(), 0, 1, mmmmm=3) + imm(), nm + ".rr")
    return forms


def int_vec(rng):
    """256 bits of integer lane data: random bytes, edge bytes, or shuffle / shift controls."""
    r = rng.random()
    if r < 0.25:
        b = bytes(rng.choice([0, 1, 2, 0x7F, 0x80, 0x81, 0xFE, 0xFF, 0x40, 0xC0]) for _ in range(32))
    elif r < 0.35:  # small shift counts / permute indices in each dword
        b = b"".join((rng.choice([0, 1, 3, 7, 15, 16, 31, 32, 33, 63, 64, 200]) | (rng.randrange(8) << 40)).to_bytes(8, "little")
                     for _ in range(4))
    else:
        b = bytes(rng.getrandbits(8) for _ in range(32))
    return [int.from_bytes(b[i:i + 8], "little") for i in range(0, 32, 8)]


def case_inputs(seed):
    rng = random.Random(seed)
    ymm = [int_vec(rng) for _ in range(16)]
    win = []
    for _ in range(WIN // 32):
        win += int_vec(rng)
    return ymm, win


def make_cases(forms, rng, per_form=6):
    cases = []
    for f in forms:
        for _ in range(per_form):
            regs = [rand_val(rng) for _ in range(16)]
            regs[RSP] = 0x80
            for r, off in f.ptrs.items():
                regs[r] = off
            for r, (lo, hi) in f.smalls.items():
                regs[r] = rng.randint(lo, hi)
            seed = rng.getrandbits(63)
            ymm, win = case_inputs(seed)
            cases.append({"name": f.name, "code": f.code.hex(), "regs": regs, "ptrs": sorted(f.ptrs) + [RSP],
                          "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "ymm": ymm, "win": win, "mx": 0x1F80,
                          "seed": seed, "ew": 1, "ints": 1})
    return cases


def main():
    rng = random.Random(0x55E4001)
    run_native(make_cases(gen_forms(rng), rng), "tests/golden/gen_sse4_vectors.py", OUT, mem_writes=True)


if __name__ == "__main__":
    main()
