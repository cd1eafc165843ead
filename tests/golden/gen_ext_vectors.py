#!/usr/bin/env python3
"""Native-execution golden vectors for the extensions beyond SSE4.1 / AVX2
(convention U45; wtf_amd/csrc/engine_ext.h, oracle/x86_oracle_ext.inc):
BMI1 / BMI2 (andn, bextr, blsi / blsmsk / blsr, bzhi, pdep, pext, mulx, rorx,
sarx / shlx / shrx), ADX (adcx, adox), MOVBE, CRC32, SSE4.2 (pcmpgtq, the
four string compares), AES, PCLMULQDQ and SHA, legacy and VEX, register and memory
forms, 32- and 64-bit operand sizes (16 for movbe / crc32).

Same machinery as gen_sse4_vectors.py (16 GPRs, RFLAGS, 16 YMM registers,
MXCSR, a 256-byte window with memory writes recorded). Control operands get
edge values (bzhi indexes and bextr fields around the operand size, shift
counts, string lengths around +-16 for the explicit-length compares), and the
string compares read strings over a small alphabet with embedded zeros, so
that every aggregation / polarity / output form meets matches, ranges and
short strings; each of the four string compares runs under all 128 control
bytes. Flags the SDM leaves undefined are masked per case ("flm").

Output: tests/golden/ext_vectors.json.gz. Re-run with
    python tests/golden/gen_ext_vectors.py
"""
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.gen_avx_vectors import vmem, vrr  # noqa: E402
from tests.golden.gen_fp_vectors import Form, leg_mem, leg_rr, run_native  # noqa: E402
from tests.golden.gen_native_vectors import WIN, rand_val  # noqa: E402

OUT = os.path.join(HERE, "ext_vectors.json.gz")
RSP = 4
M64 = (1 << 64) - 1
FL_ALL = 0x8D5
FL_NO_AP = FL_ALL & ~0x14       # AF, PF undefined
FL_BEXTR = FL_ALL & ~0x94       # AF, SF, PF undefined


class XForm(Form):
    def __init__(self, code, name, ptrs=(), smalls=(), flm=FL_ALL, strings=False, vals=()):
        super().__init__(code, name, 1, ptrs, smalls)
        self.flm = flm
        self.strings = strings
        self.vals = dict(vals)  # register -> a value chooser (rng -> int)


def gen_forms(rng):
    forms = []
    g = lambda: rng.choice([r for r in range(16) if r != RSP])  # noqa: E731
    x = lambda: rng.randrange(16)  # noqa: E731
    imm = lambda: [rng.randrange(256)]  # noqa: E731

    def small_idx(lo, hi):
        return lambda r: rng.choice([rng.randint(lo, hi), rand_val(r)]) if rng.random() < 0.5 else rng.randint(lo, hi)

    def bextr_ctl(r):
        st = rng.choice([0, 1, 7, 8, 31, 32, 33, 63, 64, 65, 200, rng.randrange(70)])
        ln = rng.choice([0, 1, 7, 8, 31, 32, 33, 63, 64, 65, 255, rng.randrange(70)])
        return (ln << 8) | st | (rng.getrandbits(40) << 16 if rng.random() < 0.3 else 0)

    def add(code, name, flm=FL_ALL, vals=(), ptrs=(), smalls=(), strings=False):
        forms.append(XForm(code, name, ptrs, smalls, flm, strings, vals))

    # ---- BMI1 / BMI2 (VEX, general registers); the vvvv operand never the stack pointer
    for w in (0, 1):
        sw = f".w{w}"
        for _ in range(3):
            d, v, r = g(), g(), x()
            add(vrr(rng, 0xF2, d, v, r, 0, 0, mmmmm=2, w=w), "andn" + sw + ".rr", FL_NO_AP)
        c, p, s = vmem(rng, 0xF2, g(), g(), 0, 0, 1, mmmmm=2, w=w)
        add(c, "andn" + sw + ".m", FL_NO_AP, ptrs=p, smalls=s)
        for r3, nm in ((1, "blsr"), (2, "blsmsk"), (3, "blsi")):
            for _ in range(3):
                add(vrr(rng, 0xF3, r3, g(), x(), 0, 0, mmmmm=2, w=w), nm + sw + ".rr", FL_NO_AP)
            c, p, s = vmem(rng, 0xF3, r3, g(), 0, 0, 1, mmmmm=2, w=w)
            add(c, nm + sw + ".m", FL_NO_AP, ptrs=p, smalls=s)
        for _ in range(4):
            v = g()
            add(vrr(rng, 0xF5, g(), v, x(), 0, 0, mmmmm=2, w=w), "bzhi" + sw + ".rr", FL_NO_AP,
                vals={v: small_idx(0, 72)})
        v = g()
        c, p, s = vmem(rng, 0xF5, g(), v, 0, 0, 1, mmmmm=2, w=w)
        if v not in p and v not in s:
            add(c, "bzhi" + sw + ".m", FL_NO_AP, vals={v: small_idx(0, 72)}, ptrs=p, smalls=s)
        for _ in range(4):
            v = g()
            add(vrr(rng, 0xF7, g(), v, x(), 0, 0, mmmmm=2, w=w), "bextr" + sw + ".rr", FL_BEXTR, vals={v: bextr_ctl})
        for pp, nm in ((1, "shlx"), (2, "sarx"), (3, "shrx")):
            for _ in range(3):
                v = g()
                add(vrr(rng, 0xF7, g(), v, x(), 0, pp, mmmmm=2, w=w), nm + sw + ".rr", vals={v: small_idx(0, 130)})
            c, p, s = vmem(rng, 0xF7, g(), g(), 0, pp, 1, mmmmm=2, w=w)
            add(c, nm + sw + ".m", ptrs=p, smalls=s)
        for pp, nm in ((2, "pext"), (3, "pdep")):
            for _ in range(3):
                add(vrr(rng, 0xF5, g(), g(), x(), 0, pp, mmmmm=2, w=w), nm + sw + ".rr")
            c, p, s = vmem(rng, 0xF5, g(), g(), 0, pp, 1, mmmmm=2, w=w)
            add(c, nm + sw + ".m", ptrs=p, smalls=s)
        for _ in range(3):
            add(vrr(rng, 0xF6, g(), g(), x(), 0, 3, mmmmm=2, w=w), "mulx" + sw + ".rr")
        r = g()
        add(vrr(rng, 0xF6, r, r, x(), 0, 3, mmmmm=2, w=w), "mulx" + sw + ".same")  # the high half wins
        c, p, s = vmem(rng, 0xF6, g(), g(), 0, 3, 1, mmmmm=2, w=w)
        add(c, "mulx" + sw + ".m", ptrs=p, smalls=s)
        for k in (0, 1, 31, 32, 63, rng.randrange(256)):
            add(vrr(rng, 0xF0, g(), 0, x(), 0, 3, mmmmm=3, w=w) + [k], "rorx" + sw + ".rr")
        c, p, s = vmem(rng, 0xF0, g(), 0, 0, 3, 1, mmmmm=3, w=w)
        add(c + imm(), "rorx" + sw + ".m", ptrs=p, smalls=s)
        # ---- ADX
        for pp, nm in ((1, "adcx"), (2, "adox")):
            for _ in range(3):
                add(leg_rr(pp, 0xF6, g(), x(), w, map3=2), nm + sw + ".rr")
            c, p, s = leg_mem(rng, pp, 0xF6, g(), 1, w, map3=2)
            add(c, nm + sw + ".m", ptrs=p, smalls=s)
    # ---- MOVBE (memory only): 16 / 32 / 64
    for pp, w, nm in ((1, 0, "movbe16"), (0, 0, "movbe32"), (0, 1, "movbe64")):
        for op, d in ((0xF0, "ld"), (0xF1, "st")):
            for _ in range(3):
                c, p, s = leg_mem(rng, pp, op, g(), 1, w, map3=2)
                add(c, f"{nm}.{d}.m", ptrs=p, smalls=s)
    # ---- CRC32: r8 / r16 / r32 / r64 sources
    for pfx, op, w, nm in (([0xF2], 0xF0, 0, "crc32b"), ([0xF2], 0xF0, 1, "crc32b.w1"), ([0x66, 0xF2], 0xF1, 0, "crc32w"),
                           ([0xF2], 0xF1, 0, "crc32d"), ([0xF2], 0xF1, 1, "crc32q")):
        for _ in range(3):
            reg, rm = g(), x()
            rex = 0x40 | (w << 3) | ((reg >> 3) << 2) | (rm >> 3)
            if op == 0xF0 and rex == 0x40 and rng.random() < 0.5:
                rex = 0x40  # sil / dil / spl / bpl instead of ah .. bh
                code = pfx + [rex, 0x0F, 0x38, op, 0xC0 | ((reg & 7) << 3) | (rm & 7)]
            else:
                code = pfx + ([rex] if rex != 0x40 else []) + [0x0F, 0x38, op, 0xC0 | ((reg & 7) << 3) | (rm & 7)]
            add(code, nm + ".rr")
        c, p, s = leg_mem(rng, 3, op, g(), 1, w, map3=2)
        if pfx[0] == 0x66:
            c = [0x66] + c
        add(c, nm + ".m", ptrs=p, smalls=s)
    # ---- SSE4.2
    for _ in range(3):
        add(leg_rr(1, 0x37, x(), x(), map3=2), "pcmpgtq.rr")
    c, p, s = leg_mem(rng, 1, 0x37, x(), 16, map3=2)
    add(c, "pcmpgtq.m", ptrs=p, smalls=s)
    for l in (0, 1):
        add(vrr(rng, 0x37, x(), x(), x(), l, 1, mmmmm=2), f"vpcmpgtq.L{l}.rr")
        c, p, s = vmem(rng, 0x37, x(), x(), l, 1, 1, mmmmm=2)
        add(c, f"vpcmpgtq.L{l}.m", ptrs=p, smalls=s)
    lens = lambda r: rng.choice([0, 1, 5, 7, 8, 9, 15, 16, 17, 100, -1, -7, -8, -9, -16, -17,  # noqa: E731
                                 -(1 << 31), (1 << 31) - 1, 1 << 32, -(1 << 40), rng.randrange(-20, 20)]) & M64
    for op, nm in ((0x60, "pcmpestrm"), (0x61, "pcmpestri"), (0x62, "pcmpistrm"), (0x63, "pcmpistri")):
        ex = op <= 0x61
        vals = {0: lens, 2: lens} if ex else {}
        for im in range(128):  # every control byte (bit 7 is ignored), 4 cases each
            w = rng.randrange(2) if ex else 0
            add(leg_rr(1, op, x(), x(), w, map3=3) + [im | (rng.randrange(2) << 7)], f"{nm}.rr", vals=vals,
                strings=True)
            forms[-1].cases = 4
        for _ in range(3):
            base = rng.choice([3, 6, 7, 9, 11])
            code = [0x66, 0x41 if base >= 8 else None, 0x0F, 0x3A, op, ((rng.randrange(8)) << 3) | (base & 7)]
            code = [b for b in code if b is not None] + imm()
            add(code, f"{nm}.m", vals=vals, ptrs={base: rng.randrange(16, WIN - 48)}, strings=True)
        for k in range(8):
            w = rng.randrange(2) if ex else 0
            add(vrr(rng, op, x(), 0, x(), 0, 1, mmmmm=3, w=w) + imm(), f"v{nm}.rr", vals=vals, strings=True)
    # ---- AES, PCLMULQDQ
    for op, nm in ((0xDB, "aesimc"), (0xDC, "aesenc"), (0xDD, "aesenclast"), (0xDE, "aesdec"), (0xDF, "aesdeclast")):
        for _ in range(3):
            add(leg_rr(1, op, x(), x(), map3=2), nm + ".rr")
        c, p, s = leg_mem(rng, 1, op, x(), 16, map3=2)
        add(c, nm + ".m", ptrs=p, smalls=s)
        add(vrr(rng, op, x(), 0 if op == 0xDB else x(), x(), 0, 1, mmmmm=2), "v" + nm + ".rr")
        c, p, s = vmem(rng, op, x(), 0 if op == 0xDB else x(), 0, 1, 1, mmmmm=2)
        add(c, "v" + nm + ".m", ptrs=p, smalls=s)
    for _ in range(4):
        add(leg_rr(1, 0xDF, x(), x(), map3=3) + imm(), "aeskeygenassist.rr")
    add(vrr(rng, 0xDF, x(), 0, x(), 0, 1, mmmmm=3) + imm(), "vaeskeygenassist.rr")
    for k in (0x00, 0x01, 0x10, 0x11, 0xFF):
        add(leg_rr(1, 0x44, x(), x(), map3=3) + [k], "pclmulqdq.rr")
        add(vrr(rng, 0x44, x(), x(), x(), 0, 1, mmmmm=3) + [k], "vpclmulqdq.rr")
    c, p, s = leg_mem(rng, 1, 0x44, x(), 16, map3=3)
    add(c + imm(), "pclmulqdq.m", ptrs=p, smalls=s)
    # ---- SHA (no prefix, legacy only); own generator, so the forms above keep their encodings
    srng = random.Random(0x5A4)
    sx = lambda: srng.randrange(16)  # noqa: E731
    for op, nm in ((0xC8, "sha1nexte"), (0xC9, "sha1msg1"), (0xCA, "sha1msg2"), (0xCB, "sha256rnds2"),
                   (0xCC, "sha256msg1"), (0xCD, "sha256msg2")):
        for _ in range(6):
            add(leg_rr(0, op, sx(), sx(), map3=2), nm + ".rr")
        for _ in range(2):
            c, p, s = leg_mem(srng, 0, op, sx(), 16, map3=2)
            add(c, nm + ".m", ptrs=p, smalls=s)
    for k in range(4):
        for _ in range(4):
            add(leg_rr(0, 0xCC, sx(), sx(), map3=3) + [k | (srng.getrandbits(6) << 2)], "sha1rnds4.rr")
    c, p, s = leg_mem(srng, 0, 0xCC, sx(), 16, map3=3)
    add(c + [srng.randrange(256)], "sha1rnds4.m", ptrs=p, smalls=s)
    return forms


def str_vec(rng):
    """32 bytes of string data: a small alphabet, zeros now and then."""
    alpha = rng.choice([b"ab", b"abc\x00", b"aAzZ09", bytes([0x80, 0x7F, 0xFF, 0x01, 0x00]), b"abcdefgh"])
    b = bytearray(rng.choice(alpha) for _ in range(32))
    if rng.random() < 0.5:  # no zero at all in the first 16 bytes now and then
        for i in range(16):
            if b[i] == 0:
                b[i] = alpha[0] or 0x61
    return [int.from_bytes(bytes(b[i:i + 8]), "little") for i in range(0, 32, 8)]


def int_vec(rng):
    return [rng.getrandbits(64) for _ in range(4)]


def case_inputs(seed, strings):
    rng = random.Random(seed)
    ymm = [str_vec(rng) if strings else int_vec(rng) for _ in range(16)]
    if strings and rng.random() < 0.5:  # two equal-ish strings
        a, b = rng.randrange(16), rng.randrange(16)
        ymm[a] = list(ymm[b])
    win = []
    for _ in range(WIN // 32):
        win += str_vec(rng) if strings else int_vec(rng)
    return ymm, win


def make_cases(forms, rng, per_form=8):
    cases = []
    for f in forms:
        for _ in range(getattr(f, "cases", per_form)):
            regs = [rand_val(rng) for _ in range(16)]
            regs[RSP] = 0x80
            for r, chooser in f.vals.items():
                regs[r] = chooser(rng) & M64
            for r, off in f.ptrs.items():
                regs[r] = off
            for r, (lo, hi) in f.smalls.items():
                regs[r] = rng.randint(lo, hi)
            seed = rng.getrandbits(63)
            ymm, win = case_inputs(seed, f.strings)
            cases.append({"name": f.name, "code": f.code.hex(), "regs": regs, "ptrs": sorted(f.ptrs) + [RSP],
                          "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "ymm": ymm, "win": win, "mx": 0x1F80,
                          "seed": seed, "ew": 1, "ints": int(f.strings), "flm": "%x" % f.flm})
    return cases


def main():
    rng = random.Random(0xE475001)
    cases = make_cases(gen_forms(rng), rng)
    run_native(cases, "tests/golden/gen_ext_vectors.py", OUT, mem_writes=True)


if __name__ == "__main__":
    main()
