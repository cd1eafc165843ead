#!/usr/bin/env python3
"""Native-execution golden vectors for FMA3, F16C and the AVX2 gathers
(convention U46; wtf_amd/csrc/engine_avx2x.h, oracle/x86_oracle_avx2x.inc).

The machinery of gen_fp_vectors.py (16 GPRs, RFLAGS, the 16 YMM registers,
MXCSR in and out, a 256-byte window with memory writes recorded, unmasked
exceptions trapping natively):

  * FMA3: the 30 opcodes (132 / 213 / 231 orders of fmadd / fmsub / fnmadd /
    fnmsub, packed and scalar, fmaddsub / fmsubadd), VEX.W 0 and 1, L 0 and 1,
    register and memory forms. Values from gen_fp_vectors.fp_value (zeros,
    infinities, NaNs, denormals, range ends, ties, tiny and huge exponents);
    in half of the register-form cases some elements get an addend equal to
    the negated rounded product, so the fused result is the product's
    rounding error (what a separate multiply and add would lose).
  * F16C: vcvtph2ps (register and memory sources; binary16 inputs with every
    class: NaNs, denormals, infinities) and vcvtps2ph (register and memory
    destinations, every imm8 rounding selection), L 0 and 1.
  * gathers: vpgatherdd / dq / qd / qq and vgatherdps / dpd / qps / qpd, L 0
    and 1, base + index * scale + disp8 with the four scales, indices
    (negative ones included) that keep every element inside the window, and
    random mask sign bits (elements with the sign clear keep the
    destination's value).

A case's YMM registers are case_inputs(seed, ew, kind) with the case's
"yset" overrides ([qword index, value]) applied on top.

Output: tests/golden/avx2x_vectors.json.gz. Re-run with
    python tests/golden/gen_avx2x_vectors.py
"""
import os
import random
import struct
import sys
from fractions import Fraction

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.gen_avx_vectors import vex_prefix  # noqa: E402
from tests.golden.gen_fp_vectors import Form, fp_value, fp_vec, rand_mx, run_native  # noqa: E402
from tests.golden.gen_native_vectors import WIN, rand_val  # noqa: E402
from tests.golden.gen_sse_vectors import enc_mem  # noqa: E402

OUT = os.path.join(HERE, "avx2x_vectors.json.gz")
RSP = 4
M64 = (1 << 64) - 1
FMA_KIND = {6: "fmaddsub", 7: "fmsubadd", 8: "fmadd", 9: "fmadd", 0xA: "fmsub", 0xB: "fmsub", 0xC: "fnmadd",
            0xD: "fnmadd", 0xE: "fnmsub", 0xF: "fnmsub"}


class AForm(Form):
    def __init__(self, code, name, ew, kind, ptrs=(), smalls=(), regs=None, gather=None):
        super().__init__(code, name, ew, ptrs, smalls)
        self.kind = kind        # "fma", "f16", "gather"
        self.regs = regs        # fma register forms: (A, B, C) registers of a * b + c
        self.gather = gather    # (dst, index, mask, base, disp, scale, ew, iw, n)


def vrr2(rng, opc, reg, vvvv, rm, l, w, mmmmm=2):
    return vex_prefix(rng, reg, 0, rm, mmmmm, w, vvvv, l, 1) + [opc, 0xC0 | ((reg & 7) << 3) | (rm & 7)]


def vmem2(rng, opc, reg, vvvv, l, w, mmmmm=2):
    """A VEX memory form (enc_mem's addressing), map 0f 38 / 0f 3a, pp 66."""
    code, p, s = enc_mem(rng, [], 0x0F, reg & 7, 1)
    i, rex = 0, 0
    if 0x40 <= code[0] <= 0x4F:
        rex, i = code[0], 1
    rest = code[i + 2:]
    return vex_prefix(rng, reg, 8 if rex & 2 else 0, 8 if rex & 1 else 0, mmmmm, w, vvvv, l, 1) + [opc] + rest, p, s


def gen_forms(rng):
    forms = []
    x = lambda: rng.randrange(16)  # noqa: E731
    # ---- FMA3
    for hi in (0x90, 0xA0, 0xB0):
        for lo in range(6, 16):
            op = hi | lo
            scalar = lo in (9, 0xB, 0xD, 0xF)
            for w in (0, 1):
                ew = 8 if w else 4
                order = {9: "132", 10: "213", 11: "231"}[op >> 4]
                nm = f"v{FMA_KIND[lo]}{order}{'s' if scalar else 'p'}{'d' if w else 's'}"
                for l in ((0,) if scalar else (0, 1)):
                    for _ in range(3):
                        d, v, r = x(), x(), x()
                        order = op >> 4
                        abc = (d, r, v) if order == 9 else (v, d, r) if order == 10 else (v, r, d)
                        forms.append(AForm(vrr2(rng, op, d, v, r, l, w), f"{nm}.L{l}.rr", ew, "fma", regs=abc))
                    c, p, s = vmem2(rng, op, x(), x(), l, w)
                    forms.append(AForm(c, f"{nm}.L{l}.m", ew, "fma", p, s))
    # ---- F16C
    for l in (0, 1):
        for _ in range(4):
            forms.append(AForm(vrr2(rng, 0x13, x(), 0, x(), l, 0), f"vcvtph2ps.L{l}.rr", 2, "f16"))
        for _ in range(2):
            c, p, s = vmem2(rng, 0x13, x(), 0, l, 0)
            forms.append(AForm(c, f"vcvtph2ps.L{l}.m", 2, "f16", p, s))
        for imm in range(8):
            forms.append(AForm(vrr2(rng, 0x1D, x(), 0, x(), l, 0, mmmmm=3) + [imm], f"vcvtps2ph.L{l}.i{imm}.rr", 4,
                               "f16"))
            c, p, s = vmem2(rng, 0x1D, x(), 0, l, 0, mmmmm=3)
            forms.append(AForm(c + [imm], f"vcvtps2ph.L{l}.i{imm}.m", 4, "f16", p, s))
    # ---- gathers: c4 <R X B map=2> <W vvvv L 01> op modrm(mod 1, rm 100) sib disp8
    names = {(0x90, 0): "vpgatherdd", (0x90, 1): "vpgatherdq", (0x91, 0): "vpgatherqd", (0x91, 1): "vpgatherqq",
             (0x92, 0): "vgatherdps", (0x92, 1): "vgatherdpd", (0x93, 0): "vgatherqps", (0x93, 1): "vgatherqpd"}
    for (op, w), nm in names.items():
        for l in (0, 1):
            for _ in range(6):
                dst, idx, msk = rng.sample(range(16), 3)
                base = rng.choice([r for r in range(16) if r != RSP])
                scale = rng.randrange(4)
                disp = rng.randrange(0, 16)
                ew, iw = (8 if w else 4), (8 if op & 1 else 4)
                n = (32 if l else 16) // max(ew, iw)
                b1 = (((dst >> 3) ^ 1) << 7) | (((idx >> 3) ^ 1) << 6) | (((base >> 3) ^ 1) << 5) | 2
                b2 = (w << 7) | ((~msk & 15) << 3) | (l << 2) | 1
                code = [0xC4, b1, b2, op, 0x44 | ((dst & 7) << 3), (scale << 6) | ((idx & 7) << 3) | (base & 7), disp]
                forms.append(AForm(code, f"{nm}.L{l}.s{1 << scale}", ew, "gather", ptrs={base: 128 - disp},
                                   gather=(dst, idx, msk, base, disp, scale, ew, iw, n)))
    return forms


# ---- values
def half_value(rng):
    s = 0x8000 if rng.random() < 0.5 else 0
    r = rng.random()
    if r < 0.08:
        return s
    if r < 0.14:
        return s | 0x7C00
    if r < 0.20:
        return s | 0x7E00 | rng.getrandbits(9)
    if r < 0.26:
        return s | 0x7C00 | (rng.getrandbits(9) or 1)
    if r < 0.40:
        return s | (rng.getrandbits(10) or 1)
    return s | (rng.randrange(1, 31) << 10) | rng.getrandbits(10)


def half_vec(rng):
    els = [half_value(rng) for _ in range(16)]
    raw = b"".join(v.to_bytes(2, "little") for v in els)
    return [int.from_bytes(raw[i:i + 8], "little") for i in range(0, 32, 8)]


def to_half_edges(rng):
    """binary32 values around binary16's range: overflow, denormal results, ties."""
    s = 1 << 31 if rng.random() < 0.5 else 0
    r = rng.random()
    if r < 0.5:
        return fp_value(rng, 4)
    if r < 0.65:  # binary16 denormal range: 2^-25 .. 2^-14
        return s | (rng.randrange(101, 114) << 23) | rng.getrandbits(23)
    if r < 0.8:  # around 65504 / 65520
        return s | (rng.choice([142, 143]) << 23) | rng.choice([0x7FE000, 0x7FF000, 0x7FEFFF, 0x7FF001, rng.getrandbits(23)])
    # ties and near-ties at binary16 precision
    return s | (rng.randrange(112, 140) << 23) | (rng.getrandbits(10) << 13) | rng.choice([0x1000, 0xFFF, 0x1001, 0])


def f32_vec_from(rng, chooser):
    raw = b"".join(chooser(rng).to_bytes(4, "little") for _ in range(8))
    return [int.from_bytes(raw[i:i + 8], "little") for i in range(0, 32, 8)]


def case_inputs(seed, ew, kind):
    """The 16 YMM registers (4 u64 each) and the window (32 u64) of a case, from its seed."""
    rng = random.Random(seed)
    if kind == "f16" and ew == 2:
        ymm = [half_vec(rng) for _ in range(16)]
        win = [v for _ in range(WIN // 32) for v in half_vec(rng)]
    elif kind == "f16":
        ymm = [f32_vec_from(rng, to_half_edges) for _ in range(16)]
        win = [v for _ in range(WIN // 32) for v in f32_vec_from(rng, to_half_edges)]
    elif kind == "gather":
        ymm = [[rng.getrandbits(64) for _ in range(4)] for _ in range(16)]
        win = [rng.getrandbits(64) for _ in range(WIN // 8)]
    else:
        ymm = [fp_vec(rng, ew) for _ in range(16)]
        win = [v for _ in range(WIN // 32) for v in fp_vec(rng, ew)]
    return ymm, win


def elems(ymm_reg, ew):
    raw = b"".join(v.to_bytes(8, "little") for v in ymm_reg)
    return [int.from_bytes(raw[i:i + ew], "little") for i in range(0, 32, ew)]


def qwords(els, ew):
    raw = b"".join(v.to_bytes(ew, "little") for v in els)
    return [int.from_bytes(raw[i:i + 8], "little") for i in range(0, 32, 8)]


def neg_rounded_product(a, b, ew):
    """-(a * b) rounded to the format (nearest even), or None if not finite / normal enough."""
    if ew == 4:
        fa, fb = struct.unpack("<f", struct.pack("<I", a))[0], struct.unpack("<f", struct.pack("<I", b))[0]
        p = fa * fb  # exact in binary64
        try:
            r = struct.unpack("<I", struct.pack("<f", -p))[0]
        except OverflowError:
            return None
    else:
        fa, fb = struct.unpack("<d", struct.pack("<Q", a))[0], struct.unpack("<d", struct.pack("<Q", b))[0]
        if fa != fa or fb != fb or abs(fa) == float("inf") or abs(fb) == float("inf"):
            return None
        try:
            p = float(Fraction(fa) * Fraction(fb))
        except OverflowError:
            return None
        r = struct.unpack("<Q", struct.pack("<d", -p))[0]
    return r


def make_cases(forms, rng, per_form=7):
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
            ymm, win = case_inputs(seed, f.ew, f.kind)
            yset = []
            if f.kind == "fma" and f.regs and rng.random() < 0.5:  # cancellations: c := -round(a * b)
                A, B, C = f.regs
                if len({A, B, C}) == 3:
                    ea, eb, ec = elems(ymm[A], f.ew), elems(ymm[B], f.ew), elems(ymm[C], f.ew)
                    for i in range(len(ec)):
                        if rng.random() < 0.6:
                            v = neg_rounded_product(ea[i], eb[i], f.ew)
                            if v is not None:
                                ec[i] = v
                    q = qwords(ec, f.ew)
                    yset += [[4 * C + k, q[k]] for k in range(4) if q[k] != ymm[C][k]]
            if f.kind == "gather":
                dst, idx, msk, base, disp, scale, ew, iw, n = f.gather
                lo = -(128 >> scale)  # element address = window + 128 + index * 2^scale
                hi = (128 - ew) >> scale
                iv = elems(ymm[idx], iw)
                for j in range(n):
                    v = rng.randint(lo, hi)
                    iv[j] = v & ((1 << (8 * iw)) - 1)
                mv = elems(ymm[msk], ew)
                for j in range(len(mv)):
                    sign = 1 << (8 * ew - 1)
                    mv[j] = (mv[j] | sign) if rng.random() < 0.7 else (mv[j] & ~sign)
                for reg, els, w in ((idx, iv, iw), (msk, mv, ew)):
                    q = qwords(els, w)
                    yset += [[4 * reg + k, q[k]] for k in range(4) if q[k] != ymm[reg][k]]
            for i, v in yset:
                ymm[i // 4][i % 4] = v
            mx = rand_mx(rng) if f.kind != "gather" else 0x1F80
            cases.append({"name": f.name, "code": bytes(f.code).hex(), "regs": regs, "ptrs": sorted(f.ptrs) + [RSP],
                          "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "ymm": ymm, "win": win, "mx": mx,
                          "seed": seed, "ew": f.ew, "ints": 0, "kind": f.kind,
                          "yset": [[i, "%x" % v] for i, v in yset]})
    return cases


def main():
    rng = random.Random(0xA2F16)
    cases = make_cases(gen_forms(rng), rng)
    run_native(cases, "tests/golden/gen_avx2x_vectors.py", OUT, mem_writes=True)


if __name__ == "__main__":
    main()
