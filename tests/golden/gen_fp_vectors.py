#!/usr/bin/env python3
"""Native-execution golden vectors for the SSE / AVX floating-point forms
(conventions U39 / U40; wtf_amd/csrc/engine_ssefp.h, oracle/x86_oracle_fp.inc).

As gen_avx_vectors.py (16 GPRs, RFLAGS, the 16 YMM registers at 256 bits, a
256-byte memory window), plus MXCSR in and out. Register and window contents
are floating-point values chosen to reach every rule: zeros, infinities, quiet
and signalling NaNs, denormals, the normal range's ends, halfway cases for the
rounding modes, near-cancellations, integer-conversion edges. MXCSR varies the
rounding control, DAZ, FTZ, the sticky flags and, for one case in six, the
exception masks: an unmasked exception traps natively (SIGFPE, caught on an
alternate stack) and the vector records the MXCSR at the trap instead of the
results. Legacy and VEX (128 / 256) encodings, register and memory forms.

Output: tests/golden/fp_vectors.json.gz. Re-run with
    python tests/golden/gen_fp_vectors.py
"""
import gzip
import json
import os
import random
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.gen_avx_vectors import YLOAD, YSTORE, vmem, vrr  # noqa: E402
from tests.golden.gen_native_vectors import WIN, rand_val  # noqa: E402
from tests.golden.gen_sse_vectors import enc_mem  # noqa: E402

OUT = os.path.join(HERE, "fp_vectors.json.gz")
RSP = 4
PFX = {0: [], 1: [0x66], 2: [0xF3], 3: [0xF2]}
ARITH = {0x51: "sqrt", 0x58: "add", 0x59: "mul", 0x5C: "sub", 0x5D: "min", 0x5E: "div", 0x5F: "max"}
SUF = {0: "ps", 1: "pd", 2: "ss", 3: "sd"}


class Form:
    def __init__(self, code, name, ew, ptrs=(), smalls=(), ints=False):
        self.code = bytes(code)
        self.name = name
        self.ew = ew  # element width of the values (4 / 8)
        self.ptrs = dict(ptrs)
        self.smalls = dict(smalls)
        self.ints = ints  # sources are integers (cvtdq2ps, cvtdq2pd)
        self.cls = "sse"  # tests/progfuzz.py's block kind


def leg_rr(pp, op, reg, rm, w=0, map3=None):
    rex = 0x40 | (w << 3) | ((reg >> 3) << 2) | (rm >> 3)
    esc = [0x0F] + ([0x38] if map3 == 2 else [0x3A] if map3 == 3 else [])
    return PFX[pp] + ([rex] if rex != 0x40 else []) + esc + [op, 0xC0 | ((reg & 7) << 3) | (rm & 7)]


def leg_mem(rng, pp, op, reg, align, w=0, map3=None):
    code, p, s = enc_mem(rng, PFX[pp], 0x0F, reg, align, w)  # ... 0f 0f modrm ...: splice the opcode in
    k = code.index(0x0F)
    esc = [0x38] if map3 == 2 else [0x3A] if map3 == 3 else []
    return code[:k + 1] + esc + [op] + code[k + 2:], p, s


def gen_forms(rng):
    forms = []
    x = lambda: rng.randrange(16)  # noqa: E731
    g = lambda: rng.choice([r for r in range(16) if r != RSP])  # noqa: E731

    def both(name, ew, rr_fn, mem_fn, n_rr=2, n_m=1, ints=False, imm=None):
        for _ in range(n_rr):
            c = rr_fn()
            forms.append(Form(c + ([imm()] if imm else []), name + ".rr", ew, ints=ints))
        for _ in range(n_m):
            c, p, s = mem_fn()
            forms.append(Form(c + ([imm()] if imm else []), name + ".m", ew, p, s, ints=ints))

    # ---- legacy
    for op, nm in ARITH.items():
        for pp in range(4):
            al = 16 if pp <= 1 else 1
            both(f"{nm}{SUF[pp]}", 8 if pp & 1 else 4, lambda: leg_rr(pp, op, x(), x()),
                 lambda: leg_mem(rng, pp, op, x(), al), n_rr=3)
    for pp in range(4):
        al = 16 if pp <= 1 else 1
        both(f"cmp{SUF[pp]}", 8 if pp & 1 else 4, lambda: leg_rr(pp, 0xC2, x(), x()),
             lambda: leg_mem(rng, pp, 0xC2, x(), al), n_rr=4, n_m=2, imm=lambda: rng.randrange(8))
    for pp in (0, 1):
        for op in (0x2E, 0x2F):
            both(("comis" if op == 0x2F else "ucomis") + ("d" if pp else "s"), 8 if pp else 4, lambda: leg_rr(pp, op, x(), x()),
                 lambda: leg_mem(rng, pp, op, x(), 1), n_rr=3)
    both("cvtps2pd", 4, lambda: leg_rr(0, 0x5A, x(), x()), lambda: leg_mem(rng, 0, 0x5A, x(), 1))
    both("cvtpd2ps", 8, lambda: leg_rr(1, 0x5A, x(), x()), lambda: leg_mem(rng, 1, 0x5A, x(), 16))
    both("cvtss2sd", 4, lambda: leg_rr(2, 0x5A, x(), x()), lambda: leg_mem(rng, 2, 0x5A, x(), 1))
    both("cvtsd2ss", 8, lambda: leg_rr(3, 0x5A, x(), x()), lambda: leg_mem(rng, 3, 0x5A, x(), 1), n_rr=3)
    both("cvtdq2ps", 4, lambda: leg_rr(0, 0x5B, x(), x()), lambda: leg_mem(rng, 0, 0x5B, x(), 16), ints=True)
    both("cvtps2dq", 4, lambda: leg_rr(1, 0x5B, x(), x()), lambda: leg_mem(rng, 1, 0x5B, x(), 16), n_rr=3)
    both("cvttps2dq", 4, lambda: leg_rr(2, 0x5B, x(), x()), lambda: leg_mem(rng, 2, 0x5B, x(), 16))
    both("cvttpd2dq", 8, lambda: leg_rr(1, 0xE6, x(), x()), lambda: leg_mem(rng, 1, 0xE6, x(), 16))
    both("cvtdq2pd", 4, lambda: leg_rr(2, 0xE6, x(), x()), lambda: leg_mem(rng, 2, 0xE6, x(), 1), ints=True)
    both("cvtpd2dq", 8, lambda: leg_rr(3, 0xE6, x(), x()), lambda: leg_mem(rng, 3, 0xE6, x(), 16), n_rr=3)
    for w in (0, 1):
        for pp in (2, 3):
            both(f"cvtsi2s{SUF[pp][1]}.w{w}", 4 if w == 0 else 8, lambda: leg_rr(pp, 0x2A, x(), g(), w),
                 lambda: leg_mem(rng, pp, 0x2A, x(), 1, w), ints=True)
            for op in (0x2C, 0x2D):
                both(f"cvt{'t' if op == 0x2C else ''}s{SUF[pp][1]}2si.w{w}", 8 if pp == 3 else 4,
                     lambda: leg_rr(pp, op, g(), x(), w), lambda: leg_mem(rng, pp, op, g(), 1, w), n_rr=3)
    for op, nm in ((0x7C, "hadd"), (0x7D, "hsub"), (0xD0, "addsub")):
        for pp in (1, 3):
            both(nm + ("pd" if pp == 1 else "ps"), 8 if pp == 1 else 4, lambda: leg_rr(pp, op, x(), x()),
                 lambda: leg_mem(rng, pp, op, x(), 16))
    both("movsldup", 4, lambda: leg_rr(2, 0x12, x(), x()), lambda: leg_mem(rng, 2, 0x12, x(), 16))
    both("movshdup", 4, lambda: leg_rr(2, 0x16, x(), x()), lambda: leg_mem(rng, 2, 0x16, x(), 16))
    both("movddup", 8, lambda: leg_rr(3, 0x12, x(), x()), lambda: leg_mem(rng, 3, 0x12, x(), 1))
    for _ in range(2):
        c, p, s = leg_mem(rng, 3, 0xF0, x(), 1)
        forms.append(Form(c, "lddqu.m", 4, p, s))
    for op, nm, ew in ((0x08, "roundps", 4), (0x09, "roundpd", 8), (0x0A, "roundss", 4), (0x0B, "roundsd", 8)):
        al = 16 if op <= 0x09 else 1
        both(nm, ew, lambda: leg_rr(1, op, x(), x(), map3=3), lambda: leg_mem(rng, 1, op, x(), al, map3=3),
             n_rr=4, n_m=2, imm=lambda: rng.randrange(16))
    for op, nm, ew in ((0x0C, "blendps", 4), (0x0D, "blendpd", 8)):
        both(nm, ew, lambda: leg_rr(1, op, x(), x(), map3=3), lambda: leg_mem(rng, 1, op, x(), 16, map3=3),
             imm=lambda: rng.randrange(256))
    for op, nm, ew in ((0x14, "blendvps", 4), (0x15, "blendvpd", 8)):
        both(nm, ew, lambda: leg_rr(1, op, x(), x(), map3=2), lambda: leg_mem(rng, 1, op, x(), 16, map3=2))
    # ---- VEX
    for op, nm in ARITH.items():
        for pp in range(4):
            ew = 8 if pp & 1 else 4
            for l in ((0, 1) if pp <= 1 else (rng.randrange(2),)):
                vv = lambda: 0 if (op == 0x51 and pp <= 1) else x()  # noqa: E731
                both(f"v{nm}{SUF[pp]}.L{l}", ew, lambda: vrr(rng, op, x(), vv(), x(), l, pp),
                     lambda: vmem(rng, op, x(), vv(), l, pp, 1))
    for pp in range(4):
        for l in ((0, 1) if pp <= 1 else (0,)):
            both(f"vcmp{SUF[pp]}.L{l}", 8 if pp & 1 else 4, lambda: vrr(rng, 0xC2, x(), x(), x(), l, pp),
                 lambda: vmem(rng, 0xC2, x(), x(), l, pp, 1), n_rr=4, n_m=2, imm=lambda: rng.randrange(32))
    for pp in (0, 1):
        for op in (0x2E, 0x2F):
            both(f"v{'c' if op == 0x2F else 'u'}omis{'d' if pp else 's'}", 8 if pp else 4,
                 lambda: vrr(rng, op, x(), 0, x(), 0, pp), lambda: vmem(rng, op, x(), 0, 0, pp, 1))
    for l in (0, 1):
        both(f"vcvtps2pd.L{l}", 4, lambda: vrr(rng, 0x5A, x(), 0, x(), l, 0), lambda: vmem(rng, 0x5A, x(), 0, l, 0, 1))
        both(f"vcvtpd2ps.L{l}", 8, lambda: vrr(rng, 0x5A, x(), 0, x(), l, 1), lambda: vmem(rng, 0x5A, x(), 0, l, 1, 1))
        for pp, nm in ((0, "vcvtdq2ps"), (1, "vcvtps2dq"), (2, "vcvttps2dq")):
            both(f"{nm}.L{l}", 4, lambda: vrr(rng, 0x5B, x(), 0, x(), l, pp), lambda: vmem(rng, 0x5B, x(), 0, l, pp, 1),
                 ints=pp == 0)
        for pp, nm, ew in ((1, "vcvttpd2dq", 8), (2, "vcvtdq2pd", 4), (3, "vcvtpd2dq", 8)):
            both(f"{nm}.L{l}", ew, lambda: vrr(rng, 0xE6, x(), 0, x(), l, pp),
                 lambda: vmem(rng, 0xE6, x(), 0, l, pp, 1), ints=pp == 2)
        for op, nm in ((0x7C, "vhadd"), (0x7D, "vhsub"), (0xD0, "vaddsub")):
            for pp in (1, 3):
                both(f"{nm}{'pd' if pp == 1 else 'ps'}.L{l}", 8 if pp == 1 else 4,
                     lambda: vrr(rng, op, x(), x(), x(), l, pp), lambda: vmem(rng, op, x(), x(), l, pp, 1), n_rr=1)
        for pp, op, nm, ew in ((2, 0x12, "vmovsldup", 4), (2, 0x16, "vmovshdup", 4), (3, 0x12, "vmovddup", 8)):
            both(f"{nm}.L{l}", ew, lambda: vrr(rng, op, x(), 0, x(), l, pp), lambda: vmem(rng, op, x(), 0, l, pp, 1),
                 n_rr=1)
        c, p, s = vmem(rng, 0xF0, x(), 0, l, 3, 1)
        forms.append(Form(c, f"vlddqu.L{l}.m", 4, p, s))
        for op, nm, ew in ((0x08, "vroundps", 4), (0x09, "vroundpd", 8), (0x0C, "vblendps", 4), (0x0D, "vblendpd", 8)):
            vv = (lambda: 0) if op <= 0x09 else x
            both(f"{nm}.L{l}", ew, lambda: vrr(rng, op, x(), vv(), x(), l, 1, mmmmm=3),
                 lambda: vmem(rng, op, x(), vv(), l, 1, 1, mmmmm=3), imm=lambda: rng.randrange(256 if op >= 0x0C else 16))
        for op, nm, ew in ((0x4A, "vblendvps", 4), (0x4B, "vblendvpd", 8)):
            both(f"{nm}.L{l}", ew, lambda: vrr(rng, op, x(), x(), x(), l, 1, mmmmm=3),
                 lambda: vmem(rng, op, x(), x(), l, 1, 1, mmmmm=3), imm=lambda: x() << 4)
    for op, nm, ew in ((0x0A, "vroundss", 4), (0x0B, "vroundsd", 8)):
        both(nm, ew, lambda: vrr(rng, op, x(), x(), x(), 0, 1, mmmmm=3), lambda: vmem(rng, op, x(), x(), 0, 1, 1, mmmmm=3),
             imm=lambda: rng.randrange(16))
    for pp in (2, 3):
        both(f"vcvts{SUF[pp][1]}2s{'d' if pp == 2 else 's'}", 4 if pp == 2 else 8,
             lambda: vrr(rng, 0x5A, x(), x(), x(), 0, pp), lambda: vmem(rng, 0x5A, x(), x(), 0, pp, 1))
        for w in (0, 1):
            both(f"vcvtsi2s{SUF[pp][1]}.w{w}", 4 if w == 0 else 8, lambda: vrr(rng, 0x2A, x(), x(), g(), 0, pp, w=w),
                 lambda: vmem(rng, 0x2A, x(), x(), 0, pp, 1, w=w), ints=True)
            for op in (0x2C, 0x2D):
                both(f"v{'t' if op == 0x2C else ''}cvts{SUF[pp][1]}2si.w{w}", 8 if pp == 3 else 4,
                     lambda: vrr(rng, op, g(), 0, x(), 0, pp, w=w), lambda: vmem(rng, op, g(), 0, 0, pp, 1, w=w))
    # ---- dpps / dppd, legacy and VEX (own generator: the forms above keep their encodings)
    drng = random.Random(0xD99)
    dx = lambda: drng.randrange(16)  # noqa: E731
    for op, nm, ew in ((0x40, "dpps", 4), (0x41, "dppd", 8)):
        for _ in range(6):
            forms.append(Form(leg_rr(1, op, dx(), dx(), map3=3) + [drng.randrange(256)], nm + ".rr", ew))
        for _ in range(2):
            c, p, s = leg_mem(drng, 1, op, dx(), 16, map3=3)
            forms.append(Form(c + [drng.randrange(256)], nm + ".m", ew, p, s))
        for l in ((0, 1) if op == 0x40 else (0,)):
            for _ in range(4):
                forms.append(Form(vrr(drng, op, dx(), dx(), dx(), l, 1, mmmmm=3) + [drng.randrange(256)],
                                  f"v{nm}.L{l}.rr", ew))
            c, p, s = vmem(drng, op, dx(), dx(), l, 1, 1, mmmmm=3)
            forms.append(Form(c + [drng.randrange(256)], f"v{nm}.L{l}.m", ew, p, s))
    # ---- rcpps / rcpss / rsqrtps / rsqrtss, legacy and VEX (own generator)
    rrng = random.Random(0x4C9)
    rx = lambda: rrng.randrange(16)  # noqa: E731
    for op, nm in ((0x53, "rcp"), (0x52, "rsqrt")):
        for pp, suf in ((0, "ps"), (2, "ss")):
            for _ in range(5):
                forms.append(Form(leg_rr(pp, op, rx(), rx()), f"{nm}{suf}.rr", 4))
            c, p, s = leg_mem(rrng, pp, op, rx(), 16 if pp == 0 else 1)
            forms.append(Form(c, f"{nm}{suf}.m", 4, p, s))
            for l in ((0, 1) if pp == 0 else (0,)):
                for _ in range(3):
                    forms.append(Form(vrr(rrng, op, rx(), 0 if pp == 0 else rx(), rx(), l, pp), f"v{nm}{suf}.L{l}.rr", 4))
                c, p, s = vmem(rrng, op, rx(), 0 if pp == 0 else rx(), l, pp, 1)
                forms.append(Form(c, f"v{nm}{suf}.L{l}.m", 4, p, s))
    return forms


# ---- values
def f32(v):
    return struct.unpack("<I", struct.pack("<f", v))[0]


def f64(v):
    return struct.unpack("<Q", struct.pack("<d", v))[0]


def fp_value(rng, ew):
    """One element of width ew: a special value or a structured random one."""
    F, E = (23, 8) if ew == 4 else (52, 11)
    emax, sb = (1 << E) - 1, 1 << (F + E)
    frac = lambda: rng.getrandbits(F)  # noqa: E731
    s = sb if rng.random() < 0.5 else 0
    r = rng.random()
    if r < 0.06:
        return s
    if r < 0.10:
        return s | (emax << F)
    if r < 0.14:  # quiet NaN (payload)
        return s | (emax << F) | (1 << (F - 1)) | rng.getrandbits(F - 1)
    if r < 0.17:  # signalling NaN
        return s | (emax << F) | (rng.getrandbits(F - 1) or 1)
    if r < 0.25:  # denormal
        return s | rng.choice([1, (1 << F) - 1, frac() or 1, 1 << (F - 1)])
    if r < 0.30:  # the normal range's ends
        return s | rng.choice([1 << F, ((emax - 1) << F) | ((1 << F) - 1), (1 << F) | frac(), ((emax - 1) << F) | frac()])
    if r < 0.42:  # small integers and halves (rounding ties, conversions)
        v = rng.choice([0.5, 1.5, 2.5, 3.5, -0.5, -2.5, 1.0, -1.0, 3.0, 7.0, 0.25, 0.75, 1e6 + 0.5])
        v = v if rng.random() < 0.7 else v * rng.choice([1, -1]) + rng.randrange(-100, 100)
        return f32(v) if ew == 4 else f64(v)
    if r < 0.50:  # integer-conversion edges: around 2^31, 2^63
        v = rng.choice([2.0 ** 31, 2.0 ** 31 - 1, -2.0 ** 31, -2.0 ** 31 - 1, 2.0 ** 63, -2.0 ** 63, 2.0 ** 32, 2.0 ** 62])
        try:
            return f32(v) if ew == 4 else f64(v)
        except OverflowError:
            return s
    if r < 0.58:  # tiny results: exponents near the bottom of the range
        return s | (rng.randrange(1, 40) << F) | frac()
    if r < 0.64:  # huge: near the top
        return s | (rng.randrange(emax - 40, emax) << F) | frac()
    # a moderate exponent
    bias = emax >> 1
    return s | (rng.randrange(bias - 30, bias + 30) << F) | frac()


def fp_vec(rng, ew, ints=False):
    """256 bits as 4 u64 of elements of width ew."""
    els = []
    for _ in range(32 // ew):
        if ints:
            v = rng.choice([0, 1, 0xFFFFFFFF, 0x7FFFFFFF, 0x80000000, rng.getrandbits(32), rng.getrandbits(24),
                            rng.getrandbits(8), (1 << 24) + 1, 0xFFFFFF01])
        else:
            v = fp_value(rng, ew)
        els.append(v)
    raw = b"".join(v.to_bytes(ew, "little") for v in els)
    return [int.from_bytes(raw[i:i + 8], "little") for i in range(0, 32, 8)]


def near(rng, v, ew):
    """v's neighbour: same exponent, a few ulps away (cancellation cases)."""
    lst = list(struct.unpack("<" + ("I" if ew == 4 else "Q") * (32 // ew), b"".join(x.to_bytes(8, "little") for x in v)))
    out = [(e + rng.randrange(-3, 4)) & ((1 << (8 * ew)) - 1) for e in lst]
    raw = struct.pack("<" + ("I" if ew == 4 else "Q") * (32 // ew), *out)
    return [int.from_bytes(raw[i:i + 8], "little") for i in range(0, 32, 8)]


def case_inputs(seed, ew, ints):
    """The 16 YMM registers (4 u64 each) and the window (32 u64) of a case, from its seed."""
    rng = random.Random(seed)
    ymm = [fp_vec(rng, ew, ints and rng.random() < 0.8) for _ in range(16)]
    if rng.random() < 0.4:
        a, b = rng.randrange(16), rng.randrange(16)
        ymm[a] = near(rng, ymm[b], ew) if rng.random() < 0.7 else list(ymm[b])
    win = []
    for _ in range(WIN // 32):
        win += fp_vec(rng, ew, ints and rng.random() < 0.8)
    return ymm, win


def rand_mx(rng):
    mx = 0x1F80 | (rng.getrandbits(6) if rng.random() < 0.3 else 0)
    mx |= rng.randrange(4) << 13
    if rng.random() < 0.25:
        mx |= 0x40  # DAZ
    if rng.random() < 0.25:
        mx |= 0x8000  # FTZ
    if rng.random() < 0.17:  # some exceptions unmasked
        mx &= ~(rng.getrandbits(6) << 7)
    return mx


def make_cases(forms, rng, per_form=9):
    cases = []
    for f in forms:
        for _ in range(per_form):
            regs = [rand_val(rng) for _ in range(16)]
            regs[RSP] = 0x80
            for r, off in f.ptrs.items():
                regs[r] = off
            for r, (lo, hi) in f.smalls.items():
                regs[r] = rng.randint(lo, hi)
            if f.ints and rng.random() < 0.5:  # the general-register integer source
                for r in range(16):
                    if r != RSP and r not in f.ptrs and r not in f.smalls:
                        regs[r] = rng.choice([0, 1, -1 & (2**64 - 1), 2**63, 2**63 - 1, 2**31, 2**31 - 1,
                                              rng.getrandbits(64), rng.getrandbits(32), rng.getrandbits(54)])
            seed = rng.getrandbits(63)
            ymm, win = case_inputs(seed, f.ew, f.ints)
            cases.append({"name": f.name, "code": f.code.hex(), "regs": regs, "ptrs": sorted(f.ptrs) + [RSP],
                          "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "ymm": ymm, "win": win, "mx": rand_mx(rng),
                          "seed": seed, "ew": f.ew, "ints": int(f.ints)})
    return cases


C_HEADER = r"""
#define _GNU_SOURCE
#include <setjmp.h>
#include <signal.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <ucontext.h>
typedef struct { uint64_t r[16]; uint64_t fl; uint64_t y[64]; uint32_t mx, pad; } st_t;
st_t g_in, g_out;
uint64_t g_host_rsp;
uint32_t g_host_mx;
uint64_t g_flagstack[64] __attribute__((aligned(32)));
uint8_t g_buf[8192] __attribute__((aligned(4096)));
"""
STUB = r"""
__asm__(
".text\n.globl t_{i}\nt_{i}:\n"
"push %rbx\npush %rbp\npush %r12\npush %r13\npush %r14\npush %r15\n"
"mov %rsp, g_host_rsp(%rip)\n"
"stmxcsr g_host_mx(%rip)\n"
""" + YLOAD + r"""
"ldmxcsr g_in+648(%rip)\n"
"lea g_flagstack+256(%rip), %rsp\n"
"pushq g_in+128(%rip)\npopfq\n"
"mov g_in+0(%rip), %rax\nmov g_in+8(%rip), %rcx\nmov g_in+16(%rip), %rdx\nmov g_in+24(%rip), %rbx\n"
"mov g_in+40(%rip), %rbp\nmov g_in+48(%rip), %rsi\nmov g_in+56(%rip), %rdi\n"
"mov g_in+64(%rip), %r8\nmov g_in+72(%rip), %r9\nmov g_in+80(%rip), %r10\nmov g_in+88(%rip), %r11\n"
"mov g_in+96(%rip), %r12\nmov g_in+104(%rip), %r13\nmov g_in+112(%rip), %r14\nmov g_in+120(%rip), %r15\n"
"mov g_in+32(%rip), %rsp\n"
".byte {bytes}\n"
"mov %rax, g_out+0(%rip)\nmov %rcx, g_out+8(%rip)\nmov %rdx, g_out+16(%rip)\nmov %rbx, g_out+24(%rip)\n"
"mov %rsp, g_out+32(%rip)\nmov %rbp, g_out+40(%rip)\nmov %rsi, g_out+48(%rip)\nmov %rdi, g_out+56(%rip)\n"
"mov %r8, g_out+64(%rip)\nmov %r9, g_out+72(%rip)\nmov %r10, g_out+80(%rip)\nmov %r11, g_out+88(%rip)\n"
"mov %r12, g_out+96(%rip)\nmov %r13, g_out+104(%rip)\nmov %r14, g_out+112(%rip)\nmov %r15, g_out+120(%rip)\n"
"lea g_flagstack+256(%rip), %rsp\npushfq\npopq g_out+128(%rip)\n"
"stmxcsr g_out+648(%rip)\n"
""" + YSTORE + r"""
"ldmxcsr g_host_mx(%rip)\n"
"vzeroupper\n"
"mov g_host_rsp(%rip), %rsp\n"
"pop %r15\npop %r14\npop %r13\npop %r12\npop %rbp\npop %rbx\nret\n");
void t_{i}(void);
"""
C_MAIN = r"""
typedef void (*fn_t)(void);
static fn_t fns[] = { FNLIST };
static sigjmp_buf g_jb;
static volatile uint32_t g_trap_mx;
static void on_fpe(int sig, siginfo_t *si, void *uc) {
  (void)sig; (void)si;
  g_trap_mx = ((ucontext_t *)uc)->uc_mcontext.fpregs->mxcsr;
  siglongjmp(g_jb, 1);
}
static char g_altstack[65536];
int main(void) {
  int form, nptr, ptrs[16]; unsigned long long flags, mx, regs[16], ym[64], wv[32];
  uint8_t *win = g_buf + 0x800;
  stack_t ss = {.ss_sp = g_altstack, .ss_size = sizeof(g_altstack)};
  sigaltstack(&ss, 0);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_fpe;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK | SA_NODEFER;
  sigaction(SIGFPE, &sa, 0);
  printf("BUF %llx\n", (unsigned long long)(uintptr_t)win);
  while (scanf("%d %llx %llx", &form, &flags, &mx) == 3) {
    for (int i = 0; i < 16; i++) if (scanf("%llx", &regs[i]) != 1) return 1;
    for (int i = 0; i < 64; i++) if (scanf("%llx", &ym[i]) != 1) return 1;
    for (int i = 0; i < 32; i++) if (scanf("%llx", &wv[i]) != 1) return 1;
    if (scanf("%d", &nptr) != 1) return 1;
    for (int i = 0; i < nptr; i++) if (scanf("%d", &ptrs[i]) != 1) return 1;
    memcpy(win, wv, 256);
    for (int i = 0; i < 16; i++) g_in.r[i] = regs[i];
    for (int i = 0; i < nptr; i++) g_in.r[ptrs[i]] = (uint64_t)(uintptr_t)win + regs[ptrs[i]];
    for (int i = 0; i < 64; i++) g_in.y[i] = ym[i];
    g_in.fl = flags;
    g_in.mx = (uint32_t)mx;
    if (sigsetjmp(g_jb, 1)) {
      __asm__ volatile("ldmxcsr %0\n vzeroupper" : : "m"(g_host_mx));
      printf("T %x\n", g_trap_mx);
      continue;
    }
    fns[form]();
    printf("R");
    for (int i = 0; i < 16; i++) printf(" %llx", (unsigned long long)g_out.r[i]);
    printf(" %llx\nY", (unsigned long long)g_out.fl);
    for (int i = 0; i < 64; i++) printf(" %llx", (unsigned long long)g_out.y[i]);
    printf(" %x\nM", g_out.mx);
    for (int i = 0; i < 256; i++) printf("%02x", win[i]);
    printf("\n");
  }
  return 0;
}
"""


def run_native(cases, generator, out_path, mem_writes=False):
    """Every case natively (one stub per encoding); the document of inputs and
    results, written to out_path."""
    uniq = {}
    for c in cases:
        uniq.setdefault(c["code"], len(uniq))
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "fv.c")
        with open(src, "w") as f:
            f.write(C_HEADER)
            for code, i in uniq.items():
                bs = ",".join("0x%02x" % b for b in bytes.fromhex(code))
                f.write(STUB.replace("{i}", str(i)).replace("{bytes}", bs))
            f.write(C_MAIN.replace("FNLIST", ",".join(f"t_{i}" for i in range(len(uniq)))))
        exe = os.path.join(td, "fv")
        subprocess.check_call(["gcc", "-O1", "-no-pie", "-o", exe, src])
        lines = []
        for c in cases:
            ys = [v for r in c["ymm"] for v in r]
            lines.append("%d %x %x %s %s %s %d %s" % (
                uniq[c["code"]], c["flags"], c["mx"], " ".join("%x" % v for v in c["regs"]),
                " ".join("%x" % v for v in ys), " ".join("%x" % v for v in c["win"]), len(c["ptrs"]),
                " ".join(str(p) for p in c["ptrs"])))
        out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
    buf_va = int(out[0].split()[1], 16)
    res = []
    k = 1
    traps = 0
    for c in cases:
        inregs = list(c["regs"])
        for p in c["ptrs"]:
            inregs[p] = (buf_va + inregs[p]) & 0xFFFFFFFFFFFFFFFF
        yin = [v for r in c["ymm"] for v in r]
        # inputs: the GPRs, RFLAGS, MXCSR; YMM and window from (seed, ew, ints) by case_inputs
        e = {"name": c["name"], "code": c["code"], "in": ["%x" % v for v in inregs], "fl": "%x" % c["flags"],
             "mx": "%x" % c["mx"], "seed": "%x" % c["seed"], "ew": c["ew"], "ints": c["ints"]}
        if "flm" in c:  # the flags the SDM defines for this form (gen_ext_vectors.py)
            e["flm"] = c["flm"]
        for key in ("kind", "yset"):  # gen_avx2x_vectors.py: the input family and YMM overrides
            if key in c:
                e[key] = c[key]
        if out[k].startswith("T"):
            e["trap_mx"] = out[k].split()[1]
            traps += 1
            k += 1
        else:
            rl, yl, ml = out[k].split(), out[k + 1].split(), out[k + 2][1:]
            k += 3
            before = b"".join(v.to_bytes(8, "little") for v in c["win"])
            after = bytes.fromhex(ml)
            assert mem_writes or after == before, c["name"]  # no FP form writes memory
            yout = [int(v, 16) for v in yl[1:65]]
            gout = [int(v, 16) for v in rl[1:17]]
            # results as changes: (index, value) of the GPRs / YMM qwords that differ from the inputs
            e.update({"gdiff": [[i, "%x" % gout[i]] for i in range(16) if gout[i] != inregs[i]], "flo": rl[17],
                      "ydiff": [[i, "%x" % yout[i]] for i in range(64) if yout[i] != yin[i]], "mxo": yl[65]})
            if mem_writes:
                e["mdiff"] = [[i, after[i]] for i in range(WIN) if after[i] != before[i]]
        res.append(e)
    doc = {"buf_va": "%x" % buf_va, "window": WIN,
           "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "generator": generator, "cases": res}
    with gzip.open(out_path, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"wrote {len(res)} vectors ({len(uniq)} encodings, {traps} trapped) to {out_path}")


def main():
    rng = random.Random(0xF10A7001)
    forms = gen_forms(rng)
    run_native(make_cases(forms, rng), "tests/golden/gen_fp_vectors.py", OUT)


if __name__ == "__main__":
    main()
