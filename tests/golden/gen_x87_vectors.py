"""x87 arithmetic vectors (convention U42): random x87 states (TOP, tags,
control word, sticky flags, register contents of every class the x87 knows:
normals, denormals, pseudo-denormals, zeros, infinities, QNaN / SNaN,
unnormals and pseudo-NaN / infinities) under every non-control d8-df form,
the register forms and the memory forms on [rsi].

The expected results come from the host CPU: the oracle runs each form
natively (oracle/x86_oracle_x87.inc: FXRSTOR, the instruction, FXSAVE), so
the committed file pins the engine's integer extended-precision arithmetic
(wtf_amd/csrc/engine_x87.h) to hardware on the CPU suite and on the GPU.

    python -m tests.golden.gen_x87_vectors   # writes tests/golden/x87_vectors.json.gz
"""
from __future__ import annotations

import gzip
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "x87_vectors.json.gz")

UD_REG = {
    0xD9: lambda m: (0xD1 <= m <= 0xD7) or m in (0xE2, 0xE3, 0xE6, 0xE7, 0xEF),
    0xDA: lambda m: m >= 0xE0 and m != 0xE9,
    0xDB: lambda m: (0xE5 <= m <= 0xE7) or m >= 0xF8,
    0xDD: lambda m: m >= 0xF0,
    0xDE: lambda m: 0xD8 <= m <= 0xDF and m != 0xD9,
    0xDF: lambda m: (0xE1 <= m <= 0xE7) or m >= 0xF8,
}
UNIMPL_D9 = {0xF0, 0xF1, 0xF2, 0xF3, 0xF9, 0xFB, 0xFE, 0xFF}
CONTROL_REG = {(0xDB, 0xE2), (0xDB, 0xE3), (0xDF, 0xE0)}


def reg_forms():
    out = []
    for op in range(0xD8, 0xE0):
        for m in range(0xC0, 0x100):
            if (op, m) in CONTROL_REG or (op == 0xD9 and m in UNIMPL_D9):
                continue
            if op in UD_REG and UD_REG[op](m):
                continue
            out.append(bytes([op, m]))
    return out


# (op, /r) -> memory operand kind
MEM_KIND = {}
for r in range(8):
    MEM_KIND[(0xD8, r)] = "f32"
    MEM_KIND[(0xDC, r)] = "f64"
    MEM_KIND[(0xDA, r)] = "i32"
    MEM_KIND[(0xDE, r)] = "i16"
for r in (0, 2, 3):
    MEM_KIND[(0xD9, r)] = "f32"
    MEM_KIND[(0xDD, r)] = "f64"
for r in (0, 1, 2, 3):
    MEM_KIND[(0xDB, r)] = "i32"
    MEM_KIND[(0xDF, r)] = "i16"
MEM_KIND[(0xDD, 1)] = "i64"
MEM_KIND[(0xDB, 5)] = MEM_KIND[(0xDB, 7)] = "f80"
MEM_KIND[(0xDF, 5)] = MEM_KIND[(0xDF, 7)] = "i64"


def mem_forms():
    return [(bytes([op, (r << 3) | 6]), k) for (op, r), k in sorted(MEM_KIND.items())]


def rand_f80(rng):
    k = rng.random()
    s = rng.getrandbits(1) << 15
    if k < 0.42:
        e = rng.choice([rng.randint(0x3FFF - 70, 0x3FFF + 70), rng.randint(1, 0x7FFE), rng.randint(1, 40),
                        rng.randint(0x7FFE - 40, 0x7FFE), rng.randint(0x3FFF - 16445, 0x3FFF - 16300) & 0x7FFF or 1])
        m = (1 << 63) | rng.getrandbits(63)
        if rng.random() < 0.4:
            m &= ~((1 << rng.randint(0, 62)) - 1)
        return m, s | e
    if k < 0.52:  # small integers and halves
        v = rng.randint(1, 1 << rng.randint(1, 20))
        sh = 63 - (v.bit_length() - 1)
        return v << sh, s | (0x3FFF + v.bit_length() - 1 - rng.choice([0, 0, 1]))
    if k < 0.58:
        return 0, s
    if k < 0.64:
        return 1 << 63, s | 0x7FFF
    if k < 0.70:
        return (3 << 62) | rng.getrandbits(62) * rng.getrandbits(1), s | 0x7FFF
    if k < 0.75:
        return (1 << 63) | (rng.getrandbits(62) or 1), s | 0x7FFF
    if k < 0.83:
        return rng.getrandbits(63) >> rng.randint(0, 62) or 1, s
    if k < 0.86:
        return (1 << 63) | rng.getrandbits(63), s
    if k < 0.93:  # unnormal
        return rng.getrandbits(63), s | rng.randint(1, 0x7FFE)
    return rng.getrandbits(63), s | 0x7FFF  # pseudo-infinity / pseudo-NaN


def rand_float(rng, w):
    F, E = (23, 0xFF) if w == 32 else (52, 0x7FF)
    s = rng.getrandbits(1) << (w - 1)
    k = rng.random()
    if k < 0.5:
        e = rng.choice([rng.randint(1, E - 1), rng.randint(E // 2 - 30, E // 2 + 30), 1, E - 1])
        f = rng.getrandbits(F)
        if rng.random() < 0.4:
            f &= ~((1 << rng.randint(0, F)) - 1)
        return s | (e << F) | f
    if k < 0.6:
        return s
    if k < 0.7:
        return s | (E << F)
    if k < 0.8:
        return s | (E << F) | (1 << (F - 1)) | rng.getrandbits(F - 1)
    if k < 0.88:
        return s | (E << F) | (rng.getrandbits(F - 1) or 1)
    return s | (rng.getrandbits(F) >> rng.randint(0, F - 1) or 1)


def rand_mem(rng, kind):
    if kind == "f32":
        return rand_float(rng, 32).to_bytes(4, "little")
    if kind == "f64":
        return rand_float(rng, 64).to_bytes(8, "little")
    if kind == "f80":
        m, se = rand_f80(rng)
        return m.to_bytes(8, "little") + se.to_bytes(2, "little")
    n = {"i16": 2, "i32": 4, "i64": 8}[kind]
    v = rng.choice([rng.getrandbits(8 * n), rng.randint(0, 1000), (1 << (8 * n)) - rng.randint(1, 1000),
                    1 << (8 * n - 1), 0])
    return v.to_bytes(n, "little")


def rand_state(rng, pending=False):
    top = rng.randrange(8)
    tw = 0
    full = rng.random()
    for p in range(8):
        empty = rng.random() > (0.85 if full < 0.7 else 0.4)
        tw |= (3 if empty else 0) << (2 * p)
    st = [rand_f80(rng) for _ in range(8)]
    masks = 0x3F if rng.random() < 0.65 else rng.getrandbits(6)
    pc = rng.choice([0, 2, 3, 3, 3, 1])
    rc = rng.randrange(4)
    fcw = 0x40 | masks | (pc << 8) | (rc << 10)
    flags = rng.getrandbits(7) & (masks if not pending else 0x7F)
    cbits = rng.choice([0, 0x4700, rng.getrandbits(16) & 0x4700])
    fsw = (top << 11) | cbits | flags
    if fsw & ~fcw & 0x3F:
        fsw |= 0x8080
    fl = rng.getrandbits(12) & 0x8D5
    return dict(fcw=fcw, fsw=fsw, ftw=tw, st=st, fl=fl)


def case_regs(c, regs):
    """Apply a case's x87 state (and rsi = the buffer) to a Regs."""
    regs.fpcw, regs.fpsw, regs.fptw = c["fcw"], c["fsw"], c["ftw"]
    for i, (m, se) in enumerate(c["st"]):
        regs.fpst[i], regs.fpse[i] = m, se
    regs.rflags = c["fl"] | 0x202
    return regs


def make_cases(seed=0x87, per_reg=5, per_mem=48):
    rng = random.Random(seed)
    cases = []
    for code in reg_forms():
        for _ in range(per_reg):
            cases.append(dict(code=code.hex(), mem="00" * 16, **rand_state(rng, pending=rng.random() < 0.03)))
    for code, kind in mem_forms():
        store = not ((code[0] in (0xD8, 0xDA, 0xDC, 0xDE)) or ((code[1] >> 3) & 7) in (0, 5))
        for _ in range(per_mem):
            m = rand_mem(rng, kind) if not store else bytes(rng.getrandbits(8) for _ in range(10))
            cases.append(dict(code=code.hex(), mem=m.ljust(16, b"\0").hex(), **rand_state(rng, rng.random() < 0.03)))
    # fbld / fbstp (own generator: the cases above keep their values)
    brng = random.Random(seed ^ 0xBCD)
    for code in (bytes([0xDF, 0x26]), bytes([0xDF, 0x36])):
        for _ in range(per_mem * 4):
            st = rand_state(brng, brng.random() < 0.03)
            if code[1] == 0x26:
                m = rand_bcd(brng)
            else:
                m = bytes(brng.getrandbits(8) for _ in range(10))
                if brng.random() < 0.7:  # ST0 in (or near) the packed-BCD range, and valid
                    st["st"][0] = bcd_range_f80(brng)
                    top = (st["fsw"] >> 11) & 7
                    st["ftw"] &= ~(3 << (2 * top))
            cases.append(dict(code=code.hex(), mem=m.ljust(16, b"\0").hex(), **st))
    return cases


def rand_bcd(rng):
    """18 packed digits (a nibble above 9 now and then) and a sign byte."""
    k = rng.random()
    if k < 0.05:
        return bytes(9) + bytes([rng.choice([0, 0x80])])
    if k < 0.1:
        return bytes([0x99] * 9) + bytes([rng.choice([0, 0x80])])
    if k < 0.15:
        return bytes([0, 0, 0, 0, 0, 0, 0, 0xC0, 0xFF, 0xFF])  # the BCD indefinite
    n = rng.randint(1, 18)
    digits = [rng.randrange(10) if i < n else 0 for i in range(18)]
    if rng.random() < 0.15:
        digits[rng.randrange(18)] = rng.randint(10, 15)
    b = bytes(digits[2 * i] | (digits[2 * i + 1] << 4) for i in range(9))
    return b + bytes([rng.choice([0, 0x80, 0x80, rng.getrandbits(8)])])


def bcd_range_f80(rng):
    """An extended value around the packed-BCD range: integers, fractions, halves, 10^18 +- 1."""
    k = rng.random()
    if k < 0.1:
        v, frac = 10**18 + rng.choice([-1, 0, 1]), 0
    else:
        v = rng.randint(0, 10**rng.randint(0, 18))
        frac = rng.choice([0, 0, 1, 2, 3])  # none, a quarter, a half, three quarters
    s = rng.getrandbits(1)
    num = v * 4 + frac
    if num == 0:
        return 0, s << 15
    e = num.bit_length() - 1  # num = 1.f * 2^e, value = num / 4
    m = (num << (63 - e)) & ((1 << 64) - 1) if e <= 63 else num >> (e - 63)
    return m, (s << 15) | (0x3FFF + e - 2)


def run_oracle(c, buf_va):
    """One case through the oracle: (status, vector, fcw, fsw, ftw, st, fl, mem)."""
    from tests.oracle_lib import Oracle
    from tests.test_sse import layout
    sp, regs = layout(bytes.fromhex(c["code"]), buf_va, bytes.fromhex(c["mem"]).ljust(256, b"\0"))
    regs.gpr[6] = buf_va
    case_regs(c, regs)
    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    o.restore(regs)
    ex = o.step()
    r = o.regs()
    return dict(status=ex.status if ex.status != 3 else 0, vector=ex.vector if ex.status == 5 else 0,
                fcw=r.fpcw, fsw=r.fpsw, ftw=r.fptw, st=[(r.fpst[i], r.fpse[i]) for i in range(8)],
                fl=r.rflags & 0x8D5, mem=o.read_virt(buf_va, 16).hex())


def main():
    from tests.test_sse import BUF
    cases = make_cases()
    doc = {"buf_va": hex(BUF), "cases": []}
    for c in cases:
        out = run_oracle(c, BUF)
        doc["cases"].append(dict(c, out=out))
    with gzip.open(OUT, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(len(doc["cases"]), "cases ->", OUT)


if __name__ == "__main__":
    main()
