#!/usr/bin/env python3
"""Generate native-execution golden vectors for x86-64 instruction semantics.

SURVEY.md §8(c)(i): bochscpu (the reference CPU core) cannot be built here, so
the oracle's per-instruction semantics are pinned by *ordinary native execution*
of assembled instructions on the x86-64 host: a generated C file holds one stub
per instruction form which loads all 16 GPRs + RFLAGS from a global, executes the
instruction bytes, and stores GPRs + RFLAGS back. Memory operands point into a
256-byte window of a page-aligned buffer; RSP points into the same window so
push/pop are observed there. Nothing is traced or single-stepped (no ptrace).

Undefined flags / results (SDM "undefined") are masked per case (`fmask`) and
documented in oracle/x86_oracle.c (U1-U13); only architecturally defined bits
are compared.

Output: tests/golden/native_vectors.json.gz. Re-run with
    python tests/golden/gen_native_vectors.py
The buffer's initial bytes are splitmix64(seed) so each vector stores only its
seed and the bytes that changed.
"""
import gzip
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "native_vectors.json.gz")

RAX, RCX, RDX, RBX, RSP, RBP, RSI, RDI = range(8)
CF, PF, AF, ZF, SF, DF, OF = 0x1, 0x4, 0x10, 0x40, 0x80, 0x400, 0x800
STATUS = CF | PF | AF | ZF | SF | OF
WIN = 256  # window size in bytes; window starts at buf + 0x800


def splitmix_bytes(seed, n):
    out = bytearray()
    x = seed & 0xFFFFFFFFFFFFFFFF
    while len(out) < n:
        x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out += z.to_bytes(8, "little")
    return bytes(out[:n])


# --------------------------------------------------------------------------
# tiny encoder
# --------------------------------------------------------------------------
class Enc:
    """One instruction form: bytes + register roles."""

    def __init__(self, code, name, ptrs=(), smalls=(), fmask=STATUS, cls="alu",
                 size=8, extra=None):
        self.code = bytes(code)
        self.name = name
        self.ptrs = dict(ptrs)     # reg -> offset into window (pointer registers)
        self.smalls = dict(smalls)  # reg -> (lo, hi) small value ranges
        self.fmask = fmask
        self.cls = cls
        self.size = size
        self.extra = extra or {}


def rex_for(w, r, x, b, force=False):
    v = 0x40 | (w << 3) | ((r >> 3) << 2) | ((x >> 3) << 1) | (b >> 3)
    return [v] if (v != 0x40 or force) else []


def pfx(size):
    return [0x66] if size == 2 else []


def rr(opc, size, reg, rm, rng, byteop=False):
    """reg/reg modrm form. Returns bytes."""
    w = 1 if size == 8 else 0
    force = False
    if byteop and (4 <= reg < 8 or 4 <= rm < 8):
        force = rng.random() < 0.5  # with REX: spl..dil; without: ah..bh
    if byteop and (reg >= 8 or rm >= 8):
        force = True
    return pfx(size) + rex_for(w, reg, 0, rm, force) + list(opc) + [0xC0 | ((reg & 7) << 3) | (rm & 7)]


def mem(opc, size, reg, rng, byteop=False, width=8):
    """reg/mem modrm form with a random addressing mode. Returns (bytes, ptrs, smalls)."""
    w = 1 if size == 8 else 0
    force = byteop and 4 <= reg < 8 and rng.random() < 0.5
    kind = rng.choice(["base", "base8", "sib", "sib32", "rbp8", "r13", "r12"])
    ptrs, smalls = {}, {}
    off = rng.randrange(16, WIN - 48)
    if kind in ("base", "base8"):
        base = rng.choice([RBX, RSI, RDI, RAX, RCX, RDX, 9, 10, 11, 14, 15])
        while base == reg:
            base = rng.choice([RBX, RSI, RDI, 9, 10, 11, 14, 15])
        disp = [] if kind == "base" else [rng.randrange(0, 16)]
        mod = 0 if kind == "base" else 1
        code = pfx(size) + rex_for(w, reg, 0, base, force) + list(opc) + [(mod << 6) | ((reg & 7) << 3) | (base & 7)] + disp
        ptrs[base] = off - (disp[0] if disp else 0)
    elif kind in ("rbp8", "r13"):
        base = RBP if kind == "rbp8" else 13
        if base == reg:
            return mem(opc, size, reg, rng, byteop, width)
        d = rng.randrange(0, 32)
        code = pfx(size) + rex_for(w, reg, 0, base, force) + list(opc) + [(1 << 6) | ((reg & 7) << 3) | (base & 7), d]
        ptrs[base] = off - d
    else:
        base = rng.choice([RBX, RSI, RDI, 12, 9])
        index = rng.choice([RCX, RDX, 8, 10])
        if base == reg or index == reg:
            return mem(opc, size, reg, rng, byteop, width)
        ss = rng.randrange(4)
        iv = rng.randrange(0, 4)
        if kind == "sib32":
            d = rng.randrange(0, 64)
            disp = list(d.to_bytes(4, "little"))
            mod = 2
        else:
            d = rng.randrange(0, 32)
            disp = [d]
            mod = 1
        code = (pfx(size) + rex_for(w, reg, index, base, force) + list(opc) +
                [(mod << 6) | ((reg & 7) << 3) | 4, (ss << 6) | ((index & 7) << 3) | (base & 7)] + disp)
        ptrs[base] = off - d - (iv << ss)
        smalls[index] = (iv, iv)
    return code, ptrs, smalls


def gen_forms(rng):
    forms = []
    sizes = [1, 2, 4, 8]
    regs = list(range(16))

    def pick_reg(exclude=()):
        while True:
            r = rng.choice(regs)
            if r != RSP and r not in exclude:
                return r

    def imm(n, sign_boundary=False):
        v = rng.getrandbits(8 * n)
        return list(v.to_bytes(n, "little"))

    # ALU 00-3f (Ex,Gx / Gx,Ex), both reg and mem
    for op in range(8):
        for form in range(4):
            opc = op * 8 + form
            byteop = (form & 1) == 0
            for size in ([1] if byteop else [2, 4, 8]):
                mask = STATUS & ~AF if op in (1, 4, 6) else STATUS
                for _ in range(3):
                    reg, rm = pick_reg(), pick_reg()
                    forms.append(Enc(rr([opc], size, reg, rm, rng, byteop), f"alu{op}.{form}.rr{size}", fmask=mask, size=size))
                code, ptrs, smalls = mem([opc], size, pick_reg(), rng, byteop)
                forms.append(Enc(code, f"alu{op}.{form}.m{size}", ptrs, smalls, fmask=mask, size=size))
        # AL/eAX, imm
        mask = STATUS & ~AF if op in (1, 4, 6) else STATUS
        forms.append(Enc([op * 8 + 4] + imm(1), f"alu{op}.al", fmask=mask))
        for size in [2, 4, 8]:
            n = 2 if size == 2 else 4
            forms.append(Enc(pfx(size) + ([0x48] if size == 8 else []) + [op * 8 + 5] + imm(n), f"alu{op}.eax{size}", fmask=mask))
        # group 1
        for size in sizes:
            for opc in ([0x80] if size == 1 else [0x81, 0x83]):
                n = 1 if opc in (0x80, 0x83) else (2 if size == 2 else 4)
                forms.append(Enc(rr([opc], size, op, pick_reg(), rng, size == 1) + imm(n), f"grp1.{op}.{opc:x}.{size}", fmask=mask))
                code, ptrs, smalls = mem([opc], size, op, rng, size == 1)
                forms.append(Enc(code + imm(n), f"grp1m.{op}.{opc:x}.{size}", ptrs, smalls, fmask=mask))
    # test / xchg / mov
    for size in sizes:
        b = size == 1
        forms.append(Enc(rr([0x84 if b else 0x85], size, pick_reg(), pick_reg(), rng, b), f"test.rr{size}", fmask=STATUS & ~AF))
        code, ptrs, smalls = mem([0x84 if b else 0x85], size, pick_reg(), rng, b)
        forms.append(Enc(code, f"test.m{size}", ptrs, smalls, fmask=STATUS & ~AF))
        forms.append(Enc(rr([0x86 if b else 0x87], size, pick_reg(), pick_reg(), rng, b), f"xchg.rr{size}"))
        code, ptrs, smalls = mem([0x86 if b else 0x87], size, pick_reg(), rng, b)
        forms.append(Enc(code, f"xchg.m{size}", ptrs, smalls))
        for opc in ([0x88, 0x8a] if b else [0x89, 0x8b]):
            forms.append(Enc(rr([opc], size, pick_reg(), pick_reg(), rng, b), f"mov{opc:x}.rr{size}"))
            code, ptrs, smalls = mem([opc], size, pick_reg(), rng, b)
            forms.append(Enc(code, f"mov{opc:x}.m{size}", ptrs, smalls))
        n = 1 if b else (2 if size == 2 else 4)
        forms.append(Enc(rr([0xC6 if b else 0xC7], size, 0, pick_reg(), rng, b) + imm(n), f"movimm.r{size}"))
        code, ptrs, smalls = mem([0xC6 if b else 0xC7], size, 0, rng, b)
        forms.append(Enc(code + imm(n), f"movimm.m{size}", ptrs, smalls))
        # f6/f7 test/not/neg/mul/imul
        for sub in (0, 2, 3, 4, 5):
            fm = {0: STATUS & ~AF, 2: STATUS, 3: STATUS, 4: CF | OF, 5: CF | OF}[sub]
            code = rr([0xF6 if b else 0xF7], size, sub, pick_reg(), rng, b) + (imm(n) if sub == 0 else [])
            forms.append(Enc(code, f"f7.{sub}.r{size}", fmask=fm))
            code, ptrs, smalls = mem([0xF6 if b else 0xF7], size, sub, rng, b)
            forms.append(Enc(code + (imm(n) if sub == 0 else []), f"f7.{sub}.m{size}", ptrs, smalls, fmask=fm))
        for sub in (6, 7):
            rm = pick_reg(exclude=(RAX, RDX))
            forms.append(Enc(rr([0xF6 if b else 0xF7], size, sub, rm, rng, b), f"div.{sub}.r{size}", fmask=0,
                             cls="div", size=size, extra={"divreg": rm, "signed": sub == 7}))
        # inc/dec
        for sub in (0, 1):
            forms.append(Enc(rr([0xFE if b else 0xFF], size, sub, pick_reg(), rng, b), f"incdec.{sub}.r{size}"))
            code, ptrs, smalls = mem([0xFE if b else 0xFF], size, sub, rng, b)
            forms.append(Enc(code, f"incdec.{sub}.m{size}", ptrs, smalls))
        # shifts
        for sub in range(8):
            for opc in ((0xC0, 0xD0, 0xD2) if b else (0xC1, 0xD1, 0xD3)):
                rm = pick_reg(exclude=(RCX,))
                code = rr([opc], size, sub, rm, rng, b)
                if opc in (0xC0, 0xC1):
                    cnt = rng.choice([0, 1, 2, 3, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, rng.randrange(256)])
                    code += [cnt]
                forms.append(Enc(code, f"shift.{sub}.{opc:x}.{size}", cls="shift", size=size,
                                 extra={"sub": sub, "opc": opc}))
            code, ptrs, smalls = mem([0xD2 if b else 0xD3], size, sub, rng, b)
            if RCX not in ptrs and RCX not in smalls:
                forms.append(Enc(code, f"shiftm.{sub}.{size}", ptrs, smalls, cls="shift", size=size,
                                 extra={"sub": sub, "opc": 0xD3}))
    for size in (2, 4, 8):
        # movzx/movsx
        for opc in (0xB6, 0xB7, 0xBE, 0xBF):
            forms.append(Enc(rr([0x0F, opc], size, pick_reg(), pick_reg(), rng, opc in (0xB6, 0xBE)), f"movx{opc:x}.{size}"))
            code, ptrs, smalls = mem([0x0F, opc], size, pick_reg(), rng)
            forms.append(Enc(code, f"movxm{opc:x}.{size}", ptrs, smalls))
        # imul 2/3 op
        forms.append(Enc(rr([0x0F, 0xAF], size, pick_reg(), pick_reg(), rng), f"imul2.{size}", fmask=CF | OF))
        n = 2 if size == 2 else 4
        forms.append(Enc(rr([0x69], size, pick_reg(), pick_reg(), rng) + imm(n), f"imul69.{size}", fmask=CF | OF))
        forms.append(Enc(rr([0x6B], size, pick_reg(), pick_reg(), rng) + imm(1), f"imul6b.{size}", fmask=CF | OF))
        # cmov / setcc
        for cc in range(16):
            forms.append(Enc(rr([0x0F, 0x40 + cc], size, pick_reg(), pick_reg(), rng), f"cmov{cc}.{size}"))
        code, ptrs, smalls = mem([0x0F, 0x40 + rng.randrange(16)], size, pick_reg(), rng)
        forms.append(Enc(code, f"cmovm.{size}", ptrs, smalls))
        # bt family
        for opc, nm in ((0xA3, "bt"), (0xAB, "bts"), (0xB3, "btr"), (0xBB, "btc")):
            forms.append(Enc(rr([0x0F, opc], size, pick_reg(), pick_reg(), rng), f"{nm}.rr{size}", fmask=CF))
        for sub in (4, 5, 6, 7):
            forms.append(Enc(rr([0x0F, 0xBA], size, sub, pick_reg(), rng) + imm(1), f"btimm{sub}.{size}", fmask=CF))
            code, ptrs, smalls = mem([0x0F, 0xBA], size, sub, rng)
            forms.append(Enc(code + imm(1), f"btimmm{sub}.{size}", ptrs, smalls, fmask=CF))
        # bsf/bsr, tzcnt/lzcnt, popcnt
        for opc in (0xBC, 0xBD):
            dst = pick_reg()
            forms.append(Enc(rr([0x0F, opc], size, dst, pick_reg(), rng), f"bs{opc:x}.{size}", fmask=ZF,
                             cls="bsx", size=size, extra={"dst": dst}))
            forms.append(Enc([0xF3] + rr([0x0F, opc], size, pick_reg(), pick_reg(), rng), f"tzlz{opc:x}.{size}", fmask=CF | ZF))
        forms.append(Enc([0xF3] + rr([0x0F, 0xB8], size, pick_reg(), pick_reg(), rng), f"popcnt.{size}"))
        # shld/shrd
        for opc in (0xA4, 0xA5, 0xAC, 0xAD):
            rm = pick_reg(exclude=(RCX,))
            code = rr([0x0F, opc], size, pick_reg(exclude=(RCX,)), rm, rng)
            if opc in (0xA4, 0xAC):
                code += [rng.randrange(0, 64)]
            forms.append(Enc(code, f"shxd{opc:x}.{size}", cls="shxd", size=size, extra={"opc": opc}))
        # xadd / cmpxchg
        forms.append(Enc(rr([0x0F, 0xC1], size, pick_reg(), pick_reg(), rng), f"xadd.{size}"))
        code, ptrs, smalls = mem([0x0F, 0xC1], size, pick_reg(), rng)
        forms.append(Enc(code, f"xaddm.{size}", ptrs, smalls))
        forms.append(Enc(rr([0x0F, 0xB1], size, pick_reg(exclude=(RAX,)), pick_reg(exclude=(RAX,)), rng), f"cmpxchg.{size}", cls="cmpxchg"))
        code, ptrs, smalls = mem([0x0F, 0xB1], size, pick_reg(exclude=(RAX,)), rng)
        if RAX not in ptrs and RAX not in smalls:
            forms.append(Enc(code, f"cmpxchgm.{size}", ptrs, smalls, cls="cmpxchg"))
        # lea
        code, ptrs, smalls = mem([0x8D], size, pick_reg(), rng)
        forms.append(Enc(code, f"lea.{size}", ptrs, smalls))
        # cbw/cwd
        forms.append(Enc(pfx(size) + ([0x48] if size == 8 else []) + [0x98], f"cbw.{size}"))
        forms.append(Enc(pfx(size) + ([0x48] if size == 8 else []) + [0x99], f"cwd.{size}"))
    # count-0 forms: the destination is still written (32-bit registers zero-extend)
    for size in (2, 4, 8):
        for opc in (0xA4, 0xAC):
            forms.append(Enc(rr([0x0F, opc], size, RBX, 13, rng) + [0], f"shxd0.{opc:x}.{size}", fmask=STATUS))
            forms.append(Enc(rr([0x0F, opc], size, RBX, 13, rng) + [32], f"shxd32.{opc:x}.{size}",
                             fmask=STATUS if size != 8 else STATUS & ~AF & ~OF))
        for sub in range(8):
            forms.append(Enc(rr([0xC1], size, sub, 14, rng) + [0], f"shift0.{sub}.{size}", fmask=STATUS))
    # same-register forms (xadd r,r: SRC := DEST then DEST := TEMP)
    for r in (RAX, RBX, 9, 13):
        for size in (1, 2, 4, 8):
            b = size == 1
            forms.append(Enc(rr([0x0F, 0xC0 if b else 0xC1], size, r, r, rng, b), f"xadd.same{size}.{r}"))
            forms.append(Enc(rr([0x0F, 0xB0 if b else 0xB1], size, r, r, rng, b), f"cmpxchg.same{size}.{r}", cls="cmpxchg"))
            forms.append(Enc(rr([0x86 if b else 0x87], size, r, r, rng, b), f"xchg.same{size}.{r}"))
    # bswap
    for r in range(16):
        if r == RSP:
            continue
        forms.append(Enc(rex_for(1, 0, 0, r, False) + [0x0F, 0xC8 + (r & 7)], f"bswap64.{r}"))
        forms.append(Enc(rex_for(0, 0, 0, r, False) + [0x0F, 0xC8 + (r & 7)], f"bswap32.{r}"))
    # setcc
    for cc in range(16):
        forms.append(Enc(rr([0x0F, 0x90 + cc], 1, 0, pick_reg(), rng, True), f"setcc{cc}"))
    code, ptrs, smalls = mem([0x0F, 0x94], 1, 0, rng, True)
    forms.append(Enc(code, "setccm", ptrs, smalls))
    # movsxd
    forms.append(Enc(rr([0x63], 8, pick_reg(), pick_reg(), rng), "movsxd"))
    forms.append(Enc(rr([0x63], 4, pick_reg(), pick_reg(), rng), "movsxd32"))
    # mov imm to reg
    for r in range(16):
        if r == RSP:
            continue
        forms.append(Enc(rex_for(1, 0, 0, r) + [0xB8 + (r & 7)] + imm(8), f"movabs.{r}"))
        forms.append(Enc(rex_for(0, 0, 0, r) + [0xB8 + (r & 7)] + imm(4), f"movimm32.{r}"))
        forms.append(Enc(rex_for(0, 0, 0, r, rng.random() < 0.5) + [0xB0 + (r & 7)] + imm(1), f"movimm8.{r}"))
    # flags ops
    for opc in (0xF5, 0xF8, 0xF9, 0xFC, 0xFD, 0x9E, 0x9F):
        forms.append(Enc([opc], f"flag{opc:x}"))
    # push / pop (rsp points into the window)
    for r in range(16):
        if r == RSP:
            continue
        forms.append(Enc(rex_for(0, 0, 0, r) + [0x50 + (r & 7)], f"push.{r}", cls="stack"))
        forms.append(Enc(rex_for(0, 0, 0, r) + [0x58 + (r & 7)], f"pop.{r}", cls="stack"))
    forms.append(Enc([0x66, 0x53], "push16", cls="stack"))
    forms.append(Enc([0x66, 0x5B], "pop16", cls="stack"))
    forms.append(Enc([0x6A] + imm(1), "push6a", cls="stack"))
    forms.append(Enc([0x68] + imm(4), "push68", cls="stack"))
    forms.append(Enc([0x9C], "pushf", cls="stack"))
    forms.append(Enc([0x9D], "popf", cls="popf"))
    forms.append(Enc([0xFF, 0xF3], "pushrm", cls="stack"))
    code, ptrs, smalls = mem([0xFF], 8, 6, rng)
    forms.append(Enc(code, "pushm", ptrs, smalls, cls="stack"))
    forms.append(Enc([0x8F, 0xC3], "poprm", cls="stack"))
    forms.append(Enc([0xC9], "leave", ptrs={RBP: 64}, cls="stack"))
    forms.append(Enc([0xD7], "xlat", ptrs={RBX: 32}))
    # xchg with rax
    for r in range(1, 16):
        if r == RSP:
            continue
        forms.append(Enc(rex_for(1, 0, 0, r) + [0x90 + (r & 7)], f"xchgrax.{r}"))
    # nops
    for code in ([0x90], [0x0F, 0x1F, 0x00], [0x0F, 0x1F, 0x44, 0x00, 0x00], [0x66, 0x0F, 0x1F, 0x44, 0x00, 0x00],
                 [0xF3, 0x90], [0xF3, 0x0F, 0x1E, 0xFA]):
        forms.append(Enc(code, "nop", ptrs={RAX: 64}))
    # strings
    for opc in (0xA4, 0xA5, 0xAA, 0xAB, 0xAC, 0xAD, 0xA6, 0xA7, 0xAE, 0xAF):
        for size in ([1] if opc % 2 == 0 else [2, 4, 8]):
            for rep in ([], [0xF3], [0xF2]) if opc in (0xA6, 0xA7, 0xAE, 0xAF) else ([], [0xF3]):
                code = rep + pfx(size) + ([0x48] if size == 8 else []) + [opc]
                forms.append(Enc(code, f"str{opc:x}.{size}.{len(rep)}", cls="string", size=size))
    # (round 3, appended so the earlier forms keep their random streams)
    # loopne / loope / loop / jrcxz with a zero displacement: the counter update
    # (rcx, or ecx zero-extended under 67) and untouched flags (U26)
    for opc in (0xE0, 0xE1, 0xE2, 0xE3):
        for p67 in ([], [0x67]):
            forms.append(Enc(p67 + [opc, 0x00], f"loop{opc:x}.{len(p67)}", smalls={RCX: (0, 3)}))
            forms.append(Enc(p67 + [opc, 0x00], f"loopr{opc:x}.{len(p67)}"))
    # cmpxchg8b / cmpxchg16b [rdi] (U28): half the cases compare equal
    forms.append(Enc([0x0F, 0xC7, 0x0F], "cmpxchg8b", ptrs={RDI: 0x40}, fmask=ZF, cls="cx"))
    forms.append(Enc([0xF0, 0x0F, 0xC7, 0x0F], "lockcmpxchg8b", ptrs={RDI: 0x48}, fmask=ZF, cls="cx"))
    forms.append(Enc([0x48, 0x0F, 0xC7, 0x0F], "cmpxchg16b", ptrs={RDI: 0x40}, fmask=ZF, cls="cx"))
    # enter iw, ib at nesting levels 0..3 (U29): rbp points into the window above rsp
    for level in (0, 1, 2, 3):
        forms.append(Enc([0xC8, 0x18, 0x00, level], f"enter.{level}", ptrs={RBP: 0xC0}, cls="stack"))
    forms.append(Enc([0xC8, 0x00, 0x01, 0x21], "enter.33", ptrs={RBP: 0xE0}, cls="stack"))
    return forms


def rand_val(rng, size=8):
    r = rng.random()
    if r < 0.15:
        return rng.choice([0, 1, 2, 0x7F, 0x80, 0xFF, 0x7FFF, 0x8000, 0xFFFF, 0x7FFFFFFF, 0x80000000,
                           0xFFFFFFFF, 0x7FFFFFFFFFFFFFFF, 0x8000000000000000, 0xFFFFFFFFFFFFFFFF])
    if r < 0.3:
        return rng.getrandbits(8)
    if r < 0.45:
        return rng.getrandbits(16) | (rng.choice([0, 0xFFFFFFFFFFFF0000]))
    if r < 0.6:
        return rng.getrandbits(32)
    return rng.getrandbits(64)


def make_cases(forms, rng, per_form=6):
    cases = []
    for f in forms:
        for _ in range(per_form):
            regs = [rand_val(rng) for _ in range(16)]
            regs[RSP] = 0x80  # offset; fixed up to buf address at run time
            ptr_regs = dict(f.ptrs)
            for r, off in ptr_regs.items():
                regs[r] = off
            for r, (lo, hi) in f.smalls.items():
                regs[r] = rng.randint(lo, hi)
            flags = 0x2 | (rng.getrandbits(16) & STATUS)
            fmask = f.fmask
            skip_regs = []
            if f.cls == "string":
                ptr_regs = {RSI: rng.randrange(32, 160), RDI: rng.randrange(32, 160)}
                regs[RSI], regs[RDI] = ptr_regs[RSI], ptr_regs[RDI]
                regs[RCX] = rng.randrange(0, 9)
                if rng.random() < 0.3:
                    flags |= DF
                    regs[RSI] += 64
                    regs[RDI] += 64
                    ptr_regs = {RSI: regs[RSI], RDI: regs[RDI]}
                if rng.random() < 0.5:
                    regs[RAX] = rng.getrandbits(8) * 0x0101010101010101  # scas hits
            if f.cls == "stack":
                pass
            if f.cls == "popf":
                pass
            if f.cls == "div":
                sz = f.size
                bits = 8 * sz
                dv = 0
                while dv == 0:
                    dv = rand_val(rng) & ((1 << bits) - 1)
                r = f.extra["divreg"]
                if sz == 1 and r in (4, 5, 6, 7) and (f.code[0] & 0xF0) != 0x40:
                    # ah..bh as divisor: keep it simple, skip this case
                    continue
                regs[r] = (regs[r] & ~((1 << bits) - 1)) | dv
                if f.extra["signed"]:
                    sdv = dv - (1 << bits) if dv >> (bits - 1) else dv
                    q = rng.randrange(-(1 << (bits - 1)) + 1, (1 << (bits - 1)) - 1) // max(1, 1)
                    q = max(min(q, (1 << (bits - 1)) - 1), -(1 << (bits - 1)) + 1)
                    rem = rng.randrange(0, abs(sdv))
                    n = q * sdv + (rem if q * sdv >= 0 else -rem)
                    if sz == 1:
                        n &= 0xFFFF
                        regs[RAX] = (regs[RAX] & ~0xFFFF) | n
                    else:
                        n &= (1 << (2 * bits)) - 1
                        lo, hi = n & ((1 << bits) - 1), n >> bits
                        regs[RAX] = (regs[RAX] & ~((1 << bits) - 1)) | lo
                        regs[RDX] = (regs[RDX] & ~((1 << bits) - 1)) | hi
                else:
                    hi = rng.randrange(0, dv)
                    lo = rng.getrandbits(bits)
                    if sz == 1:
                        regs[RAX] = (regs[RAX] & ~0xFFFF) | (hi << 8) | lo
                    else:
                        regs[RAX] = (regs[RAX] & ~((1 << bits) - 1)) | lo
                        regs[RDX] = (regs[RDX] & ~((1 << bits) - 1)) | hi
                if sz == 4:
                    pass
            if f.cls == "shift":
                # masked count 0: flags unchanged (defined). count 1: AF undefined.
                # count > 1: OF also undefined. count > operand bits: CF undefined (shl/shr).
                opc = f.extra["opc"]
                sub = f.extra["sub"]
                if opc in (0xC0, 0xC1):
                    cnt = f.code[-1]
                elif opc in (0xD0, 0xD1):
                    cnt = 1
                else:
                    cnt = regs[RCX] & 0xFF
                    if rng.random() < 0.5:
                        cnt = rng.choice([0, 1, 2, 5, 8, 9, 16, 17, 31, 32, 33, 63, 64])
                        regs[RCX] = (regs[RCX] & ~0xFF) | cnt
                m = cnt & (0x3F if f.size == 8 else 0x1F)
                bits = 8 * f.size
                if m == 0:
                    fmask = STATUS
                elif sub in (0, 1, 2, 3):
                    fmask = CF | OF if m == 1 else CF
                    if sub in (2, 3) and f.size in (1, 2):
                        fmask = CF | OF if m == 1 else CF
                else:
                    fmask = STATUS & ~AF
                    if m > 1:
                        fmask &= ~OF
                    if m > bits and sub in (4, 5, 6):
                        fmask &= ~CF
            if f.cls == "shxd":
                opc = f.extra["opc"]
                cnt = f.code[-1] if opc in (0xA4, 0xAC) else regs[RCX] & 0xFF
                m = cnt & (0x3F if f.size == 8 else 0x1F)
                if m > 8 * f.size:
                    continue
                fmask = STATUS if m == 0 else (STATUS & ~AF & ~(OF if m > 1 else 0))
            seed = rng.getrandbits(63)
            if f.cls == "popf":
                # popped rflags must keep TF/AC/NT clear so the native run stays sane
                while True:
                    v = int.from_bytes(splitmix_bytes(seed, WIN)[0x80:0x88], "little")
                    if not (v & ((1 << 8) | (1 << 18) | (1 << 14))):
                        break
                    seed = rng.getrandbits(63)
            if f.cls == "cx" and rng.random() < 0.5:  # rdx:rax = the operand: the equal case
                off = f.ptrs[RDI]
                w = splitmix_bytes(seed, WIN)
                lo = int.from_bytes(w[off:off + 8], "little")
                hi = int.from_bytes(w[off + 8:off + 16], "little")
                if f.code[0] == 0x48:
                    regs[RAX], regs[RDX] = lo, hi
                else:
                    regs[RAX] = (regs[RAX] & ~0xFFFFFFFF) | (lo & 0xFFFFFFFF)
                    regs[RDX] = (regs[RDX] & ~0xFFFFFFFF) | (lo >> 32)
            cases.append({
                "name": f.name,
                "code": f.code.hex(),
                "regs": regs,
                "ptrs": sorted(ptr_regs.keys()) + ([RSP] if RSP not in ptr_regs else []),
                "flags": flags,
                "fmask": fmask,
                "seed": seed,
                "cls": f.cls,
                "dst": f.extra.get("dst", -1),
            })
    return cases


C_HEADER = r"""
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
typedef struct { uint64_t r[16]; uint64_t fl; } st_t;
st_t g_in, g_out;
uint64_t g_host_rsp;
uint64_t g_flagstack[64] __attribute__((aligned(16)));
uint8_t g_buf[8192] __attribute__((aligned(4096)));
"""

STUB = r"""
__asm__(
".text\n.globl t_{i}\nt_{i}:\n"
"push %rbx\npush %rbp\npush %r12\npush %r13\npush %r14\npush %r15\n"
"mov %rsp, g_host_rsp(%rip)\n"
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
"mov g_host_rsp(%rip), %rsp\n"
"pop %r15\npop %r14\npop %r13\npop %r12\npop %rbp\npop %rbx\nret\n");
void t_{i}(void);
"""

C_MAIN = r"""
static uint64_t sm(uint64_t *x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
typedef void (*fn_t)(void);
static fn_t fns[] = { FNLIST };
int main(void) {
  int form; unsigned long long seed, flags; unsigned long long regs[16]; int nptr; int ptrs[16];
  uint8_t *win = g_buf + 0x800;
  printf("BUF %llx\n", (unsigned long long)(uintptr_t)win);
  while (scanf("%d %llx %llx", &form, &seed, &flags) == 3) {
    for (int i = 0; i < 16; i++) scanf("%llx", &regs[i]);
    scanf("%d", &nptr);
    for (int i = 0; i < nptr; i++) scanf("%d", &ptrs[i]);
    uint64_t x = seed;
    for (int i = 0; i < 256; i += 8) { uint64_t v = sm(&x); memcpy(win + i, &v, 8); }
    for (int i = 0; i < 16; i++) g_in.r[i] = regs[i];
    for (int i = 0; i < nptr; i++) g_in.r[ptrs[i]] = (uint64_t)(uintptr_t)win + regs[ptrs[i]];
    g_in.fl = flags;
    fns[form]();
    printf("R");
    for (int i = 0; i < 16; i++) printf(" %llx", (unsigned long long)g_out.r[i]);
    printf(" %llx\nM", (unsigned long long)g_out.fl);
    for (int i = 0; i < 256; i++) printf("%02x", win[i]);
    printf("\n");
  }
  return 0;
}
"""


def main():
    rng = random.Random(0x5EED0002)
    forms = gen_forms(rng)
    cases = make_cases(forms, rng)
    # popf: stack value with TF/AC/IF cleared to keep the native run safe
    for c in cases:
        pass
    uniq = {}
    for c in cases:
        uniq.setdefault(c["code"], len(uniq))
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "nv.c")
        with open(src, "w") as f:
            f.write(C_HEADER)
            for code, i in uniq.items():
                bs = ",".join("0x%02x" % b for b in bytes.fromhex(code))
                f.write(STUB.replace("{i}", str(i)).replace("{bytes}", bs))
            f.write(C_MAIN.replace("FNLIST", ",".join(f"t_{i}" for i in range(len(uniq)))))
        exe = os.path.join(td, "nv")
        subprocess.check_call(["gcc", "-O1", "-no-pie", "-o", exe, src])
        lines = []
        for c in cases:
            lines.append("%d %x %x %s %d %s" % (
                uniq[c["code"]], c["seed"], c["flags"], " ".join("%x" % v for v in c["regs"]),
                len(c["ptrs"]), " ".join(str(p) for p in c["ptrs"])))
        inp = "\n".join(lines) + "\n"
        # popf safety: patch the stack window bytes so popped rflags have TF/AC clear.
        out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
    buf_va = int(out[0].split()[1], 16)
    res = []
    k = 1
    for c in cases:
        rl = out[k].split()
        ml = out[k + 1][1:]
        k += 2
        outregs = [int(x, 16) for x in rl[1:17]]
        outfl = int(rl[17], 16)
        before = splitmix_bytes(c["seed"], WIN)
        after = bytes.fromhex(ml)
        diff = [[i, after[i]] for i in range(WIN) if after[i] != before[i]]
        inregs = list(c["regs"])
        for p in c["ptrs"]:
            inregs[p] = (buf_va + inregs[p]) & 0xFFFFFFFFFFFFFFFF
        res.append({
            "name": c["name"], "code": c["code"], "in": ["%x" % v for v in inregs],
            "fl": "%x" % c["flags"], "out": ["%x" % v for v in outregs], "flo": "%x" % outfl,
            "fmask": "%x" % c["fmask"], "seed": "%x" % c["seed"], "diff": diff, "cls": c["cls"], "dst": c["dst"],
        })
    doc = {"buf_va": "%x" % buf_va, "window": WIN, "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "generator": "tests/golden/gen_native_vectors.py", "cases": res}
    with gzip.open(OUT, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"wrote {len(res)} vectors ({len(uniq)} encodings) to {OUT}")


if __name__ == "__main__":
    main()
