#!/usr/bin/env python3
"""Native-execution golden vectors for the AVX-512 subset (convention U47;
wtf_amd/csrc/engine_avx512.h, oracle/x86_oracle_avx512.inc).

Every case runs once on this host's CPU (AVX512F / BW / VL / DQ): a stub
loads the 16 GPRs, RFLAGS, zmm0-31 and k0-7, executes the instruction and
stores them back. Memory is a 512-byte window that straddles a page boundary
(the last 256 bytes of one page, the first 256 of the next); in the "guard"
cases the second page (guard 1) or the first (guard 2) is PROT_NONE, so an
operand across the boundary shows memory fault suppression (masked-off
elements never touch the page) and the #PF a selected element takes. Faults are recorded from the signal
(trap number, page-fault error code, CR2); #UD is SIGILL.

Forms (EVEX, 128 / 256 / 512 bits, merging and zeroing masks, register,
memory, disp8*N and disp32, embedded broadcasts):
  vmovups / upd / aps / apd, vmovdqa32 / 64, vmovdqu8 / 16 / 32 / 64 (loads,
  stores, register moves), vmovntps / pd / dq and vmovntdqa, vpand / andn / or / xor d q, vpadd / vpsub b w d q,
  vpminub / uw, vpmaxub / uw, vpcmpeq / gt b w d q, vpcmp(u) b w d q (every
  predicate), vptestm / vptestnm b w d q, vpternlog d q, vpbroadcast b w d q
  from xmm / memory / GPR; plus the VEX opmask instructions kmov b w d q
  (k / m / r forms), kand / andn / or / xnor / xor, knot, kortest, ktest,
  kshiftl / r, kadd, kunpck, and the #UD encodings (z with a k or memory destination, b in a
  register form or a non-broadcast form, L'L = 11, vvvv in two-operand forms,
  a prefix before 62, the reserved P0 / P1 bits).

A case's zmm registers and window come from case_inputs(seed); k0-7 are
stored in the case.

Output: tests/golden/avx512_vectors.json.gz. Re-run with
    python tests/golden/gen_avx512_vectors.py
"""
import gzip
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests.golden.gen_native_vectors import rand_val  # noqa: E402

OUT = os.path.join(HERE, "avx512_vectors.json.gz")
WIN = 512          # window bytes; the page boundary is at window offset 0x100
BOUND = 0x100
RSP = 4
M64 = (1 << 64) - 1


# ---------------------------------------------------------------- encoding
def evex(mp, pp, w, ll, z, b, aaa, reg, vvvv, opc, rm=None, mem=None, imm=None, raw=None):
    """62 P0 P1 P2 opc ModRM [SIB] [disp] [imm]. rm: a 5-bit register; mem:
    (base, index or None, scale bits, disp, disp bytes 1 or 4)."""
    R, R2 = (reg >> 3) & 1, (reg >> 4) & 1
    if mem is None:
        X, B = (rm >> 4) & 1, (rm >> 3) & 1
    else:
        base, index, ss, disp, dsz = mem
        X, B = ((index >> 3) & 1) if index is not None else 0, (base >> 3) & 1
    p0 = ((R ^ 1) << 7) | ((X ^ 1) << 6) | ((B ^ 1) << 5) | ((R2 ^ 1) << 4) | mp
    p1 = (w << 7) | ((~vvvv & 15) << 3) | 4 | pp
    p2 = (z << 7) | (ll << 5) | (b << 4) | ((((vvvv >> 4) & 1) ^ 1) << 3) | aaa
    if raw:  # deliberate encoding faults: (p0 xor, p1 xor)
        p0 ^= raw[0]
        p1 ^= raw[1]
    out = [0x62, p0, p1, p2, opc]
    if mem is None:
        out.append(0xC0 | ((reg & 7) << 3) | (rm & 7))
    else:
        out += modrm_mem(reg, mem)
    if imm is not None:
        out.append(imm)
    return out


def modrm_mem(reg, mem):
    base, index, ss, disp, dsz = mem
    mod = 1 if dsz == 1 else 2
    out = []
    if index is not None or (base & 7) == 4:
        out.append((mod << 6) | ((reg & 7) << 3) | 4)
        out.append((ss << 6) | (((index if index is not None else 4) & 7) << 3) | (base & 7))
    else:
        out.append((mod << 6) | ((reg & 7) << 3) | (base & 7))
    out += list((disp & ((1 << (8 * dsz)) - 1)).to_bytes(dsz, "little"))
    return out


def vex3(mp, pp, w, l, reg, vvvv, opc, rm=None, mem=None, imm=None):
    R = (reg >> 3) & 1
    if mem is None:
        X, B = 0, (rm >> 3) & 1
    else:
        base, index, ss, disp, dsz = mem
        X, B = ((index >> 3) & 1) if index is not None else 0, (base >> 3) & 1
    b1 = ((R ^ 1) << 7) | ((X ^ 1) << 6) | ((B ^ 1) << 5) | mp
    b2 = (w << 7) | ((~vvvv & 15) << 3) | (l << 2) | pp
    out = [0xC4, b1, b2, opc]
    out += [0xC0 | ((reg & 7) << 3) | (rm & 7)] if mem is None else modrm_mem(reg, mem)
    if imm is not None:
        out.append(imm)
    return out


# ---------------------------------------------------------------- the forms
# (name, map, pp, W, opcode, kind, element bytes, extra)
# kind: ld (load / reg move, r/m source), st (store form), op (dst = vvvv op r/m),
# kd (k destination), tern, bcm (broadcast from xmm / memory), bcr (from a GPR)
def evex_forms():
    F = []
    for nm, pp, w, es in (("vmovups", 0, 0, 4), ("vmovupd", 1, 1, 8)):
        F += [(nm, 1, pp, w, 0x10, "ld", es, {}), (nm, 1, pp, w, 0x11, "st", es, {})]
    for nm, pp, w, es in (("vmovaps", 0, 0, 4), ("vmovapd", 1, 1, 8)):
        F += [(nm, 1, pp, w, 0x28, "ld", es, {"al": 1}), (nm, 1, pp, w, 0x29, "st", es, {"al": 1})]
    for nm, pp, w, es, al in (("vmovdqa32", 1, 0, 4, 1), ("vmovdqa64", 1, 1, 8, 1), ("vmovdqu32", 2, 0, 4, 0),
                              ("vmovdqu64", 2, 1, 8, 0), ("vmovdqu8", 3, 0, 1, 0), ("vmovdqu16", 3, 1, 2, 0)):
        F += [(nm, 1, pp, w, 0x6F, "ld", es, {"al": al}), (nm, 1, pp, w, 0x7F, "st", es, {"al": al})]
    for base, opc in (("vpand", 0xDB), ("vpandn", 0xDF), ("vpor", 0xEB), ("vpxor", 0xEF)):
        F += [(base + "d", 1, 1, 0, opc, "op", 4, {"bc": 1}), (base + "q", 1, 1, 1, opc, "op", 8, {"bc": 1})]
    for nm, opc, w, es, bc in (("vpaddb", 0xFC, None, 1, 0), ("vpaddw", 0xFD, None, 2, 0), ("vpaddd", 0xFE, 0, 4, 1),
                               ("vpaddq", 0xD4, 1, 8, 1), ("vpsubb", 0xF8, None, 1, 0), ("vpsubw", 0xF9, None, 2, 0),
                               ("vpsubd", 0xFA, 0, 4, 1), ("vpsubq", 0xFB, 1, 8, 1), ("vpminub", 0xDA, None, 1, 0),
                               ("vpmaxub", 0xDE, None, 1, 0)):
        F.append((nm, 1, 1, w, opc, "op", es, {"bc": bc}))
    for nm, opc, w, es, bc in (("vpcmpeqb", 0x74, None, 1, 0), ("vpcmpeqw", 0x75, None, 2, 0),
                               ("vpcmpeqd", 0x76, 0, 4, 1), ("vpcmpgtb", 0x64, None, 1, 0),
                               ("vpcmpgtw", 0x65, None, 2, 0), ("vpcmpgtd", 0x66, 0, 4, 1)):
        F.append((nm, 1, 1, w, opc, "kd", es, {"bc": bc}))
    F += [("vpcmpeqq", 2, 1, 1, 0x29, "kd", 8, {"bc": 1}), ("vpcmpgtq", 2, 1, 1, 0x37, "kd", 8, {"bc": 1}),
          ("vpminuw", 2, 1, None, 0x3A, "op", 2, {}), ("vpmaxuw", 2, 1, None, 0x3E, "op", 2, {})]
    for nm, pp, w, opc, es, bc in (("vptestmb", 1, 0, 0x26, 1, 0), ("vptestmw", 1, 1, 0x26, 2, 0),
                                   ("vptestnmb", 2, 0, 0x26, 1, 0), ("vptestnmw", 2, 1, 0x26, 2, 0),
                                   ("vptestmd", 1, 0, 0x27, 4, 1), ("vptestmq", 1, 1, 0x27, 8, 1),
                                   ("vptestnmd", 2, 0, 0x27, 4, 1), ("vptestnmq", 2, 1, 0x27, 8, 1)):
        F.append((nm, 2, pp, w, opc, "kd", es, {"bc": bc}))
    for nm, opc, w, es in (("vpbroadcastb", 0x78, 0, 1), ("vpbroadcastw", 0x79, 0, 2), ("vpbroadcastd", 0x58, 0, 4),
                           ("vpbroadcastq", 0x59, 1, 8)):
        F.append((nm, 2, 1, w, opc, "bcm", es, {}))
    for nm, opc, w, es in (("vpbroadcastb.r", 0x7A, 0, 1), ("vpbroadcastw.r", 0x7B, 0, 2),
                           ("vpbroadcastd.r", 0x7C, 0, 4), ("vpbroadcastq.r", 0x7C, 1, 8)):
        F.append((nm, 2, 1, w, opc, "bcr", es, {}))
    F += [("vpternlogd", 3, 1, 0, 0x25, "tern", 4, {"bc": 1}), ("vpternlogq", 3, 1, 1, 0x25, "tern", 8, {"bc": 1})]
    for nm, opc, w, es, bc in (("vpcmpub", 0x3E, 0, 1, 0), ("vpcmpuw", 0x3E, 1, 2, 0), ("vpcmpb", 0x3F, 0, 1, 0),
                               ("vpcmpw", 0x3F, 1, 2, 0), ("vpcmpud", 0x1E, 0, 4, 1), ("vpcmpuq", 0x1E, 1, 8, 1),
                               ("vpcmpd", 0x1F, 0, 4, 1), ("vpcmpq", 0x1F, 1, 8, 1)):
        F.append((nm, 3, 1, w, opc, "kd", es, {"bc": bc, "imm": 1}))
    # the non-temporal moves (memory only, no masking: a register form or aaa != 0 is #UD)
    F += [("vmovntps", 1, 0, 0, 0x2B, "st", 4, {"al": 1}), ("vmovntpd", 1, 1, 1, 0x2B, "st", 8, {"al": 1}),
          ("vmovntdq", 1, 1, 0, 0xE7, "st", 4, {"al": 1}), ("vmovntdqa", 2, 1, 0, 0x2A, "ld", 4, {"al": 1})]
    return F


def pick_mem(rng, regs, ptrs, smalls, toff, n_scale, use_disp8=True):
    """An addressing form whose effective address is window + toff."""
    base = rng.choice([r for r in range(16) if r != RSP])
    index = None
    ss = 0
    idx_val = 0
    if rng.random() < 0.3:
        index = rng.choice([r for r in range(16) if r not in (RSP, base)])
        ss = rng.randrange(4)
        idx_val = rng.randrange(0, 8)
        smalls[index] = idx_val
    if use_disp8 and rng.random() < 0.75:
        dd = rng.randint(-3, 3)
        disp, dsz, eff = dd, 1, dd * n_scale
    else:
        disp = rng.randint(-300, 300)
        dsz, eff = 4, disp
    ptrs[base] = toff - eff - (idx_val << ss)
    return (base, index, ss, disp, dsz)


def gen_evex_cases(rng):
    cases = []
    for (nm, mp, pp, w0, opc, kind, es, ex) in evex_forms():
        reps = 40 if kind in ("ld", "st") else 30
        for i in range(reps):
            w = w0 if w0 is not None else rng.randrange(2)
            ll = i % 3
            vlb = 16 << ll
            n = vlb // es
            mem = kind not in ("bcr",) and rng.random() < 0.5
            if kind == "bcr":
                mem = False
            aaa = 0 if rng.random() < 0.25 else rng.randrange(1, 8)
            if nm.startswith("vmovnt"):  # mostly the valid form: memory, no mask
                mem = rng.random() < 0.85
                aaa = 0 if rng.random() < 0.8 else aaa
            zok = kind not in ("kd",) and not (kind == "st" and mem)
            z = 1 if zok and rng.random() < 0.4 else 0
            b = 1 if mem and ex.get("bc") and rng.random() < 0.4 else 0
            reg, vvvv, rm = rng.randrange(32), rng.randrange(32), rng.randrange(32)
            if kind in ("ld", "st", "bcm", "bcr"):
                vvvv = 0
            if kind == "kd":
                reg = rng.randrange(8)
            imm = rng.randrange(256) if kind == "tern" else (rng.randrange(8) | (rng.randrange(32) << 3)
                                                             if ex.get("imm") else None)
            if kind == "kd" and ex.get("imm"):
                imm = (i % 8) | (rng.randrange(32) << 3)
            regs = [rand_val(rng) for _ in range(16)]
            ptrs, smalls = {RSP: 0x80}, {}
            guard = 0
            if mem:
                if kind == "bcm" or b:
                    osz, nsc = es, es
                else:
                    osz, nsc = vlb, vlb
                if rng.random() < 0.2 and osz > es:   # across the page boundary; the next page absent
                    guard = 1
                    toff = BOUND - es * rng.randrange(1, osz // es)
                elif ex.get("al") and rng.random() < 0.1:
                    toff = rng.randrange(0, WIN - osz) | 1 if es == 1 else rng.randrange(0, (WIN - osz) // es) * es
                    if toff % vlb == 0:
                        toff += es
                else:
                    al = vlb if ex.get("al") else es
                    toff = rng.randrange(0, (WIN - osz) // al + 1) * al
                m = pick_mem(rng, regs, ptrs, smalls, toff, nsc)
                code = evex(mp, pp, w, ll, z, b, aaa, reg, vvvv, opc, mem=m, imm=imm)
            else:
                code = evex(mp, pp, w, ll, z, 0, aaa, reg, vvvv, opc, rm=rm, imm=imm)
            cases.append(mk_case(rng, f"{nm}.L{ll}.{'m' if mem else 'r'}", code, regs, ptrs, smalls, guard,
                                 kmask_focus=(aaa, n, guard)))
    return cases


def gen_ud_cases(rng):
    """Encodings that are #UD natively: (name, bytes)."""
    out = []
    add = lambda nm, c: out.append((nm, c))  # noqa: E731
    for _ in range(3):
        r = rng.randrange(32)
        add("ud.z_kdest", evex(1, 1, 0, 2, 1, 0, 1, 1, r, 0x74, rm=rng.randrange(32)))           # vpcmpeqb k{z}
        add("ud.z_store", evex(1, 2, 0, 2, 1, 0, 1, r, 0, 0x7F, mem=(0, None, 0, 0, 1)))          # vmovdqu32 m{z}
        add("ud.b_reg", evex(1, 1, 0, 2, 0, 1, 0, r, 3, 0xFE, rm=rng.randrange(32)))              # vpaddd {rn-sae}
        add("ud.b_nonbcast", evex(1, 1, 0, 2, 0, 1, 0, r, 3, 0xFC, mem=(0, None, 0, 0, 1)))       # vpaddb m{1toN}
        add("ud.ll3", evex(1, 1, 0, 3, 0, 0, 0, r, 3, 0xEF, rm=rng.randrange(32)))                # vpxord L'L = 11
        add("ud.vvvv_mov", evex(1, 2, 0, 2, 0, 0, 0, r, 5, 0x6F, rm=rng.randrange(32)))           # vmovdqu32 vvvv
        add("ud.vprime_mov", evex(1, 2, 0, 2, 0, 0, 0, r, 16, 0x6F, rm=rng.randrange(32)))        # V' = 0
        add("ud.p66", [0x66] + evex(1, 1, 0, 2, 0, 0, 0, r, 3, 0xEF, rm=rng.randrange(32)))       # 66 62 ...
        add("ud.rex", [0x41] + evex(1, 1, 0, 2, 0, 0, 0, r, 3, 0xEF, rm=rng.randrange(32)))
        add("ud.p0bit3", evex(1, 1, 0, 2, 0, 0, 0, r & 15, 3, 0xEF, rm=rng.randrange(16), raw=(8, 0)))
        add("ud.p1bit2", evex(1, 1, 0, 2, 0, 0, 0, r & 15, 3, 0xEF, rm=rng.randrange(16), raw=(0, 4)))
        add("ud.map0", evex(0, 1, 0, 2, 0, 0, 0, r, 3, 0xEF, rm=rng.randrange(32)))
        add("ud.bcr_mem", evex(2, 1, 0, 2, 0, 0, 0, r, 0, 0x7C, mem=(0, None, 0, 0, 1)))          # vpbroadcastd r: m
    return out


def gen_probe_cases(rng):
    """Targeted: the aligned forms misaligned under an empty / one-element mask,
    and stores / loads across the boundary to the absent page under every mask
    shape (none, all ones, only the next page's elements, the straddling
    element highest, a low element only)."""
    cases = []

    def one(nm, code, toff, guard, kv, aaa):
        regs = [rand_val(rng) for _ in range(16)]
        c = mk_case(rng, nm, code, regs, {RSP: 0x80, 0: toff}, {}, guard)
        if aaa:
            c["k"][aaa] = kv
        cases.append(c)

    for nm, pp, w, es, opc in (("vmovdqa32", 1, 0, 4, 0x6F), ("vmovdqa64", 1, 1, 8, 0x6F), ("vmovaps", 0, 0, 4, 0x28)):
        for store in (0, 1):
            for ll in range(3):
                vlb = 16 << ll
                for kv in (0, 1, 1 << (vlb // es - 1)):
                    code = evex(1, pp, w, ll, 0, 0, 3, rng.randrange(32), 0, opc + (0x10 if store and opc == 0x6F
                                                                                      else 1 if store else 0),
                                mem=(0, None, 0, 0, 1))
                    one(f"{nm}.L{ll}.m.align{'st' if store else 'ld'}", code, 64 + es, 0, kv, 3)
    for nm, pp, w, es in (("vmovdqu8", 3, 0, 1), ("vmovdqu16", 3, 1, 2), ("vmovdqu32", 2, 0, 4),
                          ("vmovdqu64", 2, 1, 8)):
        for store in (0, 1):
            for ll in range(3):
                vlb = 16 << ll
                n = vlb // es
                for shift in (0, es // 2 if es > 1 else 0):
                    toff = BOUND - vlb // 2 - shift        # elements n/2.. on the absent page (one straddles if shift)
                    first_out = (BOUND - toff) // es       # the first element that touches the absent page
                    full = (1 << n) - 1
                    masks = [(0, 0), (full, 5), ((full >> first_out) << first_out, 5),
                             ((1 << (first_out - 1)) | (1 << first_out), 5), ((1 << first_out) - 1, 5), (1, 5),
                             (full & ~1, 5)]
                    if shift:
                        masks.append(((1 << (first_out - 1)), 5))  # the straddling element alone
                    for guard in (1, 2):
                        for kv, aaa in masks:
                            code = evex(1, pp, w, ll, 0, 0, aaa, rng.randrange(32), 0, 0x7F if store else 0x6F,
                                        mem=(0, None, 0, 0, 1))
                            one(f"{nm}.L{ll}.m.guard{'st' if store else 'ld'}", code, toff, guard, kv, aaa)
    return cases


def gen_kop_cases(rng):
    cases = []
    K = []
    for nm, opc in (("kand", 0x41), ("kandn", 0x42), ("kor", 0x45), ("kxnor", 0x46), ("kxor", 0x47)):
        for pp, w, sfx in ((0, 0, "w"), (0, 1, "q"), (1, 0, "b"), (1, 1, "d")):
            K += [(nm + sfx, lambda r, pp=pp, w=w, opc=opc: vex3(1, pp, w, 1, r.randrange(8), r.randrange(8), opc,
                                                                  rm=r.randrange(8)), {})] * 6
    for pp, w, sfx in ((0, 0, "w"), (0, 1, "q"), (1, 0, "b"), (1, 1, "d")):
        for nm, opc in (("knot", 0x44), ("kortest", 0x98), ("ktest", 0x99), ("kmov", 0x90)):
            K += [(nm + sfx, lambda r, pp=pp, w=w, opc=opc: vex3(1, pp, w, 0, r.randrange(8), 0, opc,
                                                                  rm=r.randrange(8)), {})] * 6
        K += [("kmov" + sfx + ".m", lambda r, pp=pp, w=w: ("mem", 1, pp, w, 0x90), {})] * 6
        K += [("kmov" + sfx + ".st", lambda r, pp=pp, w=w: ("mem", 1, pp, w, 0x91), {})] * 6
    for pp, w, sfx in ((0, 0, "w"), (1, 0, "b"), (3, 0, "d"), (3, 1, "q")):
        K += [("kmov" + sfx + ".fromr", lambda r, pp=pp, w=w: vex3(1, pp, w, 0, r.randrange(8), 0, 0x92,
                                                                  rm=r.randrange(16)), {})] * 6
        K += [("kmov" + sfx + ".tor", lambda r, pp=pp, w=w: vex3(1, pp, w, 0, r.randrange(16), 0, 0x93,
                                                                rm=r.randrange(8)), {})] * 6
    for pp, w, sfx in ((0, 0, "w"), (0, 1, "q"), (1, 0, "b"), (1, 1, "d")):
        K += [("kadd" + sfx, lambda r, pp=pp, w=w: vex3(1, pp, w, 1, r.randrange(8), r.randrange(8), 0x4A,
                                                         rm=r.randrange(8)), {})] * 6
    for pp, w, sfx in ((1, 0, "bw"), (0, 0, "wd"), (0, 1, "dq")):
        K += [("kunpck" + sfx, lambda r, pp=pp, w=w: vex3(1, pp, w, 1, r.randrange(8), r.randrange(8), 0x4B,
                                                           rm=r.randrange(8)), {})] * 6
    for opc, nm in ((0x30, "kshiftr"), (0x31, "kshiftr"), (0x32, "kshiftl"), (0x33, "kshiftl")):
        for w in (0, 1):
            bits = (64 if w else 32) if opc & 1 else (16 if w else 8)
            sfx = {8: "b", 16: "w", 32: "d", 64: "q"}[bits]
            K += [(nm + sfx, lambda r, opc=opc, w=w, bits=bits: vex3(
                3, 1, w, 0, r.randrange(8), 0, opc, rm=r.randrange(8),
                imm=r.choice([0, 1, 2, 7, bits - 1, bits, bits + 3, r.randrange(256)])), {})] * 6
    for nm, fn, _ in K:
        code = fn(rng)
        regs = [rand_val(rng) for _ in range(16)]
        ptrs, smalls = {RSP: 0x80}, {}
        if code[0] == "mem":
            _, mp, pp, w, opc = code
            m = pick_mem(rng, regs, ptrs, smalls, rng.randrange(0, WIN - 8), 1, use_disp8=True)
            code = vex3(mp, pp, w, 0, rng.randrange(8), 0, opc, mem=m)
        cases.append(mk_case(rng, nm, code, regs, ptrs, smalls, 0))
    return cases


# ---------------------------------------------------------------- values
def case_inputs(seed):
    """zmm0-31 (8 u64 each) and the 512-byte window of a case, from its seed:
    registers share elements with each other and with the window, so the
    compares, minimums and tests meet equal, near and extreme values."""
    rng = random.Random(seed)
    pool = [rand_val(rng) for _ in range(24)]
    zmm = []
    for r in range(32):
        v = []
        for q in range(8):
            x = rng.random()
            if x < 0.3:
                v.append(rng.getrandbits(64))
            elif x < 0.55:
                v.append(rng.choice(pool))
            elif x < 0.7 and zmm:
                v.append(zmm[rng.randrange(len(zmm))][q])
            elif x < 0.85 and zmm:  # bytes mixed from another register's qword
                o = zmm[rng.randrange(len(zmm))][q]
                mk = int.from_bytes(bytes(rng.choice((0, 0xFF)) for _ in range(8)), "little")
                v.append((o & mk) | (rng.getrandbits(64) & ~mk & M64))
            else:
                v.append(rng.choice((0, M64, 0x8080808080808080, 0x7F7F7F7F7F7F7F7F, 0x0001000100010001)))
        zmm.append(v)
    win = bytearray()
    while len(win) < WIN:
        if rng.random() < 0.5:
            win += zmm[rng.randrange(32)][rng.randrange(8)].to_bytes(8, "little")
        else:
            win += rand_val(rng).to_bytes(8, "little")
    return zmm, bytes(win[:WIN])


def kvalue(rng, n):
    x = rng.random()
    full = (1 << n) - 1 if n < 64 else M64
    if x < 0.15:
        return full
    if x < 0.25:
        return 0
    if x < 0.4:
        return rng.getrandbits(64) & full
    return rng.getrandbits(64)


def mk_case(rng, name, code, regs, ptrs, smalls, guard, kmask_focus=None):
    for r, v in smalls.items():
        regs[r] = v
    for r, off in ptrs.items():
        regs[r] = off & M64
    k = [kvalue(rng, rng.choice((8, 16, 32, 64))) for _ in range(8)]
    if kmask_focus and kmask_focus[2]:   # guard cases: a mask that stops at / reaches past the boundary
        aaa, n, _ = kmask_focus
        if aaa:
            k[aaa] = rng.getrandbits(64) if rng.random() < 0.5 else ((1 << rng.randrange(1, n)) - 1)
    return {"name": name, "code": bytes(code).hex(), "regs": regs, "ptrs": sorted(ptrs),
            "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "k": k, "seed": rng.getrandbits(63), "guard": guard}


# ---------------------------------------------------------------- native run
C_SRC = r"""
#define _GNU_SOURCE
#include <setjmp.h>
#include <signal.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <ucontext.h>
typedef struct { uint64_t r[16]; uint64_t fl; uint64_t z[256]; uint64_t k[8]; } st_t;
st_t g_in, g_out;
uint64_t g_host_rsp;
uint64_t g_flagstack[64] __attribute__((aligned(64)));
uint8_t g_buf[3 * 4096] __attribute__((aligned(4096)));
"""
ZL = "".join(f'"vmovdqu64 g_in+{136 + 64 * i}(%rip), %zmm{i}\\n"\n' for i in range(32))
KL = "".join(f'"kmovq g_in+{2184 + 8 * i}(%rip), %k{i}\\n"\n' for i in range(8))
ZS = "".join(f'"vmovdqu64 %zmm{i}, g_out+{136 + 64 * i}(%rip)\\n"\n' for i in range(32))
KS = "".join(f'"kmovq %k{i}, g_out+{2184 + 8 * i}(%rip)\\n"\n' for i in range(8))
STUB = r"""
__asm__(
".text\n.globl t_{i}\nt_{i}:\n"
"push %rbx\npush %rbp\npush %r12\npush %r13\npush %r14\npush %r15\n"
"mov %rsp, g_host_rsp(%rip)\n"
""" + ZL + KL + r"""
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
""" + ZS + KS + r"""
"vzeroupper\n"
"mov g_host_rsp(%rip), %rsp\n"
"pop %r15\npop %r14\npop %r13\npop %r12\npop %rbp\npop %rbx\nret\n");
void t_{i}(void);
"""
C_MAIN = r"""
typedef void (*fn_t)(void);
static fn_t fns[] = { FNLIST };
static sigjmp_buf g_jb;
static volatile long g_trapno, g_err;
static volatile uint64_t g_addr;
static void on_sig(int sig, siginfo_t *si, void *uc) {
  mcontext_t *mc = &((ucontext_t *)uc)->uc_mcontext;
  g_trapno = sig == SIGILL ? 6 : mc->gregs[REG_TRAPNO];
  g_err = mc->gregs[REG_ERR];
  g_addr = (uint64_t)(uintptr_t)si->si_addr;
  siglongjmp(g_jb, 1);
}
static char g_altstack[65536];
int main(void) {
  int form, nptr, ptrs[16], guard;
  unsigned long long flags, regs[16], zm[256], km[8];
  unsigned int wb[512];
  uint8_t *win = g_buf + 0xf00, *page0 = g_buf, *page1 = g_buf + 0x1000;
  stack_t ss = {.ss_sp = g_altstack, .ss_size = sizeof(g_altstack)};
  sigaltstack(&ss, 0);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_sig;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK | SA_NODEFER;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGILL, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
  printf("BUF %llx\n", (unsigned long long)(uintptr_t)win);
  while (scanf("%d %d %llx", &form, &guard, &flags) == 3) {
    for (int i = 0; i < 16; i++) if (scanf("%llx", &regs[i]) != 1) return 1;
    for (int i = 0; i < 256; i++) if (scanf("%llx", &zm[i]) != 1) return 1;
    for (int i = 0; i < 8; i++) if (scanf("%llx", &km[i]) != 1) return 1;
    for (int i = 0; i < 512; i++) if (scanf("%2x", &wb[i]) != 1) return 1;
    if (scanf("%d", &nptr) != 1) return 1;
    for (int i = 0; i < nptr; i++) if (scanf("%d", &ptrs[i]) != 1) return 1;
    mprotect(page0, 4096, PROT_READ | PROT_WRITE);
    mprotect(page1, 4096, PROT_READ | PROT_WRITE);
    memset(g_buf, 0, sizeof(g_buf));
    for (int i = 0; i < 512; i++) win[i] = (uint8_t)wb[i];
    if (guard) mprotect(guard == 2 ? page0 : page1, 4096, PROT_NONE);
    for (int i = 0; i < 16; i++) g_in.r[i] = regs[i];
    for (int i = 0; i < nptr; i++) g_in.r[ptrs[i]] = (uint64_t)(uintptr_t)win + regs[ptrs[i]];
    for (int i = 0; i < 256; i++) g_in.z[i] = zm[i];
    for (int i = 0; i < 8; i++) g_in.k[i] = km[i];
    g_in.fl = flags;
    if (sigsetjmp(g_jb, 1)) {
      __asm__ volatile("vzeroupper");
      mprotect(page0, 4096, PROT_READ | PROT_WRITE);
      mprotect(page1, 4096, PROT_READ | PROT_WRITE);
      printf("T %lx %lx %llx\nM", g_trapno, g_err, (unsigned long long)g_addr);
      for (int i = 0; i < 512; i++) printf("%02x", ((guard == 1 && i >= 256) || (guard == 2 && i < 256)) ? 0 : win[i]);
      printf("\n");
      continue;
    }
    fns[form]();
    mprotect(page0, 4096, PROT_READ | PROT_WRITE);
    mprotect(page1, 4096, PROT_READ | PROT_WRITE);
    printf("R");
    for (int i = 0; i < 16; i++) printf(" %llx", (unsigned long long)g_out.r[i]);
    printf(" %llx\nZ", (unsigned long long)g_out.fl);
    for (int i = 0; i < 256; i++) printf(" %llx", (unsigned long long)g_out.z[i]);
    printf("\nK");
    for (int i = 0; i < 8; i++) printf(" %llx", (unsigned long long)g_out.k[i]);
    printf("\nM");
    for (int i = 0; i < 512; i++) printf("%02x", ((guard == 1 && i >= 256) || (guard == 2 && i < 256)) ? 0 : win[i]);
    printf("\n");
  }
  return 0;
}
"""


def window_of(c):
    """The window a case starts with (zeros on the absent page of a guard case)."""
    _, win = case_inputs(c["seed"] if isinstance(c["seed"], int) else int(c["seed"], 16))
    return guard_window(win, c["guard"])


def guard_window(win, guard):
    if guard == 1:
        return win[:BOUND] + bytes(WIN - BOUND)
    if guard == 2:
        return bytes(BOUND) + win[BOUND:]
    return win


def run_native(cases, out_path):
    uniq = {}
    for c in cases:
        uniq.setdefault(c["code"], len(uniq))
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "z.c")
        with open(src, "w") as f:
            f.write(C_SRC)
            for code, i in uniq.items():
                bs = ",".join("0x%02x" % b for b in bytes.fromhex(code))
                f.write(STUB.replace("{i}", str(i)).replace("{bytes}", bs))
            f.write(C_MAIN.replace("FNLIST", ",".join(f"t_{i}" for i in range(len(uniq)))))
        exe = os.path.join(td, "z")
        subprocess.check_call(["gcc", "-O1", "-no-pie", "-o", exe, src])
        lines = []
        for c in cases:
            zmm, _ = case_inputs(c["seed"])
            lines.append("%d %d %x %s %s %s %s %d %s" % (
                uniq[c["code"]], c["guard"], c["flags"], " ".join("%x" % v for v in c["regs"]),
                " ".join("%x" % v for r in zmm for v in r), " ".join("%x" % v for v in c["k"]),
                window_of(c).hex(), len(c["ptrs"]), " ".join(str(p) for p in c["ptrs"])))
        out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
    buf_va = int(out[0].split()[1], 16)
    res = []
    k = 1
    nfault = 0
    for c in cases:
        inregs = list(c["regs"])
        for p in c["ptrs"]:
            inregs[p] = (buf_va + inregs[p]) & M64
        zmm, _ = case_inputs(c["seed"])
        zin = [v for r in zmm for v in r]
        before = window_of(c)
        e = {"name": c["name"], "code": c["code"], "in": ["%x" % v for v in inregs], "fl": "%x" % c["flags"],
             "seed": "%x" % c["seed"], "k": ["%x" % v for v in c["k"]], "guard": c["guard"]}
        if out[k].startswith("T"):
            t = out[k].split()
            e["fault"] = {"vec": int(t[1], 16), "err": int(t[2], 16), "addr": t[3]}
            ml = out[k + 1][1:]
            k += 2
            nfault += 1
        else:
            rl, zl, kl, ml = out[k].split(), out[k + 1].split(), out[k + 2].split(), out[k + 3][1:]
            k += 4
            gout = [int(v, 16) for v in rl[1:17]]
            zout = [int(v, 16) for v in zl[1:257]]
            e.update({"gdiff": [[i, "%x" % gout[i]] for i in range(16) if gout[i] != inregs[i]], "flo": rl[17],
                      "zdiff": [[i, "%x" % zout[i]] for i in range(256) if zout[i] != zin[i]],
                      "ko": kl[1:9]})
        after = bytes.fromhex(ml)
        e["mdiff"] = [[i, after[i]] for i in range(WIN) if after[i] != before[i]]
        res.append(e)
    doc = {"buf_va": "%x" % buf_va, "window": WIN, "bound": BOUND,
           "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "generator": "tests/golden/gen_avx512_vectors.py", "cases": res}
    with gzip.open(out_path, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"wrote {len(res)} vectors ({len(uniq)} encodings, {nfault} faulted) to {out_path}")


def main():
    rng = random.Random(0xA5125)
    cases = gen_evex_cases(rng) + gen_kop_cases(rng) + gen_probe_cases(rng)
    for nm, code in gen_ud_cases(rng):
        regs = [rand_val(rng) for _ in range(16)]
        cases.append(mk_case(rng, nm, code, regs, {RSP: 0x80, 0: 0x40}, {}, 0))
    run_native(cases, OUT)


if __name__ == "__main__":
    main()
