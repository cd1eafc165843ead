#!/usr/bin/env python3
"""Native-execution golden vectors for the SSE/SSE2 subset.

Same method as gen_native_vectors.py: one stub per instruction form loads the 16
GPRs, RFLAGS, the 16 XMM registers and MXCSR from a global, executes the
instruction bytes natively on the x86-64 host, and stores everything back.
Memory operands point into the 256-byte window at g_buf + 0x800; aligned forms
get 16-byte aligned addresses (a misaligned one would #GP the native run: those
cases are checked oracle-vs-GPU instead, tests/test_sse.py).

Output: tests/golden/sse_vectors.json.gz. Re-run with
    python tests/golden/gen_sse_vectors.py
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
from tests.golden.gen_native_vectors import WIN, rand_val, rex_for, splitmix_bytes  # noqa: E402

OUT = os.path.join(HERE, "sse_vectors.json.gz")
RSP = 4
NP, P66, F3, F2 = [], [0x66], [0xF3], [0xF2]

# xmm, xmm/m128 (16-byte aligned memory)
XX_A = [(NP, 0x14, "unpcklps"), (NP, 0x15, "unpckhps"), (P66, 0x14, "unpcklpd"), (P66, 0x15, "unpckhpd"),
        (NP, 0x28, "movaps"), (P66, 0x28, "movapd"), (NP, 0x54, "andps"), (P66, 0x54, "andpd"),
        (NP, 0x55, "andnps"), (P66, 0x55, "andnpd"), (NP, 0x56, "orps"), (P66, 0x56, "orpd"),
        (NP, 0x57, "xorps"), (P66, 0x57, "xorpd"), (P66, 0x6F, "movdqa")]
XX_A += [(P66, op, "p%02x" % op) for op in list(range(0x60, 0x6E)) + [0x74, 0x75, 0x76]]
XX_A += [(P66, op, "p%02x" % op) for op in
         [0xD1, 0xD2, 0xD3, 0xD4, 0xD5, 0xD8, 0xD9, 0xDA, 0xDB, 0xDC, 0xDD, 0xDE, 0xDF, 0xE0, 0xE1, 0xE2, 0xE3,
          0xE4, 0xE5, 0xE8, 0xE9, 0xEA, 0xEB, 0xEC, 0xED, 0xEE, 0xEF, 0xF1, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF8,
          0xF9, 0xFA, 0xFB, 0xFC, 0xFD, 0xFE]]
SHIFT_BY_XMM = {0xD1, 0xD2, 0xD3, 0xE1, 0xE2, 0xF1, 0xF2, 0xF3}
# xmm, xmm/m128 unaligned
XX_U = [(NP, 0x10, "movups"), (P66, 0x10, "movupd"), (F3, 0x6F, "movdqu")]
# xmm, xmm/m128, imm8 (aligned)
XX_IMM = [(P66, 0x70, "pshufd"), (F3, 0x70, "pshufhw"), (F2, 0x70, "pshuflw"), (NP, 0xC6, "shufps"),
          (P66, 0xC6, "shufpd")]
# xmm/m128 <- xmm
ST_A = [(NP, 0x29, "movaps.st"), (P66, 0x29, "movapd.st"), (P66, 0x7F, "movdqa.st")]
ST_A_MEM = [(NP, 0x2B, "movntps"), (P66, 0x2B, "movntpd"), (P66, 0xE7, "movntdq")]
ST_U = [(NP, 0x11, "movups.st"), (P66, 0x11, "movupd.st"), (F3, 0x7F, "movdqu.st")]
# (prefix, opcode, name, memory size): reg-reg and memory forms
SCALAR = [(F3, 0x10, "movss", 4), (F3, 0x11, "movss.st", 4), (F2, 0x10, "movsd", 8), (F2, 0x11, "movsd.st", 8),
          (F3, 0x7E, "movq.ld", 8), (P66, 0xD6, "movq.st", 8)]
# memory-only m64 forms; the np 0f 12 / 16 register forms are movhlps / movlhps
M64 = [(NP, 0x12, "movlps"), (P66, 0x12, "movlpd"), (NP, 0x13, "movlps.st"), (P66, 0x13, "movlpd.st"),
       (NP, 0x16, "movhps"), (P66, 0x16, "movhpd"), (NP, 0x17, "movhps.st"), (P66, 0x17, "movhpd.st")]
HL = [(NP, 0x12, "movhlps"), (NP, 0x16, "movlhps")]
GX = [(NP, 0x50, "movmskps"), (P66, 0x50, "movmskpd"), (P66, 0xD7, "pmovmskb")]
SHIFT_IMM = [(0x71, 2), (0x71, 4), (0x71, 6), (0x72, 2), (0x72, 4), (0x72, 6), (0x73, 2), (0x73, 3), (0x73, 6),
             (0x73, 7)]


class Form:
    def __init__(self, code, name, ptrs=(), smalls=(), xsmall=None, mx=False):
        self.code = bytes(code)
        self.name = name
        self.ptrs = dict(ptrs)
        self.smalls = dict(smalls)
        self.xsmall = xsmall  # xmm register whose low qword is a small shift count
        self.mx = mx
        self.cls = "sse"


def enc_rr(pfx, opc, reg, rm, w=0):
    return pfx + rex_for(w, reg, 0, rm) + [0x0F, opc, 0xC0 | ((reg & 7) << 3) | (rm & 7)]


def enc_mem(rng, pfx, opc, reg, align, w=0):
    """reg, [mem] with a random addressing mode; the operand lands at a window
    offset aligned to `align` bytes (1 = any)."""
    off = rng.randrange(16, WIN - 48)
    off -= off % align
    kind = rng.choice(["base", "base8", "sib", "rbp8", "r13"])
    ptrs, smalls = {}, {}
    if kind in ("base", "base8"):
        base = rng.choice([3, 6, 7, 0, 1, 2, 9, 10, 11, 14, 15])
        disp = [] if kind == "base" else [rng.randrange(0, 16)]
        mod = 0 if kind == "base" else 1
        code = pfx + rex_for(w, reg, 0, base) + [0x0F, opc, (mod << 6) | ((reg & 7) << 3) | (base & 7)] + disp
        ptrs[base] = off - (disp[0] if disp else 0)
    elif kind in ("rbp8", "r13"):
        base = 5 if kind == "rbp8" else 13
        d = rng.randrange(0, 32)
        code = pfx + rex_for(w, reg, 0, base) + [0x0F, opc, (1 << 6) | ((reg & 7) << 3) | (base & 7), d]
        ptrs[base] = off - d
    else:
        base = rng.choice([3, 6, 7, 12, 9])
        index = rng.choice([1, 2, 8, 10])
        ss, iv, d = rng.randrange(4), rng.randrange(0, 4), rng.randrange(0, 32)
        code = (pfx + rex_for(w, reg, index, base) +
                [0x0F, opc, (1 << 6) | ((reg & 7) << 3) | 4, (ss << 6) | ((index & 7) << 3) | (base & 7), d])
        ptrs[base] = off - d - (iv << ss)
        smalls[index] = (iv, iv)
    return code, ptrs, smalls


def gen_forms(rng):
    forms = []
    x = lambda: rng.randrange(16)  # noqa: E731
    g = lambda: rng.choice([r for r in range(16) if r != RSP])  # noqa: E731

    for pfx, op, nm in XX_A:
        for _ in range(3):
            src = x()
            forms.append(Form(enc_rr(pfx, op, x(), src), nm + ".rr", xsmall=src if op in SHIFT_BY_XMM else None))
        code, p, s = enc_mem(rng, pfx, op, x(), 16)
        forms.append(Form(code, nm + ".m", p, s))
    for pfx, op, nm in XX_U:
        forms.append(Form(enc_rr(pfx, op, x(), x()), nm + ".rr"))
        for _ in range(2):
            code, p, s = enc_mem(rng, pfx, op, x(), 1)
            forms.append(Form(code, nm + ".m", p, s))
    for pfx, op, nm in XX_IMM:
        for _ in range(3):
            forms.append(Form(enc_rr(pfx, op, x(), x()) + [rng.randrange(256)], nm + ".rr"))
        code, p, s = enc_mem(rng, pfx, op, x(), 16)
        forms.append(Form(code + [rng.randrange(256)], nm + ".m", p, s))
    for pfx, op, nm in ST_A + ST_U:
        forms.append(Form(enc_rr(pfx, op, x(), x()), nm + ".rr"))
    for pfx, op, nm in ST_A + ST_A_MEM:
        code, p, s = enc_mem(rng, pfx, op, x(), 16)
        forms.append(Form(code, nm + ".m", p, s))
    for pfx, op, nm in ST_U:
        for _ in range(2):
            code, p, s = enc_mem(rng, pfx, op, x(), 1)
            forms.append(Form(code, nm + ".m", p, s))
    for pfx, op, nm, _sz in SCALAR:
        for _ in range(2):
            forms.append(Form(enc_rr(pfx, op, x(), x()), nm + ".rr"))
            code, p, s = enc_mem(rng, pfx, op, x(), 1)
            forms.append(Form(code, nm + ".m", p, s))
    for pfx, op, nm in M64:
        for _ in range(2):
            code, p, s = enc_mem(rng, pfx, op, x(), 1)
            forms.append(Form(code, nm + ".m", p, s))
    for pfx, op, nm in HL:
        for _ in range(2):
            forms.append(Form(enc_rr(pfx, op, x(), x()), nm))
    # movd / movq with general registers
    for w in (0, 1):
        for _ in range(2):
            forms.append(Form(enc_rr(P66, 0x6E, x(), g(), w), f"movd.xg.w{w}"))
            forms.append(Form(enc_rr(P66, 0x7E, x(), g(), w), f"movd.gx.w{w}"))
        for op in (0x6E, 0x7E):
            code, p, s = enc_mem(rng, P66, op, x(), 1, w)
            forms.append(Form(code, f"movd.{op:x}.m.w{w}", p, s))
    for pfx, op, nm in GX:
        for _ in range(2):
            forms.append(Form(enc_rr(pfx, op, g(), x(), rng.randrange(2)), nm))
    for _ in range(3):
        forms.append(Form(enc_rr(P66, 0xC5, g(), x()) + [rng.randrange(256)], "pextrw"))
        forms.append(Form(enc_rr(P66, 0xC4, x(), g()) + [rng.randrange(256)], "pinsrw.r"))
    code, p, s = enc_mem(rng, P66, 0xC4, x(), 1)
    forms.append(Form(code + [rng.randrange(256)], "pinsrw.m", p, s))
    for op, sub in SHIFT_IMM:
        for cnt in rng.sample([0, 1, 3, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 200], 5):
            forms.append(Form(enc_rr(P66, op, sub, x()) + [cnt], f"shimm.{op:x}.{sub}"))
    # ldmxcsr / stmxcsr, fences, movnti
    for sub, nm in ((2, "ldmxcsr"), (3, "stmxcsr")):
        for _ in range(2):
            code, p, s = enc_mem(rng, NP, 0xAE, sub, 4)
            forms.append(Form(code, nm, p, s, mx=sub == 2))
    for b in (0xE8, 0xF0, 0xF8):
        forms.append(Form([0x0F, 0xAE, b], "fence%x" % b))
    for w in (0, 1):
        code, p, s = enc_mem(rng, NP, 0xC3, g(), 1, w)
        forms.append(Form(code, f"movnti.w{w}", p, s))
    return forms


def rand_xmm(rng):
    r = rng.random()
    if r < 0.1:
        return [0, 0]
    if r < 0.2:
        return [(1 << 64) - 1, (1 << 64) - 1]
    if r < 0.35:  # bytes from a small alphabet: equal / signed-boundary elements
        b = bytes(rng.choice([0, 1, 0x7F, 0x80, 0xFF, 0x41]) for _ in range(16))
        return [int.from_bytes(b[:8], "little"), int.from_bytes(b[8:], "little")]
    return [rng.getrandbits(64), rng.getrandbits(64)]


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
            xmm = [rand_xmm(rng) for _ in range(16)]
            if rng.random() < 0.4:  # sources equal to destinations in part: compare hits
                a, b = rng.randrange(16), rng.randrange(16)
                xmm[a] = [xmm[b][0], xmm[a][1]]
            if f.xsmall is not None and rng.random() < 0.7:
                xmm[f.xsmall] = [rng.choice([0, 1, 2, 7, 8, 15, 16, 31, 32, 63, 64, 65]), xmm[f.xsmall][1]]
            seed = rng.getrandbits(63)
            mx = 0x1F80 | (rng.getrandbits(16) & 0x603F & 0xFFBF)
            cases.append({
                "name": f.name, "code": f.code.hex(), "regs": regs, "ptrs": sorted(f.ptrs) + [RSP],
                "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "xmm": xmm, "mx": mx, "seed": seed, "ldmx": f.mx,
            })
    return cases


C_HEADER = r"""
#include <stdio.h>
#include <stdint.h>
#include <string.h>
typedef struct { uint64_t r[16]; uint64_t fl; uint64_t x[32]; uint32_t mx, pad; } st_t;
st_t g_in, g_out;
uint64_t g_host_rsp;
uint32_t g_host_mx;
uint64_t g_flagstack[64] __attribute__((aligned(16)));
uint8_t g_buf[8192] __attribute__((aligned(4096)));
"""

XLOAD = "".join('"movdqu g_in+%d(%%rip), %%xmm%d\\n"\n' % (136 + 16 * i, i) for i in range(16))
XSTORE = "".join('"movdqu %%xmm%d, g_out+%d(%%rip)\\n"\n' % (i, 136 + 16 * i) for i in range(16))

STUB = r"""
__asm__(
".text\n.globl t_{i}\nt_{i}:\n"
"push %rbx\npush %rbp\npush %r12\npush %r13\npush %r14\npush %r15\n"
"mov %rsp, g_host_rsp(%rip)\n"
"stmxcsr g_host_mx(%rip)\nldmxcsr g_in+392(%rip)\n"
""" + XLOAD + r"""
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
""" + XSTORE + r"""
"stmxcsr g_out+392(%rip)\nldmxcsr g_host_mx(%rip)\n"
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
  int form, nptr, ptrs[16], ldmx; unsigned long long seed, flags, mx, regs[16], xm[32];
  uint8_t *win = g_buf + 0x800;
  printf("BUF %llx\n", (unsigned long long)(uintptr_t)win);
  while (scanf("%d %llx %llx %llx %d", &form, &seed, &flags, &mx, &ldmx) == 5) {
    for (int i = 0; i < 16; i++) scanf("%llx", &regs[i]);
    for (int i = 0; i < 32; i++) scanf("%llx", &xm[i]);
    scanf("%d", &nptr);
    for (int i = 0; i < nptr; i++) scanf("%d", &ptrs[i]);
    uint64_t x = seed;
    for (int i = 0; i < 256; i += 8) { uint64_t v = sm(&x); memcpy(win + i, &v, 8); }
    if (ldmx)  /* ldmxcsr operands: valid values, exceptions masked */
      for (int i = 0; i < 256; i += 4) { uint32_t v; memcpy(&v, win + i, 4); v = 0x1f80 | (v & 0x603f & 0xffbf); memcpy(win + i, &v, 4); }
    for (int i = 0; i < 16; i++) g_in.r[i] = regs[i];
    for (int i = 0; i < nptr; i++) g_in.r[ptrs[i]] = (uint64_t)(uintptr_t)win + regs[ptrs[i]];
    for (int i = 0; i < 32; i++) g_in.x[i] = xm[i];
    g_in.fl = flags;
    g_in.mx = (uint32_t)mx;
    fns[form]();
    printf("R");
    for (int i = 0; i < 16; i++) printf(" %llx", (unsigned long long)g_out.r[i]);
    printf(" %llx\nX", (unsigned long long)g_out.fl);
    for (int i = 0; i < 32; i++) printf(" %llx", (unsigned long long)g_out.x[i]);
    printf(" %x\nM", g_out.mx);
    for (int i = 0; i < 256; i++) printf("%02x", win[i]);
    printf("\n");
  }
  return 0;
}
"""


def window_in(seed, ldmx):
    """The window bytes the stub starts from (ldmxcsr cases: valid MXCSR dwords)."""
    w = bytearray(splitmix_bytes(seed, WIN))
    if ldmx:
        for i in range(0, WIN, 4):
            v = int.from_bytes(w[i:i + 4], "little")
            w[i:i + 4] = (0x1F80 | (v & 0x603F & 0xFFBF)).to_bytes(4, "little")
    return bytes(w)


def main():
    rng = random.Random(0x55E0001)
    forms = gen_forms(rng)
    cases = make_cases(forms, rng)
    uniq = {}
    for c in cases:
        uniq.setdefault(c["code"], len(uniq))
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "sv.c")
        with open(src, "w") as f:
            f.write(C_HEADER)
            for code, i in uniq.items():
                bs = ",".join("0x%02x" % b for b in bytes.fromhex(code))
                f.write(STUB.replace("{i}", str(i)).replace("{bytes}", bs))
            f.write(C_MAIN.replace("FNLIST", ",".join(f"t_{i}" for i in range(len(uniq)))))
        exe = os.path.join(td, "sv")
        subprocess.check_call(["gcc", "-O1", "-no-pie", "-o", exe, src])
        lines = []
        for c in cases:
            xs = [v for pair in c["xmm"] for v in pair]
            lines.append("%d %x %x %x %d %s %s %d %s" % (
                uniq[c["code"]], c["seed"], c["flags"], c["mx"], int(c["ldmx"]),
                " ".join("%x" % v for v in c["regs"]), " ".join("%x" % v for v in xs),
                len(c["ptrs"]), " ".join(str(p) for p in c["ptrs"])))
        out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
    buf_va = int(out[0].split()[1], 16)
    res = []
    k = 1
    for c in cases:
        rl, xl, ml = out[k].split(), out[k + 1].split(), out[k + 2][1:]
        k += 3
        before = window_in(c["seed"], c["ldmx"])
        after = bytes.fromhex(ml)
        inregs = list(c["regs"])
        for p in c["ptrs"]:
            inregs[p] = (buf_va + inregs[p]) & 0xFFFFFFFFFFFFFFFF
        res.append({
            "name": c["name"], "code": c["code"], "in": ["%x" % v for v in inregs], "fl": "%x" % c["flags"],
            "xin": ["%x" % v for pair in c["xmm"] for v in pair], "mx": "%x" % c["mx"], "ldmx": int(c["ldmx"]),
            "out": rl[1:17], "flo": rl[17], "xout": xl[1:33], "mxo": xl[33], "seed": "%x" % c["seed"],
            "diff": [[i, after[i]] for i in range(WIN) if after[i] != before[i]],
        })
    doc = {"buf_va": "%x" % buf_va, "window": WIN,
           "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "generator": "tests/golden/gen_sse_vectors.py", "cases": res}
    with gzip.open(OUT, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"wrote {len(res)} vectors ({len(uniq)} encodings) to {OUT}")


if __name__ == "__main__":
    main()
