#!/usr/bin/env python3
"""Native-execution golden vectors for MMX (U37, oracle/x86_oracle.c exec_mmx).

Same method as gen_sse_vectors.py: one stub per instruction form loads the 16
GPRs, RFLAGS, the 16 XMM registers and mm0-7 from a global, executes the
instruction bytes natively on the x86-64 host, then FXSAVEs the x87 / MMX
state (mm values, FSW, the abridged tag byte: TOS and tags after the
instruction) and stores the GPRs, flags and XMM registers. Memory operands
point into the 256-byte window at g_buf + 0x800 (MMX memory operands need no
alignment). mm ModRM fields are drawn from 0-15 so that REX.R / REX.B are set
on some forms: the CPU ignores them for mm registers.

Output: tests/golden/mmx_vectors.json.gz. Re-run with
    python tests/golden/gen_mmx_vectors.py
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
from tests.golden.gen_sse_vectors import enc_mem, enc_rr, rand_xmm  # noqa: E402

OUT = os.path.join(HERE, "mmx_vectors.json.gz")
RSP = 4
NP, F3, F2 = [], [0xF3], [0xF2]

# mm, mm/m64
MM = list(range(0x60, 0x6C)) + [0x74, 0x75, 0x76, 0x6F]
MM += [0xD1, 0xD2, 0xD3, 0xD4, 0xD5, 0xD8, 0xD9, 0xDA, 0xDB, 0xDC, 0xDD, 0xDE, 0xDF, 0xE0, 0xE1, 0xE2, 0xE3, 0xE4,
       0xE5, 0xE8, 0xE9, 0xEA, 0xEB, 0xEC, 0xED, 0xEE, 0xEF, 0xF1, 0xF2, 0xF3, 0xF4, 0xF5, 0xF6, 0xF8, 0xF9, 0xFA,
       0xFB, 0xFC, 0xFD, 0xFE]
SHIFT_BY_MM = {0xD1, 0xD2, 0xD3, 0xE1, 0xE2, 0xF1, 0xF2, 0xF3}
SHIFT_IMM = [(0x71, 2), (0x71, 4), (0x71, 6), (0x72, 2), (0x72, 4), (0x72, 6), (0x73, 2), (0x73, 6)]


class Form:
    def __init__(self, code, name, ptrs=(), smalls=(), msmall=None):
        self.code = bytes(code)
        self.name = name
        self.ptrs = dict(ptrs)
        self.smalls = dict(smalls)
        self.msmall = msmall  # mm register holding a small shift count


def gen_forms(rng):
    forms = []
    m = lambda: rng.randrange(16)  # noqa: E731  mm field: 8-15 set REX bits, which the CPU ignores
    x = lambda: rng.randrange(16)  # noqa: E731
    g = lambda: rng.choice([r for r in range(16) if r != RSP])  # noqa: E731
    for op in MM:
        for _ in range(3):
            src = m()
            forms.append(Form(enc_rr(NP, op, m(), src), "m%02x.rr" % op,
                              msmall=(src & 7) if op in SHIFT_BY_MM else None))
        code, p, s = enc_mem(rng, NP, op, m(), 1)
        forms.append(Form(code, "m%02x.m" % op, p, s))
    for _ in range(3):
        forms.append(Form(enc_rr(NP, 0x70, m(), m()) + [rng.randrange(256)], "pshufw.rr"))
    code, p, s = enc_mem(rng, NP, 0x70, m(), 1)
    forms.append(Form(code + [rng.randrange(256)], "pshufw.m", p, s))
    for op, sub in SHIFT_IMM:
        for cnt in rng.sample([0, 1, 3, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 200], 5):
            forms.append(Form(enc_rr(NP, op, sub, m()) + [cnt], f"shimm.{op:x}.{sub}"))
    for op, nm in ((0x7F, "movq.st"), (0xE7, "movntq")):
        if op == 0x7F:
            for _ in range(2):
                forms.append(Form(enc_rr(NP, op, m(), m()), nm + ".rr"))
        for _ in range(2):
            code, p, s = enc_mem(rng, NP, op, m(), 1)
            forms.append(Form(code, nm + ".m", p, s))
    for w in (0, 1):
        for _ in range(2):
            forms.append(Form(enc_rr(NP, 0x6E, m() & 7, g(), w), f"movd.mg.w{w}"))
            forms.append(Form(enc_rr(NP, 0x7E, m() & 7, g(), w), f"movd.gm.w{w}"))
        for op in (0x6E, 0x7E):
            code, p, s = enc_mem(rng, NP, op, m(), 1, w)
            forms.append(Form(code, f"movd.{op:x}.m.w{w}", p, s))
    for _ in range(3):
        forms.append(Form(enc_rr(NP, 0xC5, g(), m()) + [rng.randrange(256)], "pextrw"))
        forms.append(Form(enc_rr(NP, 0xC4, m() & 7, g()) + [rng.randrange(256)], "pinsrw.r"))
        forms.append(Form(enc_rr(NP, 0xD7, g(), m(), rng.randrange(2)), "pmovmskb"))
    code, p, s = enc_mem(rng, NP, 0xC4, m(), 1)
    forms.append(Form(code + [rng.randrange(256)], "pinsrw.m", p, s))
    for _ in range(3):
        forms.append(Form(enc_rr(F3, 0xD6, x(), m()), "movq2dq"))
        forms.append(Form(enc_rr(F2, 0xD6, m(), x()), "movdq2q"))
    forms.append(Form([0x0F, 0x77], "emms"))
    # ---- the MMX-operand conversions (own generator: the forms above keep their cases)
    crng = random.Random(0xC7)
    cm = lambda: crng.randrange(16)  # noqa: E731
    for pfx, sfx in ((NP, "ps"), ([0x66], "pd")):
        for _ in range(4):
            forms.append(Form(enc_rr(pfx, 0x2A, cm(), cm()), f"cvtpi2{sfx}.rr"))
        code, p, s = enc_mem(crng, pfx, 0x2A, cm(), 1)
        forms.append(Form(code, f"cvtpi2{sfx}.m", p, s))
        for op, nm in ((0x2C, "cvtt"), (0x2D, "cvt")):
            for _ in range(4):
                forms.append(Form(enc_rr(pfx, op, cm(), cm()), f"{nm}{sfx}2pi.rr"))
            code, p, s = enc_mem(crng, pfx, op, cm(), 16 if sfx == "pd" else 1)
            forms.append(Form(code, f"{nm}{sfx}2pi.m", p, s))
    # ---- SSSE3 on mm registers (0f 38 00-0b / 1c-1e, 0f 3a 0f) and maskmovq (own generator)
    srng = random.Random(0x55E3)
    sm_ = lambda: srng.randrange(16)  # noqa: E731

    def three(code, op):  # 0f <esc> modrm ... -> 0f <esc> op modrm ...
        i = code.index(0x0F)
        return code[:i + 2] + [op] + code[i + 2:]
    for esc, ops in ((0x38, list(range(0x00, 0x0C)) + [0x1C, 0x1D, 0x1E]), (0x3A, [0x0F])):
        for op in ops:
            nm = "palignr" if esc == 0x3A else "ssse3.%02x" % op
            for _ in range(4):
                code = three(enc_rr(NP, esc, sm_(), sm_()), op)
                forms.append(Form(code + ([srng.choice([0, 1, 3, 7, 8, 9, 15, 16, 17, 200])] if esc == 0x3A else []),
                                  nm + ".rr"))
            for _ in range(2):
                code, p, s = enc_mem(srng, NP, esc, sm_(), 1)
                forms.append(Form(three(code, op) + ([srng.randrange(24)] if esc == 0x3A else []), nm + ".m", p, s))
    for _ in range(6):
        forms.append(Form(enc_rr(NP, 0xF7, sm_(), sm_()), "maskmovq", {7: srng.randrange(16, WIN - 24)}))
    return forms


def rand_mm(rng):
    return rand_xmm(rng)[0]


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
            mm = [rand_mm(rng) for _ in range(8)]
            if rng.random() < 0.4:
                a, b = rng.randrange(8), rng.randrange(8)
                mm[a] = mm[b]
            if f.msmall is not None and rng.random() < 0.7:
                mm[f.msmall] = rng.choice([0, 1, 2, 7, 8, 15, 16, 31, 32, 63, 64, 65])
            cases.append({"name": f.name, "code": f.code.hex(), "regs": regs, "ptrs": sorted(f.ptrs) + [RSP],
                          "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "xmm": xmm, "mm": mm,
                          "seed": rng.getrandbits(63)})
    return cases


C_HEADER = r"""
#include <stdio.h>
#include <stdint.h>
#include <string.h>
typedef struct { uint64_t r[16]; uint64_t fl; uint64_t x[32]; uint64_t mm[8]; } st_t;
st_t g_in, g_out;
uint8_t g_fx[512] __attribute__((aligned(16)));
uint64_t g_host_rsp;
uint64_t g_flagstack[64] __attribute__((aligned(16)));
uint8_t g_buf[8192] __attribute__((aligned(4096)));
"""

XLOAD = "".join('"movdqu g_in+%d(%%rip), %%xmm%d\\n"\n' % (136 + 16 * i, i) for i in range(16))
XSTORE = "".join('"movdqu %%xmm%d, g_out+%d(%%rip)\\n"\n' % (i, 136 + 16 * i) for i in range(16))
MLOAD = "".join('"movq g_in+%d(%%rip), %%mm%d\\n"\n' % (392 + 8 * i, i) for i in range(8))

STUB = r"""
__asm__(
".text\n.globl t_{i}\nt_{i}:\n"
"push %rbx\npush %rbp\npush %r12\npush %r13\npush %r14\npush %r15\n"
"mov %rsp, g_host_rsp(%rip)\n"
""" + XLOAD + MLOAD + r"""
"lea g_flagstack+256(%rip), %rsp\n"
"pushq g_in+128(%rip)\npopfq\n"
"mov g_in+0(%rip), %rax\nmov g_in+8(%rip), %rcx\nmov g_in+16(%rip), %rdx\nmov g_in+24(%rip), %rbx\n"
"mov g_in+40(%rip), %rbp\nmov g_in+48(%rip), %rsi\nmov g_in+56(%rip), %rdi\n"
"mov g_in+64(%rip), %r8\nmov g_in+72(%rip), %r9\nmov g_in+80(%rip), %r10\nmov g_in+88(%rip), %r11\n"
"mov g_in+96(%rip), %r12\nmov g_in+104(%rip), %r13\nmov g_in+112(%rip), %r14\nmov g_in+120(%rip), %r15\n"
"mov g_in+32(%rip), %rsp\n"
".byte {bytes}\n"
"fxsave g_fx(%rip)\n"
"mov %rax, g_out+0(%rip)\nmov %rcx, g_out+8(%rip)\nmov %rdx, g_out+16(%rip)\nmov %rbx, g_out+24(%rip)\n"
"mov %rsp, g_out+32(%rip)\nmov %rbp, g_out+40(%rip)\nmov %rsi, g_out+48(%rip)\nmov %rdi, g_out+56(%rip)\n"
"mov %r8, g_out+64(%rip)\nmov %r9, g_out+72(%rip)\nmov %r10, g_out+80(%rip)\nmov %r11, g_out+88(%rip)\n"
"mov %r12, g_out+96(%rip)\nmov %r13, g_out+104(%rip)\nmov %r14, g_out+112(%rip)\nmov %r15, g_out+120(%rip)\n"
"lea g_flagstack+256(%rip), %rsp\npushfq\npopq g_out+128(%rip)\n"
""" + XSTORE + r"""
"emms\n"
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
  int form, nptr, ptrs[16]; unsigned long long seed, flags, regs[16], xm[32], mm[8];
  uint8_t *win = g_buf + 0x800;
  printf("BUF %llx\n", (unsigned long long)(uintptr_t)win);
  while (scanf("%d %llx %llx", &form, &seed, &flags) == 3) {
    for (int i = 0; i < 16; i++) scanf("%llx", &regs[i]);
    for (int i = 0; i < 32; i++) scanf("%llx", &xm[i]);
    for (int i = 0; i < 8; i++) scanf("%llx", &mm[i]);
    scanf("%d", &nptr);
    for (int i = 0; i < nptr; i++) scanf("%d", &ptrs[i]);
    uint64_t x = seed;
    for (int i = 0; i < 256; i += 8) { uint64_t v = sm(&x); memcpy(win + i, &v, 8); }
    for (int i = 0; i < 16; i++) g_in.r[i] = regs[i];
    for (int i = 0; i < nptr; i++) g_in.r[ptrs[i]] = (uint64_t)(uintptr_t)win + regs[ptrs[i]];
    for (int i = 0; i < 32; i++) g_in.x[i] = xm[i];
    for (int i = 0; i < 8; i++) g_in.mm[i] = mm[i];
    g_in.fl = flags;
    fns[form]();
    uint16_t fsw; memcpy(&fsw, g_fx + 2, 2);
    printf("R");
    for (int i = 0; i < 16; i++) printf(" %llx", (unsigned long long)g_out.r[i]);
    printf(" %llx\nX", (unsigned long long)g_out.fl);
    for (int i = 0; i < 32; i++) printf(" %llx", (unsigned long long)g_out.x[i]);
    printf("\nF");
    for (int i = 0; i < 8; i++) { uint64_t v; memcpy(&v, g_fx + 32 + 16 * i, 8); printf(" %llx", (unsigned long long)v); }
    printf(" %x %x\nM", fsw, g_fx[4]);
    for (int i = 0; i < 256; i++) printf("%02x", win[i]);
    printf("\n");
  }
  return 0;
}
"""


def main():
    rng = random.Random(0x3370001)
    forms = gen_forms(rng)
    cases = make_cases(forms, rng)
    uniq = {}
    for c in cases:
        uniq.setdefault(c["code"], len(uniq))
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "mv.c")
        with open(src, "w") as f:
            f.write(C_HEADER)
            for code, i in uniq.items():
                bs = ",".join("0x%02x" % b for b in bytes.fromhex(code))
                f.write(STUB.replace("{i}", str(i)).replace("{bytes}", bs))
            f.write(C_MAIN.replace("FNLIST", ",".join(f"t_{i}" for i in range(len(uniq)))))
        exe = os.path.join(td, "mv")
        subprocess.check_call(["gcc", "-O1", "-no-pie", "-o", exe, src])
        lines = []
        for c in cases:
            xs = [v for pair in c["xmm"] for v in pair]
            lines.append("%d %x %x %s %s %s %d %s" % (
                uniq[c["code"]], c["seed"], c["flags"], " ".join("%x" % v for v in c["regs"]),
                " ".join("%x" % v for v in xs), " ".join("%x" % v for v in c["mm"]),
                len(c["ptrs"]), " ".join(str(p) for p in c["ptrs"])))
        out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
    buf_va = int(out[0].split()[1], 16)
    res = []
    k = 1
    for c in cases:
        rl, xl, fl, ml = out[k].split(), out[k + 1].split(), out[k + 2].split(), out[k + 3][1:]
        k += 4
        before = splitmix_bytes(c["seed"], WIN)
        after = bytes.fromhex(ml)
        inregs = list(c["regs"])
        for p in c["ptrs"]:
            inregs[p] = (buf_va + inregs[p]) & 0xFFFFFFFFFFFFFFFF
        res.append({
            "name": c["name"], "code": c["code"], "in": ["%x" % v for v in inregs], "fl": "%x" % c["flags"],
            "xin": ["%x" % v for pair in c["xmm"] for v in pair], "mmin": ["%x" % v for v in c["mm"]],
            "out": rl[1:17], "flo": rl[17], "xout": xl[1:33], "mmout": fl[1:9], "fsw": fl[9], "ftw": fl[10],
            "seed": "%x" % c["seed"], "diff": [[i, after[i]] for i in range(WIN) if after[i] != before[i]],
        })
    doc = {"buf_va": "%x" % buf_va, "window": WIN,
           "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "generator": "tests/golden/gen_mmx_vectors.py", "cases": res}
    with gzip.open(OUT, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"wrote {len(res)} vectors ({len(uniq)} encodings) to {OUT}")


if __name__ == "__main__":
    main()
