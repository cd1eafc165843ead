#!/usr/bin/env python3
"""Native-execution golden vectors for the AVX / AVX2 (VEX) subset and the
legacy pshufb / ptest (convention U23).

As gen_sse_vectors.py, with the 16 YMM registers (256 bits each) loaded and
stored around the instruction (vmovdqu), so VEX.128's zeroing of bits 255:128
and legacy SSE's keeping of them are both pinned. Both VEX forms (c5 and c4)
are generated. The host must have AVX2.

Output: tests/golden/avx_vectors.json.gz. Re-run with
    python tests/golden/gen_avx_vectors.py
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
from tests.golden.gen_native_vectors import WIN, rand_val, splitmix_bytes  # noqa: E402
from tests.golden.gen_sse_vectors import enc_mem, rand_xmm  # noqa: E402

OUT = os.path.join(HERE, "avx_vectors.json.gz")
RSP = 4

# 3-operand lane ops: (pp, opcode, name); L = 0 and 1
LANE = [(0, 0x14, "vunpcklps"), (1, 0x15, "vunpckhpd"), (0, 0x54, "vandps"), (1, 0x55, "vandnpd"),
        (0, 0x56, "vorps"), (1, 0x57, "vxorpd")]
LANE += [(1, op, "vp%02x" % op) for op in list(range(0x60, 0x6E)) + [0x74, 0x75, 0x76]]
LANE += [(1, op, "vp%02x" % op) for op in
         [0xD4, 0xD5, 0xD8, 0xD9, 0xDA, 0xDB, 0xDC, 0xDD, 0xDE, 0xDF, 0xE0, 0xE3, 0xE4, 0xE5, 0xE8, 0xE9, 0xEA,
          0xEB, 0xEC, 0xED, 0xEE, 0xEF, 0xF4, 0xF5, 0xF6, 0xF8, 0xF9, 0xFA, 0xFB, 0xFC, 0xFD, 0xFE]]
SHIFT_X = [0xD1, 0xD2, 0xD3, 0xE1, 0xE2, 0xF1, 0xF2, 0xF3]  # count in xmm/m128
SHIFT_IMM = [(0x71, 2), (0x71, 4), (0x71, 6), (0x72, 2), (0x72, 4), (0x72, 6), (0x73, 2), (0x73, 3), (0x73, 6),
             (0x73, 7)]


class Form:
    def __init__(self, code, name, ptrs=(), smalls=(), xsmall=None):
        self.code = bytes(code)
        self.name = name
        self.ptrs = dict(ptrs)
        self.smalls = dict(smalls)
        self.xsmall = xsmall
        self.cls = "sse"


def vex_prefix(rng, r, x, b, mmmmm, w, vvvv, l, pp):
    """c5 when it can encode the fields (and half the time then), else c4."""
    if x < 8 and b < 8 and mmmmm == 1 and w == 0 and rng.random() < 0.6:
        return [0xC5, (((r >> 3) ^ 1) << 7) | ((~vvvv & 15) << 3) | (l << 2) | pp]
    return [0xC4, (((r >> 3) ^ 1) << 7) | (((x >> 3) ^ 1) << 6) | (((b >> 3) ^ 1) << 5) | mmmmm,
            (w << 7) | ((~vvvv & 15) << 3) | (l << 2) | pp]


def vrr(rng, opc, reg, vvvv, rm, l, pp, mmmmm=1, w=0):
    return vex_prefix(rng, reg, 0, rm, mmmmm, w, vvvv, l, pp) + [opc, 0xC0 | ((reg & 7) << 3) | (rm & 7)]


def vmem(rng, opc, reg, vvvv, l, pp, align, mmmmm=1, w=0):
    """A VEX memory form: enc_mem's addressing, re-prefixed with VEX."""
    code, p, s = enc_mem(rng, [], 0x0F, reg & 7, align)  # legacy bytes: [rex] 0f 0f modrm ...
    # strip [rex] 0f <opc-placeholder>; keep modrm.. and read the REX bits back
    i = 0
    rex = 0
    if 0x40 <= code[0] <= 0x4F:
        rex = code[0]
        i = 1
    rest = code[i + 2:]
    x = 8 if rex & 2 else 0
    b = 8 if rex & 1 else 0
    return vex_prefix(rng, reg, x, b, mmmmm, w, vvvv, l, pp) + [opc] + rest, p, s


def gen_forms(rng):
    forms = []
    x = lambda: rng.randrange(16)  # noqa: E731
    g = lambda: rng.choice([r for r in range(16) if r != RSP])  # noqa: E731
    for pp, op, nm in LANE:
        for l in (0, 1):
            for _ in range(2):
                forms.append(Form(vrr(rng, op, x(), x(), x(), l, pp), f"{nm}.L{l}.rr"))
            c, p, s = vmem(rng, op, x(), x(), l, pp, 1)
            forms.append(Form(c, f"{nm}.L{l}.m", p, s))
    for op in SHIFT_X:
        for l in (0, 1):
            src = x()
            forms.append(Form(vrr(rng, op, x(), x(), src, l, 1), f"vshx{op:x}.L{l}", xsmall=src))
            c, p, s = vmem(rng, op, x(), x(), l, 1, 1)
            forms.append(Form(c, f"vshx{op:x}.L{l}.m", p, s))
    for op, sub in SHIFT_IMM:
        for l in (0, 1):
            for cnt in rng.sample([0, 1, 3, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 200], 3):
                forms.append(Form(vrr(rng, op, sub, x(), x(), l, 1) + [cnt], f"vshimm{op:x}.{sub}.L{l}"))
    for pp in (1, 2, 3):  # vpshufd / hw / lw
        for l in (0, 1):
            forms.append(Form(vrr(rng, 0x70, x(), 0, x(), l, pp) + [rng.randrange(256)], f"vpshuf.{pp}.L{l}"))
            c, p, s = vmem(rng, 0x70, x(), 0, l, pp, 1)
            forms.append(Form(c + [rng.randrange(256)], f"vpshuf.{pp}.L{l}.m", p, s))
    for pp in (0, 1):  # vshufps / pd
        for l in (0, 1):
            forms.append(Form(vrr(rng, 0xC6, x(), x(), x(), l, pp) + [rng.randrange(256)], f"vshuf.{pp}.L{l}"))
    # moves
    for l in (0, 1):
        for pp, op, al, nm in ((0, 0x10, 1, "vmovups"), (1, 0x10, 1, "vmovupd"), (0, 0x28, 32 if l else 16, "vmovaps"),
                               (1, 0x6F, 32 if l else 16, "vmovdqa"), (2, 0x6F, 1, "vmovdqu")):
            forms.append(Form(vrr(rng, op, x(), 0, x(), l, pp), f"{nm}.L{l}.rr"))
            c, p, s = vmem(rng, op, x(), 0, l, pp, al)
            forms.append(Form(c, f"{nm}.L{l}.m", p, s))
        for pp, op, al, nm in ((0, 0x11, 1, "vmovups.st"), (1, 0x29, 32 if l else 16, "vmovapd.st"),
                               (2, 0x7F, 1, "vmovdqu.st"), (1, 0x7F, 32 if l else 16, "vmovdqa.st"),
                               (1, 0xE7, 32 if l else 16, "vmovntdq"), (0, 0x2B, 32 if l else 16, "vmovntps")):
            if op not in (0xE7, 0x2B):
                forms.append(Form(vrr(rng, op, x(), 0, x(), l, pp), f"{nm}.L{l}.rr"))
            c, p, s = vmem(rng, op, x(), 0, l, pp, al)
            forms.append(Form(c, f"{nm}.L{l}.m", p, s))
        forms.append(Form(vrr(rng, 0x50, g(), 0, x(), l, rng.randrange(2)), f"vmovmsk.L{l}"))
        forms.append(Form(vrr(rng, 0xD7, g(), 0, x(), l, 1), f"vpmovmskb.L{l}"))
        forms.append(Form(vex_prefix(rng, 0, 0, 0, 1, 0, 0, l, 0) + [0x77], f"vzero.L{l}"))
    for pp, n in ((2, 4), (3, 8)):  # vmovss / vmovsd
        for op in (0x10, 0x11):
            forms.append(Form(vrr(rng, op, x(), x(), x(), rng.randrange(2), pp), f"vmovs{n}.{op:x}.rr"))
            c, p, s = vmem(rng, op, x(), 0, rng.randrange(2), pp, 1)
            forms.append(Form(c, f"vmovs{n}.{op:x}.m", p, s))
    for pp, op, nm in ((0, 0x12, "vmovlps"), (1, 0x12, "vmovlpd"), (0, 0x16, "vmovhps"), (1, 0x16, "vmovhpd")):
        c, p, s = vmem(rng, op, x(), x(), 0, pp, 1)
        forms.append(Form(c, f"{nm}.m", p, s))
    for op, nm in ((0x12, "vmovhlps"), (0x16, "vmovlhps")):
        forms.append(Form(vrr(rng, op, x(), x(), x(), 0, 0), nm))
    for pp, op, nm in ((0, 0x13, "vmovlps.st"), (0, 0x17, "vmovhps.st"), (1, 0xD6, "vmovq.st")):
        c, p, s = vmem(rng, op, x(), 0, 0, pp, 1)
        forms.append(Form(c, f"{nm}.m", p, s))
    forms.append(Form(vrr(rng, 0xD6, x(), 0, x(), 0, 1), "vmovq.d6.rr"))
    for w in (0, 1):
        forms.append(Form(vrr(rng, 0x6E, x(), 0, g(), 0, 1, w=w), f"vmovd.xg.w{w}"))
        forms.append(Form(vrr(rng, 0x7E, x(), 0, g(), 0, 1, w=w), f"vmovd.gx.w{w}"))
        c, p, s = vmem(rng, 0x6E, x(), 0, 0, 1, 1, w=w)
        forms.append(Form(c, f"vmovd.6e.m.w{w}", p, s))
    forms.append(Form(vrr(rng, 0x7E, x(), 0, x(), 0, 2), "vmovq.f3.rr"))
    forms.append(Form(vrr(rng, 0xC4, x(), x(), g(), 0, 1) + [rng.randrange(256)], "vpinsrw"))
    forms.append(Form(vrr(rng, 0xC5, g(), 0, x(), 0, 1) + [rng.randrange(256)], "vpextrw"))
    # 0f 38: vpshufb, vptest, vpbroadcast; legacy pshufb / ptest
    for l in (0, 1):
        for _ in range(2):
            forms.append(Form(vrr(rng, 0x00, x(), x(), x(), l, 1, mmmmm=2), f"vpshufb.L{l}"))
            forms.append(Form(vrr(rng, 0x17, x(), 0, x(), l, 1, mmmmm=2), f"vptest.L{l}"))
        for op in (0x58, 0x59, 0x78, 0x79):
            forms.append(Form(vrr(rng, op, x(), 0, x(), l, 1, mmmmm=2), f"vpbroadcast{op:x}.L{l}"))
            c, p, s = vmem(rng, op, x(), 0, l, 1, 1, mmmmm=2)
            forms.append(Form(c, f"vpbroadcast{op:x}.L{l}.m", p, s))
    for op, nm in ((0x00, "pshufb"), (0x17, "ptest")):
        for _ in range(3):
            reg, rm = x(), x()
            rex = 0x40 | ((reg >> 3) << 2) | (rm >> 3)
            forms.append(Form([0x66] + ([rex] if rex != 0x40 else []) + [0x0F, 0x38, op, 0xC0 | ((reg & 7) << 3) | (rm & 7)],
                              nm + ".rr"))
        c, p, s = enc_mem(rng, [0x66], 0x38, x(), 16)
        # enc_mem wrote "... 0f 38 modrm": splice the third opcode byte in after 0f 38
        k = c.index(0x38)
        forms.append(Form(c[:k + 1] + [op] + c[k + 1:], nm + ".m", p, s))
    return forms


def make_cases(forms, rng, per_form=5):
    cases = []
    for f in forms:
        for _ in range(per_form):
            regs = [rand_val(rng) for _ in range(16)]
            regs[RSP] = 0x80
            for r, off in f.ptrs.items():
                regs[r] = off
            for r, (lo, hi) in f.smalls.items():
                regs[r] = rng.randint(lo, hi)
            ymm = [rand_xmm(rng) + rand_xmm(rng) for _ in range(16)]
            if rng.random() < 0.4:
                a, b = rng.randrange(16), rng.randrange(16)
                ymm[a] = [ymm[b][0], ymm[a][1], ymm[b][2], ymm[a][3]]
            if rng.random() < 0.2:  # ptest: disjoint / covered operands
                a = rng.randrange(16)
                ymm[a] = [0, 0, 0, 0]
            if f.xsmall is not None and rng.random() < 0.7:
                ymm[f.xsmall][0] = rng.choice([0, 1, 2, 7, 8, 15, 16, 31, 32, 63, 64, 65])
            cases.append({"name": f.name, "code": f.code.hex(), "regs": regs, "ptrs": sorted(f.ptrs) + [RSP],
                          "flags": 0x2 | (rng.getrandbits(16) & 0x8D5), "ymm": ymm, "seed": rng.getrandbits(63)})
    return cases


C_HEADER = r"""
#include <stdio.h>
#include <stdint.h>
#include <string.h>
typedef struct { uint64_t r[16]; uint64_t fl; uint64_t y[64]; } st_t;
st_t g_in, g_out;
uint64_t g_host_rsp;
uint64_t g_flagstack[64] __attribute__((aligned(32)));
uint8_t g_buf[8192] __attribute__((aligned(4096)));
"""
YLOAD = "".join('"vmovdqu g_in+%d(%%rip), %%ymm%d\\n"\n' % (136 + 32 * i, i) for i in range(16))
YSTORE = "".join('"vmovdqu %%ymm%d, g_out+%d(%%rip)\\n"\n' % (i, 136 + 32 * i) for i in range(16))
STUB = r"""
__asm__(
".text\n.globl t_{i}\nt_{i}:\n"
"push %rbx\npush %rbp\npush %r12\npush %r13\npush %r14\npush %r15\n"
"mov %rsp, g_host_rsp(%rip)\n"
""" + YLOAD + r"""
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
""" + YSTORE + r"""
"vzeroupper\n"
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
  int form, nptr, ptrs[16]; unsigned long long seed, flags, regs[16], ym[64];
  uint8_t *win = g_buf + 0x800;
  printf("BUF %llx\n", (unsigned long long)(uintptr_t)win);
  while (scanf("%d %llx %llx", &form, &seed, &flags) == 3) {
    for (int i = 0; i < 16; i++) if (scanf("%llx", &regs[i]) != 1) return 1;
    for (int i = 0; i < 64; i++) if (scanf("%llx", &ym[i]) != 1) return 1;
    if (scanf("%d", &nptr) != 1) return 1;
    for (int i = 0; i < nptr; i++) if (scanf("%d", &ptrs[i]) != 1) return 1;
    uint64_t x = seed;
    for (int i = 0; i < 256; i += 8) { uint64_t v = sm(&x); memcpy(win + i, &v, 8); }
    for (int i = 0; i < 16; i++) g_in.r[i] = regs[i];
    for (int i = 0; i < nptr; i++) g_in.r[ptrs[i]] = (uint64_t)(uintptr_t)win + regs[ptrs[i]];
    for (int i = 0; i < 64; i++) g_in.y[i] = ym[i];
    g_in.fl = flags;
    fns[form]();
    printf("R");
    for (int i = 0; i < 16; i++) printf(" %llx", (unsigned long long)g_out.r[i]);
    printf(" %llx\nY", (unsigned long long)g_out.fl);
    for (int i = 0; i < 64; i++) printf(" %llx", (unsigned long long)g_out.y[i]);
    printf("\nM");
    for (int i = 0; i < 256; i++) printf("%02x", win[i]);
    printf("\n");
  }
  return 0;
}
"""


def main():
    rng = random.Random(0xA0C0001)
    forms = gen_forms(rng)
    cases = make_cases(forms, rng)
    uniq = {}
    for c in cases:
        uniq.setdefault(c["code"], len(uniq))
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "av.c")
        with open(src, "w") as f:
            f.write(C_HEADER)
            for code, i in uniq.items():
                bs = ",".join("0x%02x" % b for b in bytes.fromhex(code))
                f.write(STUB.replace("{i}", str(i)).replace("{bytes}", bs))
            f.write(C_MAIN.replace("FNLIST", ",".join(f"t_{i}" for i in range(len(uniq)))))
        exe = os.path.join(td, "av")
        subprocess.check_call(["gcc", "-O1", "-no-pie", "-o", exe, src])
        lines = []
        for c in cases:
            ys = [v for r in c["ymm"] for v in r]
            lines.append("%d %x %x %s %s %d %s" % (
                uniq[c["code"]], c["seed"], c["flags"], " ".join("%x" % v for v in c["regs"]),
                " ".join("%x" % v for v in ys), len(c["ptrs"]), " ".join(str(p) for p in c["ptrs"])))
        out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
    buf_va = int(out[0].split()[1], 16)
    res = []
    k = 1
    for c in cases:
        rl, yl, ml = out[k].split(), out[k + 1].split(), out[k + 2][1:]
        k += 3
        before = splitmix_bytes(c["seed"], WIN)
        after = bytes.fromhex(ml)
        inregs = list(c["regs"])
        for p in c["ptrs"]:
            inregs[p] = (buf_va + inregs[p]) & 0xFFFFFFFFFFFFFFFF
        res.append({
            "name": c["name"], "code": c["code"], "in": ["%x" % v for v in inregs], "fl": "%x" % c["flags"],
            "yin": ["%x" % v for r in c["ymm"] for v in r], "out": rl[1:17], "flo": rl[17], "yout": yl[1:65],
            "seed": "%x" % c["seed"], "diff": [[i, after[i]] for i in range(WIN) if after[i] != before[i]],
        })
    doc = {"buf_va": "%x" % buf_va, "window": WIN,
           "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "generator": "tests/golden/gen_avx_vectors.py", "cases": res}
    with gzip.open(OUT, "wt") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"wrote {len(res)} vectors ({len(uniq)} encodings) to {OUT}")


if __name__ == "__main__":
    main()
