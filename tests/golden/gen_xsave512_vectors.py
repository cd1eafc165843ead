#!/usr/bin/env python3
"""Native XSAVE / XSAVEC images with the AVX-512 state (convention U47;
engine_sys.h, oracle/x86_oracle_sys.inc).

A stub on this host (AVX512F) loads a known state — zmm0-31, k0-7, and
through FXRSTOR64 the x87 environment, ST0-7 and MXCSR (FIP / FDP / FOP
zero) — then runs one XSAVE-family instruction with EDX:EAX = a requested-
feature bitmap into a buffer pre-filled with 0xa5, and prints the buffer.
The host's XCR0 holds x87 | SSE | AVX | opmask | ZMM_Hi256 | Hi16_ZMM (0xe7)
and possibly more (PKRU, AMX); every bitmap here is a subset of 0xe7, so
RFBM is what a guest with XCR0 = 0xe7 gets. Every component is outside its
initial configuration (XINUSE set), so the images are the state itself.

Output: tests/golden/xsave512_vectors.json (the state, the host's
MXCSR_MASK, and per case the instruction bytes, RFBM and the buffer).
Re-run with  python tests/golden/gen_xsave512_vectors.py
"""
import json
import os
import random
import struct
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "xsave512_vectors.json")
AREA = 0x40     # the image's offset in the buffer (64-byte aligned)
SPAN = 3072     # bytes compared from the buffer start

INSNS = {"xsave": [0x0F, 0xAE, 0x27], "xsave64": [0x48, 0x0F, 0xAE, 0x27], "xsavec": [0x0F, 0xC7, 0x27],
         "xsavec64": [0x48, 0x0F, 0xC7, 0x27]}
RFBMS = [0xE7, 0xFF, 0x65, 0xA3, 0x42, 0xE0, 0x03]


def state(seed, all_valid):
    rng = random.Random(seed)
    zmm = [[rng.getrandbits(64) for _ in range(8)] for _ in range(32)]
    k = [rng.getrandbits(64) | 1 for _ in range(8)]
    st = [(rng.getrandbits(64), rng.getrandbits(16)) for _ in range(8)]
    return {"zmm": zmm, "k": k, "st": st, "fcw": 0x27F, "fsw": 0x3820, "ftw_full": 0x0000 if all_valid else 0xFFFF,
            "mxcsr": 0x1FA0}


def fx_image(s):
    img = bytearray(512)
    ftw_abridged = 0xFF if s["ftw_full"] == 0 else 0x00
    struct.pack_into("<HHB", img, 0, s["fcw"], s["fsw"], ftw_abridged)
    struct.pack_into("<I", img, 24, s["mxcsr"])
    for i, (sig, se) in enumerate(s["st"]):
        struct.pack_into("<QH", img, 32 + 16 * i, sig, se)
    for i in range(16):
        struct.pack_into("<QQ", img, 160 + 16 * i, s["zmm"][i][0], s["zmm"][i][1])
    return bytes(img)


C_SRC = r"""
#include <stdio.h>
#include <stdint.h>
#include <string.h>
uint64_t g_z[256] __attribute__((aligned(64)));
uint64_t g_k[8];
uint8_t g_fx[512] __attribute__((aligned(64)));
uint8_t g_buf[3 * 4096] __attribute__((aligned(4096)));
uint8_t g_host_fx[512] __attribute__((aligned(64)));
uint32_t g_eax, g_edx;
"""
ZL = "".join(f'"vmovdqu64 g_z+{64 * i}(%rip), %zmm{i}\\n"\n' for i in range(32))
KL = "".join(f'"kmovq g_k+{8 * i}(%rip), %k{i}\\n"\n' for i in range(8))
STUB = r"""
__asm__(".text\n.globl t_{i}\nt_{i}:\n"
""" + ZL + KL + r"""
"fxrstor64 g_fx(%rip)\n"
"push %rdi\n"
"lea g_buf+{area}(%rip), %rdi\n"
"mov g_eax(%rip), %eax\nmov g_edx(%rip), %edx\n"
".byte {bytes}\n"
"pop %rdi\n"
"vzeroupper\nfninit\nret\n");
void t_{i}(void);
"""
C_MAIN = r"""
typedef void (*fn_t)(void);
static fn_t fns[] = { FNLIST };
int main(void) {
  int form;
  unsigned int rfbm;
  __asm__ volatile("fxsave64 %0" : "=m"(g_host_fx));
  uint32_t mm;
  memcpy(&mm, g_host_fx + 28, 4);
  printf("MXCSR_MASK %x\n", mm);
  while (scanf("%d %x", &form, &rfbm) == 2) {
    for (int i = 0; i < 256; i++) if (scanf("%lx", (unsigned long *)&g_z[i]) != 1) return 1;
    for (int i = 0; i < 8; i++) if (scanf("%lx", (unsigned long *)&g_k[i]) != 1) return 1;
    for (int i = 0; i < 512; i++) { unsigned int b; if (scanf("%2x", &b) != 1) return 1; g_fx[i] = (uint8_t)b; }
    memset(g_buf, 0xa5, sizeof(g_buf));
    g_eax = rfbm;
    g_edx = 0;
    fns[form]();
    printf("B ");
    for (int i = 0; i < SPAN; i++) printf("%02x", g_buf[i]);
    printf("\n");
  }
  return 0;
}
"""


def main():
    names = list(INSNS)
    states = [state(0x5A7E0, False), state(0x5A7E1, True)]
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "x.c")
        with open(src, "w") as f:
            f.write(C_SRC)
            for i, n in enumerate(names):
                f.write(STUB.replace("{i}", str(i)).replace("{area}", str(AREA))
                        .replace("{bytes}", ",".join("0x%02x" % b for b in INSNS[n])))
            f.write(C_MAIN.replace("FNLIST", ",".join(f"t_{i}" for i in range(len(names))))
                    .replace("SPAN", str(SPAN)))
        exe = os.path.join(td, "x")
        subprocess.check_call(["gcc", "-O1", "-no-pie", "-o", exe, src])
        lines, keys = [], []
        for si, s in enumerate(states):
            fx = fx_image(s).hex()
            for ni, n in enumerate(names):
                for rfbm in RFBMS:
                    lines.append("%d %x %s %s %s" % (ni, rfbm, " ".join("%x" % v for r in s["zmm"] for v in r),
                                                     " ".join("%x" % v for v in s["k"]), fx))
                    keys.append((si, n, rfbm))
        out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
    mask = int(out[0].split()[1], 16)
    cases = [{"state": si, "insn": n, "code": bytes(INSNS[n]).hex(), "rfbm": rfbm, "buf": out[1 + j].split()[1]}
             for j, (si, n, rfbm) in enumerate(keys)]
    doc = {"generator": "tests/golden/gen_xsave512_vectors.py", "area": AREA, "span": SPAN, "mxcsr_mask": mask,
           "host": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t"),
           "states": [{"zmm": ["%x" % v for r in s["zmm"] for v in r], "k": ["%x" % v for v in s["k"]],
                       "st": [["%x" % a, b] for a, b in s["st"]], "fcw": s["fcw"], "fsw": s["fsw"],
                       "ftw_full": s["ftw_full"], "mxcsr": s["mxcsr"]} for s in states],
           "cases": cases}
    with open(OUT, "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(f"wrote {len(cases)} images (MXCSR_MASK {mask:#x}) to {OUT}")


if __name__ == "__main__":
    main()
