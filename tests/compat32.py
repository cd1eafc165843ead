"""32-bit code (compatibility mode) for the engine-vs-oracle
tests. The address space is sysprog2's (GDT with 0x23 user code32 / 0x33 user
code64, IDT, TSS, the ring-0 frame-copying handler) plus:

  KC32   a ring-0 stub: rsp := r14, SYSRET without REX.W to ecx := ebx
         (CS = STAR[63:48] | 3 = 0x23: compatibility mode), r11 := r15;
         and a CSTAR handler (syscall from 32-bit code) copying rcx / r11;
  CODE32 ring-3 32-bit snippets (GNU as, .code32), 0x80 apart, each ending
         in int3; a page of 64-bit stubs below 4 GiB for far transfers
         between the modes (call far 0x33:stub ... retf back to 0x23);
  DATA32 a user data page, STACK32 two user stack pages.

Each lane starts at KC32 in ring 0 with random registers, random status
flags (AF / CF / OF / ZF for the BCD forms) and the snippet in rbx."""
from __future__ import annotations

import functools
import os
import random
import subprocess
import tempfile

from tests import sysprog2 as S

KC32 = 0xFFFFF80000700000
CSTAR_AT = KC32 + 0x100
CODE32 = 0x00401000
STUB64 = 0x00403000
DATA32 = 0x00404000
STACK32 = 0x00600000
ESP32 = STACK32 + 0x1FF0

KSTUB = "mov rsp, r14\n mov ecx, ebx\n mov rbx, r13\n mov r11, r15\n .byte 0x0f, 0x07"
CSTAR = "mov r8, rcx\n mov r9, r11\n mov r10, rsp\n hlt"
STUBS = {  # 64-bit code below 4 GiB: the far-call target returns to 32-bit code
    "gate64": "mov r9, 0x1122334455667788\n .byte 0xcb",  # retf: 32-bit slots
    "land64": "mov r10, 0x55\n int3",
}

U32 = {
    "incdec": "inc eax\n dec ebx\n inc ecx\n dec esi\n inc edi\n int3",
    "pushpop": "push eax\n push 0x12345678\n pop ebx\n pop ecx\n push esp\n pop edx\n pushw 0x1234\n pop si\n int3",
    "callret": "push 7\n call 1f\n int3\n1: mov eax, [esp+4]\n ret 4",
    "jcc": "cmp eax, ebx\n jb 1f\n mov ecx, 1\n1: mov edx, 3\n2: dec edx\n jnz 2b\n int3",
    "loop": "mov ecx, 4\n xor eax, eax\n1: add eax, ecx\n loop 1b\n jecxz 2f\n int3\n2: inc ebx\n int3",
    "pusha": "pusha\n xor eax, eax\n xor ecx, ecx\n mov ebp, 5\n popa\n int3",
    "pusha16": "pushaw\n xor eax, eax\n popaw\n int3",
    "bcd": "daa\n das\n aaa\n aas\n aam\n aad\n int3",
    "bcd2": "daa\n int3",
    "aas": "aas\n int3",
    "aam0": "aam 0\n int3",
    "aad7": "aad 7\n int3",
    "seg": "push ds\n push es\n push ss\n push cs\n pop eax\n pop ebx\n pop es\n pop ds\n int3",
    "mem": f"mov eax, [{DATA32 + 0x10:#x}]\n mov [esi+ecx*4+8], eax\n mov ebx, [{DATA32 + 0x20:#x}]\n"
           f" lea edx, [eax+ebx*2+5]\n mov al, [esi]\n int3",
    "moffs": f"mov eax, ds:[{DATA32 + 0x40:#x}]\n mov ds:[{DATA32 + 0x44:#x}], eax\n int3",
    "xlat": f"mov ebx, {DATA32:#x}\n xlatb\n int3",
    "string": "rep movsd\n mov ecx, 3\n rep stosb\n cmpsb\n lodsw\n int3",
    "enter": "enter 0x10, 2\n mov [ebp-4], eax\n leave\n int3",
    "farcall": f"call 0x33:{STUB64:#x}\n int3",
    "farjmp": f"jmp 0x33:{STUB64 + 0x80:#x}",
    "syscall": "syscall\n int3",
    "int29": "int 0x29\n int3",
    "int23": "int 0x23\n int3",
    "into": "mov al, 0x7f\n add al, 1\n into\n int3",
    "flags": "pushfd\n popfd\n sahf\n lahf\n cwde\n cdq\n pushf\n popf\n int3",
    "mul": "imul eax, ebx, 7\n mul ecx\n div esi\n int3",
    "misc": "movzx eax, bl\n movsx ecx, dx\n shl eax, cl\n bt eax, 3\n setc dl\n cmovz esi, edi\n bswap eax\n"
            " xchg eax, ebx\n cmpxchg8b [edi]\n int3",
    "sse": "movd xmm0, eax\n paddd xmm0, xmm0\n movd ebx, xmm0\n vpaddd xmm1, xmm0, xmm0\n vmovd ecx, xmm1\n int3",
    "iretd": "pushfd\n push cs\n push offset 1f\n iretd\n1: int3",
    "retf": "push cs\n push offset 1f\n retf\n1: int3",
    "jmpind": "mov eax, offset 1f\n jmp eax\n int3\n1: call dword ptr [esi]\n int3",
    "op82": "add bl, 3\n .byte 0x82, 0xc3, 0x05\n .byte 0x82, 0xf8, 0x10\n int3",
    "les": "les eax, [esi]\n int3",
    "a16": "addr16 mov eax, [bx]\n int3",
    "bound": "bound eax, [esi]\n int3",
    "arpl": "arpl ax, bx\n int3",
    "lds": "lds ecx, [esi]\n int3",
    "salc": "stc\n .byte 0xd6\n mov ebx, eax\n clc\n .byte 0xd6\n int3",
    "jmp16": ".byte 0x66, 0xe9, 0x00, 0x00\n int3",
    "ud2": "ud2",
    # andn eax, esi, edi with VEX.W1: 32-bit code runs it at 32 bits (W1 ignored)
    "bmiw1": ".byte 0xc4, 0xe2, 0xc8, 0xf2, 0xc7\n int3",
}


def _as(src: str, code32: bool, org: int) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        s, o, b = (os.path.join(d, n) for n in ("a.s", "a.o", "a.bin"))
        with open(s, "w") as f:
            f.write(".intel_syntax noprefix\n" + (".code32\n" if code32 else ".code64\n") + src + "\n")
        subprocess.check_call(["as", "--32" if code32 else "--64", "-o", o, s])
        # link at the snippet's address so offsets / absolute labels resolve
        lnk = os.path.join(d, "a.elf")
        subprocess.check_call(["ld", "-m", "elf_i386" if code32 else "elf_x86_64", "-Ttext", hex(org), "-e", hex(org),
                               "-o", lnk, o], stderr=subprocess.DEVNULL)
        subprocess.check_call(["objcopy", "-O", "binary", "-j", ".text", lnk, b])
        return open(b, "rb").read()


@functools.lru_cache(maxsize=None)
def assemble(src: str, code32: bool, org: int) -> bytes:
    return _as(src, code32, org)


SLOT32 = {n: CODE32 + 0x80 * i for i, n in enumerate(U32)}
assert len(SLOT32) * 0x80 <= 0x2000


def build_space():
    """(address space, ring-0 state, layout, data) of sysprog2 plus the 32-bit pages."""
    sp, st, lay, data = S.build_space()
    k = bytearray(b"\xf4" * 0x1000)
    for off, src in ((0, KSTUB), (0x100, CSTAR)):
        b = S.assemble(src)
        k[off:off + len(b)] = b
    sp.map(KC32, bytes(k), user=False, write=False, nx=False)
    code = bytearray(b"\xcc" * 0x2000)
    for n, va in SLOT32.items():
        b = assemble(U32[n], True, va)
        assert len(b) <= 0x80, n
        code[va - CODE32:va - CODE32 + len(b)] = b
    sp.map(CODE32, bytes(code[:0x1000]), user=True, write=False, nx=False)
    sp.map(CODE32 + 0x1000, bytes(code[0x1000:]), user=True, write=False, nx=False)
    stubs = bytearray(b"\xcc" * 0x1000)
    for i, (n, src) in enumerate(STUBS.items()):
        b = assemble(src, False, STUB64 + 0x80 * i)
        stubs[0x80 * i:0x80 * i + len(b)] = b
    sp.map(STUB64, bytes(stubs), user=True, write=False, nx=False)
    rng = random.Random(0x3232)
    d32 = bytearray(rng.getrandbits(8) for _ in range(0x1000))
    d32[0x200:0x204] = (SLOT32["jmpind"] + 0x7F).to_bytes(4, "little")  # an indirect call target (the slot's int3 pad)
    d32[0x60:0x68] = (-5 & 0xFFFFFFFF).to_bytes(4, "little") + (100).to_bytes(4, "little")  # bound: [-5, 100]
    sp.map(DATA32, bytes(d32), user=True, write=True, nx=True)
    for i in range(2):
        sp.map(STACK32 + 0x1000 * i, b"", user=True, write=True, nx=True)
    st = dict(st)
    st["cstar"] = CSTAR_AT
    return sp, st, lay, bytes(d32)


def lanes(n: int, seed: int):
    """[(rip, 16 GPRs, rflags)]: every snippet, random registers and flags."""
    rng = random.Random(seed)
    names = list(U32)
    out = []
    for i in range(n):
        name = names[i % len(names)]
        g = [rng.getrandbits(64) if rng.random() < 0.3 else rng.getrandbits(rng.choice([4, 8, 16, 32])) for _ in
             range(16)]
        g[6] = DATA32 + rng.choice([0x100, 0x200, 0x800, 0xFF8, 0x1000, 0x7])        # esi
        g[7] = DATA32 + rng.choice([0x300, 0x400, 0x40, 0xFFC, 0x1000])              # edi
        if name in ("string", "mem", "misc"):
            g[1] = rng.choice([0, 1, 5, 0x40, 0x3FF])                               # ecx
        if name == "mul":
            g[6] = rng.choice([0, 1, 7, 0xFFFFFFFF, rng.getrandbits(32)])
        flags = 0x202 | rng.choice([0, 1, 0x10, 0x11, 0x40, 0x41, 0x800, 0x851]) | (rng.getrandbits(1) << 10)
        g[3], g[13], g[14], g[15] = SLOT32[name], rng.getrandbits(32), ESP32 - 8 * rng.randrange(4), flags
        out.append((KC32, g, 0x2))
    return out
