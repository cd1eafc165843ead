"""System, far-transfer, I/O and x87-control programs for
the engine-vs-oracle tests: INT n / INT1 through IDT gates (DPL, IST, not
present, bad type), CLI / STI against IOPL, LOOP / LOOPcc / JRCXZ, CPUID,
XGETBV / XSETBV, CMPXCHG8B / 16B, ENTER, far RET / CALL / JMP and IRET with
16- / 32-bit slots, MOV / PUSH / POP Sreg and LFS / LGS / LSS, IN / OUT /
INS / OUTS, FNINIT .. FRSTOR, FXSAVE / FXRSTOR, the XSAVE family, the
descriptor-table instructions, SYSENTER / SYSEXIT, RD / WR FS / GS base,
CLFLUSH, LOCK legality and the #UD opcodes.

The snippets are assembled with the host's GNU as (intel syntax). Each runs on
one lane of a dedicated address space: an IDT whose software-interrupt gates
lead to a ring-0 handler that copies the interrupt frame into r8..r13 and
halts (fault vectors have no gate, so a fault ends the lane in both the
oracle and the engine), a GDT with code / data / TSS / based descriptors, a
TSS with RSP0 and IST1, data pages holding prepared FXSAVE / XSAVE images and
far pointers. Ring-3 snippets are entered through an IRETQ stub. Every lane
gets random registers and random IOPL / flags."""
from __future__ import annotations

import functools
import os
import random
import struct
import subprocess
import tempfile

from wtf_amd.abi import regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, seg, user_state

KCODE = 0xFFFFF80000600000       # ring-0 snippets, 0x100 apart (+ the handlers, the user stub)
UCODE = 0x0000000140800000       # ring-3 snippets, 0x100 apart
IDT = 0xFFFFF80000004000
GDT = 0xFFFFF80000003000
TSS = 0xFFFFF80000002000
KSTACK = 0xFFFFF80000300000      # 8 pages
KSP = KSTACK + 0x7000
ISTSTACK = 0xFFFFF80000320000    # 1 page
UST = 0x00007FF000000000 - 0x4000  # user stack: 4 pages below this + 0x4000
USP = UST + 0x3000
DATA = 0x0000000150000000        # 4 pages user rw (images, far pointers, scratch); DATA + 0x4000 unmapped
KDATA = 0xFFFFF80000800000       # 1 page supervisor rw
LDT_BASE = 0xFFFFF80000005000    # the LDT descriptor's base (no page: LLDT reads only the GDT)
GDT_LIMIT = 0x9F

# GDT: 0x10 kernel code, 0x18 kernel data, 0x23 user code32, 0x2b user data,
# 0x33 user code64, 0x38 not present, 0x40 TSS (16 bytes), 0x53 data base
# 0x12345000 (DPL 3), 0x5b not-present data, 0x60 conforming code, 0x68 data
# DPL 0, 0x70 read-only data DPL 3, 0x78 data with G=1, 0x80 LDT (16 bytes),
# 0x90 a second TSS (16 bytes, at TSS + 0x800: its own RSP0 / IST1)
def _desc(base, limit, typ, s=1, dpl=0, p=1, l=0, db=1, g=0):
    return ((limit & 0xFFFF) | ((base & 0xFFFFFF) << 16) | (typ << 40) | (s << 44) | (dpl << 45) | (p << 47) |
            (((limit >> 16) & 0xF) << 48) | (l << 53) | (db << 54) | (g << 55) | (((base >> 24) & 0xFF) << 56))


def gdt_page() -> bytes:
    g = bytearray(0x1000)
    ent = {
        0x10: _desc(0, 0xFFFFF, 0xB, l=1, db=0, g=1), 0x18: _desc(0, 0xFFFFF, 0x3, g=1),
        0x20: _desc(0, 0xFFFFF, 0xB, dpl=3, g=1), 0x28: _desc(0, 0xFFFFF, 0x3, dpl=3, g=1),
        0x30: _desc(0, 0xFFFFF, 0xB, dpl=3, l=1, db=0, g=1), 0x38: _desc(0, 0xFFFF, 0x3, p=0),
        0x50: _desc(0x12345000, 0xFFF, 0x3, dpl=3), 0x58: _desc(0x4000, 0xFFF, 0x3, dpl=3, p=0),
        0x60: _desc(0, 0xFFFFF, 0xF, dpl=0, l=1, db=0, g=1), 0x68: _desc(0x1000, 0xFFFF, 0x3, dpl=0),
        0x70: _desc(0x2000, 0x1FFF, 0x1, dpl=3), 0x78: _desc(0x8000, 0x12, 0x3, dpl=3, g=1),
    }
    for off, v in ent.items():
        struct.pack_into("<Q", g, off, v)
    struct.pack_into("<QQ", g, 0x40, _desc(TSS & 0xFFFFFFFF, 0x67, 0x9, s=0, db=0), TSS >> 32)
    struct.pack_into("<QQ", g, 0x80, _desc(LDT_BASE & 0xFFFFFFFF, 0xFFF, 0x2, s=0, db=0), LDT_BASE >> 32)
    struct.pack_into("<QQ", g, 0x90, _desc((TSS + 0x800) & 0xFFFFFFFF, 0x67, 0x9, s=0, db=0), TSS >> 32)
    return bytes(g)


def _gate(off, sel=0x10, typ=0xE, dpl=0, ist=0, p=1):
    lo = (off & 0xFFFF) | (sel << 16) | (ist << 32) | (((p << 7) | (dpl << 5) | typ) << 40) | (((off >> 16) & 0xFFFF) << 48)
    return struct.pack("<QQ", lo, off >> 32)


# ---------------------------------------------------------------- snippets
HANDLER = "mov r8, [rsp]\n mov r9, [rsp+8]\n mov r10, [rsp+16]\n mov r11, [rsp+24]\n mov r12, [rsp+32]\n mov r13, rsp\n hlt"
UHANDLER = "mov r8, [rsp]\n mov r9, [rsp+8]\n mov r13, rsp\n int3"
TO_USER = "push 0x2b\n push r14\n push r15\n push 0x33\n push rbx\n iretq"

K = {  # ring 0 (each ends with hlt; a fault ends the lane)
    "int80": "int 0x80\n hlt",
    "int29": "int 0x29\n hlt",
    "int2e": "int 0x2e\n hlt",
    "int21": "int 0x21\n hlt",            # not present: #NP
    "int22": "int 0x22\n hlt",            # call gate type: #GP
    "int24": "int 0x24\n hlt",            # target selector RPL 3 from ring 0 ... (gate to ring 3): #GP(sel)
    "intff": "int 0xff\n hlt",            # beyond the IDT limit
    "int1": ".byte 0xf1\n hlt",
    "int3": "int 0x3\n hlt",
    "into": ".byte 0xce\n hlt",
    "cli": "cli\n pushfq\n pop rax\n sti\n pushfq\n pop rdx\n hlt",
    "loop": "and ecx, 0x3f\n 1: add rax, rdx\n loop 1b\n hlt",
    "loope": "and ecx, 0x1f\n 1: add rbx, 1\n cmp bl, dl\n loope 1b\n hlt",
    "loopne": "and ecx, 0x1f\n 1: add rbx, 1\n cmp bl, dl\n loopne 1b\n hlt",
    "loop32": "mov ecx, ecx\n and ecx, 7\n or rcx, r9\n 1: inc rax\n addr32 loop 1b\n hlt",
    "jrcxz": "and rcx, r9\n jrcxz 2f\n inc rax\n 2: jecxz 3f\n inc rdx\n 3: hlt",
    "cpuid": "mov eax, r8d\n mov ecx, r9d\n cpuid\n hlt",
    "xgetbv": "mov ecx, r8d\n xgetbv\n hlt",
    "xsetbv": "mov ecx, r8d\n mov eax, r9d\n mov edx, r10d\n xsetbv\n xor ecx, ecx\n xgetbv\n hlt",
    "cx16": "cmpxchg16b [rdi]\n mov r8, [rdi]\n mov r9, [rdi+8]\n hlt",
    "cx8": "lock cmpxchg8b [rdi]\n mov r8, [rdi]\n hlt",
    "enter0": "lea rbp, [rsp+0x80]\n enter 0x28, 0\n hlt",
    "enter1": "lea rbp, [rsp+0x80]\n enter 0x18, 1\n hlt",
    "enter5": "lea rbp, [rsp+0x80]\n enter 0x100, 5\n mov r8, [rsp+0x100]\n hlt",
    "enter31": "mov rbp, rsi\n enter 0x8, 31\n hlt",
    "retfq": "push r9\n push r8\n retfq",
    "retf_imm": "mov [rsp-8], r11\n mov [rsp-16], r10\n mov [rsp-40], r9\n mov [rsp-48], r8\n sub rsp, 48\n retfq 0x10",
    "retfd": "mov [rsp-4], r9d\n mov [rsp-8], r8d\n sub rsp, 8\n retf",
    "iretd": "mov [rsp-4], r12d\n mov [rsp-8], r11d\n mov [rsp-12], r10d\n mov [rsp-16], r9d\n mov [rsp-20], r8d\n"
             " sub rsp, 20\n iretd",
    "farjmp": ".byte 0xff, 0x2f\n hlt",                     # jmp far [rdi] (m16:32)
    "farcall": ".byte 0x48, 0xff, 0x1f\n hlt",             # call far [rdi] (m16:64)
    "farjmp64": ".byte 0x48, 0xff, 0x2f\n hlt",
    "movsreg": "mov rax, ds\n mov ds, r8w\n mov es, r9w\n mov bx, es\n mov rcx, cs\n mov edx, ss\n hlt",
    "movfs": "mov fs, r8w\n rdfsbase rax\n mov gs, r9w\n rdgsbase rbx\n hlt",
    "movss": "mov ss, r8w\n mov rax, ss\n hlt",
    "movcs": ".byte 0x8e, 0xc8\n hlt",                       # mov cs, ax: #UD
    "pushpop": "push fs\n pop gs\n push gs\n pop fs\n .byte 0x66\n push fs\n .byte 0x66\n pop gs\n hlt",
    "lfs": "lfs eax, [rdi]\n rdfsbase rbx\n .byte 0x48, 0x0f, 0xb5, 0x0e\n hlt",  # lfs eax,[rdi]; lgs rcx,[rsi]
    "lss": ".byte 0x48, 0x0f, 0xb2, 0x07\n mov rbx, ss\n hlt",                    # lss rax, [rdi]
    "io": "in al, 0x60\n in eax, dx\n out dx, al\n out 0x80, eax\n .byte 0x66\n in eax, dx\n hlt",
    "ins": "and ecx, 7\n rep insb\n and r9d, 3\n mov ecx, r9d\n rep insd\n hlt",
    "outs": "and ecx, 7\n rep outsb\n outsd\n hlt",
    "x87": "fninit\n fnstcw [rdi]\n fnstsw ax\n fldcw [rsi]\n fnstenv [rdi+0x40]\n fnclex\n fldenv [rsi+0x40]\n"
           " fnstsw [rdi+0x80]\n fwait\n hlt",
    "fnsave": "fnsave [rdi]\n fninit\n frstor [rsi]\n fnstcw [rdi+0x80]\n fwait\n hlt",
    "fxsave": "movq xmm0, r8\n movq xmm9, r9\n fxsave64 [rdi]\n fxrstor64 [rsi]\n movq rax, xmm3\n hlt",
    "fxsave32": "fxsave [rdi]\n fxrstor [rsi]\n hlt",
    "cr0ts": "mov cr0, r13\n fnstcw [rdi]\n fwait\n fxsave [rdi]\n hlt",
    "xsave": "movq xmm1, r9\n vpbroadcastq ymm2, xmm1\n mov eax, r11d\n mov edx, r12d\n xsave [rdi]\n xrstor [rsi]\n hlt",
    "xsaveopt": "mov eax, r11d\n mov edx, r12d\n xsaveopt [rdi]\n hlt",
    "xsavec": "movq xmm4, r9\n vpbroadcastq ymm4, xmm4\n mov eax, r11d\n mov edx, r12d\n xsavec [rdi]\n xrstor [rsi]\n hlt",
    "xsaves": "mov eax, r11d\n mov edx, r12d\n xsaves [rdi]\n xrstors [rsi]\n hlt",
    "desc": "sgdt [rdi]\n sidt [rdi+0x10]\n sldt eax\n str rbx\n smsw rcx\n smsw [rdi+0x20]\n hlt",
    "lidt": "lidt [rsi]\n sidt [rdi]\n lgdt [rsi+0x10]\n sgdt [rdi+0x10]\n int 0x80\n hlt",
    "lmsw": "lmsw r8w\n clts\n smsw rax\n wbinvd\n invlpg [rdi]\n hlt",
    "dr": "mov dr7, rax\n mov rbx, dr7\n mov rcx, dr0\n mov rdx, dr6\n hlt",
    "rdpmc": "mov ecx, r8d\n rdpmc\n hlt",
    "lar": "lar eax, r8d\n setz r9b\n lsl rbx, r8d\n setz r10b\n verr r8w\n setz r11b\n verw r8w\n setz r12b\n hlt",
    "sysenter": "mov ecx, 0x174\n mov eax, r8d\n xor edx, edx\n wrmsr\n mov ecx, 0x176\n mov eax, r9d\n mov edx, r10d\n"
                " wrmsr\n sysenter\n hlt",
    "sysexit": "mov ecx, 0x174\n mov eax, r8d\n xor edx, edx\n wrmsr\n mov rcx, r11\n mov rdx, r12\n .byte 0x48, 0x0f, 0x35",
    "fsgs": "rdfsbase rax\n wrfsbase r8\n rdfsbase rbx\n wrgsbase r9d\n rdgsbase ecx\n hlt",
    "clflush": "clflush [rdi]\n clflushopt [rsi]\n hlt",
    "lock": "lock add [rdi], eax\n lock xadd [rdi+8], rbx\n lock btc qword ptr [rdi+16], 5\n lock not byte ptr [rdi+1]\n"
            " lock xchg [rdi+24], ecx\n hlt",
    "lockbad": "lock add [rdi], eax\n .byte 0xf0, 0x03, 0x07\n hlt",      # lock add eax, [rdi]: #UD
    "locknop": ".byte 0xf0, 0x90\n hlt",
    "lockreg": ".byte 0xf0, 0x48, 0xff, 0xc0\n hlt",                     # lock inc rax
    "ud_evex": ".byte 0x62, 0xf1, 0x7c, 0x48, 0x58, 0xc1\n hlt",  # vaddps zmm0, zmm0, zmm1 (outside U47)
    "ud_0f": ".byte 0x0f, 0xff, 0xc0\n hlt",
    "ud_b9": ".byte 0x0f, 0xb9, 0xc0\n hlt",
    "ud_0e": ".byte 0x0f, 0x0e\n hlt",
    # RTM with every transaction aborted at xbegin (U48): rax = 0 at the fallback, which skips a hlt;
    # xabort outside a transaction is a no-op, xtest sets ZF
    "rtm": "mov eax, 0x1234\n .byte 0xc7, 0xf8, 1, 0, 0, 0\n hlt\n mov ebx, eax\n .byte 0xc6, 0xf8, 0x11\n"
           " .byte 0x0f, 0x01, 0xd6\n hlt",
    "xend_gp": ".byte 0x0f, 0x01, 0xd5\n hlt",  # xend outside a transaction: #GP(0)
    "ud_8f": ".byte 0x8f, 0xc8\n hlt",
    "ud_fe": ".byte 0xfe, 0xd0\n hlt",
    "ud_jmpe": ".byte 0x0f, 0xb8, 0xc0\n hlt",
    "ud_getsec": ".byte 0x0f, 0x37\n hlt",
    "rdrand16": "rdrand ax\n rdseed rbx\n hlt",
    "sysret32": "mov ecx, r8d\n mov r11d, 0x202\n .byte 0x0f, 0x07",  # to compatibility mode: the fetch faults
    "to_user": TO_USER,
    "ltr": "ltr r8w\n str r9w\n hlt",
    "ltr2": "ltr r8w\n ltr r8w\n hlt",           # the second finds the TSS busy: #GP(sel)
    "ltrist": "ltr r8w\n int 0x2e\n hlt",          # IST1 from the new TSS
    "lldt": "lldt r8w\n sldt r9w\n hlt",
    "lldtm": "lldt [rsi]\n hlt",
}
U = {  # ring 3, entered through to_user (each ends with int3)
    "u_int29": "int 0x29\n int3",
    "u_int2e": "int 0x2e\n int3",
    "u_int23": "int 0x23\n int3",
    "u_int80": "int 0x80\n int3",
    "u_int1": ".byte 0xf1\n int3",
    "u_cli": "cli\n sti\n int3",
    "u_io": "in al, dx\n out dx, al\n int3",
    "u_ins": "and ecx, 3\n rep insb\n int3",
    "u_desc": "sgdt [rdi]\n sidt [rdi+0x10]\n str rax\n smsw rbx\n int3",
    "u_lgdt": "lgdt [rsi]\n int3",
    "u_lar": "lar eax, r8d\n setz r9b\n verr r8w\n setz r11b\n verw r8w\n setz r12b\n int3",
    "u_rdpmc": "mov ecx, r8d\n rdpmc\n int3",
    "u_xsaves": "xsaves [rdi]\n int3",
    "u_retf": "push r9\n push r8\n retfq",
    "u_movfs": "mov fs, r8w\n rdfsbase rax\n int3",
    "u_cpuid": "mov eax, r8d\n cpuid\n int3",
    "u_x87": "fninit\n fnstcw [rdi]\n int3",
    "u_x87a": "fld1\n fldpi\n faddp\n fild dword ptr [rsi]\n fmul st(0), st(1)\n fstp qword ptr [rdi]\n fistp word ptr [rdi+8]\n"
              " fnstsw ax\n int3",
    "u_sysret32": ".byte 0x0f, 0x07\n int3",
    "u_wbinvd": "wbinvd\n int3",
}
HANDLER_AT = KCODE + 0x5E00
UHANDLER_AT = UCODE + 0xF00
TO_USER_AT = KCODE + 0x5F00


@functools.lru_cache(maxsize=None)
def assemble(src: str) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        s, o, b = (os.path.join(d, n) for n in ("a.s", "a.o", "a.bin"))
        with open(s, "w") as f:
            f.write(".intel_syntax noprefix\n.code64\n" + src + "\n")
        subprocess.check_call(["as", "--64", "-o", o, s])
        subprocess.check_call(["objcopy", "-O", "binary", "-j", ".text", o, b])
        return open(b, "rb").read()


def _slots(snips: dict, base: int, step: int) -> dict:
    names = [n for n in snips if n != "to_user"]
    return {n: base + step * i for i, n in enumerate(names)}


KSLOT = _slots(K, KCODE, 0x100)
USLOT = _slots(U, UCODE, 0x80)
assert len(KSLOT) * 0x100 <= 0x5E00 and len(USLOT) * 0x80 <= 0xF00


def fx_image(rng: random.Random, mxcsr_ok=True) -> bytes:
    img = bytearray(rng.getrandbits(8) for _ in range(512))
    struct.pack_into("<HHBB", img, 0, 0x37F ^ rng.getrandbits(6), rng.getrandbits(16), rng.getrandbits(8), 0)
    struct.pack_into("<I", img, 24, (0x1F80 ^ rng.getrandbits(6)) if mxcsr_ok else 0x10000)
    for i in range(8):  # sign / exponent words: zero, a normal, or the special value
        struct.pack_into("<H", img, 40 + 16 * i, rng.choice([0, 0x3FFF, 0x7FFF, 0x8001]))
    return bytes(img)


def xs_image(rng: random.Random, kind: str) -> bytes:
    img = bytearray(fx_image(rng)) + bytearray(rng.getrandbits(8) for _ in range(1088 - 512))
    hdr = bytearray(64)
    if kind == "std":
        struct.pack_into("<QQ", hdr, 0, rng.getrandbits(3), 0)
    elif kind == "cmp":
        struct.pack_into("<QQ", hdr, 0, rng.getrandbits(3), 0x8000000000000007)
    elif kind == "bad":
        struct.pack_into("<QQQ", hdr, 0, 7, 0, 1)
    else:  # a component beyond XCR0 or XCOMP_BV
        struct.pack_into("<QQ", hdr, 0, 0x20, 0)
    img[512:576] = hdr
    return bytes(img)


def build_space(seed: int = 0x5157):
    """(address space, ring-0 initial state, data layout offsets)."""
    rng = random.Random(seed)
    sp = AddressSpace()
    code = bytearray(b"\xf4" * 0x1000 * 6)
    for n, va in KSLOT.items():
        b = assemble(K[n])
        assert len(b) <= 0x100, n
        assert n in U or len(b) <= 0x100
        code[va - KCODE:va - KCODE + len(b)] = b
    h = assemble(HANDLER)
    code[HANDLER_AT - KCODE:HANDLER_AT - KCODE + len(h)] = h
    t = assemble(TO_USER)
    code[TO_USER_AT - KCODE:TO_USER_AT - KCODE + len(t)] = t
    sp.map_range(KCODE, bytes(code), user=False, write=False, nx=False)
    ucode = bytearray(b"\xcc" * 0x1000)
    for n, va in USLOT.items():
        b = assemble(U[n])
        ucode[va - UCODE:va - UCODE + len(b)] = b
    uh = assemble(UHANDLER)
    ucode[UHANDLER_AT - UCODE:UHANDLER_AT - UCODE + len(uh)] = uh
    sp.map(UCODE, bytes(ucode), user=True, write=False, nx=False)
    idt = bytearray(0x1000)
    gates = {0x80: _gate(HANDLER_AT), 0x29: _gate(HANDLER_AT, dpl=3), 0x2E: _gate(HANDLER_AT, typ=0xF, dpl=3, ist=1),
             0x01: _gate(HANDLER_AT), 0x21: _gate(HANDLER_AT, dpl=3, p=0), 0x22: _gate(HANDLER_AT, typ=0xC, dpl=3),
             0x23: _gate(UHANDLER_AT, sel=0x33, dpl=3), 0x24: _gate(UHANDLER_AT, sel=0x33, dpl=0)}
    for v, g in gates.items():
        idt[v * 16:v * 16 + 16] = g
    sp.map(IDT, bytes(idt), user=False, write=False, nx=True)
    sp.map(GDT, gdt_page(), user=False, write=True, nx=True)
    tss = bytearray(0x1000)
    struct.pack_into("<Q", tss, 4, KSP + 0x800)       # RSP0
    struct.pack_into("<Q", tss, 0x24, ISTSTACK + 0xF80)  # IST1
    struct.pack_into("<Q", tss, 0x800 + 4, KSP + 0x400)     # the second TSS: RSP0
    struct.pack_into("<Q", tss, 0x800 + 0x24, ISTSTACK + 0x780)  # and IST1
    sp.map(TSS, bytes(tss), user=False, nx=True)
    for i in range(8):
        sp.map(KSTACK + i * 0x1000, b"", user=False, nx=True)
    sp.map(ISTSTACK, b"", user=False, nx=True)
    for i in range(4):
        sp.map(UST + i * 0x1000, b"", nx=True)
    # data: page 0 scratch (random), page 1 FXSAVE images, page 2 XSAVE images, page 3 far pointers / descriptors
    data = bytearray(rng.getrandbits(8) for _ in range(0x4000))
    lay = {"fx": [], "xs": []}
    for i, ok in enumerate([True, True, True, False]):
        off = 0x1000 + 0x200 * i
        data[off:off + 512] = fx_image(rng, ok)
        lay["fx"].append(off)
    # the page's other half: x87 environments / fnsave images stay random
    for i, kind in enumerate(["std", "std", "cmp", "bad"]):
        off = 0x2000 + 0x440 * i - (0x440 * i) % 64
        data[off:off + 1088] = xs_image(rng, kind)
        lay["xs"].append(off)
    # far pointers: (offset, selector) at 0x3000 + 16 * i (m16:64) and 0x3100 + 8 * i (m16:32)
    targets = [(KSLOT["int80"], 0x10), (KSLOT["int80"], 0x13), (USLOT["u_cpuid"], 0x33), (0, 0),
               (1 << 47, 0x10), (KSLOT["cpuid"], 0x18)]
    for i, (off, sel) in enumerate(targets):
        struct.pack_into("<QH", data, 0x3000 + 16 * i, off, sel)
        struct.pack_into("<IH", data, 0x3100 + 8 * i, off & 0xFFFFFFFF, sel)
    # pseudo-descriptors for lidt / lgdt: (limit, base)
    struct.pack_into("<HQ", data, 0x3200, 0xFFF, IDT)
    struct.pack_into("<HQ", data, 0x3210, GDT_LIMIT, GDT)
    struct.pack_into("<HQ", data, 0x3220, 0x7FF, IDT)
    struct.pack_into("<HQ", data, 0x3230, 0xFFF, 1 << 48)  # non-canonical base: #GP
    for i in range(4):
        sp.map(DATA + i * 0x1000, bytes(data[i * 0x1000:(i + 1) * 0x1000]), nx=True)
    sp.map(KDATA, bytes(rng.getrandbits(8) for _ in range(0x1000)), user=False, nx=True)
    st = user_state(KSLOT["cpuid"], KSP, sp.cr3)
    st.update({"cs": seg(0x10, 0, 0, 0x209B), "ss": seg(0x18, 0, 0xFFFFFFFF, 0xC93), "rflags": 0x202,
               "gdtr": {"base": GDT, "limit": GDT_LIMIT}, "idtr": {"base": IDT, "limit": 0xFFF},
               "tr": seg(0x40, TSS, 0x67, 0x8B), "fs": seg(0x53, 0x12345000, 0xFFF, 0x4F3),
               "fpcw": 0x27F, "fptw": 0xFFFF})
    return sp, st, lay, bytes(data)


# ---------------------------------------------------------------- lanes
SELS = [0, 3, 0x10, 0x13, 0x18, 0x1B, 0x23, 0x2B, 0x33, 0x38, 0x40, 0x53, 0x5B, 0x60, 0x68, 0x6B, 0x73, 0x7B, 0x80,
        0x2C]
LEAVES = [0, 1, 7, 0xD, 0xD, 0x80000000, 0x80000001, 0x80000002, 0x80000003, 0x80000004, 0x80000008, 5, 0x12345678,
          0x8000000F]


def lanes(n: int, seed: int, st: dict, lay: dict, data: bytes):
    """[(rip, 16 GPRs, rflags)] for n lanes over every snippet."""
    rng = random.Random(seed)
    names = list(KSLOT) + list(USLOT)
    out = []
    for i in range(n):
        name = names[i % len(names)]
        g = [rng.getrandbits(64) if rng.random() < 0.5 else rng.getrandbits(rng.choice([4, 8, 16, 32])) for _ in
             range(16)]
        g[4] = KSP
        flags = 0x202 | (rng.getrandbits(2) << 12) | (rng.getrandbits(1) << 10) | rng.choice([0, 1, 0x40, 0x41])
        g[7] = DATA + rng.choice([0, 0x40, 0x80, 0x3F8, 0xFF8, 0x800, 0x3FC0, 0x3FF8, 0x4000, 0x7])  # rdi
        g[6] = DATA + rng.choice([0x100, 0x200, 0x3FFC, 0x4000])                                 # rsi
        if name in ("cx16", "cx8"):
            g[7] = DATA + rng.choice([0x10, 0x20, 0x28, 0xFF8, 0x4000, 0x3FF0])
            off = g[7] - DATA
            if off + 16 <= len(data) and rng.random() < 0.5:
                g[0], g[2] = struct.unpack_from("<QQ", data, off)
                if name == "cx8":
                    v = struct.unpack_from("<Q", data, off)[0]
                    g[0], g[2] = v & 0xFFFFFFFF | (rng.getrandbits(32) << 32), v >> 32
        elif name.startswith("enter"):
            g[6] = KSP - rng.choice([0x100, 0x10, 0x800, 0x7000 - 0x80])
        elif name in ("retfq", "u_retf"):
            g[8] = rng.choice([0x10, 0x33, 0x13, 0, 0x2B, 0x23]) if name == "retfq" else rng.choice([0x33, 0x10, 0x30])
            # 0x23: SYSRET's compatibility-mode selector (a rip past 4 GiB is #GP(0), U29)
            g[9] = rng.choice([KSLOT["cpuid"], USLOT["u_cpuid"], 1 << 47, USLOT["u_int1"], USLOT["u_cpuid"] & 0xFFFFFFFF,
                               (1 << 32) | 0x1000])
        elif name == "retf_imm":
            g[8], g[9] = rng.choice([(KSLOT["cpuid"], 0x10), (USLOT["u_cpuid"], 0x33), (USLOT["u_cpuid"], 0x33)])
            g[10], g[11] = rng.choice([USP, KSP - 0x200, 1 << 50]), rng.choice([0x2B, 0, 0x18])
        elif name == "retfd":
            g[8], g[9] = rng.choice([(KSLOT["cpuid"] & 0xFFFFFFFF, 0x10), (0x40100000, 0x33), (0x1000, 0)])
        elif name == "iretd":
            g[8], g[9] = rng.choice([(KSLOT["cpuid"] & 0xFFFFFFFF, 0x10), (USLOT["u_cpuid"] & 0xFFFFFFFF, 0x33),
                                     (0x1000, 0x33), (0x1000, 0)])
            g[10] = (rng.getrandbits(22) & 0x3F7FD7) | 2
            g[11], g[12] = rng.choice([(USP & 0xFFFFFFFF, 0x2B), (KSP & 0xFFFFFFFF, 0x18), (0x1000, 0)])
        elif name in ("farjmp", "farcall", "farjmp64"):
            g[7] = DATA + (0x3100 + 8 * rng.randrange(6) if name == "farjmp" else 0x3000 + 16 * rng.randrange(6))
            if rng.random() < 0.1:
                g[7] = DATA + 0x3FFC
        elif name in ("movsreg", "movfs", "movss", "pushpop", "u_movfs"):
            g[8], g[9] = rng.choice(SELS), rng.choice(SELS)
        elif name in ("lfs", "lss"):
            g[7] = DATA + rng.choice([0x3000 + 16 * rng.randrange(6), 0x3100 + 8 * rng.randrange(6), 0x3FFC])
            g[6] = DATA + 0x3000 + 16 * rng.randrange(6)
        elif name in ("cpuid", "u_cpuid"):
            g[8], g[9] = rng.choice(LEAVES), rng.choice([0, 1, 2, 3, 4, 5])
        elif name in ("xgetbv", "xsetbv"):
            g[8] = rng.choice([0, 0, 0, 1, 2])
            g[9] = rng.choice([0x1F, 0x7, 0x3, 0x1, 0x5, 0x0, 0x1B, 0x20, 0x17])
            g[10] = rng.choice([0, 0, 0, 1])
        elif name in ("x87", "fnsave", "u_x87"):
            g[7] = DATA + rng.choice([0x80, 0x3F80, 0x3FF0, 0x4000])
            g[6] = DATA + rng.choice([0x1000, 0x1400, 0x100, 0x3FF8])
        elif name in ("fxsave", "fxsave32", "cr0ts"):
            g[7] = DATA + rng.choice([0x400, 0x410, 0x408, 0x3E00, 0x3F00])
            g[6] = DATA + rng.choice(lay["fx"] + [lay["fx"][0] + 8])
            g[13] = st["cr0"] | rng.choice([0, 0, 8, 4, 2, 0xA])
        elif name.startswith("xsave") or name == "u_xsaves":
            g[7] = DATA + rng.choice([0x400, 0x440, 0x420, 0x3C00, 0x3E00])
            g[6] = DATA + rng.choice(lay["xs"] + [lay["xs"][0] + 0x20])
            g[11] = rng.choice([0xFFFFFFFF, 7, 3, 1, 4, 0x1F, 0x18, 0])
            g[12] = rng.choice([0, 0xFFFFFFFF])
        elif name in ("lidt", "u_lgdt"):
            g[6] = DATA + rng.choice([0x3200, 0x3220, 0x3230])
        elif name == "lmsw":
            g[8] = rng.choice([0x33, 0x3B, 0x35, 0x30, 0x3F])
        elif name in ("rdpmc", "u_rdpmc"):
            g[8] = rng.choice([0, 3, 4, 0x40000000])
        elif name in ("ltr", "ltr2", "ltrist", "lldt", "lldtm"):
            g[8] = rng.choice([0x40, 0x90, 0x80, 0, 3, 0x44, 0x38, 0x10, 0x2B, 0x1000, 0x93, 0x98])
            g[6] = DATA + 0x3000 + 16 * rng.randrange(6)
        elif name in ("lar", "u_lar"):
            g[8] = rng.choice(SELS)
        elif name == "sysenter":
            g[8] = rng.choice([0, 0x10, 0x13])
            g[9], g[10] = KSLOT["cpuid"] & 0xFFFFFFFF, KSLOT["cpuid"] >> 32
        elif name == "sysexit":
            g[8] = rng.choice([0, 0x10])
            g[11], g[12] = rng.choice([USP, 1 << 50]), rng.choice([USLOT["u_cpuid"], 1 << 47])
        elif name in ("fsgs",):
            g[8] = rng.choice([0x12340000, 1 << 47, 0xFFFFF80000000000])
        elif name in ("io", "ins", "outs", "u_io", "u_ins"):
            g[2] = rng.getrandbits(16)
        rip = KSLOT.get(name)
        if rip is None:  # ring 3 through the iretq stub: rbx = snippet, r14 = rsp, r15 = rflags
            rip = TO_USER_AT
            g[3], g[14], g[15] = USLOT[name], USP, flags | 0x200
        out.append((rip, g, flags))
    return out


def oracle_run(sp, st: dict, ln, limit=3000):
    """Final state per lane (lane_view): exit, GPRs, the register file and
    the contents of every dirty page."""
    from tests.oracle_lib import Oracle

    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    base = regs_from_state(st)
    o.set_limit(limit)
    out = []
    for va, g, flags in ln:
        r = regs_from_state(st)
        for k in range(16):
            r.gpr[k] = g[k]
        r.rip, r.rflags = va, flags
        o.restore(base)
        o.set_regs(r)
        ex = o.run()
        dirty = set(o.dirty())
        out.append(lane_view(ex.status, ex.vector, ex.error, ex.addr, ex.icount, o.nbytes(), o.regs(),
                             {gpa: o.read_phys(gpa, 4096) for gpa in dirty}))
    return out


STATE_FIELDS = ("cr0", "cr4", "xcr0", "mxcsr", "fpcw", "fpsw", "fptw", "fpop", "gdtr_base", "gdtr_limit",
                "idtr_base", "idtr_limit", "sysenter_cs", "sysenter_eip", "sysenter_esp")


def lane_view(status, vector, error, addr, icount, nbytes, r, pages: dict) -> dict:
    f = status == 5  # FAULT: vector / error / cr2 are meaningful
    return {
        "exit": (status, vector if f else 0, error if f else 0, addr if f and vector == 14 else 0, r.rip, icount),
        "nbytes": nbytes, "gpr": list(r.gpr), "rflags": r.rflags,
        "state": {k: int(getattr(r, k)) for k in STATE_FIELDS},
        "sel": [int(r.seg[i].selector) for i in range(8)], "fsgs": (int(r.seg[4].base), int(r.seg[5].base)),
        "fpst": list(r.fpst), "xmm": [int(x) for row in r.xmm for x in row],
        "ymmh": [int(x) for row in r.ymmh for x in row], "pages": pages,
    }
