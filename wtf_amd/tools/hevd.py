"""HEVD: the synthetic kernel-driver snapshot (BASELINE.json configs[4]).

No HEVD snapshot (Windows kernel + HackSysExtremeVulnerableDriver memory dump)
can be fetched offline. This builds a look-alike in wtf's on-disk
formats from two freestanding guest images compiled
with the container's gcc (Win64 calling convention):

  guest/hevd_user.c    ring 3: the program stopped at its 6-byte
                       `call [rip+x]` to DeviceIoControl (fuzzer_hevd.cc:66-67)
                       and the DeviceIoControl stub that enters the kernel
                       with SYSCALL;
  guest/hevd_kernel.c  ring 0 (supervisor pages): KiSystemCall64 (SWAPGS,
                       kernel stack from the per-processor block, SYSRETQ),
                       the IOCTL dispatcher and handlers with HEVD's bug
                       classes, nt!DbgPrintEx, nt!ExGenRandom (`rdrand rdx` at
                       +0xe0), nt!KeBugCheck2 and nt!SwapContext.

The CPU state is the reference snapshot's: rip at the call, rcx = device
handle, rdx = IOCTL code, r8 = user buffer (1024 bytes, fuzzer_hevd.cc:43-48),
r9 = its size, stack arguments 5..8 of DeviceIoControl in place (the module
writes the size at GetArgAddress(5), :50-56); EFER.SCE set, STAR / LSTAR /
SFMASK / IA32_KERNEL_GS_BASE as a Windows kernel programs them.

Layout (guest virtual):
  0x140001000                 user image (r-x / r-- / rw-)
  0x10000000                  user buffer, 2 pages (rw-)
  STACK_TOP-0x4000..STACK_TOP user stack (rw-)
  0xFFFFF80000100000          kernel image (supervisor)
  0xFFFFF80000002000          TSS (RSP0 = kernel stack), 0xFFFFF80000004000 IDT
                              (#DE/#UD/#GP/#PF gates -> KiTrapHandler)
  0xFFFFF80000200000          KPCR page (supervisor rw-)
  0xFFFFF80000300000..+0x8000 kernel stack (supervisor rw-)
"""
from __future__ import annotations

import json
import os
import struct
import subprocess

from .snapshot import PAGE, AddressSpace, user_state, write_snapshot
from .tlv import CFLAGS, _elf

HERE = os.path.dirname(os.path.abspath(__file__))
USER_SRC = os.path.join(HERE, "guest", "hevd_user.c")
KERNEL_SRC = os.path.join(HERE, "guest", "hevd_kernel.c")
USER_LD = os.path.join(HERE, "guest", "guest.ld")
KERNEL_LD = os.path.join(HERE, "guest", "hevd_kernel.ld")
USER_BUF = 0x10000000
STACK_TOP = 0x7FF000000000
KPCR = 0xFFFFF80000200000
KSTACK = 0xFFFFF80000300000
KSTACK_PAGES = 8
IDT = 0xFFFFF80000004000  # idtr (user_state), limit 0xfff
TSS = 0xFFFFF80000002000  # tr.base (user_state)
HANDLE = 0x3C
TRAPS = {0: "KiDivideErrorFault", 6: "KiInvalidOpcodeFault", 13: "KiGeneralProtectionFault", 14: "KiPageFault"}


def idt_page(ksyms: dict) -> bytes:
    """64-bit interrupt gates (present, DPL 0, type 0xE, selector 0x10) for the
    fault vectors the kernel image handles; the other vectors stay not-present."""
    idt = bytearray(PAGE)
    for vec, name in TRAPS.items():
        off = ksyms[name]
        lo = (off & 0xFFFF) | (0x10 << 16) | (0x8E << 40) | (((off >> 16) & 0xFFFF) << 48)
        struct.pack_into("<QQ", idt, vec * 16, lo, off >> 32)
    return bytes(idt)


def compile_images(work_dir: str, io: bool = False) -> tuple[str, str]:
    """io: the HEVD_IO kernel (the I/O manager's IRP path, hevd_kernel.c)."""
    os.makedirs(work_dir, exist_ok=True)
    user = os.path.join(work_dir, "hevd_user.elf")
    kernel = os.path.join(work_dir, "hevd_kernel_io.elf" if io else "hevd_kernel.elf")
    subprocess.check_call(["gcc", *CFLAGS, "-Wl,-T," + USER_LD, "-Wl,-e,UserMain", "-o", user, USER_SRC])
    subprocess.check_call(["gcc", *CFLAGS, *(["-DHEVD_IO"] if io else []), "-Wl,-T," + KERNEL_LD, "-o", kernel,
                           KERNEL_SRC])
    return user, kernel


def _map_image(sp: AddressSpace, segs, user: bool) -> None:
    for vaddr, flags, data, memsz in segs:
        assert vaddr % PAGE == 0
        sp.map_range(vaddr, data + b"\0" * (memsz - len(data)), user=user, write=bool(flags & 2),
                     nx=not (flags & 1))


def build(state_dir: str, work_dir: str | None = None, io: bool = False) -> dict:
    """Compiles both images and writes mem.dmp / regs.json / symbol-store.json
    into state_dir. Returns {name: address} of the guest symbols. io: the
    HEVD_IO kernel (wtf_amd/tools/hevd_io.py)."""
    sp, st, symbols, syms = build_space(work_dir or state_dir, io)
    write_snapshot(state_dir, sp, st, symbols)
    return syms


def build_space(work_dir: str, io: bool = False):
    """(address space, CPU state, symbol store, guest symbols) of the snapshot."""
    user_elf, kernel_elf = compile_images(work_dir, io)
    usegs, usyms = _elf(user_elf)
    ksegs, ksyms = _elf(kernel_elf)
    sp = AddressSpace()
    _map_image(sp, usegs, user=True)
    _map_image(sp, ksegs, user=False)
    # DeviceIoControl pointer (the import the call site goes through)
    sp.write(usyms["pDeviceIoControl"], struct.pack("<Q", usyms["DeviceIoControl"]))
    for i in range(2):
        sp.map(USER_BUF + i * PAGE, b"", nx=True)
    for va in range(STACK_TOP - 0x4000, STACK_TOP, PAGE):
        sp.map(va, b"", nx=True)
    sp.map(IDT, idt_page(ksyms), user=False, write=False, nx=True)
    tss = bytearray(PAGE)
    struct.pack_into("<Q", tss, 4, KSTACK + KSTACK_PAGES * PAGE - 0x40)  # RSP0
    sp.map(TSS, bytes(tss), user=False, nx=True)
    kpcr = bytearray(PAGE)
    struct.pack_into("<Q", kpcr, 0x1A8, KSTACK + KSTACK_PAGES * PAGE - 0x40)
    sp.map(KPCR, bytes(kpcr), user=False, nx=True)
    for i in range(KSTACK_PAGES):
        sp.map(KSTACK + i * PAGE, b"", user=False, nx=True)
    rsp = STACK_TOP - 0x1000 - 0x50  # UserMain's frame (sub rsp, 0x48 from an entry rsp = 8 mod 16)
    # DeviceIoControl(handle, code, in, insize, out, outsize, &returned, NULL): args 4..7
    returned = rsp + 0x40
    sp.write(rsp + 0x20, struct.pack("<QQQQ", USER_BUF, 0x400, returned, 0))
    st = user_state(usyms["CallSite"], rsp, sp.cr3, rcx=HANDLE, rdx=0x222003, r8=USER_BUF, r9=0x400)
    st.update({"lstar": ksyms["KiSystemCall64"], "kernel_gs_base": KPCR, "star": 0x0023001000000000,
               "sfmask": 0x4700, "cstar": 0})
    symbols = {
        "nt": ksegs[0][0] - 0x1000,
        "nt!DbgPrintEx": ksyms["DbgPrintEx"],
        "nt!ExGenRandom": ksyms["ExGenRandom"],
        "nt!KeBugCheck2": ksyms["KeBugCheck2"],
        "nt!SwapContext": ksyms["SwapContext"],
        "nt!KiPageFault": ksyms["KiPageFault"],
        "nt!KiGeneralProtectionFault": ksyms["KiGeneralProtectionFault"],
        "nt!KiSystemCall64": ksyms["KiSystemCall64"],
        "HEVD!IrpDeviceIoCtlHandler": ksyms["HevdIrpDeviceIoCtlHandler" if io else "NtDeviceIoControlFile"],
        "kernelbase!DeviceIoControl": usyms["DeviceIoControl"],
    }
    syms = {**{f"user:{k}": v for k, v in usyms.items()}, **{f"kernel:{k}": v for k, v in ksyms.items()}}
    return sp, st, symbols, syms


def testcase(ioctl: int, body: bytes) -> bytes:
    """The hevd module's testcase format: u32 IOCTL code + buffer (<= 1024 B,
    fuzzer_hevd.cc:20-30)."""
    return struct.pack("<I", ioctl) + body


def seed_inputs(inputs_dir: str) -> list[str]:
    """One benign seed per IOCTL (the mutator finds the bugs)."""
    os.makedirs(inputs_dir, exist_ok=True)
    seeds = {
        "stack": testcase(0x222003, b"A" * 64),
        "stack_gs": testcase(0x222007, b"B" * 64),
        "write_what_where": testcase(0x22200B, struct.pack("<QQ", USER_BUF + 0x100, USER_BUF + 0x108) + b"\0" * 16),
        "pool": testcase(0x22200F, b"C" * 32),
        "null": testcase(0x222013, struct.pack("<I", 0x11223344)),
        "integer": testcase(0x222017, b"D" * 32 + struct.pack("<I", 0xBAD0B0B0)),
        "type": testcase(0x22201B, struct.pack("<QQ", 1, 2)),
        "wait": testcase(0x22201F, b"notwait!"),
        "invalid": testcase(0x222fff, b""),
    }
    paths = []
    for name, data in seeds.items():
        p = os.path.join(inputs_dir, name)
        with open(p, "wb") as f:
            f.write(data)
        paths.append(p)
    return paths


if __name__ == "__main__":
    import sys
    d = sys.argv[1] if len(sys.argv) > 1 else "build/hevd"
    build(os.path.join(d, "state"), os.path.join(d, "work"))
    seed_inputs(os.path.join(d, "inputs"))
    os.makedirs(os.path.join(d, "outputs"), exist_ok=True)
    os.makedirs(os.path.join(d, "crashes"), exist_ok=True)
    print(json.dumps({"target": d}))
