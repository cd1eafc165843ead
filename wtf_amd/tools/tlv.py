"""TLV: the synthetic tlv_server snapshot (BASELINE.json configs[2..3]).

No real tlv_server snapshot can be fetched offline. This builds a
look-alike in wtf's on-disk formats: the guest program
`guest/tlv_server.c` (a freestanding restatement of the reference target's
ProcessPacket, src/tlv_server/tlv_server.cc:31-94) is compiled with the
container's gcc (Win64 calling convention) and mapped into a ring-3 address
space; the CPU state is the one the reference snapshot is taken at (rip =
tlv_server!ProcessPacket, [rsp] = the return address into the receive loop,
rcx = the packet page followed by a guard page, fuzzer_tlv_server.cc:80-124);
the symbol store exports every symbol the tlv module and the user-mode crash
detection ask for (Appendix B).

Layout (guest virtual):
  0x140001000  .text (r-x)   0x140002000 .rodata (r--)   0x140003000 .data (rw-)
  0x200000000  page heap: 64 slots of [page rw-][guard, unmapped]
  0x300000000  packet page (rw-), 0x300001000 guard (unmapped)
  STACK_TOP-0x4000 .. STACK_TOP   stack (rw-)
  0xFFFFF80000004000  IDT (supervisor): gate 0x29 only (64-bit interrupt gate,
                      DPL 3) -> nt!KiRaiseSecurityCheckFailure
  0xFFFFF80000002000  TSS (RSP0 = the kernel stack)
  0xFFFFF80000100000  nt!KiRaiseSecurityCheckFailure (supervisor code: hlt)
  0xFFFFF80000300000  kernel stack, 2 pages (supervisor rw-)
The guest's __fastfail (`int 0x29`, tlv_server.c Free) reaches the kernel
routine through that gate, as on Windows; no other vector has a gate, so a
fault ends the testcase with the fault (user-mode crash naming, U14).
"""
from __future__ import annotations

import json
import os
import struct
import subprocess

from .snapshot import PAGE, AddressSpace, user_state, write_snapshot

HERE = os.path.dirname(os.path.abspath(__file__))
GUEST_SRC = os.path.join(HERE, "guest", "tlv_server.c")
GUEST_LD = os.path.join(HERE, "guest", "guest.ld")
HEAP_BASE = 0x200000000
HEAP_SLOTS = 64
HEAP_STRIDE = 0x2000
PACKET_VA = 0x300000000
STACK_TOP = 0x7FF000000000
IDT = 0xFFFFF80000004000     # user_state's idtr
TSS = 0xFFFFF80000002000     # user_state's tr.base
KI_RAISE = 0xFFFFF80000100000
KSTACK = 0xFFFFF80000300000
FASTFAIL_VECTOR = 0x29
# gcc's default x86-64 code generation (SSE2 baseline): the engine runs the
# SSE / SSE2 subset (U22), so the guests are not restricted to general registers
CFLAGS = ["-O2", "-ffreestanding", "-fpie", "-fvisibility=hidden", "-mabi=ms",
          "-mno-red-zone", "-fno-stack-protector", "-fcf-protection=none", "-fno-tree-loop-distribute-patterns",
          "-fno-asynchronous-unwind-tables", "-nostdlib", "-static", "-Wl,--build-id=none"]


def compile_guest(out_elf: str) -> None:
    subprocess.check_call(["gcc", *CFLAGS, "-Wl,-T," + GUEST_LD, "-o", out_elf, GUEST_SRC])


def _elf(path: str):
    """(PT_LOAD segments [(vaddr, flags, bytes, memsz)], {symbol: value}) of a static ELF64."""
    b = open(path, "rb").read()
    assert b[:4] == b"\x7fELF" and b[4] == 2
    e_phoff, e_shoff = struct.unpack_from("<QQ", b, 0x20)
    e_phentsize, e_phnum, e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHHHH", b, 0x36)
    segs = []
    for i in range(e_phnum):
        p_type, p_flags, p_off, p_vaddr, _, p_filesz, p_memsz, _ = struct.unpack_from("<IIQQQQQQ", b, e_phoff + i * e_phentsize)
        if p_type == 1:
            segs.append((p_vaddr, p_flags, b[p_off:p_off + p_filesz], p_memsz))
    shdrs = [struct.unpack_from("<IIQQQQIIQQ", b, e_shoff + i * e_shentsize) for i in range(e_shnum)]
    syms = {}
    for sh in shdrs:
        if sh[1] != 2:  # SHT_SYMTAB
            continue
        strtab = shdrs[sh[6]]
        for off in range(sh[4], sh[4] + sh[5], 24):
            st_name, st_info, _, st_shndx, st_value, _ = struct.unpack_from("<IBBHQQ", b, off)
            if st_name and st_shndx:
                s0 = strtab[4] + st_name
                name = b[s0:b.index(b"\0", s0)].decode()
                syms[name] = st_value
    return segs, syms


def build(state_dir: str, work_dir: str | None = None, packet: str = "rw") -> dict:
    """Compiles the guest and writes mem.dmp / regs.json / symbol-store.json
    into state_dir. Returns the guest symbol table. `packet` maps the packet
    buffer page read-write ("rw", the real server), read-only ("ro": the
    module's writes still land, Backend_t::VirtWrite translates without a
    permission check, backend.cc:91-121) or not at all ("none": the module's
    write fails and its handler aborts)."""
    work_dir = work_dir or state_dir
    os.makedirs(work_dir, exist_ok=True)
    elf = os.path.join(work_dir, "tlv_server_guest.elf")
    compile_guest(elf)
    segs, syms = _elf(elf)
    sp = AddressSpace()
    for vaddr, flags, data, memsz in segs:
        assert vaddr % PAGE == 0
        img = data + b"\0" * (memsz - len(data))
        if vaddr == syms["G"] & ~0xFFF:
            # heap ready at snapshot time: free list 1 -> 2 -> ... -> 64, nothing in
            # use, no chunk freed yet, G.Initialised = 1 (tlv_server.c struct Globals)
            goff = syms["G"] - vaddr
            img = bytearray(img.ljust(goff + 0x40, b"\0"))
            struct.pack_into("<QQQQ", img, goff + 0x20, 0, 1, 0, 1)
            img = bytes(img)
        sp.map_range(vaddr, img, user=True, write=bool(flags & 2), nx=not (flags & 1))
    for i in range(HEAP_SLOTS):
        link = (i + 2) if i + 1 < HEAP_SLOTS else 0
        sp.map(HEAP_BASE + i * HEAP_STRIDE, struct.pack("<Q", link), nx=True)
    if packet != "none":
        sp.map(PACKET_VA, b"", nx=True, write=packet == "rw")
    for va in range(STACK_TOP - 0x4000, STACK_TOP, PAGE):
        sp.map(va, b"", nx=True)
    # ring 0 pieces the __fastfail path runs through (SDM vol. 3 6.14)
    sp.map(KI_RAISE, b"\xf4" * 16, user=False, write=False, nx=False)
    idt = bytearray(PAGE)
    lo = (KI_RAISE & 0xFFFF) | (0x10 << 16) | (0xEE << 40) | (((KI_RAISE >> 16) & 0xFFFF) << 48)
    struct.pack_into("<QQ", idt, FASTFAIL_VECTOR * 16, lo, KI_RAISE >> 32)
    sp.map(IDT, bytes(idt), user=False, write=False, nx=True)
    tss = bytearray(PAGE)
    struct.pack_into("<Q", tss, 4, KSTACK + 2 * PAGE - 0x40)  # RSP0
    sp.map(TSS, bytes(tss), user=False, nx=True)
    for i in range(2):
        sp.map(KSTACK + i * PAGE, b"", user=False, nx=True)
    rsp = STACK_TOP - 0x108  # rsp = 8 mod 16 at function entry
    sp.write(rsp, struct.pack("<Q", syms["ServerLoopReturn"]))
    st = user_state(syms["ProcessPacket"], rsp, sp.cr3, rcx=PACKET_VA, rdx=0x1000)
    symbols = {
        "tlv_server": segs[0][0] - 0x1000,
        "tlv_server!ProcessPacket": syms["ProcessPacket"],
        "tlv_server!printf": syms["printf"],
        "tlv_server!ServerLoop": syms["ServerLoop"],
        "hal!HalpPerfInterrupt": syms["HalpPerfInterrupt"],
        "nt!KeBugCheck2": syms["KeBugCheck2"],
        "nt!SwapContext": syms["SwapContext"],
        "ntdll!RtlDispatchException": syms["RtlDispatchException"],
        "nt!KiRaiseSecurityCheckFailure": KI_RAISE,
        "verifier": 0,
    }
    write_snapshot(state_dir, sp, st, symbols)
    return syms


def packets_json(packets: list[tuple[int, int, int, bytes]]) -> bytes:
    """A testcase as the tlv module's mutator serialises it (nlohmann dump():
    keys sorted, no spaces; fuzzer_tlv_server.cc:27-36)."""
    out = []
    for cmd, pid, body_size, body in packets:
        out.append('{"Body":[%s],"BodySize":%d,"Command":%d,"Id":%d}'
                   % (",".join(str(x) for x in body), body_size, cmd, pid))
    return ('{"Packets":[%s]}' % ",".join(out)).encode()


def seed_inputs(inputs_dir: str) -> list[str]:
    """A small seed corpus covering each command and the table-full path."""
    os.makedirs(inputs_dir, exist_ok=True)
    seeds = {
        "alloc_edit_delete": [(0, 1, 4, b"AAAA"), (1, 1, 4, b"BBBB"), (2, 1, 0, b"")],
        "alloc_many": [(0, i, 8, bytes([0x41 + i] * 8)) for i in range(4)],
        "edit_missing": [(1, 7, 2, b"zz"), (2, 9, 0, b"")],
        "short_packet": [(0, 3, 16, b"0123456789abcdef"), (1, 3, 16, b"fedcba9876543210")],
    }
    paths = []
    for name, pk in seeds.items():
        p = os.path.join(inputs_dir, name)
        with open(p, "wb") as f:
            f.write(packets_json(pk))
        paths.append(p)
    return paths


if __name__ == "__main__":
    import sys
    d = sys.argv[1] if len(sys.argv) > 1 else "build/tlv_server"
    build(os.path.join(d, "state"), os.path.join(d, "work"))
    seed_inputs(os.path.join(d, "inputs"))
    os.makedirs(os.path.join(d, "outputs"), exist_ok=True)
    os.makedirs(os.path.join(d, "crashes"), exist_ok=True)
    print(json.dumps({"target": d}))
