"""Synthetic wtf snapshots: x86-64 page tables, kdmp `mem.dmp`, `regs.json`,
`symbol-store.json`.

No real tlv_server / HEVD snapshot can be fetched offline, so the
build synthesises snapshots in exactly the on-disk formats wtf consumes:

* `mem.dmp`: kdmp 64-bit header (`HEADER64`, kdmp-parser-structs.h:558-631)
  followed either by run-ordered pages (full dump, DumpType 1, pages from file
  offset 0x2000, kdmp-parser.h:399-484) or by a BMP header + bitmap + pages
  (DumpType 5, kdmp-parser.h:490-529). The reference's own kdmp-parser,
  compiled by oracle/Makefile into oracle/_ref/kdmp_ref, checks these files in
  tests/test_snapshot_format.py.
* `regs.json`: every key `LoadCpuStateFromJSON` reads (utils.cc:57-193), hex
  strings, segments as {present, selector, base, limit, attr}.
* `symbol-store.json`: flat {"module!symbol": "0x..."} (debugger.h:351-364).
"""
from __future__ import annotations

import json
import os
import struct

PAGE = 4096
PTE_P, PTE_W, PTE_U, PTE_PS = 0x1, 0x2, 0x4, 0x80
PTE_NX = 1 << 63
ADDR_MASK = 0x000FFFFFFFFFF000


class AddressSpace:
    """Builds a 4-level x86-64 page table hierarchy over a sparse physical memory."""

    def __init__(self, first_pfn: int = 0x1000):
        self.next_pfn = first_pfn
        self.pages: dict[int, bytearray] = {}
        self.cr3 = self.alloc() << 12

    def alloc(self, data: bytes | None = None) -> int:
        pfn = self.next_pfn
        self.next_pfn += 1
        page = bytearray(PAGE)
        if data:
            page[: len(data)] = data
        self.pages[pfn] = page
        return pfn

    def _entry(self, table_pfn: int, idx: int) -> int:
        return struct.unpack_from("<Q", self.pages[table_pfn], idx * 8)[0]

    def _set_entry(self, table_pfn: int, idx: int, val: int) -> None:
        struct.pack_into("<Q", self.pages[table_pfn], idx * 8, val)

    def map_pfn(self, va: int, pfn: int, user=True, write=True, nx=False) -> None:
        assert va % PAGE == 0
        table = self.cr3 >> 12
        for level in (3, 2, 1):
            idx = (va >> (12 + 9 * level)) & 0x1FF
            e = self._entry(table, idx)
            if not e & PTE_P:
                child = self.alloc()
                e = (child << 12) | PTE_P | PTE_W | PTE_U
                self._set_entry(table, idx, e)
            table = (e & ADDR_MASK) >> 12
        idx = (va >> 12) & 0x1FF
        leaf = (pfn << 12) | PTE_P | (PTE_W if write else 0) | (PTE_U if user else 0) | (PTE_NX if nx else 0)
        self._set_entry(table, idx, leaf)

    def map(self, va: int, data: bytes = b"", user=True, write=True, nx=False) -> int:
        """Map one page at va backed by a fresh physical page holding data. Returns pfn."""
        pfn = self.alloc(data)
        self.map_pfn(va, pfn, user, write, nx)
        return pfn

    def map_range(self, va: int, data: bytes, **kw) -> list[int]:
        pfns = []
        for off in range(0, max(len(data), 1), PAGE):
            pfns.append(self.map(va + off, data[off: off + PAGE], **kw))
        return pfns

    def unmap(self, va: int) -> None:
        """Clear the leaf PTE of va (the page becomes not-present)."""
        table = self.cr3 >> 12
        for level in (3, 2, 1):
            e = self._entry(table, (va >> (12 + 9 * level)) & 0x1FF)
            if not e & PTE_P:
                return
            table = (e & ADDR_MASK) >> 12
        self._set_entry(table, (va >> 12) & 0x1FF, 0)

    def translate(self, va: int) -> int | None:
        table = self.cr3 >> 12
        for level in (3, 2, 1, 0):
            e = self._entry(table, (va >> (12 + 9 * level)) & 0x1FF)
            if not e & PTE_P:
                return None
            if level in (1, 2) and e & PTE_PS:
                mask = (1 << (12 + 9 * level)) - 1
                return (e & ADDR_MASK & ~mask) | (va & mask)
            table = (e & ADDR_MASK) >> 12
        return (table << 12) | (va & 0xFFF)

    def write(self, va: int, data: bytes) -> None:
        for i, b in enumerate(data):
            pa = self.translate(va + i)
            assert pa is not None, hex(va + i)
            self.pages[pa >> 12][pa & 0xFFF] = b

    def phys(self) -> tuple[list[int], bytes]:
        pfns = sorted(self.pages)
        return pfns, b"".join(bytes(self.pages[p]) for p in pfns)


# --------------------------------------------------------------------------
# CPU state
# --------------------------------------------------------------------------
GPRS = ["rax", "rcx", "rdx", "rbx", "rsp", "rbp", "rsi", "rdi",
        "r8", "r9", "r10", "r11", "r12", "r13", "r14", "r15"]


def user_state(rip: int, rsp: int, cr3: int, **gprs) -> dict:
    """A ring-3 64-bit Windows-like CPU state (values shaped like a bdump regs.json)."""
    st = {g: 0 for g in GPRS}
    st.update(gprs)
    st.update({
        "rip": rip, "rsp": rsp, "rflags": 0x202, "cr0": 0x80050031, "cr2": 0, "cr3": cr3,
        "cr4": 0x370678, "cr8": 0, "efer": 0xD01, "xcr0": 0x1F, "tsc": 0x1000, "tsc_aux": 0,
        "apic_base": 0xFEE00900, "pat": 0x0007010600070106, "sysenter_cs": 0, "sysenter_esp": 0,
        "sysenter_eip": 0, "star": 0x0023001000000000, "lstar": 0xFFFFF80000001000,
        "cstar": 0xFFFFF80000001040, "sfmask": 0x4700, "kernel_gs_base": 0,
        "fpcw": 0x27F, "fpsw": 0, "fptw": 0, "fpop": 0, "mxcsr": 0x1F80, "mxcsr_mask": 0xFFBF,
        "dr0": 0, "dr1": 0, "dr2": 0, "dr3": 0, "dr6": 0, "dr7": 0,
        "es": seg(0x2B, 0, 0xFFFFFFFF, 0xCF3), "cs": seg(0x33, 0, 0, 0x20FB),
        "ss": seg(0x2B, 0, 0xFFFFFFFF, 0xCF3), "ds": seg(0x2B, 0, 0xFFFFFFFF, 0xCF3),
        "fs": seg(0x53, 0, 0x3C00, 0x4F3), "gs": seg(0x2B, 0x7FF000000000, 0xFFFFFFFF, 0xCF3),
        "tr": seg(0x40, 0xFFFFF80000002000, 0x67, 0x8B), "ldtr": seg(0, 0, 0, 0),
        "gdtr": {"base": 0xFFFFF80000003000, "limit": 0x57},
        "idtr": {"base": 0xFFFFF80000004000, "limit": 0xFFF},
        "fpst": ["0x-Infinity"] * 8,
    })
    return st


def seg(selector, base, limit, attr, present=True) -> dict:
    # SanitizeCpuState (utils.cc:234-243) wants attr bits 8-11 == (limit >> 16) & 0xf
    attr = (attr & ~0xF00) | (((limit >> 16) & 0xF) << 8)
    return {"present": present, "selector": selector, "base": base, "limit": limit, "attr": attr}


def regs_json(state: dict) -> dict:
    out = {}
    for k, v in state.items():
        if isinstance(v, dict):
            out[k] = {kk: (vv if isinstance(vv, bool) else hex(vv)) for kk, vv in v.items()}
        elif isinstance(v, list):
            out[k] = v
        else:
            out[k] = hex(v)
    return out


# --------------------------------------------------------------------------
# kdmp writer
# --------------------------------------------------------------------------
def _runs(pfns: list[int]) -> list[tuple[int, int]]:
    runs = []
    for p in pfns:
        if runs and runs[-1][0] + runs[-1][1] == p:
            runs[-1] = (runs[-1][0], runs[-1][1] + 1)
        else:
            runs.append((p, 1))
    return runs


def _context(state: dict) -> bytes:
    ctx = bytearray(0x4D0)
    struct.pack_into("<I", ctx, 0x30, 0x10001F)  # ContextFlags
    struct.pack_into("<I", ctx, 0x34, state.get("mxcsr", 0x1F80))
    for i, name in enumerate(["cs", "ds", "es", "fs", "gs", "ss"]):
        struct.pack_into("<H", ctx, 0x38 + 2 * i, state[name]["selector"])
    struct.pack_into("<I", ctx, 0x44, state["rflags"] & 0xFFFFFFFF)
    for i, g in enumerate(["rax", "rcx", "rdx", "rbx", "rsp", "rbp", "rsi", "rdi",
                           "r8", "r9", "r10", "r11", "r12", "r13", "r14", "r15"]):
        struct.pack_into("<Q", ctx, 0x78 + 8 * i, state[g])
    struct.pack_into("<Q", ctx, 0xF8, state["rip"])
    struct.pack_into("<H", ctx, 0x100, state.get("fpcw", 0x27F))
    struct.pack_into("<I", ctx, 0x118, state.get("mxcsr", 0x1F80))  # MxCsr2 == MxCsr
    struct.pack_into("<I", ctx, 0x11C, state.get("mxcsr_mask", 0xFFBF))
    return bytes(ctx)


def write_kdmp(path: str, pfns: list[int], pages: bytes, state: dict, bmp: bool | None = None) -> None:
    runs = _runs(pfns)
    if bmp is None:
        bmp = len(runs) > 40
    hdr = bytearray(0x2000)
    struct.pack_into("<IIII", hdr, 0, 0x45474150, 0x34365544, 15, 19041)
    struct.pack_into("<Q", hdr, 0x10, state["cr3"])
    struct.pack_into("<II", hdr, 0x30, 0x8664, 1)
    hdr[0x348: 0x348 + 0x4D0] = _context(state)
    if not bmp:
        struct.pack_into("<IIQ", hdr, 0x88, len(runs), 0, len(pfns))
        for i, (base, count) in enumerate(runs):
            struct.pack_into("<QQ", hdr, 0x98 + 16 * i, base, count)
        struct.pack_into("<I", hdr, 0xF98, 1)  # FullDump
        body = pages
    else:
        struct.pack_into("<IIQ", hdr, 0x88, 0x45474150, 0x45474150, 0x4547415045474150)
        struct.pack_into("<I", hdr, 0xF98, 5)  # BMPDump
        maxpfn = (max(pfns) + 64) & ~63
        bitmap = bytearray(maxpfn // 8)
        for p in pfns:
            bitmap[p // 8] |= 1 << (p % 8)
        bmph = bytearray(0x38)
        first_page = 0x2000 + 0x38 + len(bitmap)
        first_page = (first_page + PAGE - 1) & ~(PAGE - 1)
        struct.pack_into("<II", bmph, 0, 0x504D4446, 0x504D5544)
        struct.pack_into("<QQQ", bmph, 0x20, first_page, len(pfns), maxpfn)
        body = bytes(bmph) + bytes(bitmap)
        body += b"\x00" * (first_page - 0x2000 - len(body)) + pages
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(body)


def read_kdmp(path: str) -> tuple[dict[int, int], memoryview, int]:
    """Minimal reader: returns ({gpfn: file offset}, mapped bytes, cr3)."""
    with open(path, "rb") as f:
        data = memoryview(f.read())
    sig, valid = struct.unpack_from("<II", data, 0)
    assert sig == 0x45474150 and valid == 0x34365544, "not a 64-bit kdmp"
    cr3 = struct.unpack_from("<Q", data, 0x10)[0]
    dtype = struct.unpack_from("<I", data, 0xF98)[0]
    index = {}
    if dtype == 1:
        nruns = struct.unpack_from("<I", data, 0x88)[0]
        off = 0x2000
        for i in range(nruns):
            base, count = struct.unpack_from("<QQ", data, 0x98 + 16 * i)
            for k in range(count):
                index.setdefault(base + k, off)
                off += PAGE
    elif dtype == 5:
        first, _present, npages = struct.unpack_from("<QQQ", data, 0x2020)
        off = first
        for byte_i in range(npages // 8):
            b = data[0x2038 + byte_i]
            for bit in range(8):
                if b >> bit & 1:
                    index.setdefault(byte_i * 8 + bit, off)
                    off += PAGE
    else:
        raise ValueError(f"unsupported dump type {dtype}")
    return index, data, cr3


def write_snapshot(state_dir: str, space: AddressSpace, state: dict, symbols: dict[str, int],
                   bmp: bool | None = None) -> None:
    os.makedirs(state_dir, exist_ok=True)
    pfns, pages = space.phys()
    write_kdmp(os.path.join(state_dir, "mem.dmp"), pfns, pages, state, bmp=bmp)
    with open(os.path.join(state_dir, "regs.json"), "w") as f:
        json.dump(regs_json(state), f, indent=1)
    with open(os.path.join(state_dir, "symbol-store.json"), "w") as f:
        json.dump({k: hex(v) for k, v in symbols.items()}, f, indent=1)
