"""ctypes wrapper of the CPU oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

from wtf_amd.abi import Exit, Regs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from tests.cpu_bins import ALT, ORACLE_SO  # noqa: E402

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not ALT and not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])
    L = C.CDLL(ORACLE_SO)
    P, U32, U64 = C.c_void_p, C.c_uint32, C.c_uint64
    sig = {
        "orc_create": ([], P), "orc_destroy": ([P], None),
        "orc_add_page": ([P, U64, C.c_char_p], C.c_int),
        "orc_set_regs": ([P, C.POINTER(Regs)], None), "orc_get_regs": ([P, C.POINTER(Regs)], None),
        "orc_set_limit": ([P, U64], None), "orc_set_edges": ([P, C.c_int], None),
        "orc_set_breakpoints": ([P, C.POINTER(U64), U32], C.c_int),
        "orc_restore": ([P, C.POINTER(Regs)], None),
        "orc_run": ([P, C.c_int, C.POINTER(Exit)], C.c_int),
        "orc_step": ([P, C.POINTER(Exit)], C.c_int),
        "orc_icount": ([P], U64), "orc_bytes": ([P], U64),
        "orc_coverage": ([P, C.POINTER(U64), U64], U64),
        "orc_dirty": ([P, C.POINTER(U64), U64], U64),
        "orc_translate": ([P, U64, C.POINTER(U64)], C.c_int),
        "orc_read_phys": ([P, U64, P, U64], C.c_int),
        "orc_write_phys": ([P, U64, P, U64], C.c_int),
        "orc_read_virt": ([P, U64, P, U64], C.c_int),
        "orc_write_virt": ([P, U64, P, U64], C.c_int),
        "orc_inject_fault": ([P, U32, U32, U64], C.c_int),
        "orc_set_tenet": ([P, C.c_int], None), "orc_tenet_event": ([P], None),
        "orc_tenet": ([P, C.POINTER(U64), U64], U64),
    }
    for n, (a, r) in sig.items():
        f = getattr(L, n)
        f.argtypes, f.restype = a, r
    _lib = L
    return L


class Oracle:
    """One oracle lane over a set of physical pages."""

    def __init__(self, pages: dict[int, bytes] | None = None, pfns=None, blob: bytes | None = None):
        self.L = lib()
        self.m = self.L.orc_create()
        if pages:
            for pfn, data in pages.items():
                self.L.orc_add_page(self.m, pfn, bytes(data))
        if pfns is not None:
            for i, pfn in enumerate(pfns):
                self.L.orc_add_page(self.m, pfn, blob[i * 4096:(i + 1) * 4096])

    def __del__(self):
        try:
            self.L.orc_destroy(self.m)
        except Exception:
            pass

    def restore(self, regs: Regs):
        self.L.orc_restore(self.m, C.byref(regs))

    def set_regs(self, regs: Regs):
        self.L.orc_set_regs(self.m, C.byref(regs))

    def regs(self) -> Regs:
        r = Regs()
        self.L.orc_get_regs(self.m, C.byref(r))
        return r

    def set_edges(self, on: bool):
        self.L.orc_set_edges(self.m, 1 if on else 0)

    def set_limit(self, n):
        self.L.orc_set_limit(self.m, n)

    def set_breakpoints(self, gvas):
        arr = (C.c_uint64 * max(1, len(gvas)))(*gvas)
        self.L.orc_set_breakpoints(self.m, arr, len(gvas))

    def run(self, skip_bp=False) -> Exit:
        e = Exit()
        self.L.orc_run(self.m, int(skip_bp), C.byref(e))
        return e

    def step(self) -> Exit:
        e = Exit()
        self.L.orc_step(self.m, C.byref(e))
        return e

    def set_tenet(self, on: bool):
        self.L.orc_set_tenet(self.m, 1 if on else 0)

    def tenet(self) -> bytes:
        """The Tenet stream (U38) as bytes."""
        n = self.L.orc_tenet(self.m, None, 0)
        arr = (C.c_uint64 * max(1, n))()
        self.L.orc_tenet(self.m, arr, n)
        return bytes(arr)[:8 * n]

    def icount(self):
        return self.L.orc_icount(self.m)

    def nbytes(self):
        return self.L.orc_bytes(self.m)

    def coverage(self) -> list[int]:
        n = self.L.orc_coverage(self.m, None, 0)
        arr = (C.c_uint64 * max(1, n))()
        self.L.orc_coverage(self.m, arr, n)
        return list(arr[:n])

    def dirty(self) -> list[int]:
        n = self.L.orc_dirty(self.m, None, 0)
        arr = (C.c_uint64 * max(1, n))()
        self.L.orc_dirty(self.m, arr, n)
        return list(arr[:n])

    def read_virt(self, gva, n) -> bytes:
        b = C.create_string_buffer(n)
        if self.L.orc_read_virt(self.m, gva, b, n):
            raise ValueError(f"translate failed {gva:#x}")
        return b.raw

    def write_virt(self, gva, data: bytes):
        if self.L.orc_write_virt(self.m, gva, data, len(data)):
            raise ValueError(f"translate failed {gva:#x}")

    def read_phys(self, gpa, n) -> bytes:
        b = C.create_string_buffer(n)
        self.L.orc_read_phys(self.m, gpa, b, n)
        return b.raw

    def inject_fault(self, vector, error, addr) -> bool:
        return bool(self.L.orc_inject_fault(self.m, vector, error, addr))

    def translate(self, gva):
        out = C.c_uint64()
        if self.L.orc_translate(self.m, gva, C.byref(out)):
            return None
        return out.value
