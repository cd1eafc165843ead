"""Python handle on the HIP engine (libwtfgpu.so) through its C ABI.

Used by tests and bench.py to drive lanes directly; the C++ GpuBackend_t
(wtf_amd/host) is the drop-in for wtf's Backend_t. Every call goes to the HIP
library; a missing library or device raises instead of falling back.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class EngineError(RuntimeError):
    pass


def _chk(rc, what):
    if rc != 0:
        raise EngineError(f"{what} failed: {rc}")


class Engine:
    def __init__(self, device: int = 0):
        self.L = abi.load_hip_library()
        ctx = C.c_void_p()
        _chk(self.L.wtfgpu_create(device, C.byref(ctx)), "wtfgpu_create")
        self.ctx = ctx
        self.nlanes = 0

    def close(self):
        if self.ctx:
            self.L.wtfgpu_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- setup
    def load_pool(self, pfns, blob: bytes):
        arr = (C.c_uint64 * max(1, len(pfns)))(*pfns)
        _chk(self.L.wtfgpu_load_pool(self.ctx, arr, blob, len(pfns)), "load_pool")

    def alloc_lanes(self, n, overlay_pages=16, cov_entries=1024):
        _chk(self.L.wtfgpu_alloc_lanes(self.ctx, n, overlay_pages, cov_entries), "alloc_lanes")
        self.nlanes = n

    def set_initial_state(self, regs: abi.Regs):
        _chk(self.L.wtfgpu_set_initial_state(self.ctx, C.byref(regs)), "set_initial_state")

    def set_limit(self, n):
        _chk(self.L.wtfgpu_set_limit(self.ctx, n), "set_limit")

    def set_breakpoints(self, gvas):
        arr = (C.c_uint64 * max(1, len(gvas)))(*gvas)
        _chk(self.L.wtfgpu_set_breakpoints(self.ctx, arr, len(gvas)), "set_breakpoints")

    def set_edges(self, on: bool):
        _chk(self.L.wtfgpu_set_edges(self.ctx, 1 if on else 0), "set_edges")

    def set_code_pages(self, vpns):
        arr = (C.c_uint64 * max(1, len(vpns)))(*vpns)
        _chk(self.L.wtfgpu_set_code_pages(self.ctx, arr, len(vpns)), "set_code_pages")

    def restore(self, first=0, count=None):
        count = self.nlanes - first if count is None else count
        _chk(self.L.wtfgpu_restore(self.ctx, first, count), "restore")

    # ---- registers
    def read_gprs(self, first=0, count=None) -> np.ndarray:
        count = self.nlanes - first if count is None else count
        out = np.zeros((count, 18), dtype=np.uint64)
        _chk(self.L.wtfgpu_read_gprs(self.ctx, first, count, out.ctypes.data_as(C.POINTER(C.c_uint64))),
             "read_gprs")
        return out

    def write_gprs(self, g: np.ndarray, first=0):
        g = np.ascontiguousarray(g, dtype=np.uint64)
        _chk(self.L.wtfgpu_write_gprs(self.ctx, first, g.shape[0], g.ctypes.data_as(C.POINTER(C.c_uint64))),
             "write_gprs")

    def read_regs(self, first=0, count=1):
        arr = (abi.Regs * count)()
        _chk(self.L.wtfgpu_read_regs(self.ctx, first, count, arr), "read_regs")
        return list(arr)

    def write_regs(self, regs, first=0):
        arr = (abi.Regs * len(regs))(*regs)
        _chk(self.L.wtfgpu_write_regs(self.ctx, first, len(regs), arr), "write_regs")

    # ---- run
    def run(self, first=0, count=None, max_steps=1 << 40) -> abi.RunStats:
        count = self.nlanes - first if count is None else count
        st = abi.RunStats()
        _chk(self.L.wtfgpu_run(self.ctx, first, count, max_steps, C.byref(st)), "run")
        return st

    def exits(self, first=0, count=None):
        count = self.nlanes - first if count is None else count
        arr = (abi.Exit * count)()
        _chk(self.L.wtfgpu_read_exits(self.ctx, first, count, arr), "read_exits")
        return list(arr)

    EXIT_DTYPE = np.dtype([("status", "<u4"), ("vector", "<u4"), ("error", "<u4"), ("opcode", "<u4"),
                           ("addr", "<u8"), ("rip", "<u8"), ("icount", "<u8")])

    def exits_np(self, first=0, count=None) -> np.ndarray:
        """read_exits as a numpy structured array (one record per lane)."""
        count = self.nlanes - first if count is None else count
        out = np.zeros(count, dtype=self.EXIT_DTYPE)
        assert out.itemsize == C.sizeof(abi.Exit)
        _chk(self.L.wtfgpu_read_exits(self.ctx, first, count, out.ctypes.data_as(C.POINTER(abi.Exit))),
             "read_exits")
        return out

    def resume(self, lanes, skip):
        n = len(lanes)
        la = (C.c_uint32 * max(1, n))(*lanes)
        sk = (C.c_uint8 * max(1, n))(*[1 if s else 0 for s in skip])
        _chk(self.L.wtfgpu_resume(self.ctx, la, n, sk), "resume")

    def inject_fault(self, lanes, vector, error, addrs) -> list[bool]:
        n = len(lanes)
        la = (C.c_uint32 * max(1, n))(*lanes)
        aa = (C.c_uint64 * max(1, n))(*addrs)
        ok = (C.c_int32 * max(1, n))()
        _chk(self.L.wtfgpu_inject_fault(self.ctx, la, n, vector, error, aa, ok), "inject_fault")
        return [bool(ok[i]) for i in range(n)]

    def stop(self, lanes, status=abi.EXIT_STOPPED):
        n = len(lanes)
        la = (C.c_uint32 * max(1, n))(*lanes)
        _chk(self.L.wtfgpu_stop(self.ctx, la, n, status), "stop")

    # ---- memory
    def apply_writes(self, writes):
        """writes: list of (lane, gva, bytes)."""
        if not writes:
            return
        recs = (abi.Write * len(writes))()
        blob = bytearray()
        for i, (lane, gva, data) in enumerate(writes):
            recs[i].lane, recs[i].len, recs[i].gva, recs[i].data_off = lane, len(data), gva, len(blob)
            blob += data
        st = (C.c_int32 * len(writes))()
        _chk(self.L.wtfgpu_apply_writes(self.ctx, recs, len(writes), bytes(blob), len(blob), st), "apply_writes")

    def read_virt(self, lane, gva, n) -> bytes:
        b = C.create_string_buffer(n)
        _chk(self.L.wtfgpu_lane_read_virt(self.ctx, lane, gva, b, n), "read_virt")
        return b.raw

    def write_virt(self, lane, gva, data: bytes):
        _chk(self.L.wtfgpu_lane_write_virt(self.ctx, lane, gva, data, len(data)), "write_virt")

    def read_phys(self, lane, gpa, n) -> bytes:
        b = C.create_string_buffer(n)
        _chk(self.L.wtfgpu_lane_read_phys(self.ctx, lane, gpa, b, n), "read_phys")
        return b.raw

    def translate(self, lane, gva):
        out = C.c_uint64()
        rc = self.L.wtfgpu_lane_translate(self.ctx, lane, gva, C.byref(out))
        return None if rc else out.value

    def dirty(self, lane) -> list[int]:
        n = C.c_uint32()
        cap = 4096
        arr = (C.c_uint64 * cap)()
        _chk(self.L.wtfgpu_read_dirty(self.ctx, lane, arr, cap, C.byref(n)), "read_dirty")
        return list(arr[: min(n.value, cap)])

    def coverage(self, first=0, count=None, cap=None):
        """{lane: set(rips)} of rips absent from the coverage map when executed
        (a first call sizes the buffers: after warm-up the log is usually empty)."""
        count = self.nlanes - first if count is None else count
        n = C.c_uint64()
        ovf = C.c_uint32()
        dummy_l, dummy_r = (C.c_uint32 * 1)(), (C.c_uint64 * 1)()
        _chk(self.L.wtfgpu_read_coverage(self.ctx, first, count, dummy_l, dummy_r, 0, C.byref(n), C.byref(ovf)),
             "read_coverage")
        out: dict[int, set] = {}
        total = n.value
        if total:
            lanes = np.zeros(total, dtype=np.uint32)
            rips = np.zeros(total, dtype=np.uint64)
            _chk(self.L.wtfgpu_read_coverage(self.ctx, first, count, lanes.ctypes.data_as(C.POINTER(C.c_uint32)),
                                             rips.ctypes.data_as(C.POINTER(C.c_uint64)), total, C.byref(n),
                                             C.byref(ovf)), "read_coverage")
            for ln, rp in zip(lanes.tolist(), rips.tolist()):
                out.setdefault(ln, set()).add(rp)
        return out, bool(ovf.value)

    def commit_coverage(self, rips):
        arr = np.ascontiguousarray(np.array(sorted(rips), dtype=np.uint64))
        _chk(self.L.wtfgpu_commit_coverage(self.ctx, arr.ctypes.data_as(C.POINTER(C.c_uint64)), len(arr)),
             "commit_coverage")

    def nbytes(self, first=0, count=None) -> np.ndarray:
        count = self.nlanes - first if count is None else count
        out = np.zeros(count, dtype=np.uint64)
        _chk(self.L.wtfgpu_read_bytes(self.ctx, first, count, out.ctypes.data_as(C.POINTER(C.c_uint64))),
             "read_bytes")
        return out

    def dirty_counts(self, first=0, count=None) -> np.ndarray:
        count = self.nlanes - first if count is None else count
        out = np.zeros(count, dtype=np.uint32)
        _chk(self.L.wtfgpu_read_dirty_counts(self.ctx, first, count, out.ctypes.data_as(C.POINTER(C.c_uint32))),
             "read_dirty_counts")
        return out

    def gather_pages(self, lanes, gpas) -> np.ndarray:
        """[n, 4096] u8: each lane's current view of each guest-physical page."""
        lanes = np.ascontiguousarray(lanes, dtype=np.uint32)
        gpas = np.ascontiguousarray(gpas, dtype=np.uint64)
        out = np.zeros((len(lanes), 4096), dtype=np.uint8)
        _chk(self.L.wtfgpu_gather_pages(self.ctx, lanes.ctypes.data_as(C.POINTER(C.c_uint32)),
                                        gpas.ctypes.data_as(C.POINTER(C.c_uint64)), len(lanes),
                                        out.ctypes.data_as(C.c_void_p)), "gather_pages")
        return out

    def get_cr(self, lane, cr) -> int:
        out = C.c_uint64()
        _chk(self.L.wtfgpu_lane_get_cr(self.ctx, lane, cr, C.byref(out)), "lane_get_cr")
        return out.value

    def set_cr(self, lane, cr, value):
        _chk(self.L.wtfgpu_lane_set_cr(self.ctx, lane, cr, value), "lane_set_cr")
