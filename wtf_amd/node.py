"""ctypes handle on libwtfnode.so (include/wtfnode.h): one fuzzing node on one
GPU, stepped one batch at a time. bench.py drives the headline workload with
it; the product node is the same C++ (`wtfgpu fuzz`). A missing library
raises: there is no Python or CPU fallback."""
from __future__ import annotations

import ctypes as C
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "wtf_amd", "host", "libwtfnode.so")
RCCL_ID_BYTES = 128


class Opts(C.Structure):
    _fields_ = [("name", C.c_char_p), ("target", C.c_char_p), ("lanes", C.c_uint32), ("overlay_pages", C.c_uint32),
                ("limit", C.c_uint64), ("seed", C.c_uint64), ("max_len", C.c_uint64), ("device", C.c_int32),
                ("rank", C.c_int32), ("world", C.c_int32), ("rccl_id", C.POINTER(C.c_uint8)),
                ("slice_steps", C.c_uint64), ("regroup_steps", C.c_uint64)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "execs", "retired", "batches", "crashes", "unique_crashes", "timeouts", "cr3", "errors",
        "coverage", "corpus", "merged_rips", "kernel_launches", "group_steps", "alg_bytes",
        "breakpoint_hits", "rounds", "error_retired")] + [(n, C.c_double) for n in (
        "run_s", "kernel_ms", "merge_ms", "insert_ms", "coverage_ms", "service_ms", "total_ms")]

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"node library missing: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.wtfnode_rccl_unique_id.argtypes = [C.POINTER(C.c_uint8)]
        L.wtfnode_open.argtypes = [C.POINTER(Opts), C.POINTER(P)]
        L.wtfnode_step.argtypes = [P]
        L.wtfnode_stats.argtypes = [P, C.POINTER(Stats)]
        L.wtfnode_summary_json.argtypes = [P, C.c_char_p, C.c_uint64]
        L.wtfnode_close.argtypes = [P]
        for f in ("wtfnode_rccl_unique_id", "wtfnode_open", "wtfnode_step", "wtfnode_stats",
                  "wtfnode_summary_json", "wtfnode_close"):
            getattr(L, f).restype = C.c_int
        _lib = L
    return _lib


def rccl_unique_id() -> bytes:
    buf = (C.c_uint8 * RCCL_ID_BYTES)()
    if lib().wtfnode_rccl_unique_id(buf) != 0:
        raise RuntimeError("ncclGetUniqueId failed")
    return bytes(buf)


class Node:
    def __init__(self, name: str, target: str, lanes: int, limit: int, seed: int = 1337, max_len: int = 0x1000,
                 device: int = 0, rank: int = 0, world: int = 1, rccl_id: bytes | None = None,
                 overlay_pages: int = 0, slice_steps: int = 0, regroup_steps: int | None = None):
        self.L = lib()
        self._id = (C.c_uint8 * RCCL_ID_BYTES)(*rccl_id) if rccl_id else None
        o = Opts(name.encode(), target.encode(), lanes, overlay_pages, limit, seed, max_len, device, rank, world,
                 C.cast(self._id, C.POINTER(C.c_uint8)) if self._id is not None else None,
                 slice_steps, (1 << 64) - 1 if regroup_steps is None else regroup_steps)
        h = C.c_void_p()
        rc = self.L.wtfnode_open(C.byref(o), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"wtfnode_open({name}, {target}) failed: {rc}")
        self.h = h

    def step(self):
        rc = self.L.wtfnode_step(self.h)
        if rc != 0:
            raise RuntimeError(f"wtfnode_step failed: {rc}")

    def stats(self) -> dict:
        s = Stats()
        self.L.wtfnode_stats(self.h, C.byref(s))
        return s.as_dict()

    def summary(self) -> dict:
        buf = C.create_string_buffer(1 << 16)
        self.L.wtfnode_summary_json(self.h, buf, len(buf))
        return json.loads(buf.value.decode())

    def close(self):
        if getattr(self, "h", None):
            self.L.wtfnode_close(self.h)
            self.h = None
