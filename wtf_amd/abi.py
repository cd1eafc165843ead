"""ctypes view of the C ABI in include/wtfgpu.h (struct layouts + library loader).

The product path is the HIP library `wtf_amd/csrc/libwtfgpu.so`. Loading fails
loudly when it is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WTFGPU_LIB") or os.path.join(HERE, "csrc", "libwtfgpu.so")
HOST_LIB_PATH = os.path.join(HERE, "host", "libwtf_host.so")

RUNNING, EXIT_BREAKPOINT, EXIT_TIMEOUT, EXIT_INT3, EXIT_HLT, EXIT_FAULT, EXIT_UNIMPLEMENTED, \
    EXIT_CR3, EXIT_OVERLAY_FULL, EXIT_STOPPED, EXIT_IDLE, EXIT_STOP_OK, EXIT_FEED_FAULT, EXIT_STOP_ARGS = range(14)
STATUS_NAMES = ["running", "breakpoint", "timeout", "int3", "hlt", "fault", "unimplemented",
                "cr3", "overlay_full", "stopped", "idle", "stop_ok", "feed_fault"]


class Seg(C.Structure):
    _fields_ = [("base", C.c_uint64), ("limit", C.c_uint32), ("selector", C.c_uint16),
                ("attr", C.c_uint16), ("present", C.c_uint8), ("pad", C.c_uint8 * 7)]


class Regs(C.Structure):
    _fields_ = [
        ("gpr", C.c_uint64 * 16), ("rip", C.c_uint64), ("rflags", C.c_uint64),
        ("cr0", C.c_uint64), ("cr2", C.c_uint64), ("cr3", C.c_uint64), ("cr4", C.c_uint64),
        ("cr8", C.c_uint64), ("efer", C.c_uint64), ("xcr0", C.c_uint64),
        ("kernel_gs_base", C.c_uint64), ("star", C.c_uint64), ("lstar", C.c_uint64),
        ("cstar", C.c_uint64), ("sfmask", C.c_uint64), ("tsc", C.c_uint64), ("tsc_aux", C.c_uint64),
        ("apic_base", C.c_uint64), ("pat", C.c_uint64), ("sysenter_cs", C.c_uint64),
        ("sysenter_eip", C.c_uint64), ("sysenter_esp", C.c_uint64), ("seg", Seg * 8),
        ("gdtr_base", C.c_uint64), ("idtr_base", C.c_uint64), ("gdtr_limit", C.c_uint32),
        ("idtr_limit", C.c_uint32), ("mxcsr", C.c_uint32), ("mxcsr_mask", C.c_uint32),
        ("fpcw", C.c_uint16), ("fpsw", C.c_uint16), ("fptw", C.c_uint16), ("fpop", C.c_uint16),
        ("pad0", C.c_uint32), ("fpst", C.c_uint64 * 8), ("xmm", (C.c_uint64 * 2) * 16),
        ("ymmh", (C.c_uint64 * 2) * 16), ("fpse", C.c_uint16 * 8),
        ("zmmh", (C.c_uint64 * 4) * 16), ("zmm_hi", (C.c_uint64 * 8) * 16), ("k", C.c_uint64 * 8),
    ]


class Exit(C.Structure):
    _fields_ = [("status", C.c_uint32), ("vector", C.c_uint32), ("error", C.c_uint32),
                ("opcode", C.c_uint32), ("addr", C.c_uint64), ("rip", C.c_uint64),
                ("icount", C.c_uint64)]

    def tuple(self):
        return (self.status, self.vector, self.error, self.addr, self.rip, self.icount)


class RunStats(C.Structure):
    _fields_ = [("kernel_launches", C.c_uint64), ("group_steps", C.c_uint64),
                ("lane_retired", C.c_uint64), ("kernel_ms", C.c_double)]


class BpAction(C.Structure):
    """wtfgpu_bp_action_t: a breakpoint handler's device-side register effect."""
    _fields_ = [("gva", C.c_uint64), ("kind", C.c_uint32), ("pad", C.c_uint32),
                ("value", C.c_uint64), ("gprs", C.c_uint64 * 17)]


BPACT_HOST, BPACT_RETURN, BPACT_SET_GPRS, BPACT_FEED = 0, 1, 2, 3


class Write(C.Structure):
    _fields_ = [("lane", C.c_uint32), ("len", C.c_uint32), ("gva", C.c_uint64),
                ("data_off", C.c_uint64)]


SEG_ORDER = ["es", "cs", "ss", "ds", "fs", "gs", "tr", "ldtr"]
GPR_ORDER = ["rax", "rcx", "rdx", "rbx", "rsp", "rbp", "rsi", "rdi",
             "r8", "r9", "r10", "r11", "r12", "r13", "r14", "r15"]


def regs_from_state(st: dict) -> Regs:
    """Build a Regs from a snapshot state dict (wtf_amd.tools.snapshot.user_state)."""
    r = Regs()
    for i, g in enumerate(GPR_ORDER):
        r.gpr[i] = st.get(g, 0)
    r.rip, r.rflags = st["rip"], st["rflags"]
    for k in ("cr0", "cr2", "cr3", "cr4", "cr8", "efer", "xcr0", "kernel_gs_base", "star", "lstar",
              "cstar", "sfmask", "tsc", "tsc_aux", "apic_base", "pat", "sysenter_cs",
              "sysenter_eip", "sysenter_esp", "mxcsr", "mxcsr_mask", "fpcw", "fpsw", "fptw", "fpop"):
        if k in st:
            setattr(r, k, st[k])
    for i, s in enumerate(SEG_ORDER):
        if s in st:
            v = st[s]
            r.seg[i].base, r.seg[i].limit = v["base"], v["limit"]
            r.seg[i].selector, r.seg[i].attr, r.seg[i].present = v["selector"], v["attr"], int(v["present"])
    if "gdtr" in st:
        r.gdtr_base, r.gdtr_limit = st["gdtr"]["base"], st["gdtr"]["limit"]
    if "idtr" in st:
        r.idtr_base, r.idtr_limit = st["idtr"]["base"], st["idtr"]["limit"]
    return r


def load_hip_library(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise RuntimeError(f"HIP extension missing: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    P, U32, U64, I32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "wtfgpu_abi_version": ([], C.c_int),
        "wtfgpu_device_count": ([], C.c_int),
        "wtfgpu_create": ([C.c_int, C.POINTER(P)], C.c_int),
        "wtfgpu_destroy": ([P], C.c_int),
        "wtfgpu_stream": ([P], P),
        "wtfgpu_load_pool": ([P, C.POINTER(U64), C.c_char_p, U64], C.c_int),
        "wtfgpu_alloc_lanes": ([P, U32, U32, U32], C.c_int),
        "wtfgpu_lane_count": ([P], U32),
        "wtfgpu_set_initial_state": ([P, C.POINTER(Regs)], C.c_int),
        "wtfgpu_set_limit": ([P, U64], C.c_int),
        "wtfgpu_set_regroup": ([P, U64], C.c_int),
        "wtfgpu_set_edges": ([P, C.c_int], C.c_int),
        "wtfgpu_set_trace": ([P, U32], C.c_int),
        "wtfgpu_read_trace": ([P, U32, C.POINTER(U64), U64, C.POINTER(U64)], C.c_int),
        "wtfgpu_read_stop_args": ([P, C.POINTER(U32), U32, C.POINTER(U64)], C.c_int),
        "wtfgpu_select_queue": ([P, U32], C.c_int),
        "wtfgpu_lane_seeds": ([P, C.POINTER(U32), U32, C.POINTER(U64), C.c_int], C.c_int),
        "wtfgpu_run_async": ([P, U32, U32, U64], C.c_int),
        "wtfgpu_run_wait": ([P, C.POINTER(RunStats)], C.c_int),
        "wtfgpu_prefetch_results": ([P, U32, U32, C.POINTER(Exit), C.POINTER(U64), C.POINTER(U32), C.POINTER(U64)],
                                    C.c_int),
        "wtfgpu_prefetch_coverage": ([P, U32, U32, C.POINTER(U64)], C.c_int),
        "wtfgpu_prefetched_coverage": ([P, C.POINTER(U32), C.POINTER(U64), U64], C.c_int),
        "wtfgpu_clear_coverage_lanes": ([P, C.POINTER(U32), U32], C.c_int),
        "wtfgpu_set_breakpoints": ([P, C.POINTER(U64), U32], C.c_int),
        "wtfgpu_set_breakpoint_actions": ([P, C.POINTER(BpAction), U32], C.c_int),
        "wtfgpu_set_feed": ([P, U32, U32, C.POINTER(U64), C.c_char_p, C.c_char_p, U64], C.c_int),
        "wtfgpu_set_code_pages": ([P, C.POINTER(U64), U32], C.c_int),
        "wtfgpu_restore": ([P, U32, U32], C.c_int),
        "wtfgpu_read_regs": ([P, U32, U32, C.POINTER(Regs)], C.c_int),
        "wtfgpu_write_regs": ([P, U32, U32, C.POINTER(Regs)], C.c_int),
        "wtfgpu_read_gprs": ([P, U32, U32, C.POINTER(U64)], C.c_int),
        "wtfgpu_write_gprs": ([P, U32, U32, C.POINTER(U64)], C.c_int),
        "wtfgpu_read_exits": ([P, U32, U32, C.POINTER(Exit)], C.c_int),
        "wtfgpu_resume": ([P, C.POINTER(U32), U32, C.POINTER(C.c_uint8)], C.c_int),
        "wtfgpu_inject_fault": ([P, C.POINTER(U32), U32, U32, U32, C.POINTER(U64), C.POINTER(C.c_int32)], C.c_int),
        "wtfgpu_stop": ([P, C.POINTER(U32), U32, U32], C.c_int),
        "wtfgpu_run": ([P, U32, U32, U64, C.POINTER(RunStats)], C.c_int),
        "wtfgpu_lane_translate": ([P, U32, U64, C.POINTER(U64)], C.c_int),
        "wtfgpu_lane_read_phys": ([P, U32, U64, P, U64], C.c_int),
        "wtfgpu_lane_write_phys": ([P, U32, U64, P, U64], C.c_int),
        "wtfgpu_lane_read_virt": ([P, U32, U64, P, U64], C.c_int),
        "wtfgpu_lane_write_virt": ([P, U32, U64, P, U64], C.c_int),
        "wtfgpu_apply_writes": ([P, C.POINTER(Write), U32, C.c_char_p, U64, C.POINTER(I32)], C.c_int),
        "wtfgpu_read_dirty": ([P, U32, C.POINTER(U64), U32, C.POINTER(U32)], C.c_int),
        "wtfgpu_read_coverage": ([P, U32, U32, C.POINTER(U32), C.POINTER(U64), U64, C.POINTER(U64),
                                  C.POINTER(U32)], C.c_int),
        "wtfgpu_commit_coverage": ([P, C.POINTER(U64), U64], C.c_int),
        "wtfgpu_reset_coverage": ([P], C.c_int),
        "wtfgpu_coverage_device_map": ([P, C.POINTER(P), C.POINTER(U64)], C.c_int),
        "wtfgpu_coverage_rips": ([P, C.POINTER(U64), U64, C.POINTER(U64)], C.c_int),
        "wtfgpu_read_bytes": ([P, U32, U32, C.POINTER(U64)], C.c_int),
        "wtfgpu_read_dirty_counts": ([P, U32, U32, C.POINTER(U32)], C.c_int),
        "wtfgpu_gather_pages": ([P, C.POINTER(U32), C.POINTER(U64), U32, P], C.c_int),
        "wtfgpu_lane_get_cr": ([P, U32, U32, C.POINTER(U64)], C.c_int),
        "wtfgpu_lane_set_cr": ([P, U32, U32, U64], C.c_int),
        "wtfgpu_coverage_absorb": ([P, C.POINTER(U64), U64, C.POINTER(U64)], C.c_int),
    }
    for name, (args, ret) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ret
    return lib


def exported_symbols_from_header(header: str) -> list[str]:
    import re
    text = open(header).read()
    return sorted(set(re.findall(r"\b(wtfgpu_[a-z_0-9]+)\s*\(", text)))
