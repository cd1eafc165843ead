"""32-bit code in compatibility mode: SYSRET without REX.W
enters it, far transfers and interrupts leave it and come back. Hand-checked
oracle cases (the SDM's arithmetic for the BCD forms, stack and branch widths,
the mode switches), the engine's device code built for the host against the
oracle lane by lane, and the GPU engine against the oracle lane by lane (-m gpu).

Parity unpinned against real hardware: this container cannot execute 32-bit
code natively (no 32-bit code segment for user processes here), so the
restatement is pinned by the SDM's definitions checked below and by the
engine / oracle agreement."""
import pytest

from tests import compat32 as T
from tests import sysprog2 as S
from tests.test_sys2 import _diff, sim_lanes, sim_lib
from wtf_amd import abi
from wtf_amd.abi import regs_from_state

HLT, INT3, FAULT, UNIMPL = abi.EXIT_HLT, abi.EXIT_INT3, abi.EXIT_FAULT, abi.EXIT_UNIMPLEMENTED
M32 = 0xFFFFFFFF


@pytest.fixture(scope="module")
def space():
    return T.build_space()


def _one(space, name, flags=0x202, esp=T.ESP32, **regs):
    sp, st, lay, data = space
    g = [0] * 16
    for k, v in regs.items():
        g[abi.GPR_ORDER.index(k)] = v
    g[3], g[14], g[15] = T.SLOT32[name], esp, flags
    g[13] = regs.get("rbx", 0)
    return S.oracle_run(sp, st, [(T.KC32, g, 0x2)], limit=500)[0]


def test_sysret_enters_32_bit_code(space):
    r = _one(space, "incdec", rax=0xFFFFFFFF_00000010, rcx=0xFFFFFFFF, rsi=0, rdi=5, rbx=0x100000000)
    g = r["gpr"]
    assert r["exit"][0] == INT3 and r["exit"][4] == T.SLOT32["incdec"] + 5 and r["sel"][1] == 0x23
    # 32-bit results zero-extend (ecx held the entry point: the stub's sysret target)
    assert g[0] == 0x11 and g[1] == T.SLOT32["incdec"] + 1 and g[3] == 0xFFFFFFFF and g[6] == 0xFFFFFFFF
    assert g[7] == 6


def test_stack_and_branch_widths(space):
    r = _one(space, "pushpop", rax=0xAABBCCDD_11223344, rsi=0x77778888_99990000)
    g = r["gpr"]
    assert r["exit"][0] == INT3
    assert g[3] == 0x12345678 and g[1] == 0x11223344 and g[2] == T.ESP32  # push esp: the value before
    assert g[6] == 0x77778888_99991234 and g[4] == T.ESP32  # pop si keeps the upper bits; esp balanced
    r = _one(space, "callret")
    assert r["exit"][0] == INT3 and r["gpr"][0] == 7 and r["gpr"][4] == T.ESP32  # ret 4 releases the argument
    r = _one(space, "loop", rbx=1)
    assert r["exit"][0] == INT3 and r["gpr"][0] == 10 and r["gpr"][3] == 2
    r = _one(space, "pusha", rax=1, rbp=3, rdi=4)
    g = r["gpr"]
    assert (g[0], g[1], g[5], g[7], g[4]) == (1, T.SLOT32["pusha"], 3, 4, T.ESP32)
    r = _one(space, "enter", rbp=T.ESP32 - 0x100)  # level 2: one frame pointer copied from [ebp - 4]
    assert r["exit"][0] == INT3 and r["gpr"][5] == T.ESP32 - 0x100 and r["gpr"][4] == T.ESP32


def test_bcd_adjustments_follow_the_sdm(space):
    AF, CF = 0x10, 0x1
    r = _one(space, "bcd2", rax=0x7B)  # 0x35 + 0x46 = 0x7B -> daa -> 0x81, AF
    assert r["gpr"][0] & 0xFF == 0x81 and r["rflags"] & AF and not r["rflags"] & CF
    r = _one(space, "bcd2", rax=0x9A, flags=0x202)  # both nibbles adjust: 0x00, CF, ZF
    assert r["gpr"][0] & 0xFF == 0x00 and r["rflags"] & CF and r["rflags"] & 0x40
    r = _one(space, "aas", rax=0x0203, flags=0x202 | AF)  # AX - 6 borrows into AH, then AH - 1
    assert r["gpr"][0] & 0xFFFF == 0x000D and r["rflags"] & CF and r["rflags"] & AF
    r = _one(space, "aad7", rax=0x0305)  # 3 * 7 + 5 = 26
    assert r["gpr"][0] & 0xFFFF == 26
    r = _one(space, "aam0")
    assert r["exit"][:2] == (FAULT, 0)


def test_mode_switches(space):
    r = _one(space, "farcall")  # 32 -> 64 (call far 0x33:stub) -> retf -> 32
    assert r["exit"][0] == INT3 and r["exit"][4] == T.SLOT32["farcall"] + 7
    assert r["gpr"][9] == 0x1122334455667788 and r["sel"][1] == 0x23 and r["gpr"][4] == T.ESP32
    r = _one(space, "farjmp")
    assert r["exit"][0] == INT3 and r["gpr"][10] == 0x55 and r["sel"][1] == 0x33
    r = _one(space, "syscall", flags=0x203)  # from 32-bit code: CSTAR
    assert r["exit"][0] == HLT and r["gpr"][8] == T.SLOT32["syscall"] + 2 and r["gpr"][9] & 1
    assert r["sel"][1] == 0x10
    r = _one(space, "int29")  # a 64-bit gate: 64-bit frame on RSP0, cs 0x23 in it
    assert r["exit"][0] == HLT and r["gpr"][8] == T.SLOT32["int29"] + 2 and r["gpr"][9] == 0x23
    assert r["gpr"][11] == T.ESP32
    r = _one(space, "iretd")  # iret at the same privilege from 32-bit code: no SS:ESP
    assert r["exit"][0] == INT3 and r["gpr"][4] == T.ESP32 and r["sel"][1] == 0x23
    r = _one(space, "retf")
    assert r["exit"][0] == INT3 and r["gpr"][4] == T.ESP32


def test_outside_forms_and_ud(space):
    for n in ("a16", "jmp16"):
        assert _one(space, n, rsi=T.DATA32)["exit"][0] == UNIMPL, n
    assert _one(space, "ud2")["exit"][:2] == (FAULT, 6)


def _sx32(v):
    return v - (1 << 32) if v & 0x80000000 else v


def test_bound_arpl_les_lds_salc(space):
    """The one-byte forms only 32-bit code has (SDM BOUND, ARPL, LDS / LES,
    SALC; U29 / U30): bound faults #BR (vector 5) outside [lower, upper]
    (signed) and is a no-op inside; arpl raises the destination's RPL to the
    source's with ZF; les / lds load the offset and the selector (es / ds keep
    only the selector, U30); salc sets AL from CF."""
    sp, st, lay, data = space
    for off in (0x40, 0x60):  # random bounds (here lower > upper: always #BR), and [-5, 100]
        esi = T.DATA32 + off
        lo = _sx32(int.from_bytes(data[off:off + 4], "little"))
        hi = _sx32(int.from_bytes(data[off + 4:off + 8], "little"))
        for ix in (lo, hi, lo - 1, hi + 1, (lo + hi) // 2, -1, 0):
            if not -(1 << 31) <= ix < (1 << 31):
                continue
            want = (INT3, 0) if lo <= ix <= hi else (FAULT, 5)
            assert _one(space, "bound", rsi=esi, rax=ix & M32)["exit"][:2] == want, (ix, lo, hi)
    r = _one(space, "arpl", rax=0x10, rbx=0x3)
    assert r["exit"][0] == INT3 and r["gpr"][0] & 0xFFFF == 0x13 and r["rflags"] & 0x40
    r = _one(space, "arpl", rax=0x13, rbx=0x1)
    assert r["gpr"][0] & 0xFFFF == 0x13 and not r["rflags"] & 0x40
    for n, reg, sreg in (("les", 0, 0), ("lds", 1, 3)):
        r = _one(space, n, rsi=T.DATA32 + 0x10)
        assert r["exit"][0] == INT3, n
        assert r["gpr"][reg] == int.from_bytes(data[0x10:0x14], "little"), n
        assert r["sel"][sreg] == int.from_bytes(data[0x14:0x16], "little"), n
    r = _one(space, "salc", rax=0x12345600)
    assert r["exit"][0] == INT3 and r["gpr"][3] & 0xFF == 0xFF and r["gpr"][0] == 0x12345600


def test_vex_w1_gpr_form_is_32_bit(space):
    """BMI's VEX.W1 selects a 64-bit operand in 64-bit mode only ("the operand
    size is always 32 bits if not in 64-bit mode", SDM ANDN / RORX / ...):
    ~esi & edi with edi's upper half set is 0 at 32 bits (ZF, not SF), where a
    64-bit andn would give 0xffffffff00000000 with SF."""
    ZF, SF = 0x40, 0x80
    r = _one(space, "bmiw1", rax=0x1234, rsi=0, rdi=0xFFFFFFFF_00000000)
    assert r["exit"][0] == INT3
    assert r["gpr"][0] == 0 and r["rflags"] & ZF and not r["rflags"] & SF
    r = _one(space, "bmiw1", rsi=0x0F0F0F0F, rdi=0xFFFFFFFF_FFFFFFFF)
    assert r["gpr"][0] == 0xF0F0F0F0 and r["rflags"] & SF and not r["rflags"] & ZF


def test_engine_code_matches_oracle(space):
    sp, st, lay, data = space
    ln = T.lanes(37 * 24, 21)
    want = S.oracle_run(sp, st, ln, limit=500)
    got = sim_lanes(sim_lib(), sp, st, ln, limit=500)
    names = {v: k for k, v in T.SLOT32.items()}
    bad = []
    for i, (w, g) in enumerate(zip(want, got)):
        d = _diff(g, w)
        if d:
            bad.append((i, names[ln[i][1][3]], d, {k: (g[k], w[k]) for k in d if k not in ("pages", "xmm", "ymmh")}))
    assert not bad, f"{len(bad)}/{len(ln)} lanes differ; first: {bad[:3]}"
    kinds = {(w["exit"][0], w["exit"][1]) for w in want}
    assert {(HLT, 0), (INT3, 0), (UNIMPL, 0), (FAULT, 0), (FAULT, 6), (FAULT, 14)} <= kinds, kinds
    # most lanes run their snippet to its int3
    assert sum(w["exit"][0] == INT3 for w in want) > len(ln) // 2


@pytest.mark.gpu
def test_gpu_matches_oracle(space):
    import numpy as np
    from wtf_amd.engine import Engine

    sp, st, lay, data = space
    n = 37 * 32
    ln = T.lanes(n, 22)
    want = S.oracle_run(sp, st, ln, limit=500)
    eng = Engine(0)
    try:
        pfns, blob = sp.phys()
        eng.load_pool(pfns, blob)
        eng.alloc_lanes(n, overlay_pages=16, cov_entries=256)
        eng.set_initial_state(regs_from_state(st))
        eng.set_limit(500)
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
        assert sum(w["exit"][0] == INT3 for w in want) > n // 2
    finally:
        eng.close()


def _random_32bit_programs(n=256, seed=0x3232F):
    """progfuzz's random programs (64-bit encodings: REX bytes become inc / dec,
    imm64 tails become instructions) placed below 4 GiB and entered with CS =
    SYSRET's 32-bit selector: (space, state, lanes)."""
    import random as _r

    from tests import progfuzz as PF
    from tests.golden.gen_native_vectors import gen_forms
    from wtf_amd.tools.snapshot import AddressSpace, seg, user_state

    rng = _r.Random(seed)
    forms = gen_forms(_r.Random(seed ^ 0xABCDEF))
    sp = AddressSpace()
    code_va, win_va, stack_va = 0x10000000, 0x20000000, 0x30000000
    lanes = []
    for i in range(n):
        va = code_va + i * PF.SLOT
        code = PF.make_program(rng, forms)
        sp.map_range(va, code + b"\xcc" * (PF.SLOT - len(code)), write=False)
        g = [rng.getrandbits(32) if rng.random() < 0.7 else rng.getrandbits(64) for _ in range(16)]
        g[4] = stack_va + 0x1F00
        g[6], g[7] = win_va + rng.randrange(0x40, 0x1F00), win_va + rng.randrange(0x40, 0x1F00)
        lanes.append((va, g, 0x202 | (rng.getrandbits(12) & 0x8D5)))
    sp.map_range(win_va, bytes(rng.getrandbits(8) for _ in range(0x2000)), nx=True)
    sp.map_range(stack_va, bytes(0x2000), nx=True)
    st = user_state(code_va, stack_va + 0x1F00, sp.cr3)
    st["cs"] = seg(0x23, 0, 0xFFFFFFFF, 0xCFB)  # SYSRET's 32-bit selector (STAR[63:48] = 0x23)
    st["ss"] = seg(0x2B, 0, 0xFFFFFFFF, 0xCF3)
    return sp, st, lanes


def test_random_instruction_bytes_in_32_bit_mode_engine_equals_oracle():
    """Differential fuzz of the 32-bit decoder and executor (~100 instructions
    per lane before most end in a page fault): the engine code and the oracle
    agree lane by lane on every exit, register and page."""
    sp, st, lanes = _random_32bit_programs()
    want = S.oracle_run(sp, st, lanes, limit=2000)
    got = sim_lanes(sim_lib(), sp, st, lanes, limit=2000)
    bad = [(i, _diff(g, w)) for i, (g, w) in enumerate(zip(got, want)) if _diff(g, w)]
    assert not bad, f"{len(bad)}/{len(lanes)} lanes differ; first: {bad[:3]}"
    kinds = {(w["exit"][0], w["exit"][1]) for w in want}
    assert len(kinds) >= 4, kinds
    assert sum(w["exit"][5] for w in want) > 50 * len(lanes)


@pytest.mark.gpu
def test_gpu_random_instruction_bytes_in_32_bit_mode():
    import numpy as np
    from wtf_amd.engine import Engine

    sp, st, lanes = _random_32bit_programs(1024, 0x3232E)
    n = len(lanes)
    want = S.oracle_run(sp, st, lanes, limit=2000)
    eng = Engine(0)
    try:
        pfns, blob = sp.phys()
        eng.load_pool(pfns, blob)
        eng.alloc_lanes(n, overlay_pages=16, cov_entries=1024)
        eng.set_initial_state(regs_from_state(st))
        eng.set_limit(2000)
        eng.restore()
        g = eng.read_gprs()
        for i, (va, regs, flags) in enumerate(lanes):
            g[i, :16] = np.array(regs, dtype=np.uint64)
            g[i, 16], g[i, 17] = va, flags
        eng.write_gprs(g)
        eng.run()
        ex = eng.exits()
        out = eng.read_regs(0, n)
        nb = eng.nbytes()
        bad = []
        for i, w in enumerate(want):
            e = ex[i]
            pg = {gpa: eng.read_phys(i, gpa, 4096) for gpa in eng.dirty(i)}
            got = S.lane_view(e.status, e.vector, e.error, e.addr, e.icount, int(nb[i]), out[i], pg)
            d = _diff(got, w)
            if d:
                bad.append((i, d))
        assert not bad, f"{len(bad)}/{n} lanes differ; first: {bad[:3]}"
    finally:
        eng.close()
