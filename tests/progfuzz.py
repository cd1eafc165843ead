"""Random x86-64 programs for GPU-vs-oracle differential tests.

A program is a chain of blocks; each block re-establishes the pointer
registers its instruction form needs (mov r64, imm64 into a data window) and
then runs one random form drawn from the native-vector generator's encodings
(tests/golden/gen_native_vectors.py). Some blocks are guarded by a forward
conditional jump, some jump backwards through a counted loop. Programs end in
int3. Faults (#DE, #PF on a read-only page, ...) end a lane early; both
engines must agree on that too. With sse=True the SSE / SSE2 forms of
tests/golden/gen_sse_vectors.py join the pool (aligned forms sometimes get a
misaligned window: #GP) and every lane starts from its own XMM registers.
"""
from __future__ import annotations

import random

from tests.golden.gen_native_vectors import RCX, RDI, RSI, RSP, gen_forms
from wtf_amd.abi import regs_from_state
from wtf_amd.tools.snapshot import AddressSpace, user_state

CODE_VA = 0x100000000
SLOT = 0x2000
WIN_VA = 0x200000000     # two RW pages
RO_VA = 0x200002000      # one read-only page right after (writes fault)
STACK_VA = 0x300000000   # two pages
STACK_TOP = STACK_VA + 0x2000 - 0x100


def mov_imm64(r, v):
    return bytes([0x48 | (r >> 3), 0xB8 + (r & 7)]) + (v & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")


def make_program(rng: random.Random, forms, n_blocks=24) -> bytes:
    code = bytearray()
    for _ in range(n_blocks):
        f = rng.choice(forms)
        if f.cls == "div" and rng.random() < 0.7:
            continue
        setup = bytearray()
        base = WIN_VA + rng.choice([0x100, 0x800, 0xF00, 0xFF8 - 0x80])
        for r, off in f.ptrs.items():
            setup += mov_imm64(r, base + off)
        for r, (lo, hi) in f.smalls.items():
            setup += mov_imm64(r, rng.randint(lo, hi))
        if f.cls == "string":
            setup += mov_imm64(RSI, WIN_VA + rng.randrange(0x40, 0x1F00))
            setup += mov_imm64(RDI, rng.choice([WIN_VA + rng.randrange(0x40, 0x1F00), RO_VA - 4]))
            setup += mov_imm64(RCX, rng.randrange(0, 12))
        if f.cls in ("stack", "popf"):
            setup += mov_imm64(RSP, STACK_TOP - rng.randrange(0, 32) * 8)
        block = bytes(setup) + f.code
        r = rng.random()
        if r < 0.15 and len(block) < 120:
            code += bytes([0x70 + rng.randrange(16), len(block)])  # jcc over the block
        elif r < 0.2 and len(block) < 100:
            # a short counted loop around the block: mov ecx, k ; block ; dec ecx ; jnz
            k = rng.randrange(1, 4)
            code += bytes([0xB9]) + k.to_bytes(4, "little")
            body = block + bytes([0xFF, 0xC9])
            code += body + bytes([0x75, (-(len(body) + 2)) & 0xFF])
            continue
        code += block
        if len(code) > SLOT - 64:
            break
    code += b"\xcc"
    return bytes(code[:SLOT])


def build(n_programs: int, seed: int, sse: bool = False, fp: bool = False):
    """Returns (AddressSpace, base state, list of (code_va, regs dict)). fp:
    the SSE / AVX floating-point (U39 / U40) and SSE4 / AVX2 (U41) forms join
    the SSE pool."""
    rng = random.Random(seed)
    forms = gen_forms(random.Random(seed ^ 0xABCDEF))
    if fp:
        from tests.golden.gen_fp_vectors import gen_forms as gen_fp_forms
        from tests.golden.gen_sse4_vectors import gen_forms as gen_sse4_forms

        forms = forms + (gen_fp_forms(random.Random(seed ^ 0xF9)) + gen_sse4_forms(random.Random(seed ^ 0x54))) * 2
    if sse:
        from tests.golden.gen_sse_vectors import gen_forms as gen_sse_forms

        from tests.golden.gen_avx_vectors import gen_forms as gen_avx_forms

        sse_forms = gen_sse_forms(random.Random(seed ^ 0x55E)) + gen_avx_forms(random.Random(seed ^ 0xA0C))
        forms = forms + sse_forms * 3  # mostly SSE / AVX
    sp = AddressSpace()
    progs = []
    for i in range(n_programs):
        code = make_program(rng, forms)
        va = CODE_VA + i * SLOT
        sp.map_range(va, code + b"\xcc" * (SLOT - len(code)), write=False)
        progs.append(va)
    win = bytes(rng.getrandbits(8) for _ in range(0x2000))
    sp.map_range(WIN_VA, win, nx=True)
    sp.map(RO_VA, bytes(rng.getrandbits(8) for _ in range(0x1000)), write=False, nx=True)
    sp.map_range(STACK_VA, bytes(0x2000), nx=True)
    st = user_state(CODE_VA, STACK_TOP, sp.cr3)
    lanes = []
    for i, va in enumerate(progs):
        regs = [rng.getrandbits(64) for _ in range(16)]
        regs[RSP] = STACK_TOP
        flags = 0x202 | (rng.getrandbits(12) & 0x8D5)
        lanes.append((va, regs, flags))
    return sp, st, lanes


def lane_xmm(n: int, seed: int, salt: int = 0x3E3):
    """Initial XMM registers per lane (32 u64 each); salt 0x4E4: the YMM upper halves."""
    rng = random.Random(seed ^ salt)
    return [[rng.getrandbits(64) for _ in range(32)] for _ in range(n)]


def lane_mxcsr(n: int, seed: int):
    """Initial MXCSR per lane: rounding control, DAZ, FTZ, sometimes unmasked exceptions."""
    rng = random.Random(seed ^ 0x3C5)
    out = []
    for _ in range(n):
        mx = 0x1F80 | (rng.randrange(4) << 13) | (0x40 if rng.random() < 0.3 else 0) | (0x8000 if rng.random() < 0.3 else 0)
        if rng.random() < 0.2:
            mx &= ~(rng.getrandbits(6) << 7)
        out.append(mx)
    return out


def oracle_run(sp: AddressSpace, st: dict, lanes, limit=20000, breakpoints=(), xmm=None, ymmh=None, mxcsr=None):
    """Runs every lane on the CPU oracle; returns per-lane result dicts."""
    from tests.oracle_lib import Oracle

    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    base = regs_from_state(st)
    o.set_limit(limit)
    o.set_breakpoints(list(breakpoints))
    out = []
    for i, (va, regs, flags) in enumerate(lanes):
        r = regs_from_state(st)
        for k in range(16):
            r.gpr[k] = regs[k]
        if xmm is not None:
            for k in range(16):
                r.xmm[k][0], r.xmm[k][1] = xmm[i][2 * k], xmm[i][2 * k + 1]
        if ymmh is not None:
            for k in range(16):
                r.ymmh[k][0], r.ymmh[k][1] = ymmh[i][2 * k], ymmh[i][2 * k + 1]
        if mxcsr is not None:
            r.mxcsr = mxcsr[i]
        r.rip = va
        r.rflags = flags
        o.restore(base)
        o.set_regs(r)
        ex = o.run()
        rr = o.regs()
        out.append({
            "status": ex.status, "vector": ex.vector, "error": ex.error, "addr": ex.addr, "rip": rr.rip,
            "icount": ex.icount, "gpr": list(rr.gpr), "rflags": rr.rflags, "cov": set(o.coverage()),
            "dirty": set(o.dirty()), "bytes": o.nbytes(),
            "win": o.read_virt(WIN_VA, 0x2000), "stack": o.read_virt(STACK_VA, 0x2000),
            "xmm": [rr.xmm[k][h] for k in range(16) for h in range(2)], "mxcsr": rr.mxcsr,
            "ymmh": [rr.ymmh[k][h] for k in range(16) for h in range(2)],
        })
    return out
