"""Ring-0 system-instruction programs for the engine-vs-oracle tests
(DESIGN.md U19-U21): RDMSR / WRMSR over CpuState_t's MSRs, RDTSC / RDTSCP,
MOV to and from control registers (a cr3 write that ends the testcase with
Cr3Change_t, bochscpu_backend.cc:628-657) and IRETQ to ring 0 / ring 3 with
valid and invalid frames. The programs run on the HEVD look-alike's address
space (its IDT / TSS deliver the faults they raise); every lane starts at one
of the snippets below with its own random operands."""
from __future__ import annotations

import random

from wtf_amd.abi import regs_from_state
from wtf_amd.tools import hevd
from wtf_amd.tools.snapshot import seg

SYS_CODE = 0xFFFFF80000600000   # supervisor code page: the snippets, 0x100 apart
USER_CODE = 0x0000000140800000  # user code page: rdtsc; hlt
KSP = hevd.KSTACK + 0x5000
USTACK = hevd.STACK_TOP - 0x2000

MSRS = [0x10, 0x1B, 0x174, 0x175, 0x176, 0x277, 0xC0000080, 0xC0000081, 0xC0000082, 0xC0000083,
        0xC0000084, 0xC0000100, 0xC0000101, 0xC0000102, 0xC0000103]
BAD_MSRS = [0x0, 0x3A, 0xC0000085, 0x12345678]

SNIPPETS = {
    # rcx = r8; rdmsr; keep; edx:eax = r10:r9; wrmsr; rdmsr; hlt
    "msr": bytes.fromhex("4c89c1 0f32 4889c6 4889d7 4c89c8 4c89d2 0f30 0f32 f4"),
    # rdtsc; keep; rdtscp; hlt
    "tsc": bytes.fromhex("0f31 4889c6 4889d7 0f01f9 f4"),
    # cr3 -> rax -> cr3 (same: goes on); cr0 / cr4 read and written back;
    # cr2 = r8 and read back; cr8 = r9 and read back; cr3 = r10 (another
    # value ends the testcase); mov rdi, r11; mov cr5, rax (#UD); hlt
    "cr": bytes.fromhex("0f20d8 0f22d8 0f20c3 0f22c3 0f20e1 0f22e1 410f22d0 0f20d2 450f22c1 440f20c6"
                        " 410f22da 4c89df 0f22e8 f4"),
    # cr4 = r13; push ss, rsp, rflags, cs, rip (r8..r12); iretq
    "iret": bytes.fromhex("410f22e5 4150 4151 4152 4153 4154 48cf f4"),
}
SLOT = {name: SYS_CODE + 0x100 * i for i, name in enumerate(SNIPPETS)}
HLT_TARGET = SYS_CODE + 0x100 * len(SNIPPETS)     # rdtsc; hlt (ring 0 target)


def build_space(work_dir: str):
    sp, st, _, _ = hevd.build_space(work_dir)
    code = bytearray(0x1000)
    for name, blob in SNIPPETS.items():
        off = SLOT[name] - SYS_CODE
        code[off:off + len(blob)] = blob
    off = HLT_TARGET - SYS_CODE
    code[off:off + 3] = bytes.fromhex("0f31f4")
    sp.map(SYS_CODE, bytes(code), user=False, write=False, nx=False)
    sp.map(USER_CODE, bytes.fromhex("0f31f4") + b"\xcc" * 0xffd, user=True, write=False, nx=False)
    st = dict(st)
    st.update({"rip": SLOT["tsc"], "rsp": KSP, "cs": seg(0x10, 0, 0, 0x209B), "ss": seg(0x18, 0, 0xFFFFFFFF, 0xC93),
               "rflags": 0x202})
    return sp, st


def _canon(rng):
    return rng.choice([rng.getrandbits(47), (1 << 64) - 1 - rng.getrandbits(47), rng.getrandbits(64)])


def lanes(n: int, seed: int, st: dict):
    """[(rip, 16 GPRs, rflags)] for n lanes."""
    rng = random.Random(seed)
    out = []
    names = list(SNIPPETS)
    for i in range(n):
        name = names[i % len(names)]
        g = [rng.getrandbits(64) for _ in range(16)]
        g[4] = KSP
        if name == "msr":
            g[8] = rng.choice(MSRS * 3 + BAD_MSRS)
            v = _canon(rng) if rng.random() < 0.8 else rng.getrandbits(32)
            if g[8] == 0xC0000080:  # EFER: the snapshot's with a bit or two flipped
                v = st["efer"] ^ rng.choice([0, 1, 0x800, 0x400, 0x100])
            if g[8] in (0xC0000084, 0xC0000103) and rng.random() < 0.7:
                v &= 0xFFFFFFFF
            g[9], g[10] = v & 0xFFFFFFFF | (rng.getrandbits(32) << 32), v >> 32
        elif name == "cr":
            g[10] = st["cr3"] if rng.random() < 0.5 else rng.getrandbits(40) << 12
        elif name == "iret":
            g[13] = st["cr4"] | rng.choice([0, 0, 4])                    # CR4.TSD for ring-3 rdtsc
            g[8] = rng.choice([0, 0x18, 0x2B])                           # ss
            g[9] = rng.choice([KSP - 0x100, USTACK, _canon(rng)])       # rsp
            g[10] = (rng.getrandbits(22) & 0x3F7FD7) | 2                # rflags
            g[11] = rng.choice([0x10, 0x33, 0x33, 0x13, 0x0, 0x30, 0x2B])  # cs
            g[12] = rng.choice([HLT_TARGET, USER_CODE, USER_CODE, 1 << 47, 0xFFFFF80000700000])  # rip
        out.append((SLOT[name], g, 0x202 | (rng.getrandbits(1) << 11)))
    return out


REG_FIELDS = ("cr0", "cr2", "cr3", "cr4", "cr8", "efer", "star", "lstar", "cstar", "sfmask", "kernel_gs_base",
              "tsc", "tsc_aux", "apic_base", "pat", "sysenter_cs", "sysenter_eip", "sysenter_esp")


def reg_view(r) -> dict:
    d = {k: int(getattr(r, k)) for k in REG_FIELDS}
    d["fs_base"], d["gs_base"] = int(r.seg[4].base), int(r.seg[5].base)
    d["cs"], d["ss"] = int(r.seg[1].selector), int(r.seg[2].selector)
    return d


def oracle_run(sp, st: dict, ln, limit=2000):
    from tests.oracle_lib import Oracle

    pfns, blob = sp.phys()
    o = Oracle(pfns=pfns, blob=blob)
    base = regs_from_state(st)
    o.set_limit(limit)
    out = []
    for va, regs, flags in ln:
        r = regs_from_state(st)
        for k in range(16):
            r.gpr[k] = regs[k]
        r.rip, r.rflags = va, flags
        o.restore(base)
        o.set_regs(r)
        ex = o.run()
        rr = o.regs()
        out.append({"status": ex.status, "vector": ex.vector, "error": ex.error, "addr": ex.addr,
                    "rip": rr.rip, "icount": ex.icount, "gpr": list(rr.gpr), "rflags": rr.rflags,
                    "regs": reg_view(rr), "cov": set(o.coverage()), "dirty": set(o.dirty())})
    return out

