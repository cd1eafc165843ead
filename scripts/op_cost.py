"""Per-form cost of k_run's step loop (a measurement aid, not a test): a ring-3
loop of one instruction form repeated 8 times + dec rcx / jnz, every lane on
the same trip count (converged waves, 64 lanes a wave-step), 65,536 lanes (one
wave per SIMD). Each case runs twice (the second run, warm shared uop cache, is
the one reported): kernel ms, wave-steps, ns per wave-step of one wave.

Run under `rocprofv3 --pmc SQ_...` as well: k_run dispatches come two per case
in the order printed, so the instruction mix per wave-step of each form is the
second dispatch's counters / its wave-steps."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from wtf_amd.abi import regs_from_state  # noqa: E402
from wtf_amd.engine import Engine  # noqa: E402
from wtf_amd.tools.snapshot import AddressSpace, user_state  # noqa: E402

CODE_VA, EXIT_VA, TABLE_VA, SCRATCH_VA, STACK_TOP = 0x140001000, 0x140002000, 0x150000000, 0x160000000, 0x7FF000000000
CASES = {
    "nop": "90",
    "mov_rr": "4889d8",            # mov rax, rbx
    "add_rr": "4801d8",            # add rax, rbx
    "add_ri": "4883c005",          # add rax, 5
    "and_r32i": "81e2f8010000",    # and edx, 0x1f8
    "lea": "4c8d545810",           # lea r10, [rax+rbx*2+0x10]
    "load": "488b4708",            # mov rax, [rdi+8]   (read-only table page)
    "store": "48894608",           # mov [rsi+8], rax   (the lane's private page)
    "pushpop": "5058",             # push rax; pop rax
    "cmp_jz": "4839d87400",        # cmp rax, rbx; jz +0
    "movaps_ld": "0f2807",         # movaps xmm0, [rdi]
    "bswap": "480fc8",             # bswap rax       (generic: the slow step's exec)
    "imul_rr": "480fafc3",         # imul rax, rbx   (generic)
}
SYN_LOOP = ("4889c2" "81e2f8010000" "4c8b0417" "4c01c0" "4831c3" "4929d9" "4c8d545810" "4181e2f80f0000" "4e890c16")


def build(body: bytes, rep: int):
    code = body * rep + bytes.fromhex("48ffc9")  # dec rcx
    code += bytes([0x75, (-(len(code) + 2)) & 0xFF]) if len(code) + 2 <= 128 else \
        bytes([0x0F, 0x85]) + (-(len(code) + 6) & 0xFFFFFFFF).to_bytes(4, "little")
    code += b"\xc3"
    sp = AddressSpace()
    sp.map(CODE_VA, code, write=False)
    sp.map(EXIT_VA, b"\xcc", write=False)
    sp.map(TABLE_VA, bytes(range(256)) * 16, write=False, nx=True)
    sp.map(SCRATCH_VA, b"", nx=True)
    stack = bytearray(4096)
    stack[4088:4096] = EXIT_VA.to_bytes(8, "little")
    sp.map(STACK_TOP - 0x1000, bytes(stack), nx=True)
    st = user_state(CODE_VA, STACK_TOP - 8, sp.cr3, rdi=TABLE_VA, rsi=SCRATCH_VA, rax=1, rbx=2)
    return sp, st


def run_case(name, body, rep, lanes, trips):
    sp, st = build(body, rep)
    eng = Engine(0)
    pfns, blob = sp.phys()
    eng.load_pool(pfns, blob)
    eng.alloc_lanes(lanes, overlay_pages=4, cov_entries=256)
    eng.set_initial_state(regs_from_state(st))
    eng.set_limit(0)
    eng.set_breakpoints([EXIT_VA])
    eng.set_code_pages([CODE_VA >> 12, EXIT_VA >> 12])
    out = None
    for _ in range(2):
        eng.restore()
        g = eng.read_gprs()
        g[:, 1] = trips
        eng.write_gprs(g)
        r = eng.run()
        waves = lanes // 64
        out = {"case": name, "kernel_ms": r.kernel_ms, "launches": r.kernel_launches, "wave_steps": r.group_steps,
               "retired": r.lane_retired, "lanes_per_step": r.lane_retired / max(1, r.group_steps),
               "ns_per_wave_step": r.kernel_ms * 1e6 / max(1, r.group_steps / waves)}
    eng.close()
    return out


def main():
    lanes = int(os.environ.get("OPC_LANES", "65536"))
    trips = int(os.environ.get("OPC_TRIPS", "256"))
    only = sys.argv[1:]
    cases = [(k, bytes.fromhex(v), 8) for k, v in CASES.items()] + [("syn", bytes.fromhex(SYN_LOOP), 1)]
    for name, body, rep in cases:
        if only and name not in only:
            continue
        print(json.dumps(run_case(name, body, rep, lanes, trips)), flush=True)


if __name__ == "__main__":
    main()
