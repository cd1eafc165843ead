"""SYN: the synthetic ring-3 ALU / branch / load-store loop snapshot
(BASELINE.json configs[1]).

Guest program (11 instructions per iteration, one 8-byte load from a read-only
table page, one 8-byte store into a scratch page that every testcase dirties):

    loop: mov rdx, rax ; and edx, 0x1f8 ; mov r8, [rdi+rdx] ; add rax, r8
          xor rbx, rax ; sub r9, rbx ; lea r10, [rax+rbx*2+0x10]
          and r10d, 0xff8 ; mov [rsi+r10], r9 ; dec rcx ; jnz loop
          ret                     -> EXIT_VA, where a breakpoint stops the testcase

Testcase (64 bytes): trip count = 1 + (in[0] | in[1] << 8) % 4096, rax / rbx / r9
seeded from in[2:10] / in[10:18] / in[18:26]. Inputs are uniform random bytes
(numpy default_rng(0x5EED0001)); the reference plan's std::mt19937_64 stream is
not reproduced bit for bit, only its distribution.
"""
from __future__ import annotations

import numpy as np

from .snapshot import AddressSpace, user_state

CODE_VA = 0x140001000
EXIT_VA = 0x140002000
TABLE_VA = 0x150000000
SCRATCH_VA = 0x160000000
STACK_TOP = 0x7FF000000000
INPUT_SIZE = 64
SEED = 0x5EED0001

LOOP = bytes.fromhex(
    "4889c2"          # mov rdx, rax
    "81e2f8010000"    # and edx, 0x1f8
    "4c8b0417"        # mov r8, [rdi+rdx]
    "4c01c0"          # add rax, r8
    "4831c3"          # xor rbx, rax
    "4929d9"          # sub r9, rbx
    "4c8d545810"      # lea r10, [rax+rbx*2+0x10]
    "4181e2f80f0000"  # and r10d, 0xff8
    "4e890c16"        # mov [rsi+r10], r9
    "48ffc9"          # dec rcx
    "75d5"            # jnz loop
    "c3"              # ret
)
INSNS_PER_ITER = 11
BYTES_PER_ITER = len(LOOP) - 1 + 16  # instruction bytes + 8 loaded + 8 stored


def build():
    """Returns (AddressSpace, cpu state dict, symbols)."""
    sp = AddressSpace()
    sp.map(CODE_VA, LOOP, write=False)
    sp.map(EXIT_VA, b"\xcc", write=False)
    table = np.random.default_rng(1).integers(0, 2**63, size=512, dtype=np.int64).astype(np.uint64).tobytes()
    sp.map(TABLE_VA, table, write=False, nx=True)
    sp.map(SCRATCH_VA, b"", nx=True)
    stack = bytearray(4096)
    stack[4096 - 8: 4096] = EXIT_VA.to_bytes(8, "little")
    sp.map(STACK_TOP - 0x1000, bytes(stack), nx=True)
    st = user_state(CODE_VA, STACK_TOP - 8, sp.cr3, rdi=TABLE_VA, rsi=SCRATCH_VA)
    symbols = {"syn!loop": CODE_VA, "syn!exit": EXIT_VA, "syn": CODE_VA}
    return sp, st, symbols


def inputs(n: int, seed: int = SEED) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, size=(n, INPUT_SIZE), dtype=np.uint8)


def insert(gprs: np.ndarray, inp: np.ndarray) -> None:
    """InsertTestcase for a batch: writes rcx / rax / rbx / r9 of each lane
    (gprs: [n, 18] u64 in wtfgpu order, rows already at the snapshot state)."""
    inp = np.ascontiguousarray(inp, dtype=np.uint8)
    trip = 1 + ((inp[:, 0].astype(np.uint64) | (inp[:, 1].astype(np.uint64) << np.uint64(8))) % np.uint64(4096))
    gprs[:, 1] = trip
    gprs[:, 0] = inp[:, 2:10].copy().view("<u8")[:, 0]
    gprs[:, 3] = inp[:, 10:18].copy().view("<u8")[:, 0]
    gprs[:, 9] = inp[:, 18:26].copy().view("<u8")[:, 0]


def expected_instructions(inp: np.ndarray) -> np.ndarray:
    trip = 1 + ((inp[:, 0].astype(np.int64) | (inp[:, 1].astype(np.int64) << 8)) % 4096)
    return trip * INSNS_PER_ITER + 1


def model(inp: np.ndarray, table: bytes):
    """The SYN loop restated over whole batches in numpy (a test checker):
    final rax, rbx, rcx, rdx, r8, r9, r10 of every testcase, and the scratch
    page each one leaves (uint64[n, 512]). Same insert as `insert`."""
    n = len(inp)
    g = np.zeros((n, 18), dtype=np.uint64)
    insert(g, inp)
    tab = np.frombuffer(table, dtype=np.uint64)
    rax, rbx, r9, rcx = g[:, 0].copy(), g[:, 3].copy(), g[:, 9].copy(), g[:, 1].copy()
    rdx = np.zeros(n, np.uint64)
    r8 = np.zeros(n, np.uint64)
    r10 = np.zeros(n, np.uint64)
    scratch = np.zeros((n, 512), dtype=np.uint64)
    idx = np.arange(n)
    live = np.ones(n, dtype=bool)
    with np.errstate(over="ignore"):
        while live.any():
            k = idx[live]
            rdx[k] = rax[k] & np.uint64(0x1F8)
            r8[k] = tab[(rdx[k] >> np.uint64(3)).astype(np.int64)]
            rax[k] = rax[k] + r8[k]
            rbx[k] = rbx[k] ^ rax[k]
            r9[k] = r9[k] - rbx[k]
            r10[k] = (rax[k] + rbx[k] * np.uint64(2) + np.uint64(0x10)) & np.uint64(0xFF8)
            scratch[k, (r10[k] >> np.uint64(3)).astype(np.int64)] = r9[k]
            rcx[k] = rcx[k] - np.uint64(1)
            live[k] = rcx[k] != 0
    return {"rax": rax, "rbx": rbx, "rcx": rcx, "rdx": rdx, "r8": r8, "r9": r9, "r10": r10}, scratch
