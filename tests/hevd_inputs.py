"""Seeded HEVD testcases for the parity tests: crafted inputs that reach each
handler's bug (the crash each one must produce is asserted by
tests/test_hevd_cpu.py), and random ones shaped like the hevd module's inputs
(u32 IOCTL code + up to 1024 bytes, fuzzer_hevd.cc:20-30)."""
from __future__ import annotations

import os
import random
import struct

from wtf_amd.tools.hevd import USER_BUF, testcase

IOCTLS = [0x222003, 0x222007, 0x22200B, 0x22200F, 0x222013, 0x222017, 0x22201B, 0x22201F]


def crafted() -> dict[str, bytes]:
    return {
        "stack_ret_overrun": testcase(0x222003, b"A" * 512 + b"B" * 240),   # return address -> 0x4242.. (#GP)
        "stack_gs_cookie": testcase(0x222007, b"A" * 520),                  # cookie -> KeBugCheck2(0xF7)
        "write_what_where_bad": testcase(0x22200B, struct.pack("<QQ", USER_BUF, 0xFFFF800000000000)),
        "write_what_where_ok": testcase(0x22200B, struct.pack("<QQ", USER_BUF + 0x10, USER_BUF + 0x20)),
        # a user address that faults inside __try: the trap resumes the handler through IRETQ
        "write_what_where_user_fault": testcase(0x22200B, struct.pack("<QQ", 0x20000000, USER_BUF + 0x20)),
        "pool_overflow": testcase(0x22200F, b"P" * 0x210),                  # next header -> KeBugCheck2(0x19)
        "null_deref": testcase(0x222013, struct.pack("<I", 0xBAD0B0B0)),     # callback through NULL (#PF)
        "integer_wrap": testcase(0x222017, struct.pack("<I", 0xFFFFFFFC) + b"I" * 600 + struct.pack("<I", 0xBAD0B0B0)),
        "integer_ok": testcase(0x222017, struct.pack("<I", 64) + b"i" * 64),
        "type_confusion": testcase(0x22201B, struct.pack("<QQ", 0x4242424242424242, 0x0000000140001000)),
        "type_confusion_bad": testcase(0x22201B, struct.pack("<QQ", 0x4242424242424242, 0x4141414141414141)),
        "wait_swapcontext": testcase(0x22201F, b"TIAWTIAW"),
        "short": b"\x03\x20",
        "too_long": testcase(0x222003, b"Z" * 1025),
        "empty_body": testcase(0x222003, b""),
    }


def write_inputs(d: str, n: int, seed: int = 0x4E7D) -> list[str]:
    os.makedirs(d, exist_ok=True)
    rng = random.Random(seed)
    out = dict(crafted())
    for i in range(n):
        ioctl = rng.choice(IOCTLS + [rng.getrandbits(32)])
        size = rng.choice([rng.randint(0, 64), rng.randint(0, 1024), rng.choice([512, 520, 528, 0x1f8, 0x200, 0x210])])
        body = bytes(rng.getrandbits(8) for _ in range(size))
        if rng.randint(0, 3) == 0 and size >= 16:  # plausible pointers for the pointer-taking handlers
            body = struct.pack("<QQ", USER_BUF + rng.randint(0, 0x1ff8), rng.choice([USER_BUF + 0x100, 0, 1 << 63])) + body[16:]
        out[f"rand_{i:05d}"] = testcase(ioctl, body)
    for name, data in out.items():
        with open(os.path.join(d, name), "wb") as f:
            f.write(data)
    return list(out)
