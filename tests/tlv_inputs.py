"""Seeded TLV testcases for the parity tests: what the tlv module's mutator
produces (fuzzer_tlv_server.cc:243-262: 1..10 packets, commands 0..10, bodies
0..100 bytes, BodySize with one bit flipped one time in three), plus the edge
cases the module handles specially (no packet, a packet of 0x1000 bytes or
more, malformed JSON, more than four allocations, short packets)."""
from __future__ import annotations

import os
import random

from wtf_amd.tools.tlv import packets_json


def random_packets(rng: random.Random) -> list:
    pk = []
    for idx in range(rng.randint(1, 11)):
        cmd = rng.choice([0, 0, 0, 1, 1, 2, 2, rng.randint(3, 10)])
        body = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 100)))
        size = len(body)
        if rng.randint(1, 3) == 1:
            size ^= 1 << rng.randint(0, 15)
        pid = rng.choice([idx, rng.randint(0, 4)])
        pk.append((cmd, pid & 0xFFFF, size & 0xFFFF, body))
    return pk


def edge_cases() -> dict[str, bytes]:
    return {
        "edge_no_packets": packets_json([]),
        "edge_too_big": packets_json([(0, 1, 4, b"\x41" * 0x1000)]),
        "edge_bad_json": b'{"Packets":[{"Body":[1,2',
        "edge_five_allocs": packets_json([(0, i, 8, bytes([i] * 8)) for i in range(5)] + [(1, 2, 8, b"x" * 8)]),
        "edge_header_only": packets_json([(0, 1, 0, b"")]),
        "edge_big_edit": packets_json([(0, 1, 4, b"abcd"), (1, 1, 64, b"y" * 64)]),
        "edge_delete_twice": packets_json([(0, 1, 4, b"abcd"), (2, 1, 0, b""), (2, 1, 0, b"")]),
        # the stale LastFreed deleted by an allocation past the table: a free of a
        # pointer the heap does not own -> __fastfail -> int 0x29 -> nt!KiRaiseSecurityCheckFailure
        "edge_fastfail": packets_json([(0, i, 16, bytes([0x30 + i] * 16)) for i in range(1, 5)] + [(2, 1, 0, b"")] +
                                      [(0, 5, 16, b"5" * 16), (0, 6, 16, b"6" * 16)]),
    }


def write_inputs(d: str, n: int, seed: int = 0x71F) -> list[str]:
    os.makedirs(d, exist_ok=True)
    rng = random.Random(seed)
    names = []
    for name, data in edge_cases().items():
        with open(os.path.join(d, name), "wb") as f:
            f.write(data)
        names.append(name)
    for i in range(n):
        name = f"rand_{i:05d}"
        with open(os.path.join(d, name), "wb") as f:
            f.write(packets_json(random_packets(rng)))
        names.append(name)
    return names
