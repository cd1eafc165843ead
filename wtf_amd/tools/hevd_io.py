"""hevd_io: the HEVD look-alike with the I/O manager's request path (the
bench's HEVD leg, BASELINE.json configs[4] on one GPU).

The kernel image is wtf_amd/tools/guest/hevd_kernel.c built with -DHEVD_IO:
the same user program, SYSCALL entry, HEVD bug classes and nt exports the
fuzzer_hevd module breakpoints (so the reference module runs unchanged), but a
DeviceIoControl reaches the driver the way Windows sends a METHOD_NEITHER
request: a trap frame, ObReferenceObjectByHandle through the handle table, an
IRP from a lookaside list with a stack location per device, IofCallDriver
through a filter device to HEVD's IRP_MJ_DEVICE_CONTROL handler via the driver
object's MajorFunction table, and IofCompleteRequest (completion routines, the
I/O status block, the event, the IRP freed, the file object dereferenced);
reference shape: fuzzer_hevd.cc:61-142, README.md:42,58.

The driver also answers four benign requests (a CRC over the input buffer, a
record parser, a bounded copy, a command list over a kernel table), and the
seed corpus is mostly those: most
mutated testcases return a status, as most of a real campaign's do, instead of
bugchecking. The bare variant (wtf_amd/tools/hevd.py: the IOCTL handlers
called straight from the system-call entry) stays as the "hevd" workload."""
from __future__ import annotations

import json
import os
import struct

from . import hevd
from .hevd import USER_BUF, testcase

CHECKSUM, PARSE, SECURE_COPY, COMMANDS = 0x222023, 0x222027, 0x22202B, 0x22202F


def build(state_dir: str, work_dir: str | None = None) -> dict:
    return hevd.build(state_dir, work_dir, io=True)


def build_space(work_dir: str):
    return hevd.build_space(work_dir, io=True)


def records(*items: tuple[int, bytes]) -> bytes:
    """The record parser's input: [u16 length][u8 type][payload] per record."""
    return b"".join(struct.pack("<HB", 3 + len(p), t) + p for t, p in items)


def seed_inputs(inputs_dir: str) -> list[str]:
    """Mostly benign requests (checksums, record lists, bounded copies), and
    benign seeds of two bug IOCTLs (the mutator still reaches every bug: the
    IOCTL code is part of the testcase)."""
    os.makedirs(inputs_dir, exist_ok=True)
    seeds = {
        "crc_64": testcase(CHECKSUM, bytes(range(64))),
        "crc_256": testcase(CHECKSUM, bytes((i * 7) & 255 for i in range(256))),
        "crc_512": testcase(CHECKSUM, b"HEVD" * 128),
        "crc_900": testcase(CHECKSUM, bytes((i * 13 + 5) & 255 for i in range(900))),
        "crc_1000": testcase(CHECKSUM, bytes((i ^ 0x5A) & 255 for i in range(1000))),
        "records_3": testcase(PARSE, records((1, b"alpha"), (2, b"beta" * 4), (3, b""))),
        "records_16": testcase(PARSE, records(*[(i & 15, bytes([0x41 + i]) * (8 + i)) for i in range(16)])),
        "records_big": testcase(PARSE, records(*[(7, b"x" * 60) for _ in range(12)])),
        "cmds_set": testcase(COMMANDS, bytes([0, 1, 2, 3, 0, 2, 5, 6, 2, 1, 2, 0, 1, 1, 0, 0])),
        "cmds_mix": testcase(COMMANDS, bytes(sum(([op, (op * 3) & 63, (op * 5 + 1) & 63, op] for op in range(16)), []))),
        "cmds_sort": testcase(COMMANDS, bytes([12, 0, 32, 7, 3, 4, 9, 8, 10, 5, 3, 1, 7, 0, 31, 0, 4, 0, 31, 40])),
        "copy_64": testcase(SECURE_COPY, b"S" * 64),
        "copy_512": testcase(SECURE_COPY, b"T" * 512),
        "copy_800": testcase(SECURE_COPY, b"U" * 800),
        "crc_1024": testcase(CHECKSUM, bytes((i * 31 + 7) & 255 for i in range(1024))),
        "records_40": testcase(PARSE, records(*[((i * 5) & 15, bytes([0x30 + (i & 63)]) * 20) for i in range(40)])),
        "records_types": testcase(PARSE, records(*[(t, bytes((t * 17 + j) & 255 for j in range(24))) for t in range(16)])),
        "write_what_where": testcase(0x22200B, struct.pack("<QQ", USER_BUF + 0x100, USER_BUF + 0x108) + b"\0" * 16),
        "integer": testcase(0x222017, b"D" * 32 + struct.pack("<I", 0xBAD0B0B0)),
        "invalid": testcase(0x222fff, b""),
    }
    paths = []
    for name, data in seeds.items():
        p = os.path.join(inputs_dir, name)
        with open(p, "wb") as f:
            f.write(data)
        paths.append(p)
    return paths


if __name__ == "__main__":
    import sys
    d = sys.argv[1] if len(sys.argv) > 1 else "build/hevd_io"
    build(os.path.join(d, "state"), os.path.join(d, "work"))
    seed_inputs(os.path.join(d, "inputs"))
    os.makedirs(os.path.join(d, "outputs"), exist_ok=True)
    os.makedirs(os.path.join(d, "crashes"), exist_ok=True)
    print(json.dumps({"target": d}))
