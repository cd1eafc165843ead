"""Snapshot files vs the reference's own kdmp-parser.

wtf_amd/tools/snapshot.py writes the mem.dmp files every synthetic snapshot
uses (full dumps and BMP dumps); wtf_amd/host/kdmp.cc reads them for the gpu
backend. Both are checked against kdmp-parser as the reference vendors it
(src/libs/kdmp-parser/src/lib: Parse kdmp-parser.h:51-94, full-dump runs
:399-484, BMP bitmap :490-529, GetPhysicalPage :233-254, VirtTranslate
:269-345), compiled into oracle/_ref/kdmp_ref by oracle/Makefile:

  * header type, DirectoryTableBase, context rip;
  * every physical page (address + FNV-1a of its 4096 bytes);
  * VirtTranslate of mapped, unmapped, large-page (2 MiB / 1 GiB) and
    non-canonical addresses.

The SYN and large-page dumps are built here from Python alone, and kdmp_ref's
output on them is committed (tests/golden/kdmp_fixtures.json, written by
`python tests/test_snapshot_format.py --regen`), so the comparison runs without
the reference build too. The tlv / HEVD dumps (gcc-built guests) are compared
live when oracle/_ref exists.
"""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from wtf_amd.tools import snapshot, syn  # noqa: E402

from tests.cpu_bins import ALT, HOSTCHECK as TOOL  # noqa: E402
REF = os.path.join(ROOT, "oracle", "_ref", "kdmp_ref")
FIXTURES = os.path.join(ROOT, "tests", "golden", "kdmp_fixtures.json")
PREFIXES = ("TYPE ", "CR3 ", "RIP ", "PAGE ", "VT ", "PARSE_FAIL")


def _tool():
    if not ALT and not os.path.exists(TOOL):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "hostcheck"])
    return TOOL


def lines(out: str) -> list[str]:
    """The comparable lines (kdmp-parser also prints diagnostics)."""
    return [ln for ln in out.splitlines() if ln.startswith(PREFIXES)]


def ours(dump: str, gvas: list[int]) -> list[str]:
    r = subprocess.run([_tool(), "kdmp", dump, *map(hex, gvas)], capture_output=True, text=True)
    return lines(r.stdout)


def reference(dump: str, gvas: list[int]) -> list[str]:
    r = subprocess.run([REF, dump, *map(hex, gvas)], capture_output=True, text=True)
    return lines(r.stdout)


def large_page_space():
    """Page tables with a 1 GiB leaf (PDPTE.PS) and a 2 MiB leaf (PDE.PS),
    the kdmp-parser walk's large-page branches (kdmp-parser.h:300-330)."""
    sp = snapshot.AddressSpace()
    sp.map(0x140000000, b"\x90" * 16)               # an ordinary 4 KiB page
    pml4 = sp.cr3 >> 12
    # 1 GiB leaf at 0x7f8000000000 -> gpa 0x40000000
    pdpt = sp.alloc()
    struct.pack_into("<Q", sp.pages[pml4], 0xFF * 8, (pdpt << 12) | 0x7)
    struct.pack_into("<Q", sp.pages[pdpt], 0, 0x40000000 | 0x87)
    # 2 MiB leaf at 0x7f8040000000 -> gpa 0x200000
    pd = sp.alloc()
    struct.pack_into("<Q", sp.pages[pdpt], 1 * 8, (pd << 12) | 0x7)
    struct.pack_into("<Q", sp.pages[pd], 3 * 8, 0x200000 | 0x87)
    # a few pages inside both large mappings, so GetPhysicalPage sees them
    for gpa in (0x40000000, 0x40001000, 0x200000, 0x3FF000):
        sp.pages[gpa >> 12] = bytearray(struct.pack("<Q", gpa) * 512)
    gvas = [0x140000000, 0x140000FFF, 0x7F8000000000, 0x7F8000001234, 0x7F803FFFFFFF, 0x7F8040600000,
            0x7F80407FFFFF, 0x7F8040800000, 0x7F9000000000, 0x0, 0xFFFF800000000000, 0x800000000000]
    return sp, gvas


def syn_space():
    sp, st, _ = syn.build()
    gvas = [syn.CODE_VA, syn.EXIT_VA, syn.TABLE_VA + 0x123, syn.SCRATCH_VA, syn.STACK_TOP - 8, syn.STACK_TOP,
            0x0, 0x7FFFFFFFF000, 0xFFFFF80000000000]
    return sp, st, gvas


def python_dumps(tmp: str) -> dict[str, tuple[str, list[int]]]:
    out = {}
    sp, st, gvas = syn_space()
    for bmp in (False, True):
        d = os.path.join(tmp, f"syn_{int(bmp)}")
        snapshot.write_snapshot(d, sp, st, {}, bmp=bmp)
        out[f"syn_{'bmp' if bmp else 'full'}"] = (os.path.join(d, "mem.dmp"), gvas)
    lp, lgvas = large_page_space()
    st2 = snapshot.user_state(0x140000000, 0x7F8000000100, lp.cr3)
    for bmp in (False, True):
        d = os.path.join(tmp, f"lp_{int(bmp)}")
        snapshot.write_snapshot(d, lp, st2, {}, bmp=bmp)
        out[f"large_{'bmp' if bmp else 'full'}"] = (os.path.join(d, "mem.dmp"), lgvas)
    return out


@pytest.fixture(scope="module")
def py_dumps():
    with tempfile.TemporaryDirectory() as d:
        yield python_dumps(d)


def test_fixtures_cover_python_dumps(py_dumps):
    fx = json.load(open(FIXTURES))
    assert set(fx) == set(py_dumps)


@pytest.mark.parametrize("name", ["syn_full", "syn_bmp", "large_full", "large_bmp"])
def test_kdmp_reader_matches_reference_fixture(py_dumps, name):
    path, gvas = py_dumps[name]
    expect = json.load(open(FIXTURES))[name]
    got = ours(path, gvas)
    assert got == expect
    assert any(ln.startswith("VT ") and not ln.endswith(" -1") for ln in got)


@pytest.mark.skipif(not os.path.exists(REF), reason="reference build absent (oracle/_ref)")
@pytest.mark.parametrize("name", ["syn_full", "syn_bmp", "large_full", "large_bmp"])
def test_python_dumps_live_reference(py_dumps, name):
    path, gvas = py_dumps[name]
    assert reference(path, gvas) == json.load(open(FIXTURES))[name]


@pytest.mark.skipif(not os.path.exists(REF), reason="reference build absent (oracle/_ref)")
@pytest.mark.parametrize("target", ["tlv", "hevd"])
@pytest.mark.parametrize("bmp", [False, True])
def test_guest_snapshots_live_reference(target, bmp, tmp_path):
    """The gcc-built tlv_server / HEVD look-alike snapshots, both dump kinds,
    parsed by kdmp-parser and by kdmp.cc, with a walk of every symbol."""
    import importlib

    mod = importlib.import_module(f"wtf_amd.tools.{target}")
    state = tmp_path / "state"
    mod.build(str(state), str(tmp_path / "work"))
    syms = {k: int(v, 16) for k, v in json.load(open(state / "symbol-store.json")).items()}
    regs = json.load(open(state / "regs.json"))
    gvas = sorted({v for v in syms.values() if v} | {int(regs["rsp"], 16), int(regs["rip"], 16), 0x0})
    dump = str(state / "mem.dmp")
    if bmp:  # re-write the same pages as a BMP dump
        index, data, cr3 = snapshot.read_kdmp(dump)
        pfns = sorted(index)
        pages = b"".join(bytes(data[index[p]:index[p] + 4096]) for p in pfns)
        st = {k: (int(v, 16) if isinstance(v, str) and v.startswith("0x") else v) for k, v in regs.items()}
        for s in ("cs", "ds", "es", "fs", "gs", "ss"):
            st[s] = {"selector": int(regs[s]["selector"], 16)}
        dump = str(tmp_path / "bmp.dmp")
        snapshot.write_kdmp(dump, pfns, pages, st, bmp=True)
    ref = reference(dump, gvas)
    assert ref and ref[0] == ("TYPE 5" if bmp else "TYPE 1")
    assert ours(dump, gvas) == ref


if __name__ == "__main__" and "--regen" in sys.argv:
    with tempfile.TemporaryDirectory() as d:
        fx = {name: reference(path, gvas) for name, (path, gvas) in python_dumps(d).items()}
    json.dump(fx, open(FIXTURES, "w"), indent=0)
    print(f"wrote {FIXTURES}: {', '.join(f'{k} ({len(v)} lines)' for k, v in fx.items())}")
