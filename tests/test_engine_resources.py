"""k_run's resource budget, read from the built engine's gfx950 code object
(no GPU needed): the occupancy DESIGN.md §3 is measured at — two 256-thread
blocks per CU — needs at most 256 VGPRs with none spilled and at most half
the CU's 160 KiB of LDS per block (the uop cache takes all that is left,
DESIGN §3 item 3). A change that grows k_run's LDS or VGPRs past these would
halve its occupancy silently; this catches it at build time."""
from __future__ import annotations

import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "wtf_amd", "csrc", "libwtfgpu.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
LDS_PER_CU = 160 * 1024


def _tool(name: str) -> str:
    p = os.path.join(LLVM, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not in this image")
    return p


def _kernels(tmp_path) -> dict[str, dict[str, str]]:
    if not os.path.exists(LIB):
        pytest.skip("engine not built (run __graft_entry__.build())")
    fb, co = str(tmp_path / "fb.bin"), str(tmp_path / "k.o")
    subprocess.check_call([_tool("llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", LIB,
                           str(tmp_path / "copy.so")])
    subprocess.check_call([_tool("clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                           f"--targets={TARGET}", f"--output={co}"])
    notes = subprocess.check_output([_tool("llvm-readelf"), "--notes", co], text=True)
    out = {}
    # kernel maps: "  - .agpr_count: ..." opens one; kernel-level keys sit at 4 spaces
    for block in re.split(r"\n  - (?=\.agpr_count)", notes)[1:]:
        fields = dict(re.findall(r"^(?:    |)\.([a-z_]+):\s+(\S+)$", block, re.M))
        if "name" in fields:
            out[fields["name"]] = fields
    return out


def test_k_run_fits_two_blocks_per_cu(tmp_path):
    ks = _kernels(tmp_path)
    k = [v for n, v in ks.items() if "5k_run" in n]
    assert len(k) == 1, sorted(ks)
    k = k[0]
    assert int(k["max_flat_workgroup_size"]) == 256
    assert int(k["wavefront_size"]) == 64
    assert int(k["vgpr_count"]) <= 256 and int(k["vgpr_spill_count"]) == 0, k
    lds = int(k["group_segment_fixed_size"])
    # 4 waves x UC_N x 64-byte entries + 4 x UC_U uop slots: 312 entries today
    assert 256 * 64 * 4 <= lds <= LDS_PER_CU // 2, lds
    # scratch (stack frames and arrays the compiler could not keep in
    # registers): 1,344 bytes a lane today; a jump means something new spilled
    assert int(k["private_segment_fixed_size"]) <= 2048, k["private_segment_fixed_size"]


def test_every_kernel_is_wave64(tmp_path):
    ks = _kernels(tmp_path)
    assert len(ks) > 5
    assert {v["wavefront_size"] for v in ks.values()} == {"64"}
