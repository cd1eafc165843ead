"""CPU-side checks of the C ABI: the HIP library exists, loads and exports
every entry point include/wtfgpu.h declares (no GPU calls)."""
import ctypes
import os

from wtf_amd.abi import LIB_PATH, exported_symbols_from_header, load_hip_library

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    syms = exported_symbols_from_header(os.path.join(ROOT, "include", "wtfgpu.h"))
    assert len(syms) >= 30
    lib = ctypes.CDLL(LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_abi_version_and_loader():
    lib = load_hip_library()
    assert lib.wtfgpu_abi_version() == 4


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the ABI structs agree with the C compiler's layout."""
    import subprocess
    from wtf_amd import abi
    src = tmp_path / "sz.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n'
        'int main(){printf("%%zu %%zu %%zu %%zu %%zu %%zu %%zu\\n", sizeof(wtfgpu_seg_t), sizeof(wtfgpu_regs_t),'
        'sizeof(wtfgpu_exit_t), sizeof(wtfgpu_write_t), sizeof(wtfgpu_run_stats_t), offsetof(wtfgpu_regs_t, seg),'
        'offsetof(wtfgpu_regs_t, xmm));}\n' % os.path.join(ROOT, "include", "wtfgpu.h"))
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", str(src), "-o", str(exe)])
    want = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    got = [ctypes.sizeof(abi.Seg), ctypes.sizeof(abi.Regs), ctypes.sizeof(abi.Exit), ctypes.sizeof(abi.Write),
           ctypes.sizeof(abi.RunStats), abi.Regs.seg.offset, abi.Regs.xmm.offset]
    assert got == want
