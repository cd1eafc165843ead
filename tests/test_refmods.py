"""The reference's own fuzzer modules, unchanged, on this repository's backends.

`north_star` asks for fuzzer_tlv_server and fuzzer_hevd to run unchanged on
the gpu backend. oracle/Makefile compiles the reference's fuzzer_hevd.cc and
crash_detection_umode.cc, byte for byte as they lie under /root/reference,
against this repository's Backend_t / Target_t interface
(wtf_amd/host/compat/, README there) and links them:
  * into the gpu node: oracle/_ref/wtfgpu_refmods;
  * into the oracle twin: oracle/_ref/wtf_twin_refmods.
Every HEVD parity input must then end exactly as it does with the restated
modules (wtf_amd/host/modules/) on the twin: result, crash name, retired
count, final registers, coverage set. The reference hevd module declares no
device-side breakpoint actions, so on the GPU every one of its breakpoints is a
host round trip (the host service path, exercised by an unmodified module).

The reference's fuzzer_tlv_server.cc keeps its packet queue in a plain
global: linked into the executable it runs unchanged wherever one testcase is
in flight at a time (the twin; the gpu node at one lane per batch). Batched,
it runs unchanged too as per-lane copies (module_instances.h):
oracle/Makefile also builds it as oracle/_ref/fuzzer_tlv_server_ref.so, and
`--module-so` loads one private copy per lane (own globals, own handlers),
512 lanes per batch on the GPU. Either way it must match the restated module.
Malformed-JSON inputs are left out: the reference module throws on them
(nlohmann parse, uncaught).
"""
import os
import subprocess

import pytest

from tests import tlv_harness as H
from tests.hevd_inputs import write_inputs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"
TWIN_REF = os.path.join(ROOT, "oracle", "_ref", "wtf_twin_refmods")
GPU_REF = os.path.join(ROOT, "oracle", "_ref", "wtfgpu_refmods")
TLV_SO = os.path.join(ROOT, "oracle", "_ref", "fuzzer_tlv_server_ref.so")
FIELDS = ("result", "crash", "error", "icount", "gprs", "coverage")


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("hevd_refmods"))
    H.build_hevd_target(d)
    write_inputs(os.path.join(d, "parity"), 400)
    return d


def _diff(a, b):
    assert len(a) == len(b) and len(a) > 0
    return [(x["input"], k) for x, y in zip(a, b) for k in FIELDS if x[k] != y[k] or x["input"] != y["input"]]


@pytest.mark.skipif(not os.path.exists(TWIN_REF), reason="reference build absent (oracle/_ref)")
def test_reference_hevd_module_matches_restated_module(target, tmp_path):
    inp = os.path.join(target, "parity")
    ref = H.run(TWIN_REF, target, inp, str(tmp_path / "ref.jsonl"), lanes=64, name="hevd")
    ours = H.run(H.TWIN, target, inp, str(tmp_path / "ours.jsonl"), lanes=64, name="hevd")
    assert not _diff(ref, ours)
    assert any(r["crash"].startswith("crash-0xf7-") for r in ref)   # nt!KeBugCheck2 handler
    assert any(r["result"] == "cr3" for r in ref)                    # nt!SwapContext handler


@pytest.fixture(scope="module")
def tlv_target(tmp_path_factory):
    from tests.tlv_inputs import write_inputs as tlv_inputs

    d = str(tmp_path_factory.mktemp("tlv_refmods"))
    H.build_target(d)
    inp = os.path.join(d, "parity")
    tlv_inputs(inp, 1100)
    os.remove(os.path.join(inp, "edge_bad_json"))
    return d


@pytest.mark.skipif(not os.path.exists(TWIN_REF), reason="reference build absent (oracle/_ref)")
def test_reference_tlv_module_matches_restated_module(tlv_target, tmp_path):
    inp = os.path.join(tlv_target, "parity")
    ref = H.run(TWIN_REF, tlv_target, inp, str(tmp_path / "ref.jsonl"), lanes=1)
    ours = H.run(H.TWIN, tlv_target, inp, str(tmp_path / "ours.jsonl"), lanes=64)
    assert not _diff(ref, ours)
    assert any(r["crash"].startswith("crash-EXCEPTION_") for r in ref)  # user-mode crash detection


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
def test_reference_tlv_module_compiles_against_backend_interface(tmp_path):
    src = os.path.join(REF, "wtf", "fuzzer_tlv_server.cc")
    host = os.path.join(ROOT, "wtf_amd", "host")
    cmd = ["g++", "-std=c++20", "-fsyntax-only", "-w", "-x", "c++", "-DFMT_HEADER_ONLY",
           "-include", f"{host}/compat/pch.h", f"-I{host}/compat", f"-I{host}", f"-I{REF}/libs/fmt/include", f"-I{REF}/libs/json/single_include",
           "-idirafter", f"{REF}/wtf", "-"]
    with open(src, "rb") as f:
        r = subprocess.run(cmd, stdin=f, cwd=str(tmp_path), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(GPU_REF), reason="oracle/_ref/wtfgpu_refmods not built")
def test_reference_hevd_module_on_gpu(target, tmp_path):
    inp = os.path.join(target, "parity")
    g = H.run(GPU_REF, target, inp, str(tmp_path / "g.jsonl"), lanes=512, name="hevd")
    t = H.run(H.TWIN, target, inp, str(tmp_path / "t.jsonl"), lanes=512, name="hevd")
    assert not _diff(g, t)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(GPU_REF), reason="oracle/_ref/wtfgpu_refmods not built")
def test_reference_tlv_module_on_gpu_one_lane(tlv_target, tmp_path):
    inp = os.path.join(tlv_target, "parity")
    names = sorted(os.listdir(inp))[:60]
    sub = tmp_path / "sub"
    sub.mkdir()
    for n in names:
        (sub / n).write_bytes(open(os.path.join(inp, n), "rb").read())
    g = H.run(GPU_REF, tlv_target, str(sub), str(tmp_path / "g.jsonl"), lanes=1)
    t = H.run(H.TWIN, tlv_target, str(sub), str(tmp_path / "t.jsonl"), lanes=1)
    assert not _diff(g, t)


@pytest.mark.skipif(not os.path.exists(TLV_SO), reason="reference build absent (oracle/_ref)")
def test_reference_tlv_module_copies_on_twin(tlv_target, tmp_path):
    inp = os.path.join(tlv_target, "parity")
    ref = H.run(TWIN_REF, tlv_target, inp, str(tmp_path / "ref.jsonl"), lanes=512, extra=("--module-so", TLV_SO))
    ours = H.run(H.TWIN, tlv_target, inp, str(tmp_path / "ours.jsonl"), lanes=512)
    assert not _diff(ref, ours)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(GPU_REF) or not os.path.exists(TLV_SO), reason="oracle/_ref not built")
@pytest.mark.parametrize("lanes", [512, 1024])
def test_reference_tlv_module_batched_on_gpu(tlv_target, tmp_path, lanes):
    """The unchanged module, one copy per lane, `lanes` testcases in flight:
    every copy's packet queue is its own lane's (a shared queue would hand
    one lane's packets to another and change results)."""
    inp = os.path.join(tlv_target, "parity")
    g = H.run(GPU_REF, tlv_target, inp, str(tmp_path / "g.jsonl"), lanes=lanes, extra=("--module-so", TLV_SO))
    t = H.run(H.TWIN, tlv_target, inp, str(tmp_path / "t.jsonl"), lanes=512)
    assert len(g) > lanes
    assert not _diff(g, t)
