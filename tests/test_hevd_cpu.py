"""HEVD on the CPU: the synthetic ring-0 snapshot (SYSCALL / SWAPGS / SYSRETQ,
supervisor pages, ExGenRandom's rdrand), the hevd module and the batched
runner, driven through the oracle twin (no GPU). Each crafted input must end
the way the reference module classifies it (fuzzer_hevd.cc:64-139)."""
import os

import pytest

from tests import tlv_harness as H
from tests.hevd_inputs import write_inputs
from wtf_amd.tools.snapshot import read_kdmp

pytestmark = pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")


@pytest.fixture(scope="module")
def target(tmp_path_factory):
    return H.build_hevd_target(str(tmp_path_factory.mktemp("hevd")))


def _run(target, d, out, lanes=16):
    return {r["input"]: r for r in H.run(H.TWIN, target, d, out, lanes=lanes, name="hevd")}


def test_snapshot_layout(target):
    index, _, cr3 = read_kdmp(os.path.join(target, "state", "mem.dmp"))
    assert cr3 and len(index) > 20


def test_seeds_return_to_user_mode(target, tmp_path):
    res = _run(target, os.path.join(target, "inputs"), str(tmp_path / "r.jsonl"))
    assert all(r["result"] == "ok" for r in res.values()), res
    # every seed went through the kernel (syscall ... sysretq) and stopped
    # after the 6-byte call, back in ring 3 with the caller's stack
    rips = {r["gprs"][16] for r in res.values()}
    assert len(rips) == 1
    assert all(r["icount"] > 40 for r in res.values())


def test_crafted_bug_classes(target, tmp_path):
    d = str(tmp_path / "in")
    write_inputs(d, 0)
    res = _run(target, d, str(tmp_path / "r.jsonl"))
    assert res["stack_gs_cookie"]["crash"].startswith("crash-0xf7-")           # DRIVER_OVERRAN_STACK_BUFFER
    # a user-address fault inside __try: KiPageFault resumes the handler through
    # IRETQ, which returns STATUS_ACCESS_VIOLATION to user mode
    assert res["write_what_where_user_fault"]["result"] == "ok"
    assert res["write_what_where_user_fault"]["gprs"][0] == 0xC0000005
    assert res["integer_wrap"]["crash"].startswith("crash-0xf7-")
    assert res["pool_overflow"]["crash"].startswith("crash-0x19-0x21-")        # BAD_POOL_HEADER
    assert res["wait_swapcontext"]["result"] == "cr3"                          # nt!SwapContext
    # ring-0 faults are named as the bugcheck the kernel raises
    assert res["stack_ret_overrun"]["crash"] == "crash-0x1e-0xc0000005-0x4242424242424242-0x0-0x0-0x0"
    assert res["null_deref"]["crash"].startswith("crash-0x50-0x8-0x0-0xfffff800")      # read of NULL->Callback
    assert res["write_what_where_bad"]["crash"].startswith("crash-0x50-0xffff800000000000-0x2-")
    assert res["write_what_where_ok"]["result"] == "ok"
    assert res["integer_ok"]["result"] == "ok"
    assert res["too_long"]["crash"] == "insert-testcase-failed"               # > 1024 bytes: InsertTestcase fails
    assert not any(r["error"] for r in res.values())


def test_kernel_faults_delivered_through_idt(target, tmp_path):
    """Ring-0 faults go through the guest IDT (U18): the #PF / #GP handlers run
    (their rips are covered) and the bugcheck comes from nt!KeBugCheck2."""
    import json
    d = str(tmp_path / "in")
    write_inputs(d, 0)
    res = _run(target, d, str(tmp_path / "r.jsonl"))
    sym = {k: int(v, 16) for k, v in json.load(open(os.path.join(target, "state", "symbol-store.json"))).items()}
    assert sym["nt!KiPageFault"] in res["null_deref"]["coverage"]
    assert sym["nt!KiGeneralProtectionFault"] in res["stack_ret_overrun"]["coverage"]
    assert sym["nt!KeBugCheck2"] in res["null_deref"]["coverage"]


def test_batch_size_does_not_change_results(target, tmp_path):
    d = str(tmp_path / "in")
    write_inputs(d, 150)
    a = H.run(H.TWIN, target, d, str(tmp_path / "a.jsonl"), lanes=1, name="hevd")
    b = H.run(H.TWIN, target, d, str(tmp_path / "b.jsonl"), lanes=64, name="hevd")
    assert a == b


def test_fuzz_default_mutator(target):
    st = H.fuzz(H.TWIN, target, runs=4000, lanes=512, name="hevd", max_len=1028)
    assert st["execs"] == 4000 and st["errors"] == 0
    assert st["unique_crashes"] >= 1 and st["coverage"] > 200


def test_parallel_mutation_is_deterministic(target, tmp_path):
    """Batches of >= 8192 new testcases are mutated in fixed chunks on the host
    threads (runner.cc MakeBatch): the corpus and crash set of a seed must not
    depend on the thread count."""
    import shutil
    import subprocess

    out = []
    for threads in ("1", "4"):
        d = str(tmp_path / f"t{threads}")
        shutil.copytree(target, d, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
        subprocess.run([H.TWIN, "fuzz", "--name", "hevd", "--target", d, "--runs", "24576", "--lanes", "8192",
                        "--seed", "7", "--limit", "100000", "--max_len", "1028"], check=True, capture_output=True,
                       timeout=600, env={**os.environ, "OMP_NUM_THREADS": threads})
        out.append((sorted(os.listdir(os.path.join(d, "outputs"))), sorted(os.listdir(os.path.join(d, "crashes")))))
    assert out[0] == out[1]
    assert len(out[0][0]) > 10


def test_dbgprintex_engine_error_path(target, tmp_path):
    """The HEVD leg's engine errors (U43): an input 1-2 bytes longer than
    TriggerBufferOverflowStack's frame (IOCTL 0x222003, no cookie) overwrites the
    low bytes of the saved return address, the `ret` lands on nt!DbgPrintEx's
    entry, and the module's handler reads a format pointer (r8) the guest never
    set, which does not translate: the reference would __debugbreak there
    (backend.cc:39-42); here the testcase ends as a handler fault.
    tests/golden/hevd_dbgprint_error.bin was kept by a twin HEVD campaign
    (all 21 errors of six 150 s campaigns were this IOCTL at 745-746 bytes)."""
    import shutil
    import struct

    d = tmp_path / "in"
    d.mkdir()
    src = os.path.join(os.path.dirname(__file__), "golden", "hevd_dbgprint_error.bin")
    shutil.copy(src, d / "err")
    data = open(src, "rb").read()
    assert struct.unpack_from("<I", data)[0] == 0x222003 and len(data) - 4 in (745, 746)
    res = _run(target, str(d), str(tmp_path / "r.jsonl"))
    r = res["err"]
    assert r["error"] and r["handler_fault"], r
    tr = tmp_path / "tr"
    H.run(H.TWIN, target, str(d), str(tmp_path / "r2.jsonl"), lanes=1, name="hevd",
          extra=("--trace-path", str(tr), "--trace-type", "rip"))
    rips = [int(x, 16) for x in open(tr / "err.trace").read().split()]
    import json
    sym = json.load(open(os.path.join(target, "state", "symbol-store.json")))
    assert rips[-1] == int(sym["nt!DbgPrintEx"], 16)                     # the last rip: the handler's
    # the rip before it is the driver's: TriggerBufferOverflowStack's own ret
    # (the look-alike links the driver into nt's image, right after nt!DbgPrintEx)
    from wtf_amd.tools import hevd
    ks = {k[7:]: v for k, v in hevd.build_space(str(tmp_path / "img"))[3].items() if k.startswith("kernel:")}
    f = ks["TriggerBufferOverflowStack"]
    end = min(v for v in ks.values() if v > f)
    assert f <= rips[-2] < end, (hex(rips[-2]), hex(f), hex(end))
