"""Record reference outputs of the host logic the gpu backend restates, from the
reference's own sources compiled where they lie (oracle/_ref/ref_hostcheck,
recipe oracle/Makefile `ref`; driver oracle/hostcheck.cc):

  * LoadCpuStateFromJSON + SanitizeCpuState (src/wtf/utils.cc:57-258) on
    regs.json variants: the synthetic snapshots' states and edge cases
    (x87 "Infinity" strings, a segment attr that fails the sanitiser, user-mode
    cr8 / debug registers the sanitiser zeroes, a missing mxcsr_mask);
  * LibfuzzerMutator_t (src/wtf/mutator.cc:8-54 over libFuzzer's
    MutationDispatcher, src/libs/libfuzzer/FuzzerMutate.cpp) on the hevd seed
    corpus and on short binary corpora, with OnNewCoverage feedback;
  * the tlv_server CustomMutator_t (src/wtf/fuzzer_tlv_server.cc:204-365) on
    the tlv seed corpus;
  * Blake3HexDigest (src/wtf/utils.cc:279-300).

Inputs are stored in the fixture itself (data only); each mutator output is
kept as a sha256 of its bytes (the first few also in full) so the file stays
small. Run here (the reference tree is needed):
    python tests/golden/gen_host_fixtures.py
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

REF_TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_hostcheck")
OUT = os.path.join(HERE, "host_fixtures.json")


def regs_variants() -> dict[str, dict]:
    from wtf_amd.tools.snapshot import regs_json, seg, user_state

    base = user_state(0x140001000, 0x7FF0000FFF00, 0x1AB000, rcx=0x1234, rdx=0x1000, r15=0xFFFFFFFFFFFFFFFF)
    v = {"user": regs_json(base)}
    k = dict(base)
    k.update({"rip": 0xFFFFF80000101000, "rsp": 0xFFFFF80000F00000, "cr8": 2,
              "cs": seg(0x10, 0, 0, 0x209B), "ss": seg(0x18, 0, 0xFFFFFFFF, 0xC93)})
    v["kernel_cr8"] = regs_json(k)
    u = dict(base)
    u.update({"cr8": 0xF, "dr0": 0x1000, "dr7": 0x401, "dr6": 0xFFFF0FF0})
    v["user_cr8_dr"] = regs_json(u)
    f = regs_json(base)
    f["fpst"] = ["Infinity", "-Infinity", "0x3fff8000000000000000", "0x0", "0x1", "0x-Infinity", "Infinity",
                 "0xffffffffffffffff"]
    v["fpst_mixed"] = f
    m = regs_json(base)
    m["mxcsr_mask"] = "0x0"
    v["mxcsr_mask_zero"] = m
    b = regs_json(base)
    b["ds"] = dict(b["ds"], attr="0x4f3")  # attr bits 8-11 != (limit >> 16) & 0xf
    v["bad_attr"] = b
    n = regs_json(base)
    n["rax"] = "12345"  # decimal, strtoull base 0
    n["rbx"] = "0777"   # octal
    v["number_bases"] = n
    return v


def corpora() -> dict[str, list[bytes]]:
    from wtf_amd.tools import hevd, tlv

    with tempfile.TemporaryDirectory() as d:
        tl = [open(p, "rb").read() for p in tlv.seed_inputs(os.path.join(d, "tlv"))]
        hv = [open(p, "rb").read() for p in hevd.seed_inputs(os.path.join(d, "hevd"))]
    small = [b"", b"A", b"hello world 1234 5678", bytes(range(64)), b"\xff" * 9 + b"12" * 8]
    # the reference copies a pick into a max_len scratch buffer: picks must fit
    tiny = [b"", b"A", b"12345678", b"\x00\xff\x7f"]
    return {"tlv": tl, "hevd": hv, "small": small, "tiny": tiny}


# (name, mutator, seed, maxlen, count, newcov_every, corpus)
MUTATE_RUNS = [
    ("hevd_libfuzzer_1337", "libfuzzer", 1337, 1028, 4000, 97, "hevd"),
    ("hevd_libfuzzer_7", "libfuzzer", 7, 1028, 1000, 0, "hevd"),
    ("small_libfuzzer_max64", "libfuzzer", 99, 64, 4000, 13, "small"),
    ("tiny_libfuzzer_max8", "libfuzzer", 5, 8, 2000, 7, "tiny"),
    ("tlv_custom_1337", "tlv_server", 1337, 0x1000, 600, 0, "tlv"),
    ("tlv_custom_42", "tlv_server", 42, 0x1000, 600, 0, "tlv"),
]
KEEP_FULL = 8


def ref_rdrand_chain(seed: int, n: int) -> list[str]:
    """BochscpuBackend_t::Rdrand (bochscpu_backend.cc:874-885) over the
    reference's BLAKE3 (oracle/_ref/libblake3_ref.so, built from
    src/libs/BLAKE3/c): h = blake3(le64(seed))[0:16]; seed = h[0:8]; value = h[8:16]."""
    import ctypes as C

    lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libblake3_ref.so"))
    out = []
    for _ in range(n):
        hasher = C.create_string_buffer(4096)
        lib.blake3_hasher_init(hasher)
        lib.blake3_hasher_update(hasher, seed.to_bytes(8, "little"), C.c_size_t(8))
        h = C.create_string_buffer(16)
        lib.blake3_hasher_finalize(hasher, h, C.c_size_t(16))
        seed = int.from_bytes(h.raw[:8], "little")
        out.append("%016x" % int.from_bytes(h.raw[8:16], "little"))
    return out


def run_tool(tool: str, args: list[str]) -> str:
    return subprocess.run([tool, *args], check=True, capture_output=True, text=True).stdout


def mutate_outputs(tool: str, run, files: list[str]) -> list[str]:
    _, mut, seed, maxlen, count, every, _ = run
    out = run_tool(tool, ["mutate", mut, str(seed), str(maxlen), str(count), str(every), *files])
    return [ln[2:] for ln in out.splitlines() if ln.startswith("T ")]


def main():
    if not os.path.exists(REF_TOOL):
        raise SystemExit(f"{REF_TOOL} missing: run `make -C oracle ref` with /root/reference present")
    fx = {"generator": "tests/golden/gen_host_fixtures.py", "tool": "oracle/_ref/ref_hostcheck",
          "cpustate": {}, "corpora": {}, "mutate": [], "blake3": []}
    with tempfile.TemporaryDirectory() as d:
        for name, doc in regs_variants().items():
            p = os.path.join(d, name + ".json")
            json.dump(doc, open(p, "w"), indent=1)
            fx["cpustate"][name] = {"regs": doc, "out": run_tool(REF_TOOL, ["cpustate", p])}
        cps = corpora()
        files = {}
        for cname, items in cps.items():
            fx["corpora"][cname] = [x.hex() for x in items]
            files[cname] = []
            for i, x in enumerate(items):
                p = os.path.join(d, f"{cname}_{i:02d}")
                open(p, "wb").write(x)
                files[cname].append(p)
        for run in MUTATE_RUNS:
            outs = mutate_outputs(REF_TOOL, run, files[run[6]])
            fx["mutate"].append({"name": run[0], "mutator": run[1], "seed": run[2], "maxlen": run[3],
                                 "count": run[4], "newcov_every": run[5], "corpus": run[6],
                                 "sha256": [hashlib.sha256(bytes.fromhex(o)).hexdigest()[:32] for o in outs],
                                 "full": outs[:KEEP_FULL]})
    for data in [b"", b"\x00", bytes(range(251)) * 5, b"wtf"]:
        fx["blake3"].append({"in": data.hex(), "digest": run_tool(REF_TOOL, ["blake3", data.hex() or "-"]).strip()})
    fx["rdrand"] = {str(seed): ref_rdrand_chain(seed, 64) for seed in (0, 1, 0xDEADBEEFCAFEBABE)}
    json.dump(fx, open(OUT, "w"), indent=0)
    print(f"wrote {OUT}: {len(fx['cpustate'])} states, {len(fx['mutate'])} mutator runs")


if __name__ == "__main__":
    main()
