"""Host restatements vs the reference's own host code.

The gpu backend's host side restates pieces of wtf that sit on the hot path's
edges: the snapshot CPU-state loader (LoadCpuStateFromJSON / SanitizeCpuState,
src/wtf/utils.cc:57-258), the Rdrand BLAKE3 chain (bochscpu_backend.cc:874-885),
Blake3HexDigest (utils.cc:279-300), libFuzzer's MutationDispatcher behind
LibfuzzerMutator_t (mutator.cc:8-54; the hevd target's mutator, targets.h:25)
and the tlv_server CustomMutator_t (fuzzer_tlv_server.cc:204-365).

Each is checked, through oracle/hostcheck (oracle/hostcheck.cc over
libwtfhost.a), against
  * tests/golden/host_fixtures.json: outputs recorded from the same driver
    linked against the reference's sources (tests/golden/gen_host_fixtures.py);
  * the official BLAKE3 test vectors the reference vendors
    (tests/golden/blake3_vectors.json);
  * when present, the reference build itself (oracle/_ref/ref_hostcheck), live.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
from tests.cpu_bins import ALT, HOSTCHECK as TOOL  # noqa: E402
REF_TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_hostcheck")

FX = json.load(open(os.path.join(GOLD, "host_fixtures.json")))

# CpuState_t fields the checker prints (the sanitiser's diagnostics are not compared)
FIELDS = None


def _tool() -> str:
    if not ALT and not os.path.exists(TOOL):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "hostcheck"])
    return TOOL


def run(tool: str, *args: str) -> str:
    return subprocess.run([tool, *args], check=True, capture_output=True, text=True).stdout


def state_lines(out: str) -> list[str]:
    """The OK line and the field lines (anything else is a printed diagnostic)."""
    keep = []
    started = False
    for ln in out.splitlines():
        if ln.startswith("OK ") or ln == "LOAD_FAIL":
            started = True
        if started and ln and not ln.startswith("Setting") and " " in ln and ln.split()[0].replace(".", "").isalnum():
            keep.append(ln)
    return keep


@pytest.mark.parametrize("name", sorted(FX["cpustate"]))
def test_cpustate_matches_reference(name, tmp_path):
    case = FX["cpustate"][name]
    p = tmp_path / "regs.json"
    p.write_text(json.dumps(case["regs"]))
    ours = state_lines(run(_tool(), "cpustate", str(p)))
    assert ours == state_lines(case["out"])
    assert len(ours) > 60


def _corpus_files(tmp: str, name: str) -> list[str]:
    files = []
    for i, h in enumerate(FX["corpora"][name]):
        p = os.path.join(tmp, f"{name}_{i:02d}")
        with open(p, "wb") as f:
            f.write(bytes.fromhex(h))
        files.append(p)
    return files


def _mutate(tool: str, case: dict, files: list[str]) -> list[str]:
    out = run(tool, "mutate", case["mutator"], str(case["seed"]), str(case["maxlen"]), str(case["count"]),
              str(case["newcov_every"]), *files)
    return [ln[2:] for ln in out.splitlines() if ln.startswith("T ")]


@pytest.mark.parametrize("idx", range(len(FX["mutate"])), ids=[c["name"] for c in FX["mutate"]])
def test_mutator_stream_matches_reference(idx):
    """Bit-exact mutation streams for a seed: every output of `count`
    GetNewTestcase calls, OnNewCoverage feedback included."""
    case = FX["mutate"][idx]
    with tempfile.TemporaryDirectory() as d:
        outs = _mutate(_tool(), case, _corpus_files(d, case["corpus"]))
    assert outs[:len(case["full"])] == case["full"]
    got = [hashlib.sha256(bytes.fromhex(o)).hexdigest()[:32] for o in outs]
    first_bad = next((i for i, (a, b) in enumerate(zip(got, case["sha256"])) if a != b), None)
    assert first_bad is None, f"diverges at output {first_bad}"
    assert len(got) == case["count"]


def test_blake3_hexdigest_matches_reference():
    for c in FX["blake3"]:
        assert run(_tool(), "blake3", c["in"] or "-").strip() == c["digest"]


def test_blake3_official_vectors():
    """blake3_lite against BLAKE3's official vectors (hash mode, extended
    output): input = the repeating byte pattern 0..250."""
    doc = json.load(open(os.path.join(GOLD, "blake3_vectors.json")))
    for c in doc["cases"]:
        data = bytes(i % 251 for i in range(c["input_len"]))
        # long inputs go through the command line as hex: keep the cases that fit
        if c["input_len"] > 31744:
            continue
        out = run(_tool(), "xof", data.hex() or "-", str(len(c["hash"]) // 2)).strip()
        assert out == c["hash"], f"input_len {c['input_len']}"


def test_rdrand_chain_matches_reference_blake3():
    for seed, chain in FX["rdrand"].items():
        assert run(_tool(), "rdrand", seed, str(len(chain))).split() == chain


@pytest.mark.skipif(not os.path.exists(REF_TOOL), reason="reference build absent (oracle/_ref)")
def test_live_reference_agrees_with_fixtures():
    """The committed fixtures still match the reference build (when it exists)."""
    case = FX["mutate"][0]
    with tempfile.TemporaryDirectory() as d:
        outs = _mutate(REF_TOOL, dict(case, count=300), _corpus_files(d, case["corpus"]))
    assert [hashlib.sha256(bytes.fromhex(o)).hexdigest()[:32] for o in outs] == case["sha256"][:300]


ODD_TLV = [
    # the general parser's forms: whitespace, reordered keys, a leading zero
    b'{ "Packets" : [ {"Id":2,"Command":3,"BodySize":1,"Body":[7]} ] }',
    b'{"Packets":[{"Body":[1,2,300],"BodySize":070,"Command":1,"Id":1}]}',
    # no packets, one packet too many to insert into, a truncated testcase
    b'{"Packets":[]}',
    b'{"Packets":[' + b",".join(b'{"Body":[%d],"BodySize":1,"Command":%d,"Id":%d}' % (i, i, i)
                                for i in range(12)) + b']}',
    b'{"Packets":[{"Body":[65,65],"BodySize":2,"Command":0,"Id":0},{"Body":[6',
    b'not json at all',
]


@pytest.mark.parametrize("seed", [1, 1337, 0xC0FFEE])
def test_tlv_mutator_parsed_cache_matches_plain(seed, tmp_path):
    """The tlv mutator's fast path (corpus testcases parsed once, outputs
    written from packet references) gives the stream of the plain path, which
    parses and rewrites every pick as the reference does (the reference-pinned
    one above), over a corpus that grows as the campaign's does and holds
    testcases only the general parser reads."""
    files = _corpus_files(str(tmp_path), "tlv")
    for i, b in enumerate(ODD_TLV):
        p = tmp_path / f"odd_{i}"
        p.write_bytes(b)
        files.append(str(p))
    args = ["mutate-grow", "tlv_server", str(seed), "4096", "6000", "7", *files]
    fast = run(_tool(), *args)
    plain = subprocess.run([_tool(), *args], check=True, capture_output=True, text=True,
                           env={**os.environ, "WTF_TLV_MUTATOR_PLAIN": "1"}).stdout
    assert fast.count("\n") == 6000
    assert fast == plain
