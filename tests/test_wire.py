"""The master <-> node wire protocol (wtf_amd/host/wire.h,
remote.h).

1. The codec against the reference's own yas encoding (server.h:720-737,
   client.cc:187-200): fixtures recorded from oracle/_ref/ref_hostcheck
   (tests/golden/gen_wire_fixtures.py), and the live reference build when it
   is present (each side decodes the other's messages).
2. A master and two batched nodes (oracle twins) over TCP: the same corpus,
   crashes and execs as the in-process loop with the same total lanes (the
   master admits a testcase only when its own aggregate grows, server.h:816-854).
3. The reference protocol (one testcase per round trip) between the same
   master and nodes.
"""
import json
import os
import shutil
import socket
import subprocess
import time

import pytest

from tests import tlv_harness as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
from tests.cpu_bins import HOSTCHECK as TOOL  # noqa: E402
REF_TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_hostcheck")
FX = json.load(open(os.path.join(ROOT, "tests", "golden", "wire_fixtures.json")))


def run(tool, *args):
    return subprocess.run([tool, *args], check=True, capture_output=True, text=True).stdout


def test_testcase_message_matches_reference():
    for c in FX["testcases"]:
        assert run(TOOL, "wire-testcase", c["in"] or "-").strip() == c["msg"]


def test_result_message_matches_reference():
    for c in FX["results"]:
        args = [c["tc"] or "-", str(c["idx"]), c["name"], *[hex(v) for v in c["cov"]]]
        mine = run(TOOL, "wire-result", *args).strip()
        if len(c["cov"]) <= 1:  # a robin_set's iteration order is the reference's own: compare bytes up to one element
            assert mine == c["msg"], c
        assert run(TOOL, "wire-decode", c["msg"]).splitlines() == c["decoded"]  # the reference's bytes, decoded here
        assert run(TOOL, "wire-decode", mine).splitlines() == c["decoded"]


@pytest.mark.skipif(not os.path.exists(REF_TOOL), reason="reference build absent (oracle/_ref)")
def test_reference_decodes_our_messages():
    for c in FX["results"]:
        args = [c["tc"] or "-", str(c["idx"]), c["name"], *[hex(v) for v in c["cov"]]]
        mine = run(TOOL, "wire-result", *args).strip()
        assert run(REF_TOOL, "wire-decode", mine).splitlines() == c["decoded"]


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def tlv_target(tmp_path_factory):
    return H.build_target(str(tmp_path_factory.mktemp("tlvw")))


def fresh(target, dst):
    """A copy of the target with empty outputs / crashes."""
    shutil.copytree(target, dst, ignore=shutil.ignore_patterns("outputs", "crashes", "work"))
    return dst


def master_with_nodes(target, runs, lanes, batched, nodes=2):
    addr = f"tcp://127.0.0.1:{free_port()}"
    common = ["--name", "tlv_server", "--target", target, "--limit", "100000", "--max_len", "4096"]
    flag = ["--batched"] if batched else []
    m = subprocess.Popen([H.TWIN, "master", *common, "--address", addr, "--nodes", str(nodes), "--runs", str(runs),
                          "--seed", "1337", *flag], stdout=subprocess.PIPE, text=True)
    ns = []
    for _ in range(nodes):
        for _attempt in range(100):  # the master may not listen yet
            p = subprocess.Popen([H.TWIN, "fuzz", *common, "--address", addr, "--lanes", str(lanes), *flag],
                                 stdout=subprocess.PIPE, text=True)
            time.sleep(0.05)
            if p.poll() is None or p.returncode == 0:
                break
        ns.append(p)
    out, _ = m.communicate(timeout=600)
    assert m.returncode == 0, out
    node_out = [json.loads(p.communicate(timeout=60)[0].strip().splitlines()[-1]) for p in ns]
    return json.loads(out.strip().splitlines()[-1]), node_out


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_batched_master_and_two_nodes_equal_in_process(tlv_target, tmp_path):
    runs, lanes = 6000, 256
    a = fresh(tlv_target, str(tmp_path / "local"))
    local = H.fuzz(H.TWIN, a, runs=runs, lanes=2 * lanes, max_len=4096)
    b = fresh(tlv_target, str(tmp_path / "remote"))
    master, nodes = master_with_nodes(b, runs, lanes, batched=True)
    assert master["execs"] == local["execs"] == runs
    assert sum(n["execs"] for n in nodes) == runs
    assert master["backend"]["kind"] == "remote" and master["backend"]["nodes"] == 2
    assert master["batches"] == local["batches"]
    assert master["retired"] == local["retired"]
    assert sorted(os.listdir(os.path.join(b, "crashes"))) == sorted(os.listdir(os.path.join(a, "crashes")))
    assert sorted(os.listdir(os.path.join(b, "outputs"))) == sorted(os.listdir(os.path.join(a, "outputs")))
    assert master["crashes"] == local["crashes"] and master["corpus"] == local["corpus"]


@pytest.mark.skipif(not os.path.exists(H.TWIN), reason="oracle/wtf_twin not built")
def test_reference_protocol_master_and_nodes(tlv_target, tmp_path):
    """One testcase per round trip, the testcase echoed with its result: the
    protocol a reference client / master speaks."""
    runs = 400
    a = fresh(tlv_target, str(tmp_path / "local"))
    local = H.fuzz(H.TWIN, a, runs=runs, lanes=2, max_len=4096)
    b = fresh(tlv_target, str(tmp_path / "remote"))
    master, nodes = master_with_nodes(b, runs, 1, batched=False)
    assert master["execs"] == runs and sum(n["execs"] for n in nodes) == runs
    assert master["backend"]["batched"] == 0 and master["backend"]["frames"] == runs
    assert sorted(os.listdir(os.path.join(b, "crashes"))) == sorted(os.listdir(os.path.join(a, "crashes")))
    assert master["corpus"] == local["corpus"]


@pytest.mark.gpu
def test_gpu_node_behind_a_batched_master(tlv_target, tmp_path):
    """The product node (wtfgpu, one MI355X) serving a master over the batched
    protocol: the same results as its own in-process loop in batch mode."""
    runs, lanes = 8192, 4096
    common = ["--name", "tlv_server", "--limit", "100000", "--max_len", "4096"]
    a = fresh(tlv_target, str(tmp_path / "local"))
    local = H.fuzz(H.WTFGPU, a, runs=runs, lanes=lanes, max_len=4096, extra=["--slice-steps", "0"])
    b = fresh(tlv_target, str(tmp_path / "remote"))
    addr = f"tcp://127.0.0.1:{free_port()}"
    m = subprocess.Popen([H.TWIN, "master", *common, "--target", b, "--address", addr, "--nodes", "1",
                          "--runs", str(runs), "--seed", "1337", "--batched"], stdout=subprocess.PIPE, text=True)
    time.sleep(0.5)
    node = subprocess.run([H.WTFGPU, "fuzz", *common, "--target", b, "--address", addr, "--lanes", str(lanes),
                           "--batched"], capture_output=True, text=True, timeout=300)
    out, _ = m.communicate(timeout=300)
    assert m.returncode == 0 and node.returncode == 0, (out, node.stdout, node.stderr)
    master = json.loads(out.strip().splitlines()[-1])
    assert master["execs"] == local["execs"] == runs
    assert master["retired"] == local["retired"]
    assert sorted(os.listdir(os.path.join(b, "crashes"))) == sorted(os.listdir(os.path.join(a, "crashes")))
    assert sorted(os.listdir(os.path.join(b, "outputs"))) == sorted(os.listdir(os.path.join(a, "outputs")))
