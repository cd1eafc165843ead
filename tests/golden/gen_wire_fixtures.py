"""Record the reference's wire messages (yas binary, no header; socket.h:124,
server.h:720-737, client.cc:187-200) from its own headers compiled where they
lie (oracle/_ref/ref_hostcheck: yas + socket.h's Gva_t / robin_set / result
serializers). Inputs and outputs are stored as hex. Run here (the reference
tree is needed):
    python tests/golden/gen_wire_fixtures.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_TOOL = os.path.join(ROOT, "oracle", "_ref", "ref_hostcheck")
OUT = os.path.join(HERE, "wire_fixtures.json")

# (testcase hex, result index, crash name, coverage rips)
RESULTS = [
    ("", 0, "-", []),
    ("41", 1, "-", []),
    ("00ff7f", 2, "-", [0x140001000]),
    ("7b2274797065223a31327d", 3, "crash-EXCEPTION_ACCESS_VIOLATION_WRITE-0x140001234", [0x140001234]),
    ("deadbeef" * 64, 3, "-", [0xFFFFF80000100610]),
    ("0322200041414141", 3, "crash-0x1e-0xc0000005-0x4242424242424242-0x0-0x0-0x0",
     [0x140001000, 0x140001003, 0xFFFFF80000100A60, 0x7FF000000000]),
]


def run(*args):
    return subprocess.run([REF_TOOL, *args], check=True, capture_output=True, text=True).stdout


def main():
    doc = {"tool": "oracle/_ref/ref_hostcheck", "testcases": [], "results": []}
    for tc in ["", "41", "00" * 300, bytes(range(256)).hex()]:
        doc["testcases"].append({"in": tc, "msg": run("wire-testcase", tc or "-").strip()})
    for tc, idx, name, cov in RESULTS:
        msg = run("wire-result", tc or "-", str(idx), name, *[hex(c) for c in cov]).strip()
        dec = run("wire-decode", msg).splitlines()
        doc["results"].append({"tc": tc, "idx": idx, "name": name, "cov": cov, "msg": msg, "decoded": dec})
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
