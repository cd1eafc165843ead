"""Extract the official BLAKE3 test vectors (hash mode) that the reference tree
vendors at src/libs/BLAKE3/test_vectors/test_vectors.json into a small fixture:
input lengths and the expected extended hash. The input of each case is the
repeating byte pattern 0, 1, ..., 250 (documented in that file). Data only.
Re-run: python tests/golden/gen_blake3_vectors.py /root/reference"""
import json
import os
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
src = os.path.join(ref, "src/libs/BLAKE3/test_vectors/test_vectors.json")
doc = json.load(open(src))
out = {"source": "src/libs/BLAKE3/test_vectors/test_vectors.json (BLAKE3 1.2.0, vendored by the reference)",
       "cases": [{"input_len": c["input_len"], "hash": c["hash"]} for c in doc["cases"]]}
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "blake3_vectors.json")
json.dump(out, open(dst, "w"), indent=0)
print(f"{len(out['cases'])} cases -> {dst}")
