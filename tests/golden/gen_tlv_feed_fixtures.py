"""Generates tests/golden/tlv_feed_fixtures.json: tlv_server testcases (the
canonical JSON the tlv mutator writes, and hand-made variants the general JSON
parser decides: key order, whitespace, duplicates, missing keys, large /
negative / non-integer numbers, truncations, trailing bytes) with the packet
chunks the reference's InsertTestcase deserializes from each
(fuzzer_tlv_server.cc:36-40, 67-75, nlohmann::json), as printed by
oracle/_ref/ref_hostcheck tlv-feed (built from /root/reference by
oracle/Makefile). Run from the repository root:
    python tests/golden/gen_tlv_feed_fixtures.py
"""
import json
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def packet(rng, body_max):
    n = rng.choice([0, 1, 2, 3, rng.randint(0, body_max)])
    body = [rng.choice([rng.randint(0, 255), rng.randint(0, 9), rng.randint(10, 99)]) for _ in range(n)]
    return {"Body": body, "BodySize": rng.choice([n, rng.randint(0, 65535)]), "Command": rng.randint(0, 6),
            "Id": rng.randint(0, 65535)}


def canonical(pk):
    return json.dumps({"Packets": pk}, separators=(",", ":"), sort_keys=True).encode()


def cases(seed=2024):
    rng = random.Random(seed)
    out = [b'{"Packets":[]}']
    for _ in range(300):
        out.append(canonical([packet(rng, 48) for _ in range(rng.randint(1, 6))]))
    base = canonical([packet(rng, 6) for _ in range(2)])
    out += [base[:i] for i in range(0, len(base), 3)]  # truncations
    out += [base + b" ", base + b"x", b" " + base]
    hand = [
        b'{"Packets":[{"Id":7,"Command":1,"BodySize":2,"Body":[1,2]}]}',             # other key order
        b'{ "Packets" : [ { "Body" : [ 1 , 2 ] , "BodySize" : 2 , "Command" : 1 , "Id" : 3 } ] }',
        b'{"Packets":[{"Body":[1],"Body":[2],"BodySize":1,"Command":1,"Id":1}]}',   # duplicate key
        b'{"Packets":[{"Body":[1],"BodySize":1,"Command":1}]}',                    # missing key
        b'{"Packets":[{"Body":[1],"BodySize":1,"Command":1,"Id":1,"X":5}]}',        # extra key
        b'{"Packets":[{"Body":[256,300,65535,1000,4294967296],"BodySize":5,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[1234567890123456789],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[12345678901234567890],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[007],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[-1],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[1.5],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[1e2],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[1],"BodySize":70000,"Command":4294967297,"Id":65537}]}',
        b'{"Packets":[{"Body":[],"BodySize":0,"Command":0,"Id":0}]}',
        b'{"Packets":{}}',
        b'{"Packets":[{"Body":[1,],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[1 2],"BodySize":1,"Command":1,"Id":1}]}',
        b'{"Packets":[{"Body":[1],"BodySize":1,"Command":1,"Id":1}],"More":1}',
        b'{"Packets":[{"Body":[1],"BodySize":1,"Command":1,"Id":1}]}]',
        b'',
    ]
    return out + hand


def encode(tcs):
    return b"".join(len(t).to_bytes(4, "little") + t for t in tcs)


def feeds(exe, tcs):
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(encode(tcs))
        path = f.name
    try:
        out = subprocess.run([exe, "tlv-feed", path], check=True, capture_output=True, text=True).stdout
    finally:
        os.unlink(path)
    return [None if x == "F -" else x[2:] for x in out.splitlines()]


def main():
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_hostcheck")
    if not os.path.exists(exe):
        sys.exit("oracle/_ref/ref_hostcheck is not built (make -C oracle ref)")
    tcs = cases()
    got = feeds(exe, tcs)
    doc = {"source": "oracle/_ref/ref_hostcheck tlv-feed (reference fuzzer_tlv_server.cc Deserialize)",
           "cases": [{"tc": t.hex(), "feed": f} for t, f in zip(tcs, got)]}
    with open(os.path.join(HERE, "tlv_feed_fixtures.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print(len(tcs), "cases,", sum(1 for x in got if x is None), "rejected")


if __name__ == "__main__":
    main()
