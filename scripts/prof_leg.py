"""One bench workload on its own, for rocprofv3 (scripts/gpu_pmc.sh): the tlv
node for a number of steps, or the SYN batches. (HEVD is profiled on the
wtfgpu binary directly.) Prints the workload's lanes / limit / k_run launches
as one JSON line."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    leg = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    limit = 100000
    lanes = 65536 if leg == "syn" else 262144  # bench.py's --syn-lanes / --lanes defaults
    if leg == "syn":
        s = bench.syn_leg(lanes, limit, steps, 0)
        # syn_leg's one untimed step: one launch in the fixed order (gpu_pmc.sh)
        print(json.dumps({"leg": "syn", "lanes": lanes, "limit": limit, "launches": s.get("launches"),
                          "warm_launches": 1, "value": s.get("value")}))
        return
    from wtf_amd import node as wn
    d = bench.build_target("tlv_server", tempfile.mkdtemp())
    n = wn.Node("tlv_server", d, lanes, limit, seed=1337, max_len=bench.TARGETS["tlv_server"][2])
    # bench.py's warm-up first: the summary leaves these launches out, as the
    # bench's timed window does (the cold start logs every new rip per lane)
    warm = int(os.environ.get("PROF_WARMUP", "6"))
    for _ in range(warm):
        n.step()
    warm_launches = n.stats()["kernel_launches"]
    for _ in range(steps):
        n.step()
    s = n.stats()
    print(json.dumps({"leg": "tlv", "lanes": lanes, "limit": limit, "launches": s["kernel_launches"],
                      "warm_launches": warm_launches, "execs": s["execs"]}))
    n.close()


if __name__ == "__main__":
    main()
