"""SYN leg under one engine setting (env), printed as one line: ms/step, lanes per wave-step, launches."""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

r = bench.syn_leg(65536, 100000, 10, 0)
print(json.dumps({"tag": sys.argv[1] if len(sys.argv) > 1 else "", "ms_per_step": round(r["ms_per_step"], 2),
                  "lpws": round(r["lanes_per_wave_step"], 2), "avg_launch_ms": round(r["roofline"]["avg_launch_ms"], 3),
                  "alg_per_launch": r["roofline"]["alg_bytes_per_launch"]}))
