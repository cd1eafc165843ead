# GPU round (parity suite + tlv/hevd fuzz rates) and a short SYN bench line (no CPU baselines).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash scripts/gpu_round.sh || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-tlv > gpurun_out/bench_syn.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench_syn.log; exit 1; }
tail -1 gpurun_out/bench_syn.log | cut -c1-400
grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/bench_syn.log
