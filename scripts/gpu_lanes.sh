# tlv headline leg at several lane counts (no CPU baselines, no other legs).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for n in ${LANES:-262144 393216 524288}; do
  timeout -k 10 240 python -u bench.py --no-cpu --no-legs --lanes $n > gpurun_out/l$n.log 2>&1 || { echo BENCH_FAIL $n; tail -20 gpurun_out/l$n.log; exit 1; }
  tail -1 gpurun_out/l$n.log > gpurun_out/l$n.json
  python3 -c "
import json; d=json.load(open('gpurun_out/l$n.json'))
print($n, round(d['value']), 'ms/step', round(d['ms_per_step'], 2), 'busy', round(d['kernel_busy_frac'], 3), 'launch_ms', round(d['roofline']['avg_launch_ms'], 3))"
done
