# Throughput exploration: bench.py variants (no CPU baselines), one JSON summary line each.
#   scripts/gpu_explore.sh <name>:<lanes>[:ENV=V,...] ...
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for spec in "$@"; do
  IFS=: read -r name lanes envs <<< "$spec"
  envargs=(); [ -n "$envs" ] && IFS=, read -ra envargs <<< "$envs"
  env "${envargs[@]}" timeout -k 10 400 python -u bench.py --no-cpu --steps 30 --warmup 4 --lanes "$lanes" > gpurun_out/x_$name.log 2>&1 || { echo "$name FAILED rc=$?"; tail -5 gpurun_out/x_$name.log; exit 1; }
  tail -1 gpurun_out/x_$name.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
def f(x): return 'cpu=%.2f ' % x.get('host_cpu_frac', -1) + 'v=%.0f busy=%.2f frac=%.4f lpws=%.1f avg_ms=%.2f' % (x['value'], x.get('kernel_busy_frac',0), x['roofline']['frac'], x['lanes_per_wave_step'], x['roofline']['avg_launch_ms'])
print('$name', 'tlv', f(d), '| hevd', f(d['hevd']) if 'hevd' in d else '', '| syn %.0f %.1fms lpws %.1f' % (d['syn']['value'], d['syn']['ms_per_step'], d['syn']['lanes_per_wave_step']) if 'syn' in d else '')"
done
