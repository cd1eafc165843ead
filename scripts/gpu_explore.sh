# Throughput exploration: bench.py variants (no CPU baselines), one JSON summary line each.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python -u bench.py --no-cpu --steps 30 --warmup 4 "$@" > gpurun_out/x_$name.log 2>&1 || { echo "$name FAILED rc=$?"; tail -5 gpurun_out/x_$name.log; return 1; }
  tail -1 gpurun_out/x_$name.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
def f(x): return 'v=%.0f busy=%.2f frac=%.4f lpws=%.1f avg_ms=%.2f' % (x['value'], x.get('kernel_busy_frac',0), x['roofline']['frac'], x['lanes_per_wave_step'], x['roofline']['avg_launch_ms'])
print('$name', 'tlv', f(d), '| hevd', f(d['hevd']) if 'hevd' in d else '', '| syn %.0f %.1fms' % (d['syn']['value'], d['syn']['ms_per_step']) if 'syn' in d else '')"
}
run base A=1 -- "$@"
run l262k A=1 -- --lanes 262144 "$@"
run lpw32 WTFGPU_LPW=32 -- "$@"
