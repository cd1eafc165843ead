# Headline leg only (no CPU baselines, no hevd / syn legs), twice, plus the HEVD node for 6 s.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-cpu --no-legs ${BENCH_ARGS:-} > gpurun_out/q$i.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/q$i.log; exit 1; }
  tail -1 gpurun_out/q$i.log > gpurun_out/q$i.json
done
python3 - <<'P'
import json
for i in (1, 2):
    d = json.load(open(f'gpurun_out/q{i}.json'))
    t = d['node_timed']; b = t['backend']
    print(round(d['value']), 'ms/step', round(d['ms_per_step'], 2), 'busy', round(d['kernel_busy_frac'], 3), 'cpu', round(d.get('host_cpu_frac', 0), 3))
    n = d['steps']
    print(' node', {k: round(v / n, 2) for k, v in t.items() if k.endswith('_ms')})
    print(' backend', {k: round(v / n, 2) for k, v in b.items() if k.endswith('_ms')})
P
if [ -n "${HEVD:-}" ]; then
  python -c "
from tests import tlv_harness as H
H.build_hevd_target('/tmp/hq')" || exit 1
  timeout -k 10 60 wtf_amd/host/wtfgpu fuzz --name hevd --target /tmp/hq --lanes 131072 --seconds 6 --seed 1337 --limit 10000000 --max_len 1028 > gpurun_out/hq.log 2>&1 || { echo HEVD_FAIL; tail -5 gpurun_out/hq.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/hq.log').read().strip().splitlines()[-1]); b=d['backend']
print('hevd', d['execs']/d['wall_s'], 'kernel busy', b['kernel_ms']/1e3/d['wall_s'])
print({k: v for k, v in d.items() if k.endswith('_ms')}); print({k: v for k, v in b.items() if k.endswith('_ms')})"
fi
