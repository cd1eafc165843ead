# Is the tlv headline host-bound? bench.py's tlv leg (--no-cpu --no-legs) at
# OMP_NUM_THREADS = 8 / 12 / 16 host threads, default regrouping and every
# 256 wave-steps: throughput that scales with the threads is host-bound.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/hb
for rg in -1 256; do for t in 8 12 16; do
  OMP_NUM_THREADS=$t timeout -k 10 240 python -u bench.py --no-cpu --no-legs --regroup-steps $rg > gpurun_out/hb/t${t}_rg$rg.log 2>&1 || { echo FAIL; tail -5 gpurun_out/hb/t${t}_rg$rg.log; exit 1; }
  tail -1 gpurun_out/hb/t${t}_rg$rg.log > gpurun_out/hb/t${t}_rg$rg.json
  python3 -c "
import json; d=json.load(open('gpurun_out/hb/t${t}_rg$rg.json')); r=d['roofline']
print('threads $t regroup $rg', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'busy', round(d['kernel_busy_frac'],3), 'host', round(d['host_cpu_frac'],3), 'launch_ms', round(r['avg_launch_ms'],3), 'lpws', round(d['lanes_per_wave_step'],1))"
done; done
