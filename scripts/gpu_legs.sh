# Every bench leg (tlv headline, hevd, syn; no CPU baselines) at each regroup setting in $RG_LIST.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for R in ${RG_LIST:-0 256}; do
  WTFGPU_REGROUP_STEPS=$R timeout -k 10 400 python -u bench.py --no-cpu --regroup-steps $R --lanes ${LANES:-131072} > gpurun_out/legs_$R.log 2>&1 || { echo FAIL $R; tail -20 gpurun_out/legs_$R.log; exit 1; }
  tail -1 gpurun_out/legs_$R.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('R=$R tlv', round(d['value']), 'lpws', round(d['lanes_per_wave_step'],1))
for k in ('hevd','syn'):
    x=d.get(k) or {}
    b=x.get('backend') or {}
    print('   ', k, round(x.get('value',0)), x.get('unit'), 'lpws', round(x.get('lanes_per_wave_step',0),1), 'ipe', round(x.get('instr_per_exec',0)), 'errors', x.get('errors'), {kk: b.get(kk) for kk in ('kernel_ms','total_ms','breakpoint_hits','err_unimpl','err_overlay','err_other','last_unimpl_op','last_unimpl_rip','upload_ms','service_ms')})"
done
