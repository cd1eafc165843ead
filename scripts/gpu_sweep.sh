# tlv headline sweep over lanes x regroup launch length x slice length ($SWEEP: "lanes:regroup:slice ...").
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in ${SWEEP:-65536:0:4096}; do
  IFS=: read L R S <<< "$cfg"
  log=gpurun_out/sw_${L}_${R}_${S}.log
  timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup 6 --no-cpu --no-legs --lanes $L --regroup-steps $R --slice-steps $S > $log 2>&1 || { echo FAIL $cfg; tail -20 $log; exit 1; }
  tail -1 $log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); n=d['node']; ns=d['node_timed']; b=ns['backend']
print('$cfg', round(d['value']), round(d['ms_per_step'],1), round(d.get('lanes_per_wave_step'),1), round(n['kernel_ms'],1), n['kernel_launches'], round(n['insert_ms'],1), round(n['node_ms'],1))
print('   timed ms:', {k: round(ns[k]) for k in ('make_ms','fill_ms','step_ms','account_ms','produce_wait_ms','run_s')}, {k: round(b[k]) for k in ('total_ms','insert_ms','restore_ms','module_ms','upload_ms','run_ms','kernel_ms','exits_ms','regs_ms','coverage_ms','covlog_ms','attrib_ms','target_restore_ms','bytes_ms')})"
done
