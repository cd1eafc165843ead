# Round record: GPU suite, the default bench line (all legs, CPU baselines), then PMC of k_run on tlv / hevd.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/c_pytest.txt 2>&1; echo "pytest rc=$?"; grep -E "FAILED|ERROR" gpurun_out/c_pytest.txt | head; tail -1 gpurun_out/c_pytest.txt
timeout -k 10 500 python -u bench.py > gpurun_out/c_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/c_bench.log; exit 1; }
tail -1 gpurun_out/c_bench.log > gpurun_out/c_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/c_bench.json'))
print('tlv', round(d['value']), 'cpu', d.get('cpu_baseline',{}).get('value'), 'busy', round(d['kernel_busy_frac'],3), 'roof', d['roofline'])
for k in ('hevd','syn'):
    x=d[k]; print(k, round(x['value']), 'vs_cpu', x.get('vs_cpu'), 'lpws', x.get('lanes_per_wave_step'), 'err', x.get('errors'))"
LEGS="tlv hevd" STEPS=12 HEVD_SECS=3 bash scripts/gpu_pmc.sh
