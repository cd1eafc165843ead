# Round record: the GPU test suite, then the default bench line (all legs, CPU baselines).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/rec_pytest.txt 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/rec_pytest.txt
timeout -k 10 600 python -u bench.py > gpurun_out/rec_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/rec_bench.log; exit 1; }
tail -1 gpurun_out/rec_bench.log > gpurun_out/rec_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/rec_bench.json'))
print('tlv', round(d['value']), 'cpu', d.get('cpu_baseline',{}).get('value'), 'vs_cpu', d.get('vs_cpu'), 'roof', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
for k in ('hevd','syn'):
    x=d[k]; print(k, round(x['value']), 'cpu', (x.get('cpu_baseline') or {}).get('value'), 'vs_cpu', x.get('vs_cpu'), 'lpws', x.get('lanes_per_wave_step'))"
