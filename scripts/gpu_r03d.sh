# x87 (U42) on the GPU: its vectors first, then the whole GPU suite and the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sse.py -k x87 > gpurun_out/d_x87.txt 2>&1; rc=$?; tail -3 gpurun_out/d_x87.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/d_pytest.txt 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/d_pytest.txt | head; tail -1 gpurun_out/d_pytest.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u bench.py > gpurun_out/d_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/d_bench.log; exit 1; }
tail -1 gpurun_out/d_bench.log > gpurun_out/d_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/d_bench.json'))
print('tlv', round(d['value']), 'busy', round(d['kernel_busy_frac'],3), 'roof', d['roofline'])
for k in ('hevd','syn'):
    x=d[k]; print(k, round(x['value']), 'err', x.get('errors'), x.get('backend',{}).get('unimpl_ops'))"
