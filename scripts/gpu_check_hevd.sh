# HEVD / node / wire GPU tests, then a short bench (no CPU baselines): device actions and the wire node.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hevd.py tests/test_refmods.py tests/test_gpu_node.py tests/test_wire.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/hevd_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/hevd_pytest.log; exit 1; }
tail -3 gpurun_out/hevd_pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_hevd.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench_hevd.log; exit 1; }
tail -1 gpurun_out/bench_hevd.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d['hevd']
print('tlv', round(d['value']), 'hevd', round(x['value']), 'ipe', round(x['instr_per_exec']), 'err', x['errors'], 'uc', x['unique_crashes'])
print(json.dumps(x['backend'])[:700])"
