# Per-lane coverage sets + cross-wave regrouping: GPU parity suite, then the
# tlv headline / hevd fuzz with several regroup chunk sizes.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -z "$QUICK" ]; then
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/rg_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/rg_pytest.log; exit 1; }
tail -3 gpurun_out/rg_pytest.log
fi
WTFGPU_REGROUP_STEPS=256 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tlv.py tests/test_gpu_hevd.py > gpurun_out/rg_pytest_rg.log 2>&1 || { echo PYTEST_RG_FAIL; tail -40 gpurun_out/rg_pytest_rg.log; exit 1; }
tail -3 gpurun_out/rg_pytest_rg.log
for R in ${RG_LIST:-0 64 256 1024}; do
  WTFGPU_REGROUP_STEPS=$R timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-legs > gpurun_out/rg_bench_$R.log 2>&1 || { echo BENCH_FAIL $R; tail -20 gpurun_out/rg_bench_$R.log; exit 1; }
  echo "R=$R"; tail -1 gpurun_out/rg_bench_$R.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); n=d['node']; print(d['value'], d['ms_per_step'], d.get('lanes_per_wave_step'), n['kernel_ms'], n['kernel_launches'], n['group_steps'])"
done
