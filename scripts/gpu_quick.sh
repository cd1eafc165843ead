# Quick GPU iteration: parity tests, then a short bench (extra bench args via $BENCH_ARGS).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu $BENCH_ARGS > gpurun_out/bench_quick.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ('value','instr_per_s','ms_per_step','gpu_kernel_ms_per_step')}, d['roofline']['frac'])"
