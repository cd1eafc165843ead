# Occupancy probe: 64K lanes at 64 and 32 lanes per wave, 128K lanes at 64.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {  # lanes lpw
  WTFGPU_LPW=$2 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu --lanes $1 > gpurun_out/occ_$1_$2.log 2>&1 || { tail -5 gpurun_out/occ_$1_$2.log; exit 1; }
  echo "lanes=$1 lpw=$2"; tail -1 gpurun_out/occ_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ('value','instr_per_s','gpu_kernel_ms_per_step')})"
}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run 65536 64 && run 65536 32 && run 131072 64 && run 65536 16
