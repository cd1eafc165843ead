set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_quick.sh || exit 1
for L in 64 16; do
  WTFGPU_LPW=$L timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/lpw_$L.log 2>&1 || { tail -5 gpurun_out/lpw_$L.log; exit 1; }
  echo "lpw=$L"; tail -1 gpurun_out/lpw_$L.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ('value','instr_per_s','gpu_kernel_ms_per_step')})"
done
