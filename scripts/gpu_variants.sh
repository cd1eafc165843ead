# Time k_run build variants (wtf_amd/csrc/variants/*) on the SYN bench, one process each.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for V in v11 v10 v21 v20; do
  WTFGPU_LIB=$GRAFT_REPO_ROOT/wtf_amd/csrc/variants/$V/libwtfgpu.so timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu $BENCH_ARGS > gpurun_out/var_$V.log 2>&1 || { tail -5 gpurun_out/var_$V.log; exit 1; }
  echo "$V"; tail -1 gpurun_out/var_$V.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:d[k] for k in ('value','gpu_kernel_ms_per_step')})"
done
