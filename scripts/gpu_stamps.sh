set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
WTFGPU_LIB=$GRAFT_REPO_ROOT/wtf_amd/csrc/stamps/libwtfgpu.so timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu $BENCH_ARGS > gpurun_out/stamps.log 2>&1 || { tail -20 gpurun_out/stamps.log; exit 1; }
grep stamps gpurun_out/stamps.log | tail -2
