# TLV parity + fuzz rates, then the default bench line (SYN + tlv leg + CPU baselines).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash scripts/gpu_tlv.sh || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
