# Default bench line (SYN + tlv leg + CPU baselines) and rocprofv3 kernel stats of the SYN bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/prof
timeout -k 10 500 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/stats -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-tlv > $R/gpurun_out/prof/bench_stats.log 2>&1 || { echo STATS_FAIL; tail -20 $R/gpurun_out/prof/bench_stats.log; exit 1; }
tail -1 $R/gpurun_out/prof/bench_stats.log
find $R/gpurun_out/prof/stats -name '*stats*'
