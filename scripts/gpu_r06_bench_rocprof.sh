# Round 6: rocprofv3 kernel trace + stats of the bench command itself (the
# tlv headline, --no-legs --no-cpu); the kernel statistics come back
# to gpurun_out/benchprof.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/benchprof && cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bprof -o run -- python3 $R/bench.py --no-cpu --no-legs > $R/gpurun_out/benchprof/bench.log 2>&1 || { echo FAIL; tail -20 $R/gpurun_out/benchprof/bench.log; exit 1; }
cp $(find /tmp/bprof -name '*kernel_stats.csv' | head -1) $R/gpurun_out/benchprof/kernel_stats.csv
tail -1 $R/gpurun_out/benchprof/bench.log > $R/gpurun_out/benchprof/bench.json
head -5 $R/gpurun_out/benchprof/kernel_stats.csv
