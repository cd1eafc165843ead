# Profile pass: kernel-trace stats (CSV) + PMC HBM traffic passes + lane-count sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/stats -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof/bench_stats.log 2>&1 || { echo STATS_FAIL; tail -20 $R/gpurun_out/prof/bench_stats.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/prof/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; tail -20 $R/gpurun_out/prof/pmc_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/prof/pmc_write.log 2>&1 || { echo PMC2_FAIL; tail -20 $R/gpurun_out/prof/pmc_write.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --output-format csv -d $R/gpurun_out/prof/pmc_sq -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/prof/pmc_sq.log 2>&1 || { echo PMC3_FAIL; tail -20 $R/gpurun_out/prof/pmc_sq.log; exit 1; }
cd $R
for L in 131072 262144; do
  timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu --lanes $L > gpurun_out/prof/lanes_$L.log 2>&1 || { echo LANES_FAIL $L; tail -20 gpurun_out/prof/lanes_$L.log; exit 1; }
done
find gpurun_out/prof -name '*.csv' | head -30
