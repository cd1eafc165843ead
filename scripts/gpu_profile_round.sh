# Round profile: parity tests, full bench (with CPU baseline), rocprofv3 kernel stats
# (CSV) and PMC HBM traffic passes for k_run, summarised into gpurun_out/prof/*.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/prof/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -20 gpurun_out/prof/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/prof/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/prof/bench.json.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/prof/bench.json.log; exit 1; }
tail -1 gpurun_out/prof/bench.json.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/stats -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/prof/bench_stats.log 2>&1 || { echo STATS_FAIL; tail -20 $R/gpurun_out/prof/bench_stats.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/prof/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; tail -20 $R/gpurun_out/prof/pmc_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/prof/pmc_write.log 2>&1 || { echo PMC2_FAIL; tail -20 $R/gpurun_out/prof/pmc_write.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/gpurun_out/prof/pmc_mix -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/prof/pmc_mix.log 2>&1 || { echo PMC3_FAIL; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/prof/pmc_wait -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/prof/pmc_wait.log 2>&1 || { echo PMC4_FAIL; exit 1; }
cd $R && python3 scripts/pmc_summary.py gpurun_out/prof > gpurun_out/prof/pmc_k_run.json && cat gpurun_out/prof/pmc_k_run.json
