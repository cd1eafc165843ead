# Round 6: the GPU suite, then bench.py without the CPU legs (tlv headline,
# HEVD and SYN legs) twice; one summary line per run.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
fi
for i in ${RUNS:-1 2}; do
  timeout -k 10 300 python -u bench.py --no-cpu $BENCH_ARGS > gpurun_out/bench_$i.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$i.log; exit 1; }
  tail -1 gpurun_out/bench_$i.log > gpurun_out/bench_$i.json
  python3 scripts/bench_brief.py gpurun_out/bench_$i.json
done
