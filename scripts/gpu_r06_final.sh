# Round 6 close: the GPU suite, smoke(), then the default bench.py (CPU
# baselines included, as the driver runs it); results under gpurun_out/final.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/final/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/final/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/final/smoke.txt; exit 1; }
tail -1 gpurun_out/final/smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log > gpurun_out/final/bench.json
python3 scripts/bench_brief.py gpurun_out/final/bench.json
