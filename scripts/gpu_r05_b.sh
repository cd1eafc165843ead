# Round 5: bench, then the whole GPU suite (one process, per-test timeouts).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash scripts/gpu_r05_bench.sh ${1:-b} || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05_${1:-b}_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/r05_${1:-b}_pytest.log; exit 1; }
tail -3 gpurun_out/r05_${1:-b}_pytest.log
