# GPU test suite, then every bench leg without CPU baselines (one line per leg).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/q_pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/q_pytest.txt; exit 1; }
tail -1 gpurun_out/q_pytest.txt
RG_LIST=${RG_LIST:-1024} bash scripts/gpu_legs.sh
