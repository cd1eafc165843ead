# Full GPU parity suite, k_run stamps with/without regrouping, then the tlv headline sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/rg_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/rg_pytest.log; exit 1; }
tail -2 gpurun_out/rg_pytest.log
bash scripts/gpu_rg_stamps.sh || exit 1
QUICK=1 bash scripts/gpu_regroup.sh
