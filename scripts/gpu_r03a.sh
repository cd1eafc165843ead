# Tenet GPU tests, then k_run PMC on tlv and the stamps build on tlv / HEVD.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_trace.py tests/test_tenet.py > gpurun_out/a_pytest.txt 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/a_pytest.txt
LEGS="tlv hevd" bash scripts/gpu_pmc.sh || exit 1
bash scripts/gpu_stamps.sh > gpurun_out/stamps_summary.txt 2>&1; echo "stamps rc=$?"; tail -40 gpurun_out/stamps_summary.txt
