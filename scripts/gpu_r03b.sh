# GPU suite (one process, per-test timeouts), then the headline leg twice (host timing split).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/b_pytest.txt 2>&1; echo "pytest rc=$?"; grep -E "FAILED|ERROR" gpurun_out/b_pytest.txt | head; tail -2 gpurun_out/b_pytest.txt
bash scripts/gpu_tlvq.sh
