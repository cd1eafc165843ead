# The GPU parity suite (one pytest process, per-test timeouts), then bench.py variants via gpu_explore.sh.
#   scripts/gpu_check.sh "<pytest selection>" [explore specs...]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
sel=$1; shift
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $sel > gpurun_out/chk_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/chk_pytest.txt | tail -2
grep -E "FAILED|ERROR" gpurun_out/chk_pytest.txt | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ $# -gt 0 ] && bash scripts/gpu_explore.sh "$@"
exit 0
