# Round 5, first GPU pass: bench (driver's shape), HEVD errors for replay, the new vector tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash scripts/gpu_r05_bench.sh a || exit 1
bash scripts/gpu_r05_hevd_errors.sh || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_sse.py -k "avx2x or ext or fp_vectors" > gpurun_out/r05_a_pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r05_a_pytest.log; exit 1; }
tail -2 gpurun_out/r05_a_pytest.log
