# Round 6: the AVX-512 GPU vectors first, then the GPU suite and one bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sse.py -k avx512 -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/pytest_avx512.txt 2>&1 || { echo AVX512_FAIL; tail -30 gpurun_out/pytest_avx512.txt; exit 1; }
tail -3 gpurun_out/pytest_avx512.txt
RUNS="${RUNS:-1}" bash scripts/gpu_r06_b.sh
