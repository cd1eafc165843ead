# Round 6, first GPU call: the forced world-1 RCCL merge test, then an
# occupancy A/B (in-tree build vs abx/<variant> libraries) on SYN and the
# tlv headline + HEVD (gpu_ab.sh). Usage: scripts/gpu_r06_a.sh variant...
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_rccl.txt 2>&1 || { tail -40 gpurun_out/pytest_rccl.txt; exit 1; }
tail -4 gpurun_out/pytest_rccl.txt
specs="base:.:"; for v in "$@"; do specs="$specs $v:abx/$v:"; done
STEPS=8 bash scripts/syn_ab.sh $specs || exit 1
abspecs=":262144"; for v in "$@"; do abspecs="$abspecs abx/$v:262144"; done; abspecs="$abspecs $EXTRA_AB"
bash scripts/gpu_ab.sh $abspecs > gpurun_out/ab_tlv.txt 2>&1 || { cat gpurun_out/ab_tlv.txt; exit 1; }
cat gpurun_out/ab_tlv.txt
