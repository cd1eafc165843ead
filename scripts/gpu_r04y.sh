# Round 4: a new k_run step loop, checked in stages: smoke + the tlv / HEVD
# parity files first (short limits), then the whole suite + bench, stamps and
# an A/B of engine builds (scripts/gpu_ab.sh specs).
#   scripts/gpu_r04y.sh <tag> "<ab specs ...>"
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=$1; specs=$2
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${tag}_smoke.txt; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tlv.py tests/test_gpu_hevd.py > gpurun_out/${tag}_first.txt 2>&1
rc=$?; echo "first rc=$rc"; grep -E " passed| failed" gpurun_out/${tag}_first.txt | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${tag}_first.txt | head; exit $rc; }
bash scripts/gpu_r04.sh $tag tests; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
STAMPLIB=exp/stamps timeout -k 10 300 bash scripts/gpu_stamps.sh || { echo STAMPS_FAIL; exit 1; }
[ -n "$specs" ] && timeout -k 10 600 bash scripts/gpu_ab.sh $specs
exit 0
