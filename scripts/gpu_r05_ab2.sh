# A/B of an engine variant (abx/$V) against the in-tree build: SYN, the tlv
# headline and HEVD, then the GPU suite on the in-tree build.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=${V:-base}
STEPS=8 bash scripts/syn_ab.sh "$V:abx/$V:" "tree:.:" || exit 1
bash scripts/gpu_ab.sh "abx/$V:262144" ":262144" > gpurun_out/ab2.txt 2>&1 || { cat gpurun_out/ab2.txt; exit 1; }
cat gpurun_out/ab2.txt
[ -n "$NOTEST" ] && exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.txt; exit $rc
