# Round 4: GPU suite + bench (gpu_r04.sh), stamps of the current build, then an
# A/B of engine build variants (scripts/gpu_ab.sh), in one call.
#   scripts/gpu_r04x.sh <tag> "<variant lib dirs ...>"
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=$1; variants=$2
bash scripts/gpu_r04.sh $tag tests; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
STAMPLIB=exp/stamps timeout -k 10 300 bash scripts/gpu_stamps.sh || { echo STAMPS_FAIL; exit 1; }
[ -n "$variants" ] && timeout -k 10 600 bash scripts/gpu_ab.sh "" $variants
exit 0
