# Round 4: stamps of the current build, then an A/B of engine builds (no suite).
#   scripts/gpu_r04z.sh "<ab specs ...>"
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
STAMPLIB=exp/stamps timeout -k 10 300 bash scripts/gpu_stamps.sh || { echo STAMPS_FAIL; exit 1; }
[ -n "$1" ] && timeout -k 10 700 bash scripts/gpu_ab.sh $1
exit 0
