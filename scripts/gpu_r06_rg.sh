# Round 6: regroup launch length on the GPU-bound node (host plumbing async):
# bench.py --no-cpu (tlv headline + hevd / hevd_bare / syn legs) per
# --regroup-steps value given (-1 = the engine default, 1024).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/rg
for rg in "$@"; do
  timeout -k 10 300 python -u bench.py --no-cpu --regroup-steps $rg $BENCH_ARGS > gpurun_out/rg/b_$rg.log 2>&1 || { echo BENCH_FAIL $rg; tail -20 gpurun_out/rg/b_$rg.log; exit 1; }
  tail -1 gpurun_out/rg/b_$rg.log > gpurun_out/rg/b_$rg.json
  echo "== regroup $rg"; python3 scripts/bench_brief.py gpurun_out/rg/b_$rg.json
done
