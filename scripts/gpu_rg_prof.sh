# rocprofv3 kernel stats of the tlv headline with and without cross-wave regrouping.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
for R in ${RG_LIST:-0 64}; do
  WTFGPU_REGROUP_STEPS=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rgprof_$R -o run -- python -u bench.py --steps 10 --warmup 2 --no-cpu --no-legs > gpurun_out/rgprof_$R.log 2>&1 || { echo PROF_FAIL $R; tail -20 gpurun_out/rgprof_$R.log; exit 1; }
  f=$(find gpurun_out/rgprof_$R -name '*kernel_stats.csv' | head -1)
  echo "R=$R"; head -12 "$f" | cut -c1-200
done
