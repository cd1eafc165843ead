# Round 5: the driver's bench command (no CPU baselines) + a condensed view.
# $1 = tag for the output files; extra bench args via $BENCH_ARGS.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-b}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu $BENCH_ARGS > gpurun_out/r05_$T.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r05_$T.log; exit 1; }
python3 scripts/bench_brief.py gpurun_out/r05_$T.log
