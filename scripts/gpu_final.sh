# Round-end evidence: parity suite + fuzz rates, the default bench line, rocprofv3 kernel stats of the SYN bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash scripts/gpu_round.sh || exit 1
bash scripts/gpu_bench_prof.sh || exit 1
