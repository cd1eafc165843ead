# Round 6: environment A/B of bench.py (BENCH_ARGS, default --no-cpu --no-legs,
# 120 timed steps): HOSTVARS is a list of name=ENV1=v1,ENV2=v2 entries ('-' = none),
# each run twice in opposite orders; results under gpurun_out/hab.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/hab
set -- $HOSTVARS
order="$* $(echo "$@" | tr ' ' '\n' | tac | tr '\n' ' ')"
for v in $order; do
  name=${v%%=*}; envs=${v#*=}
  i=$(ls gpurun_out/hab | grep -c "^$name\.")
  ( [ "$envs" != "-" ] && for kv in $(echo $envs | tr ',' ' '); do export "$kv"; done
    timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-cpu --no-legs --steps 120} > gpurun_out/hab/$name.$i.log 2>&1 ) \
    || { echo "FAIL $name"; tail -20 gpurun_out/hab/$name.$i.log; exit 1; }
  tail -1 gpurun_out/hab/$name.$i.log > gpurun_out/hab/$name.$i.json
  echo "== $name ($envs)"; python3 scripts/bench_brief.py gpurun_out/hab/$name.$i.json | grep -v "node/step\|backend/step"
done
