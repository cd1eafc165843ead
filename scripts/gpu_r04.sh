# Round 4: the GPU parity suite (one pytest process, per-test timeouts), then the default bench line.
#   scripts/gpu_r04.sh <tag> ["<pytest selection>"] [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=$1; sel=${2:-tests}; shift; [ $# -gt 0 ] && shift
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $sel > gpurun_out/${tag}_pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E " passed| failed" gpurun_out/${tag}_pytest.txt | tail -2
grep -E "FAILED|ERROR" gpurun_out/${tag}_pytest.txt | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "$1" = "nobench" ] && exit $rc
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log > gpurun_out/${tag}_bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_bench.json')); r=d['roofline']
print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'launch_ms', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],4), 'lpws', round(d['lanes_per_wave_step'],1), 'busy', d.get('kernel_busy_frac'))
for k in ('legs',):
  print(json.dumps(d.get(k))[:1500])"
exit $rc
