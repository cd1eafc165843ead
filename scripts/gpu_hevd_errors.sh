# HEVD fuzz campaign with regrouping; the testcases the engine could not finish are replayed on
# the GPU node and on the oracle twin (one lane at a time) to check they agree.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
python -c "
import sys; sys.path.insert(0,'.')
from tests import tlv_harness as H
H.build_hevd_target('/tmp/hevdt')
" || exit 1
timeout -k 10 120 ./wtf_amd/host/wtfgpu fuzz --name hevd --target /tmp/hevdt --lanes 65536 --seconds ${SECS:-10} --seed 1337 --limit 10000000 --max_len 1028 --regroup-steps ${RG:-256} > gpurun_out/he_fuzz.log 2>&1 || { tail -5 gpurun_out/he_fuzz.log; exit 1; }
grep '^{' gpurun_out/he_fuzz.log | tail -1 | cut -c1-400
n=$(ls /tmp/hevdt/errors 2>/dev/null | wc -l); echo "errors saved: $n"
[ "$n" -gt 0 ] || exit 0
mkdir -p gpurun_out/he_errors && cp /tmp/hevdt/errors/* gpurun_out/he_errors/
timeout -k 10 120 ./wtf_amd/host/wtfgpu run --name hevd --target /tmp/hevdt --input /tmp/hevdt/errors --results gpurun_out/he_err_gpu.jsonl --lanes 256 --limit 10000000 --full-coverage > gpurun_out/he_err_gpu.log 2>&1 || { tail -5 gpurun_out/he_err_gpu.log; exit 1; }
timeout -k 10 300 ./oracle/wtf_twin run --name hevd --target /tmp/hevdt --input /tmp/hevdt/errors --results gpurun_out/he_err_twin.jsonl --lanes 256 --limit 10000000 --full-coverage > gpurun_out/he_err_twin.log 2>&1 || { tail -5 gpurun_out/he_err_twin.log; exit 1; }
python - <<'PY'
import json
g=[json.loads(l) for l in open('gpurun_out/he_err_gpu.jsonl')]
t=[json.loads(l) for l in open('gpurun_out/he_err_twin.jsonl')]
bad=[(a['input'],k,a[k] if k!='coverage' else len(a[k]),b[k] if k!='coverage' else len(b[k])) for a,b in zip(g,t) for k in ('result','crash','error','icount','gprs','coverage') if a[k]!=b[k]]
print('replayed', len(g), 'gpu errors', sum(1 for a in g if a['error']), 'twin errors', sum(1 for b in t if b['error']), 'mismatches', len(bad), bad[:5])
PY
