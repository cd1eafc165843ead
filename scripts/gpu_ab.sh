# A/B of engine builds on the headline leg and the HEVD node: for each library directory given
# (empty string = the in-tree build), bench.py --no-cpu --no-legs twice, then HEVD for 6 s.
#   scripts/gpu_ab.sh "" variantlib/l2w2 variantlib/l2w2:262144 ...   (lib[:lanes])
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
python -c "
from tests import tlv_harness as H
H.build_hevd_target('/tmp/hab')" || exit 1
# spec = lib[:lanes[:slice[:regroup]]]
for spec in "$@"; do
  lib=${spec%%:*}; rest=${spec#*:}; [ "$rest" = "$spec" ] && rest=131072
  lanes=${rest%%:*}; rest2=${rest#*:}; [ "$rest2" = "$rest" ] && rest2=0
  slice=${rest2%%:*}; rg=${rest2#*:}; [ "$rg" = "$rest2" ] && rg=-1
  tag=$(echo "${lib:-default}_${lanes}_${slice}_$rg" | tr / _)
  for i in 1 2; do
    LD_LIBRARY_PATH=${lib:+$PWD/$lib} timeout -k 10 240 python -u bench.py --no-cpu --no-legs --lanes $lanes --slice-steps $slice --regroup-steps $rg > gpurun_out/ab_$tag.$i.log 2>&1 || { echo "BENCH_FAIL $tag"; tail -20 gpurun_out/ab_$tag.$i.log; exit 1; }
    tail -1 gpurun_out/ab_$tag.$i.log > gpurun_out/ab_$tag.$i.json
    python3 -c "
import json; d=json.load(open('gpurun_out/ab_$tag.$i.json')); r=d['roofline']
print('$tag', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'busy', round(d['kernel_busy_frac'],3), 'launch_ms', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],4), 'lpws', round(d['lanes_per_wave_step'],1))"
  done
  LD_LIBRARY_PATH=${lib:+$PWD/$lib} timeout -k 10 60 wtf_amd/host/wtfgpu fuzz --name hevd --target /tmp/hab --lanes $lanes $( [ $slice -gt 0 ] && echo --slice-steps $slice) $( [ $rg -ge 0 ] && echo --regroup-steps $rg) --seconds 6 --seed 1337 --limit 10000000 --max_len 1028 > gpurun_out/ab_hevd_$tag.log 2>&1 || { echo "HEVD_FAIL $tag"; tail -5 gpurun_out/ab_hevd_$tag.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab_hevd_$tag.log').read().strip().splitlines()[-1]); b=d['backend']
print('$tag hevd', round(d['execs']/d['wall_s']), 'kernel busy', round(b['kernel_ms']/1e3/d['wall_s'],3), 'launch ms', round(b['kernel_ms']/max(1,b['kernel_launches']),3), 'err', d['errors'])"
done
