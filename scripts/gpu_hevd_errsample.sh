# A 10 s HEVD leg on the GPU node; the first 300 engine-error testcases it kept
# come back under gpurun_out/hevd_errs/ for classification on the CPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/hevd_errs
python -c "
import sys; sys.path.insert(0,'.')
from tests import tlv_harness as H
H.build_hevd_target('/tmp/hevde')
" || exit 1
timeout -k 10 120 $R/wtf_amd/host/wtfgpu fuzz --name hevd --target /tmp/hevde --lanes 131072 --seconds 10 --seed 1337 --limit 10000000 --max_len 1028 > gpurun_out/hevd_errs/run.log 2>&1 || exit 1
ls /tmp/hevde/errors | head -300 | while read f; do cp /tmp/hevde/errors/$f gpurun_out/hevd_errs/; done
ls /tmp/hevde/errors | wc -l
