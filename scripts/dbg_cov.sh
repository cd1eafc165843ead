set -e
cd $GRAFT_REPO_ROOT
python - <<'PY'
import sys; sys.path.insert(0,'.')
from tests import tlv_harness as H
d=H.build_target('/tmp/tlvdbg')
PY
WTFGPU_DEBUG_COV=1 timeout -k 10 120 ./wtf_amd/host/wtfgpu fuzz --name tlv_server --target /tmp/tlvdbg --lanes 4096 --runs 40960 --seed 1337 > gpurun_out/dbg_cov.out 2> gpurun_out/dbg_cov.err
WTFGPU_DEBUG_COV=1 timeout -k 10 120 ./wtf_amd/host/wtfgpu fuzz --name tlv_server --target /tmp/tlvdbg --lanes 4096 --runs 40960 --seed 1337 --slice-steps 0 > gpurun_out/dbg_cov0.out 2> gpurun_out/dbg_cov0.err
