# Focused GPU check: the named tests, then an HEVD fuzz window for the engine-error sample.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/focus_pytest.txt 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/focus_pytest.txt
python3 -c "
from tests import tlv_harness as H; H.build_hevd_target('gpurun_out/hv')" &&
timeout -k 10 300 wtf_amd/host/wtfgpu fuzz --name hevd --target gpurun_out/hv --runs 30000000 --lanes 131072 --seed 1337 --limit 10000000 --max_len 1028 > gpurun_out/focus_hevd.txt 2>&1; echo "hevd rc=$?"
rm -rf gpurun_out/hv
tail -1 gpurun_out/focus_hevd.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['backend']; print(d['execs'], d['errors'], b.get('unimpl_ops'), b.get('unimpl_raw'))"
