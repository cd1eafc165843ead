# The HEVD leg's engine errors (U43 handler faults), kept for replay on the twin:
# a 10 s `wtfgpu fuzz` at the leg's configuration; errors/ copied to gpurun_out.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
T=$(mktemp -d)
python3 -c "import sys; sys.path.insert(0,'.'); from tests import tlv_harness as H; H.build_hevd_target('$T')" || exit 1
timeout -k 10 120 wtf_amd/host/wtfgpu fuzz --name hevd --target $T --lanes 131072 --seconds 10 --seed 1337 \
  --limit 10000000 --max_len 1028 > gpurun_out/r05_hevd_fuzz.log 2>&1 || { echo FUZZ_FAIL; tail -20 gpurun_out/r05_hevd_fuzz.log; exit 1; }
tail -1 gpurun_out/r05_hevd_fuzz.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('execs', d['execs'], 'errors', d['errors'], 'handler', d['backend']['err_handler'])"
rm -rf gpurun_out/r05_hevd_errors && cp -r $T/errors gpurun_out/r05_hevd_errors && ls gpurun_out/r05_hevd_errors | wc -l
