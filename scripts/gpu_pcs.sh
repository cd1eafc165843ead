# Stochastic PC sampling of k_run on the tlv fuzz workload (build with line
# tables in exp/pcs), for the stall map of the step loop.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
python -c "
from tests import tlv_harness as H
H.build_target('/tmp/pc_tlv')" || exit 1
export TMPDIR=/tmp
LD_LIBRARY_PATH=$PWD/exp/pcs timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-stochastic} --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-1048576} -d $PWD/gpurun_out/pcs -o pcs --output-format csv -- $PWD/wtf_amd/host/wtfgpu fuzz --name tlv_server --target /tmp/pc_tlv --lanes 131072 --seconds 3 --seed 1337 --limit 100000 --max_len 4096 > gpurun_out/pcs_run.log 2>&1
rc=$?; echo "pcs rc=$rc"; tail -5 gpurun_out/pcs_run.log; find gpurun_out/pcs -type f | head; exit $rc
