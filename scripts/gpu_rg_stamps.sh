# Per-phase cycle stamps of k_run (diagnostic build) on the tlv node, with and without regrouping.
set -o pipefail
R0=$GRAFT_REPO_ROOT
cd $R0 && mkdir -p gpurun_out
python -m wtf_amd.tools.tlv gpurun_out/tlvt > /dev/null || exit 1
for R in ${RG_LIST:-0 64}; do
  LD_LIBRARY_PATH=$R0/wtf_amd/csrc/stamps WTFGPU_REGROUP_STEPS=$R timeout -k 10 200 $R0/wtf_amd/host/wtfgpu fuzz --name tlv_server --target $R0/gpurun_out/tlvt --runs 262144 --lanes 65536 --limit 100000 > gpurun_out/rgstamps_$R.log 2>&1 || { echo FAIL $R; tail -20 gpurun_out/rgstamps_$R.log; exit 1; }
  echo "R=$R $(grep -c stamps gpurun_out/rgstamps_$R.log) stamp lines"; grep '^{' gpurun_out/rgstamps_$R.log | tail -1 | cut -c1-300
done
