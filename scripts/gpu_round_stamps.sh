# GPU round (parity suite + tlv/hevd fuzz rates), then the tlv fuzz run on the per-phase stamps build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && bash scripts/gpu_round.sh || exit 1
LD_LIBRARY_PATH=$R/wtf_amd/csrc/stamps timeout -k 10 200 wtf_amd/host/wtfgpu fuzz --name tlv_server --target gpurun_out/tlv --runs 131072 --lanes 65536 --limit 100000 > gpurun_out/tlv_stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/tlv_stamps.log; exit 1; }
grep stamps gpurun_out/tlv_stamps.log | head -3
grep stamps gpurun_out/tlv_stamps.log | tail -3
