# Full GPU parity suite, then TLV fuzz throughput of the gpu node at two batch sizes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
python -m wtf_amd.tools.tlv gpurun_out/tlv > /dev/null
for L in 16384 65536; do
  timeout -k 10 200 wtf_amd/host/wtfgpu fuzz --name tlv_server --target gpurun_out/tlv --runs $((L*8)) --lanes $L --limit 100000 > gpurun_out/tlv_fuzz_$L.log 2>&1 || { echo FUZZ_FAIL; tail -20 gpurun_out/tlv_fuzz_$L.log; exit 1; }
  tail -1 gpurun_out/tlv_fuzz_$L.log
done
