# TLV on one MI355X: parity tests, then a fuzz throughput run of the gpu node.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tlv.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_tlv.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_tlv.log; exit 1; }
tail -5 gpurun_out/pytest_tlv.log
python -m wtf_amd.tools.tlv gpurun_out/tlv > /dev/null
for L in 16384 65536; do
  timeout -k 10 200 wtf_amd/host/wtfgpu fuzz --name tlv_server --target gpurun_out/tlv --runs $((L*8)) --lanes $L --limit 100000 > gpurun_out/tlv_fuzz_$L.log 2>&1 || { echo FUZZ_FAIL; tail -20 gpurun_out/tlv_fuzz_$L.log; exit 1; }
  tail -1 gpurun_out/tlv_fuzz_$L.log
done
