# Full GPU parity suite, then tlv_server and HEVD fuzz rates of the gpu node (64K lanes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
python -m wtf_amd.tools.tlv gpurun_out/tlv > /dev/null
timeout -k 10 200 wtf_amd/host/wtfgpu fuzz --name tlv_server --target gpurun_out/tlv --runs 524288 --lanes 65536 --limit 100000 > gpurun_out/tlv_fuzz.log 2>&1 || { echo FUZZ_FAIL; tail -20 gpurun_out/tlv_fuzz.log; exit 1; }
tail -1 gpurun_out/tlv_fuzz.log
python -m wtf_amd.tools.hevd gpurun_out/hevd > /dev/null
timeout -k 10 200 wtf_amd/host/wtfgpu fuzz --name hevd --target gpurun_out/hevd --runs 524288 --lanes 65536 --limit 100000 --max_len 1028 > gpurun_out/hevd_fuzz.log 2>&1 || { echo FUZZ_FAIL; tail -20 gpurun_out/hevd_fuzz.log; exit 1; }
tail -1 gpurun_out/hevd_fuzz.log
