# Round 6, ADVICE (inline actions): the SetGprs + StopOk test and the tlv
# parity tests against the in-tree build and three A/B builds:
#   abx/nest    the nested action block, -structurizecfg-skip-uniform-regions=1
#   abx/nestnu  the nested action block, without that option
#   abx/nu      the split blocks (in-tree source), without that option
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for lib in "" abx/nest abx/nestnu abx/nu; do
  tag=${lib:-intree}; tag=${tag//\//_}
  if [ -n "$lib" ]; then export LD_LIBRARY_PATH=$PWD/$lib WTFGPU_LIB=$PWD/$lib/libwtfgpu.so; else unset LD_LIBRARY_PATH WTFGPU_LIB; fi
  timeout -k 10 400 python -u -m pytest tests/test_gpu_actions.py "tests/test_gpu_tlv.py::test_tlv_full_coverage_parity" \
    "tests/test_gpu_tlv.py::test_tlv_streaming_parity" -q --timeout 300 --timeout-method thread > gpurun_out/act_$tag.txt 2>&1
  rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/act_$tag.txt)"
  grep -E "^FAILED|lanes wrong" gpurun_out/act_$tag.txt | head -5
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit 1; fi
done
