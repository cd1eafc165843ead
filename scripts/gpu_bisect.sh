# One GPU test (TEST) against engine builds: the in-tree build and each
# abx/<variant> given, through LD_LIBRARY_PATH (wtfgpu's RUNPATH yields to it).
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = "." ]; then lp=""; else lp=$PWD/$v; fi
  LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 300 python -u -m pytest "$TEST" -x -q --timeout 240 --timeout-method thread > gpurun_out/bisect_$(echo $v | tr / _).txt 2>&1
  echo "== $v rc=$? $(tail -1 gpurun_out/bisect_$(echo $v | tr / _).txt)"
done
