# Round 6 A/B: sequential prefetch on uop-cache fills and the fast loop after
# coverage logging (abp/<variant>),
# bench.py --no-cpu (tlv headline, HEVD I/O and bare, SYN), two passes in
# opposite orders.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abp
for v in ${VARIANTS:-pf0 pf2 pf4 pf4 pf2 pf0}; do
  export LD_LIBRARY_PATH=$PWD/abp/$v WTFGPU_LIB=$PWD/abp/$v/libwtfgpu.so
  i=$(ls gpurun_out/abp | grep -c "^$v\.") 
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/abp/$v.$i.log 2>&1 || { echo "FAIL $v"; tail -20 gpurun_out/abp/$v.$i.log; exit 1; }
  tail -1 gpurun_out/abp/$v.$i.log > gpurun_out/abp/$v.$i.json
  echo "== $v"; python3 scripts/bench_brief.py gpurun_out/abp/$v.$i.json | grep -v "node/step\|backend/step"
done
