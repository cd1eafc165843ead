# Quick A/B of engine builds: op_cost.py timings (one line per form) for each
# library dir given ("." = the in-tree build), then SYN, then the tlv headline
# (gpu_ab.sh) unless QUICK is set, then the GPU suite on the in-tree build
# when TESTS is set.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/abq.txt; : > $out
for v in "$@"; do
  if [ "$v" = "." ]; then lib=$PWD/wtf_amd/csrc/libwtfgpu.so; else lib=$PWD/$v/libwtfgpu.so; fi
  d=gpurun_out/opc_$(echo $v | tr / _ | tr -d .); [ "$v" = "." ] && d=gpurun_out/opc_tree
  mkdir -p $d
  echo "== $v" | tee -a $out
  WTFGPU_LIB=$lib timeout -k 10 120 python3 -u scripts/op_cost.py $OPC_CASES > $d/times.jsonl 2> $d/times.err || { echo OPC_FAIL; tail $d/times.err; exit 1; }
  if [ -n "$PMC" ]; then
    (cd /tmp && export TMPDIR=/tmp && WTFGPU_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d /tmp/opcp -o opc -- python3 $GRAFT_REPO_ROOT/scripts/op_cost.py $OPC_CASES > $GRAFT_REPO_ROOT/$d/pmc.log 2>&1) || { echo PMC_FAIL; tail -5 $d/pmc.log; exit 1; }
    f=$(find /tmp/opcp -name '*counter_collection.csv' | head -1)
    grep k_run $f > $d/k_run_counters.csv; rm -rf /tmp/opcp
    python3 scripts/opc_summary.py $d | tee -a $out
  else
    python3 -c "
import json
for l in open('$d/times.jsonl'):
    d=json.loads(l); print(f\"{d['case']:10s} {d['ns_per_wave_step']:7.0f} ns/ws\")" | tee -a $out
  fi
done
specs=""; for v in "$@"; do specs="$specs $v:$v:"; done
if [ -z "$NOSYN" ]; then STEPS=8 bash scripts/syn_ab.sh $specs | tee -a $out || exit 1; fi
if [ -z "$QUICK" ]; then
  abspecs=""; for v in "$@"; do [ "$v" = "." ] && abspecs="$abspecs :262144" || abspecs="$abspecs $v:262144"; done
  bash scripts/gpu_ab.sh $abspecs > gpurun_out/ab_tlv.txt 2>&1 || { cat gpurun_out/ab_tlv.txt; exit 1; }
  cat gpurun_out/ab_tlv.txt | tee -a $out
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
  tail -3 gpurun_out/pytest_gpu.txt; exit $rc
fi
