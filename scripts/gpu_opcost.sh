# op_cost.py on the GPU: plain timings, then the SQ instruction mix of each
# case (rocprofv3 --pmc, its own pass under its own time limit).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/opc
timeout -k 10 200 python3 -u scripts/op_cost.py > gpurun_out/opc/times.jsonl 2> gpurun_out/opc/times.err || { tail gpurun_out/opc/times.err; exit 1; }
cat gpurun_out/opc/times.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d /tmp/opc -o opc -- python3 $R/scripts/op_cost.py > $R/gpurun_out/opc/pmc.log 2>&1 || { echo PMC_FAIL; tail -5 $R/gpurun_out/opc/pmc.log; exit 1; }
f=$(find /tmp/opc -name '*counter_collection.csv' | head -1)
grep k_run $f > $R/gpurun_out/opc/k_run_counters.csv; head -1 $f > $R/gpurun_out/opc/header.csv
wc -l $R/gpurun_out/opc/k_run_counters.csv
