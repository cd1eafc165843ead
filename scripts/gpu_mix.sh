# Instruction-mix PMC passes for k_run (one counter set per rocprofv3 run).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/mix
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SMEM SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $SET --output-format csv -d $R/gpurun_out/mix/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/mix/p$i.log 2>&1 || { echo PMC_FAIL $i; tail -20 $R/gpurun_out/mix/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv,collections,glob,os
R=os.environ['GRAFT_REPO_ROOT']
for f in sorted(glob.glob(R+'/gpurun_out/mix/p*/run_counter_collection.csv')):
    agg=collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if 'k_run' in r['Kernel_Name']: agg[r['Counter_Name']]+=float(r['Counter_Value'])
    print(dict(agg))
PY
