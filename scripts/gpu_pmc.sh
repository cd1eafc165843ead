# rocprofv3 kernel stats + PMC passes (HBM fetch / write, instruction mix, wave cycles) of k_run on
# each workload (tlv node, hevd node binary, SYN batches), one counter group per run, summarised into
# gpurun_out/pmc/pmc_<leg>_k_run$TAG.json by scripts/pmc_summary.py (TAG: an optional suffix).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/pmc
python -c "
import sys; sys.path.insert(0,'.')
from tests import tlv_harness as H
H.build_hevd_io_target('/tmp/hevdp')
H.build_hevd_target('/tmp/hevdb')
" || exit 1
cd /tmp && export TMPDIR=/tmp
run() {  # leg pass-name timeout rocprof-args...
  local leg=$1 pass=$2 t=$3; shift 3
  local out=/tmp/pmc/$leg/$pass
  mkdir -p $out
  if [ $leg = hevd ] || [ $leg = hevd_bare ]; then
    local tgt=/tmp/hevdp; [ $leg = hevd_bare ] && tgt=/tmp/hevdb
    timeout -s KILL $t rocprofv3 "$@" --output-format csv -d $out -o run -- $R/wtf_amd/host/wtfgpu fuzz --name hevd --target $tgt --lanes 131072 --seconds ${HEVD_SECS:-10} --seed 1337 --limit 10000000 --max_len 1028 > $out.log 2>&1
  else
    timeout -s KILL $t rocprofv3 "$@" --output-format csv -d $out -o run -- python3 $R/scripts/prof_leg.py $leg ${STEPS:-20} > $out.log 2>&1
  fi
  local rc=$?
  [ $rc -eq 0 ] || { echo "FAIL $leg $pass rc=$rc"; tail -5 $out.log; exit 1; }
}
for leg in ${LEGS:-tlv hevd hevd_bare syn}; do
  # SYN's runs go to completion: after one probe of each schedule the run
  # policy keeps the fixed lane order (wtfgpu_ctx::nspi_sched), so every
  # profiled launch is measured in that steady state
  if [ $leg = syn ]; then export WTFGPU_REGROUP_STEPS=0; else unset WTFGPU_REGROUP_STEPS; fi
  run $leg stats 240 --kernel-trace --stats
  run $leg fetch 180 --pmc FETCH_SIZE
  run $leg write 180 --pmc WRITE_SIZE
  run $leg mix 180 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
  run $leg wait 180 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES
  cd $R && python3 scripts/pmc_summary.py /tmp/pmc/$leg $leg $([ $leg = syn ] && echo 65536 || ([ ${leg%_bare} = hevd ] && echo 131072 || echo 262144)) $([ ${leg%_bare} = hevd ] && echo 10000000 || echo 100000) > gpurun_out/pmc/pmc_${leg}_k_run${TAG}.json && cd /tmp || { echo SUMMARY_FAIL $leg; exit 1; }
  # the raw CSVs stay on the box (large); the kernel statistics and logs come back
  cp $(find /tmp/pmc/$leg/stats -name '*kernel_stats.csv' | head -1) $R/gpurun_out/pmc/${leg}_kernel_stats${TAG}.csv
  cp /tmp/pmc/$leg/stats.log $R/gpurun_out/pmc/${leg}_stats${TAG}.log
  rm -rf /tmp/pmc/$leg
  echo "== $leg$TAG"; python3 -c "import json; d=json.load(open('$R/gpurun_out/pmc/pmc_${leg}_k_run${TAG}.json')); print({k: d[k] for k in ('hbm_bytes_per_launch','hbm_write_bytes','valu_util','wait_frac','kernel_trace')})"
done
