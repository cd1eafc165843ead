# Per-phase cycle stamps of k_run on the SYN leg (diagnostic build in
# $STAMPLIB, default exp/stamps), fixed lane order and regrouped.
set -o pipefail
mkdir -p gpurun_out
for mode in ${MODES:-"WTFGPU_REGROUP_STEPS=0" "WTFGPU_REGROUP_AUTO=0"}; do
  echo "== $mode"
  timeout -k 10 180 env $mode WTFGPU_LIB=$PWD/${STAMPLIB:-exp/stamps}/libwtfgpu.so python -u -c "
import bench
r = bench.syn_leg(65536, 100000, 3, 0)
print({k: r[k] for k in ('value', 'ms_per_step', 'lanes_per_wave_step')})
" > gpurun_out/syn_stamps.log 2>&1 || exit 1
  python scripts/stamps_summary.py gpurun_out/syn_stamps.log || exit 1
  tail -1 gpurun_out/syn_stamps.log
done
