#!/bin/bash
# A/B of the SYN leg (BASELINE.json configs[1]). Each spec is
# "name:lib dir:env"; lib dir "." is the in-tree build. Every leg is its own
# process with its own time limit.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/syn_ab.txt
: > "$out"
for spec in "$@"; do
  IFS=: read -r name lib envs <<< "$spec"
  echo "== $name ($lib, $envs)" | tee -a "$out"
  if [ "$lib" = "." ]; then libp=$PWD/wtf_amd/csrc/libwtfgpu.so; else libp=$PWD/$lib/libwtfgpu.so; fi
  timeout -k 10 240 env $envs WTFGPU_LIB=$libp python -u -c "
import json, bench
r = bench.syn_leg(65536, 100000, ${STEPS:-12}, 0)
print(json.dumps({k: r[k] for k in ('value', 'ms_per_step', 'lanes_per_wave_step')} | {'launch_ms': r['roofline'].get('avg_launch_ms'), 'frac': r['roofline'].get('frac')}))
" 2>&1 | grep -v "^wtfgpu stamps" | tee -a "$out" || exit 1
done
