#!/bin/bash
# rocprofv3 kernel stats of one wtfgpu fuzz run on the synthetic tlv_server
# snapshot (the bench.py tlv leg: 64K lanes, 6 batches, seed 1337). GPU box only.
set -euo pipefail
cd "$(dirname "$0")/.."
T=gpurun_out/tlvt
rm -rf "$T" && mkdir -p "$T"
python3 -c "
import wtf_amd.tools.tlv as m
m.build('$T/state', '$T/work'); m.seed_inputs('$T/inputs')"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tlv -o tlv -- \
  wtf_amd/host/wtfgpu fuzz --name tlv_server --target "$T" --lanes 65536 --runs 393216 --seed 1337 \
  --limit 100000 --max_len 4096 > gpurun_out/prof_tlv.log 2>&1
rm -rf "$T"
