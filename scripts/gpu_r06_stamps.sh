# Round 6: per-phase stamps and the generic-op histogram (stamps build,
# `make -C wtf_amd/csrc stamps`) on tlv and the HEVD I/O-manager look-alike.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
python -c "
from tests import tlv_harness as H
H.build_target('/tmp/st_tlv'); H.build_hevd_io_target('/tmp/st_hevd')" || exit 1
# ST: stamps builds under st6/<name> (one build: st6/ itself)
for v in ${ST:-.}; do
  export LD_LIBRARY_PATH=$PWD/st6/$v
  o=gpurun_out/stamps_$(basename $(realpath st6/$v))
  timeout -k 10 120 wtf_amd/host/wtfgpu fuzz --name tlv_server --target /tmp/st_tlv --lanes 131072 --seconds 4 --seed 1337 --limit 100000 --max_len 4096 > ${o}_tlv.log 2>&1 || exit 1
  timeout -k 10 120 wtf_amd/host/wtfgpu fuzz --name hevd --target /tmp/st_hevd --lanes 131072 --seconds 4 --seed 1337 --limit 10000000 --max_len 1028 > ${o}_hevd.log 2>&1 || exit 1
  python scripts/stamps_summary.py ${o}_tlv.log ${o}_hevd.log
done
