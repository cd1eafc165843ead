# rocprofv3 kernel stats of the gpu node fuzzing the synthetic tlv_server snapshot.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/tlvprof
python -m wtf_amd.tools.tlv gpurun_out/tlvt > /dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tlvprof/stats -o run -- $R/wtf_amd/host/wtfgpu fuzz --name tlv_server --target $R/gpurun_out/tlvt --runs 262144 --lanes 65536 --limit 100000 > $R/gpurun_out/tlvprof/fuzz.log 2>&1 || { echo PROF_FAIL; tail -20 $R/gpurun_out/tlvprof/fuzz.log; exit 1; }
grep '^{' $R/gpurun_out/tlvprof/fuzz.log | tail -1
cut -c1-160 $R/gpurun_out/tlvprof/stats/run_kernel_stats.csv
