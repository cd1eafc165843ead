cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/syn_probe.py default &&
WTFGPU_REGROUP_STEPS=0 timeout -k 10 120 python -u scripts/syn_probe.py regroup0 &&
WTFGPU_REGROUP_AUTO=0 timeout -k 10 120 python -u scripts/syn_probe.py auto0
