# SYN leg under several regrouping settings (scripts/syn_probe.py prints one line each).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/syn_probe.py default &&
WTFGPU_REGROUP_STEPS=0 timeout -k 10 120 python -u scripts/syn_probe.py regroup0 &&
WTFGPU_REGROUP_AUTO=0 timeout -k 10 120 python -u scripts/syn_probe.py auto0_1024 &&
WTFGPU_REGROUP_AUTO=0 WTFGPU_REGROUP_STEPS=4096 timeout -k 10 120 python -u scripts/syn_probe.py auto0_4096 &&
WTFGPU_REGROUP_AUTO=0 WTFGPU_REGROUP_STEPS=16384 timeout -k 10 120 python -u scripts/syn_probe.py auto0_16384
