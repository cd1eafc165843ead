set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_ab.sh ":262144:0:1024" ":262144:0:512" ":262144:0:384" ":262144:0:256" > gpurun_out/ab1.txt 2>&1 || { cat gpurun_out/ab1.txt; exit 1; }
cat gpurun_out/ab1.txt
STEPS=8 bash scripts/syn_ab.sh "lpw64:.:WTFGPU_LPW=64" "lpw32:.:WTFGPU_LPW=32"
