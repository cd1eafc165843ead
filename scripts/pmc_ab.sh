cd $GRAFT_REPO_ROOT
LEGS=tlv TAG=_lds bash scripts/gpu_pmc.sh &&
LEGS=tlv TAG=_scr LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/wtf_amd/csrc/ab_scratch WTFGPU_LIB=$GRAFT_REPO_ROOT/wtf_amd/csrc/ab_scratch/libwtfgpu.so bash scripts/gpu_pmc.sh
