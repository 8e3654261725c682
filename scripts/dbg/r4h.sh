cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4.sh r4h "tests:g0_lds or tile or model or dp_exchange or dp_rccl or tensor_parallel" g0ldsab j3ab dpprof rehearse trace pmc
