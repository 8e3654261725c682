cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4.sh r4h "tests:tile or model or dp_exchange or dp_rccl or tensor_parallel" j3ab dpprof trace pmc
