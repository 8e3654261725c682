cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4.sh r4e "tests:tensor_parallel_bf16 or rruff_fused or fused_g0" mnistab rruffab && bash scripts/gpu_r4.sh r4e tests libbench
