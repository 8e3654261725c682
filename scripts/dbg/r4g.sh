cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4.sh r4g "tests:tile or tn_update or fused_g0" earlyab mnistab pmc && bash scripts/gpu_r4.sh r4g tests learn fpsteps dpforce
