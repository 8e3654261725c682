cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg6
timeout -k 10 120 python scripts/dbg/g0_x.py > gpurun_out/dbg6/g0_x.log 2>&1; echo g0_x rc=$?
grep -v amdgpu.ids gpurun_out/dbg6/g0_x.log | tail -12
bash scripts/gpu_r4.sh r4f "tests:fragment_major or fused_g0 or tile" mnistab rruffab2 prof prof0 prof_rruff trace pmc && bash scripts/gpu_r4.sh r4f tests
