cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg6
timeout -k 10 120 python scripts/dbg/g0_x.py > gpurun_out/dbg6/g0_x.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/dbg6/g0_x.log | tail -20
