cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg4
timeout -k 10 120 python scripts/dbg/g0_slabs.py > gpurun_out/dbg4/slabs.log 2>&1; echo rc=$?
grep -v amdgpu.ids gpurun_out/dbg4/slabs.log | tail -40
