cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg5
timeout -k 10 120 python scripts/dbg/g0_cols.py > gpurun_out/dbg5/g0_cols.log 2>&1 || { echo "g0_cols rc=$?"; tail -20 gpurun_out/dbg5/g0_cols.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dbg5/g0_cols.log | grep -E "G0|G12"
bash scripts/gpu_r4.sh r4d "tests:tile or bplan or wide or fused or capi or tp or learn" tests bench rruff rruffab
