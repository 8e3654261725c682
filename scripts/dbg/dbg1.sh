cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg1
timeout -k 10 120 python scripts/dbg/g0_cols.py > gpurun_out/dbg1/g0_cols.log 2>&1; echo rc=$? >> gpurun_out/dbg1/g0_cols.log
tail -40 gpurun_out/dbg1/g0_cols.log
