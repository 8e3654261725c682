cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg3
for p in 0 1 2 3 4 7; do
  echo "== HPNN_G0_PROTO=$p"
  HPNN_G0_PROTO=$p timeout -k 10 120 python scripts/dbg/g0_cols.py > gpurun_out/dbg3/p$p.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/dbg3/p$p.log; exit 1; }
  grep -E "G0 max" gpurun_out/dbg3/p$p.log
done
