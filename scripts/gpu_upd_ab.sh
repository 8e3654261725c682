#!/bin/bash
# A/B of the update kernel's early W / V fetch (HPNN_UPD_PREFETCH), alternating bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for rep in 1 2 3; do
  for p in 1 0; do
    HPNN_UPD_PREFETCH=$p timeout -k 10 200 python bench.py --steps 400 --warmup 40 2>&1 | grep metric | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("prefetch='$p'", round(d["ms_per_step"]*1e3,2), "us")' | tee -a gpurun_out/upd_ab.txt || exit 1
  done
done
