#!/bin/bash
# per-kernel microbench + PMC counters (separate rocprofv3 run, counters only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kbench.py --reps 10 ${KB_ARGS:---mid-grid 128,256} > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$PMC" ]; then
  timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/pmc -o pmc -- python3 scripts/kbench.py --reps 3 --mid-grid 256 > gpurun_out/pmc.log 2>&1
  echo "pmc rc=$?"
fi
