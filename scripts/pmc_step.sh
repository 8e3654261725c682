#!/bin/bash
# PMC counters of the training-step kernels of one bench.py config (eager launches): memory-side
# bytes (FETCH_SIZE / WRITE_SIZE), L2 hit rate, MFMA busy, waits and LDS bank conflicts.
# One rocprofv3 pass per counter group (kernel-trace only, each within the per-block limits).
# usage: scripts/pmc_step.sh [bench args...]   summary: gpurun_out/pmc_step<TAG>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${PMC_TAG:-}
D=gpurun_out/pmcs$TAG
mkdir -p $D && export TMPDIR=/tmp
groups=("FETCH_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
        "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE")
i=0
for grp in "${groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D/g$i -o p -- python3 bench.py --graph 0 --steps 6 --warmup 2 "$@" > $D/g$i.log 2>&1 || exit $?
  i=$((i+1))
done
D=$D python3 - <<'PY' | tee gpurun_out/pmc_step$TAG.txt
import csv, glob, collections, os, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.environ["D"] + "/g*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        if k.startswith("at::") or "rocclr" in k:
            continue
        k = re.sub(r"\(.*", "", k)
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):14.4g}   (n={len(v)})")
PY
