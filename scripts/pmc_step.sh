#!/bin/bash
# PMC counters of one MNIST training step (bench.py, eager launches): HBM/L2 bytes,
# MFMA busy, waits and LDS conflicts of mlp3_fused, gemm_tn_pipe and sgd_update_multi.
# One rocprofv3 pass per counter group (kernel-trace only).  Summary: gpurun_out/pmc_step.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcs && export TMPDIR=/tmp
groups=("FETCH_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
        "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE")
i=0
for grp in "${groups[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcs/g$i -o p -- python3 bench.py --graph 0 --steps 6 --warmup 2 > gpurun_out/pmcs/g$i.log 2>&1 || exit $?
  i=$((i+1))
done
python3 - <<'PY' | tee gpurun_out/pmc_step.txt
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmcs/g*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        m = re.search(r"(mlp3_fused_kernel|gemm_tn_pipe_kernel<[^>]*>|sgd_update_multi_wide_kernel)", k)
        if not m: continue
        acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):14.4g}")
PY
