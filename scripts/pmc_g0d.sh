#!/bin/bash
# PMC counters of the first-layer gradient kernels (scripts/g0_direct.py): LDS-DMA TN, register-staged, fragment-major
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmcg && export TMPDIR=/tmp
rm -rf gpurun_out/pmcg/*
groups=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"
        "SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM"
        "FETCH_SIZE TCC_HIT_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum")
i=0
for grp in "${groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcg/g$i -o p -- python3 scripts/g0_direct.py 48 > gpurun_out/pmcg/g$i.log 2>&1 || { echo "group $i failed"; tail -5 gpurun_out/pmcg/g$i.log; }
  i=$((i+1))
done
python3 - <<'PY'
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmcg/g*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        m = re.search(r"(gemm_fm_direct_kernel|gemm_tn_pipe_kernel|gemm_tn_rs_kernel<[^>]*>)", k)
        if not m: continue
        acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:34s} {sum(v)/len(v):14.4g}")
PY
