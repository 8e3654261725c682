#!/bin/bash
# PMC counters of the direct-load G0 kernel vs the LDS-staged TN kernel (scripts/g0_direct.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/pmcg && export TMPDIR=/tmp
groups=("FETCH_SIZE TCC_HIT_sum" "TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum")
i=0
for grp in "${groups[@]}"; do
  HPNN_G0D=${VAR:-1} timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmcg/g$i -o p -- python3 scripts/g0_direct.py 48 > gpurun_out/pmcg/g$i.log 2>&1 || { echo "group $i failed"; tail -5 gpurun_out/pmcg/g$i.log; }
  i=$((i+1))
done
python3 - <<'PY'
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmcg/g*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        m = re.search(r"(gemm_nt_direct\w*|gemm_tn_pipe_kernel)", k)
        if not m: continue
        acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:34s} {sum(v)/len(v):14.4g}")
PY
