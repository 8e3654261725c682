#!/bin/bash
# PMC counters of the 8-phase NT / TN GEMMs (8192x4096x4096): MFMA busy, waits, LDS
# activity and bank conflicts, L2 traffic.  One rocprofv3 pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc8 && export TMPDIR=/tmp
groups=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
        "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum")
i=0
for grp in "${groups[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc8/g$i -o p -- python3 scripts/gemm8_once.py > gpurun_out/pmc8/g$i.log 2>&1 || exit $?
  i=$((i+1))
done
python3 - <<'PY' | tee gpurun_out/pmc_8ph.txt
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmc8/g*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(gemm_nt8_kernel|gemm_tn8_kernel)", r["Kernel_Name"])
        if m:
            acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    v = {c: sum(x) / len(x) for c, x in d.items()}
    for c in sorted(v):
        print(f"   {c:28s} {v[c]:14.4g}")
    if "GRBM_GUI_ACTIVE" in v and "SQ_VALU_MFMA_BUSY_CYCLES" in v:
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        print(f"   MFMA busy per SIMD / kernel cycles: {v['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / cyc:.3f}"
              f" (kernel ~{cyc:.0f} cycles)")
    if "SQ_LDS_IDX_ACTIVE" in v and "SQ_LDS_BANK_CONFLICT" in v:
        print(f"   LDS bank-conflict cycles / LDS active cycles: {v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_LDS_IDX_ACTIVE']):.3f}")
PY
