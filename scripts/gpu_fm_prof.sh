#!/bin/bash
# per-kernel times of the MNIST step, fragment-major G0 vs LDS-staged TN G0 (HPNN_G0_FM=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for fm in 1 0; do
  HPNN_G0_FM=$fm timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fmp$fm -o run -- python3 bench.py --steps 50 --warmup 10 --graph 0 > gpurun_out/fmp$fm.log 2>&1 || exit 1
  python3 - $fm <<'PY'
import csv, sys
fm = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/fmp{fm}/run_kernel_stats.csv")):
    n = r["Name"]
    for k in ["mlp3_fused", "gemm_tn", "gemm_fm", "sgd_update"]:
        if k in n: print(f"fm={fm} {k:12s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1000:7.2f} us")
PY
done
