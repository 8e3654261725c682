#!/bin/bash
# mlp3_fused duration with row-major vs fragment-major delta1 (float input; HPNN_G0_FM toggles d1fm)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for fm in 0 1 0 1; do
  HPNN_G0_FM=$fm timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fd$fm -o run -- python3 bench.py --steps 40 --warmup 10 --graph 0 --input float > gpurun_out/fd.log 2>&1 || exit 1
  python3 - $fm <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/fd{sys.argv[1]}/run_kernel_stats.csv")):
    if "mlp3_fused" in r["Name"]: print(f"d1fm={sys.argv[1]} front avg {float(r['AverageNs'])/1000:.2f} min {float(r['MinNs'])/1000:.2f} us")
PY
done
