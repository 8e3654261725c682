#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
for p in ${PADS:-0 64 128 256 1024}; do for v in ${VARS:-0 1 3}; do
  G0D_PAD=$p HPNN_G0D=$v timeout -k 10 120 python scripts/g0_direct.py ${SPLITS:-48} || exit $?
done; done
