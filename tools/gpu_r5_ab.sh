#!/bin/bash
# GPU box: config-4 int8 contraction A/B (diag modes), with a bitwise check of the given modes against w32t.
# Usage: MODES=900,2000,... CHECK="2032" bash tools/gpu_r5_ab.sh <tag>
set -o pipefail
TAG=${1:-r5_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$CHECK" ]; then
  timeout -k 10 200 python -u tools/diag_w32r.py 1 $CHECK > $OUT/bitwise.txt 2>&1 || { echo "bitwise check failed"; tail -20 $OUT/bitwise.txt; exit 1; }
  cat $OUT/bitwise.txt | cut -c1-200
fi
DIAG_KERNELS=w32t W32T_MODES=${MODES} DIAG_ROUNDS=${ROUNDS:-7} DIAG_STREAMS=0 timeout -k 10 300 \
  python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/ab.txt 2>&1 || { echo "diag failed"; tail -20 $OUT/ab.txt; exit 1; }
grep -v "stream grid" $OUT/ab.txt
echo "run $TAG ok"
