#!/bin/bash
# GPU box, round 5 first run: smoke, the GPU suite on the product's HIP runtime, the scatter attribution
# (diagnostic build), the default bench.  Usage: bash tools/gpu_r5_a.sh <tag>
set -o pipefail
TAG=${1:-r5_a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
STAGES="smoke pytest" bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 300 python -u tools/diag_scatter.py --attribute > $OUT/scatter_attribution.txt 2>&1 || { echo "attribution failed"; tail -20 $OUT/scatter_attribution.txt; exit 1; }
cat $OUT/scatter_attribution.txt
STAGES="bench" bash tools/gpu_check.sh $TAG || exit 1
echo "run $TAG ok"
