#!/bin/bash
# GPU box, round-4 evidence: smoke, the GPU suite, the default bench (+ rocprof re-run, PMC, ceilings, CPU baseline),
# the rocprofv3 kernel-trace summary, PMC of the config-4 kernels, the LDS-DMA probe and the generator timing.
# Usage: bash tools/gpu_round4_final.sh <tag>
set -o pipefail
TAG=${1:-r4_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
STAGES="smoke pytest bench prof" bash tools/gpu_check.sh $TAG || exit 1
bash tools/gpu_pmc_cfg4.sh $OUT/pmc || { echo "pmc failed"; exit 1; }
timeout -k 10 60 ./build/lds_dma_high > $OUT/lds_dma_high.txt 2>&1 || { echo "lds probe failed"; cat $OUT/lds_dma_high.txt; }
DIAG_KERNELS=w32t W32T_MODES=-1,900 DIAG_ROUNDS=5 timeout -k 10 200 python -u tools/diag_fused.py 1 4096 256 256 64 \
  > $OUT/gen.txt 2>&1 || { echo "gen timing failed"; exit 1; }
grep "w32t mode" $OUT/gen.txt
echo "round $TAG ok"
