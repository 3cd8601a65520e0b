#!/bin/bash
# GPU box, round 5 evidence run: smoke, the GPU suite, a config-4 A/B, the default bench (+ rocprof re-run, PMC
# traffic, ceilings, CPU baseline), the rocprofv3 kernel-trace summary, PMC of the config-4 kernels.
# Usage: MODES=... CHECK=... bash tools/gpu_r5_full.sh <tag>
set -o pipefail
TAG=${1:-r5_full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
STAGES="smoke pytest" bash tools/gpu_check.sh $TAG || exit 1
tail -1 $OUT/pytest_gpu.log
if [ -n "$MODES" ]; then
  MODES=$MODES CHECK=$CHECK bash tools/gpu_r5_ab.sh $TAG/ab || exit 1
fi
STAGES="bench prof" bash tools/gpu_check.sh $TAG || exit 1
bash tools/gpu_pmc_cfg4.sh $OUT/pmc || { echo "pmc failed"; exit 1; }
echo "run $TAG ok"
