#!/bin/bash
# GPU box: the GPU suite, then same-process A/Bs of this tree's libbf.so against a saved build (build/libbf_<old>.so).
# Usage: OLD=r5a CASES="cfg3:0xb cfg3:0x1" bash tools/gpu_r5_ab_libs.sh <tag>
set -o pipefail
TAG=${1:-r5_abl}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  STAGES="pytest" bash tools/gpu_check.sh $TAG || exit 1
  tail -1 $OUT/pytest_gpu.log
fi
for cs in ${CASES:-cfg3:0xb}; do
  timeout -k 10 240 python -u tools/ab_libs.py ${cs%%:*} ${cs##*:} 0.015625 new=dpdk_dc_sand_amd/libbf.so \
    old=build/libbf_${OLD:-r5a}.so >> $OUT/ab_libs.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_libs.txt; exit 1; }
done
cat $OUT/ab_libs.txt
echo "run $TAG ok"
