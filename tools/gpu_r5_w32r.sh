#!/bin/bash
# GPU box, round 5: the LDS-DMA ring contraction (w32r) -- bitwise against w32t (3 runs), parity on the config-4
# tests, then the same-process A/B against the table kernel (w32t) on one kLayoutW32 table.
set -o pipefail
TAG=${1:-r5_w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/diag_w32r.py 3 2000 > $OUT/w32r_vs_w32t.txt 2>&1 || { echo "diag_w32r failed"; tail -20 $OUT/w32r_vs_w32t.txt; exit 1; }
cat $OUT/w32r_vs_w32t.txt | cut -c1-200
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_q14table.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $OUT/pytest_cfg4.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_cfg4.log; exit 1; }
tail -2 $OUT/pytest_cfg4.log
DIAG_KERNELS=w32t W32T_MODES=${MODES:-900,2000,2004,2008,2012,2016,2024,908,901,904} DIAG_ROUNDS=5 timeout -k 10 300 \
  python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/w32r_ab.txt 2>&1 || { echo "diag failed"; tail -20 $OUT/w32r_ab.txt; exit 1; }
cat $OUT/w32r_ab.txt

# the int8-via-f32 drift: round-3 tree, round-4 tree and this tree in one process
for fl in 0xb 0x3 0x1; do
  timeout -k 10 240 python -u tools/ab_libs.py cfg3 $fl 0.015625 r5=dpdk_dc_sand_amd/libbf.so \
    r4=build/libbf_r4.so r3=build/libbf_r3.so >> $OUT/ab_rounds.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_rounds.txt; exit 1; }
done
cat $OUT/ab_rounds.txt
echo "run $TAG ok"
