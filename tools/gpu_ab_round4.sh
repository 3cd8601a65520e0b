# GPU box, round 4 A/B batch: config-4 contraction forms (int8 w32t, f32 wide, MatrixMultiply output-stationary),
# the hardware sin/cos probe, then the GPU suite and the default bench.  Usage: bash tools/gpu_ab_round4.sh <out dir>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
DIAG_KERNELS=w32t W32T_MODES=-1,240,900,920,940,908,928,901,921,904 DIAG_ROUNDS=3 \
  timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > "$OUT/w32t_ab.txt" 2>&1 && \
DIAG_KERNELS=w32chunk W32_CHUNKS=1,o2,o4,o8,2 DIAG_ROUNDS=3 \
  timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > "$OUT/w32_overlap_ab.txt" 2>&1 && \
DIAG_KERNELS=wide WIDE_TW=2 WIDE_MODES=0,1000,1,1001,4,1004,64,1064 DIAG_ROUNDS=3 \
  timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > "$OUT/wide_ab.txt" 2>&1 && \
DIAG_KERNELS=table TABLE_MODES=400,500,600 TABLE_NTS=2 DIAG_ROUNDS=3 \
  timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > "$OUT/table_os_ab.txt" 2>&1 && \
timeout -k 10 120 ./build/sincos_hw_probe > "$OUT/sincos_hw_probe.txt" 2>&1 && \
bash tools/gpu_suite_bench.sh "$OUT"
