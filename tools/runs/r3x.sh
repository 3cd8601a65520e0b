set -o pipefail
OUT=gpurun_out/r3_x
mkdir -p $OUT
export TMPDIR=/tmp
DIAG_KERNELS=w32chunk W32_CHUNKS=1,2,4,8,16 DIAG_STREAMS=0 DIAG_ROUNDS=5 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/chunks.txt 2>&1 || { echo diag failed; tail $OUT/chunks.txt; exit 1; }
cat $OUT/chunks.txt
