set -o pipefail
OUT=gpurun_out/r3_y
mkdir -p $OUT
export TMPDIR=/tmp
DIAG_KERNELS=w32t W32T_MODES=300,600,304,604,301,601 DIAG_STREAMS=0 DIAG_ROUNDS=5 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/l16_ab.txt 2>&1 || { echo diag failed; tail $OUT/l16_ab.txt; exit 1; }
cat $OUT/l16_ab.txt
