set -o pipefail
OUT=gpurun_out/r3_ag
mkdir -p $OUT
export TMPDIR=/tmp
DIAG_KERNELS=w32t W32T_MODES=240,280 DIAG_STREAMS=0 DIAG_ROUNDS=9 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/early_ab.txt 2>&1 || { echo diag failed; tail $OUT/early_ab.txt; exit 1; }
cat $OUT/early_ab.txt
