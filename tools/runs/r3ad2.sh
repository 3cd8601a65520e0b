set -o pipefail
OUT=gpurun_out/r3_ad2
mkdir -p $OUT
export TMPDIR=/tmp
DIAG_KERNELS=w32t W32T_MODES=200,220,240,260 DIAG_STREAMS=0 DIAG_ROUNDS=5 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/ch_per_wg.txt 2>&1 || { echo diag failed; tail $OUT/ch_per_wg.txt; exit 1; }
cat $OUT/ch_per_wg.txt
