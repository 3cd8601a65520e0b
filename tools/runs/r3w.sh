set -o pipefail
OUT=gpurun_out/r3_w
mkdir -p $OUT
export TMPDIR=/tmp
DIAG_KERNELS=w32t W32T_MODES=300,800,813,829,845,861,832,700,713,729,745,761 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/os_floor.txt 2>&1 || { echo diag failed; tail $OUT/os_floor.txt; exit 1; }
cat $OUT/os_floor.txt
