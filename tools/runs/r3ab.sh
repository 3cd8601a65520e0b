# (modes as built for this run: 1000 = the 16-byte load form at NB 2, 1100 = NB 2 -- adopted, now diag mode 200 and the product form; the 16-byte form was removed)
set -o pipefail
OUT=gpurun_out/r3_ab
mkdir -p $OUT
export TMPDIR=/tmp
DIAG_KERNELS=w32t W32T_MODES=300,1000,1100,600,304,1004,1104 DIAG_STREAMS=0 DIAG_ROUNDS=5 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/nb2_ab.txt 2>&1 || { echo diag failed; tail $OUT/nb2_ab.txt; exit 1; }
cat $OUT/nb2_ab.txt
