set -o pipefail
OUT=gpurun_out/r3_aa
mkdir -p $OUT
export TMPDIR=/tmp
for nt in 0 1 0 1 0 1; do
  echo "nt stores $nt" >> $OUT/gen_nt.txt
  BF_Q14_NT=$nt DIAG_KERNELS=w32t,w32chunk W32T_MODES=-1 W32_CHUNKS=1 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 120 python -u tools/diag_fused.py 1 4096 256 256 64 >> $OUT/gen_nt.txt 2>&1 || { echo diag failed; tail $OUT/gen_nt.txt; exit 1; }
done
grep -E "nt stores|generator" $OUT/gen_nt.txt
