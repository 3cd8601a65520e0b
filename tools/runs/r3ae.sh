set -o pipefail
mkdir -p gpurun_out/r3_ae
export TMPDIR=/tmp
for u in 1 0 1 0 1 0; do
  echo "unit_fast $u" >> gpurun_out/r3_ae/gen.txt
  BF_Q14_UNIT=$u DIAG_KERNELS=w32t W32T_MODES=-1 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 120 python -u tools/diag_fused.py 1 4096 256 256 64 >> gpurun_out/r3_ae/gen.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_ae/gen.txt; exit 1; }
done
grep -E "unit_fast|generator" gpurun_out/r3_ae/gen.txt
