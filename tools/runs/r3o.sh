set -o pipefail
mkdir -p gpurun_out/r3_o2
export TMPDIR=/tmp
for v in x1:64:1 x1:128:1 x1:256:1 x4:64:0 x4:128:0 x4:128:1 x1:64:1; do
  IFS=: read f r n <<< "$v"
  echo "form $f run $r nt $n" >> gpurun_out/r3_o2/gen.txt
  BF_Q14_FORM=$f BF_Q14_RUN=$r BF_Q14_NT=$n DIAG_KERNELS=w32t W32T_MODES=-1 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 120 python -u tools/diag_fused.py 1 4096 256 256 64 >> gpurun_out/r3_o2/gen.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_o2/gen.txt; exit 1; }
done
grep -E "form|generator" gpurun_out/r3_o2/gen.txt
echo done
