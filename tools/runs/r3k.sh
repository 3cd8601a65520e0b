set -o pipefail
mkdir -p gpurun_out/r3_k
export TMPDIR=/tmp
REORDER_NT=0,3 REORDER_TT=256 timeout -k 10 400 python -u tools/diag_ops.py > gpurun_out/r3_k/ops_ab.txt 2>&1 || { echo diag_ops failed; tail -20 gpurun_out/r3_k/ops_ab.txt; exit 1; }
cat gpurun_out/r3_k/ops_ab.txt
TABLE_MODES=200,228,240,268,250,278 TABLE_NTS=2 DIAG_KERNELS=table DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_k/table_ablation.txt 2>&1 || { echo table diag failed; tail gpurun_out/r3_k/table_ablation.txt; exit 1; }
cat gpurun_out/r3_k/table_ablation.txt
echo done
