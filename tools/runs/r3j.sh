set -o pipefail
mkdir -p gpurun_out/r3_j
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/diag_ops.py > gpurun_out/r3_j/ops_ab.txt 2>&1 || { echo diag_ops failed; tail -20 gpurun_out/r3_j/ops_ab.txt; exit 1; }
cat gpurun_out/r3_j/ops_ab.txt
TABLE_MODES=200,201,204,208,216,217,220,228 TABLE_NTS=2 DIAG_KERNELS=table DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_j/table_ablation.txt 2>&1 || { echo table diag failed; tail gpurun_out/r3_j/table_ablation.txt; exit 1; }
cat gpurun_out/r3_j/table_ablation.txt
echo done
