set -o pipefail
mkdir -p gpurun_out/r3_m
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "matrix_multiply or op_sequence" > gpurun_out/r3_m/pytest_mm.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_m/pytest_mm.log; exit 1; }
tail -2 gpurun_out/r3_m/pytest_mm.log
TABLE_MODES=200,400,404,408,416,428,500,528 TABLE_NTS=2 DIAG_KERNELS=table DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_m/table_ablation.txt 2>&1 || { echo table diag failed; tail gpurun_out/r3_m/table_ablation.txt; exit 1; }
cat gpurun_out/r3_m/table_ablation.txt
echo done
