set -o pipefail
OUT=gpurun_out/r3_v2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_q14table.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_q14.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_q14.log; exit 1; }
tail -3 $OUT/pytest_q14.log
DIAG_KERNELS=w32t W32T_MODES=300,700,800,701,704,708,709,713,715,815 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/os_ablation.txt 2>&1 || { echo diag failed; tail $OUT/os_ablation.txt; exit 1; }
cat $OUT/os_ablation.txt
