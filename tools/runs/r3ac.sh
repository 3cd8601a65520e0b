set -o pipefail
OUT=gpurun_out/r3_ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_q14table.py tests/test_gpu_fullsize.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_wide.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_wide.log; exit 1; }
tail -2 $OUT/pytest_wide.log
DIAG_KERNELS=w32t W32T_MODES=300,200,304,204 DIAG_STREAMS=0 DIAG_ROUNDS=5 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/nb2_confirm.txt 2>&1 || { echo diag failed; tail $OUT/nb2_confirm.txt; exit 1; }
cat $OUT/nb2_confirm.txt
STAGES="bench" BENCH_ARGS="--prof-out gpurun_out/r3_ac/benchprof" bash tools/gpu_check.sh r3_ac
