set -o pipefail
OUT=gpurun_out/r3_ae2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_q14table.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_wide.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_wide.log; exit 1; }
tail -2 $OUT/pytest_wide.log
STAGES="bench" BENCH_ARGS="--prof-out gpurun_out/r3_ae2/benchprof" bash tools/gpu_check.sh r3_ae2
