set -o pipefail
mkdir -p gpurun_out/r3_c
timeout -k 10 300 python -u -m pytest tests/test_gpu_q14table.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_c/pytest_q14.log 2>&1 || { echo "q14 tests failed"; tail -30 gpurun_out/r3_c/pytest_q14.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "int8 or cfg4" > gpurun_out/r3_c/pytest_int8.log 2>&1 || { echo "int8 tests failed"; tail -30 gpurun_out/r3_c/pytest_int8.log; exit 1; }
for ct in on off on off; do
  timeout -k 10 200 python bench.py --workload cfg4 --coeff-table $ct --no-secondary --no-pmc --no-cpu-baseline --no-ceiling --no-rocprof >> gpurun_out/r3_c/cfg4_ab.jsonl 2>> gpurun_out/r3_c/bench.err || { echo "bench failed"; tail gpurun_out/r3_c/bench.err; exit 1; }
done
echo done
