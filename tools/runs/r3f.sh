set -o pipefail
mkdir -p gpurun_out/r3_f
export TMPDIR=/tmp
DIAG_KERNELS=w32t DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_f/w32t_ablation.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_f/w32t_ablation.txt; exit 1; }
cat gpurun_out/r3_f/w32t_ablation.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_q14table.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "int8 or cfg4 or q14" > gpurun_out/r3_f/pytest_int8.log 2>&1 || { echo "int8 tests failed"; tail -30 gpurun_out/r3_f/pytest_int8.log; exit 1; }
tail -2 gpurun_out/r3_f/pytest_int8.log
for ct in on off on off; do
  timeout -k 10 200 python bench.py --workload cfg4 --coeff-table $ct --no-secondary --no-pmc --no-cpu-baseline --no-ceiling --no-rocprof >> gpurun_out/r3_f/cfg4_ab.jsonl 2>> gpurun_out/r3_f/bench.err || { echo "bench failed"; tail gpurun_out/r3_f/bench.err; exit 1; }
done
echo done
