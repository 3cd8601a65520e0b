set -o pipefail
mkdir -p gpurun_out/r3_n
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_q14table.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "int8 or cfg4 or q14" > gpurun_out/r3_n/pytest_int8.log 2>&1 || { echo "int8 tests failed"; tail -30 gpurun_out/r3_n/pytest_int8.log; exit 1; }
tail -2 gpurun_out/r3_n/pytest_int8.log
DIAG_KERNELS=w32t W32T_MODES=-1,300 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 200 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_n/w32t.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_n/w32t.txt; exit 1; }
cat gpurun_out/r3_n/w32t.txt
timeout -k 10 300 python -u bench.py --workload cfg4 --no-secondary --no-cpu-baseline --no-pmc --no-ceiling > gpurun_out/r3_n/bench_cfg4.json 2> gpurun_out/r3_n/bench_cfg4.err || { echo bench failed; tail gpurun_out/r3_n/bench_cfg4.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r3_n/bench_cfg4.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r.get('rocprof',{}).get('kernels_us_per_step'), r.get('rocprof',{}).get('avg_us'))"
echo done
