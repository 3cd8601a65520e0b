# r2: int8-from-f32 row stores: parity subset + bench cfg3 --int8-contract f32
mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "requantised or int8 or fused" > gpurun_out/$1/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$1/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAIL" gpurun_out/$1/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py --int8-contract f32 --no-cpu-baseline --no-pmc --no-secondary > gpurun_out/$1/bench_f32c.json 2> gpurun_out/$1/bench.err; cat gpurun_out/$1/bench_f32c.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('frac_of_ceiling'))"
