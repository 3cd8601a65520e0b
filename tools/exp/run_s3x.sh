set -o pipefail
O=gpurun_out/s3x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DIAG_KERNELS=item,i8 DIAG_MODES=0,2097152,160 DIAG_ROUNDS=7 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
timeout -k 10 600 python bench.py --no-cpu-baseline --no-pmc > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; b=json.load(open('$O/bench.json')); print('headline', b['value'], b['roofline']['avg_launch_us'], b['roofline']['frac'])
for s in b['secondary']: print(s['workload'][:5], s['output'], s['value'], s['avg_launch_us'], s['roofline_frac'])"
