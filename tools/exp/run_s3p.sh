set -o pipefail
O=gpurun_out/s3p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/bench_ops.py --only cfg3,cfg4 > $O/ops_ring4.jsonl 2> $O/ops.err || { echo "ops failed"; tail -20 $O/ops.err; exit 1; }
BF_TABLE_RING4=0 timeout -k 10 300 python tools/bench_ops.py --only cfg3 > $O/ops_basic.jsonl 2>> $O/ops.err || { echo "ops failed"; tail -20 $O/ops.err; exit 1; }
grep -E "matrix|sequence" $O/ops_ring4.jsonl $O/ops_basic.jsonl
