set -o pipefail
O=gpurun_out/s4h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "matrix or op_sequence or drop_in or golden" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
for ord in xcd channel; do
BF_TABLE_ORDER=$ord timeout -k 10 300 python tools/bench_ops.py --only cfg2,cfg3,cfg4 > $O/ops_${ord}_$r.jsonl 2> $O/ops.err || { echo "ops failed"; tail -20 $O/ops.err; exit 1; }
grep matrix $O/ops_${ord}_$r.jsonl | sed "s/^/$ord $r /"
done; done
