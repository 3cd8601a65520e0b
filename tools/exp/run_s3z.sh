set -o pipefail
O=gpurun_out/s3z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
for ord in 2 1; do
for out in int8 f32; do
X=""; [ $ord = 1 ] && X="BF_FUSED_XCD_ORDER=1"
env $X timeout -k 10 300 python bench.py --workload cfg4 --output $out --no-cpu-baseline --no-pmc --no-secondary > $O/b_${out}_${ord}_$r.json 2> $O/b.err || { echo "bench failed"; tail -20 $O/b.err; exit 1; }
python3 -c "import json; b=json.load(open('$O/b_${out}_${ord}_$r.json')); print('cfg4 $out order$ord $r', b['roofline']['avg_launch_us'], b['roofline']['frac'])"
done; done; done
