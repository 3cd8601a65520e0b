set -o pipefail
O=gpurun_out/s3y; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for ord in xcd channel; do
for wl in cfg2 cfg3; do
BF_ITEM_ORDER=$ord timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-pmc --no-secondary --steps 100 > $O/b_${wl}_${ord}_$r.json 2> $O/b.err || { echo "bench failed"; tail -20 $O/b.err; exit 1; }
python3 -c "import json; b=json.load(open('$O/b_${wl}_${ord}_$r.json')); print('$wl $ord $r', b['roofline']['avg_launch_us'], b['roofline']['frac'])"
done; done; done
