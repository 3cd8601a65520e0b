set -o pipefail
O=gpurun_out/s3o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DIAG_KERNELS=w8 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py 1 4096 256 256 64 > $O/diag_w8.txt 2>&1 || { echo "diag w8 failed"; tail -20 $O/diag_w8.txt; exit 1; }
cat $O/diag_w8.txt
timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline --no-pmc > $O/bench_cfg4.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench_cfg4.json
