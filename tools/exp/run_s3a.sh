set -o pipefail
mkdir -p gpurun_out/s3a
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s3a/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/s3a/pytest.log; exit 1; }
tail -2 gpurun_out/s3a/pytest.log
DIAG_KERNELS=i8 DIAG_MODES=0,8192,11264,10240,4096,7168,6144,1024,2048 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > gpurun_out/s3a/diag.txt 2>&1 || { echo "diag failed"; tail -20 gpurun_out/s3a/diag.txt; exit 1; }
cat gpurun_out/s3a/diag.txt
timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-pmc > gpurun_out/s3a/bench.json 2> gpurun_out/s3a/bench.err || { echo "bench failed"; tail -20 gpurun_out/s3a/bench.err; exit 1; }
cat gpurun_out/s3a/bench.json
