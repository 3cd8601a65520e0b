set -o pipefail
O=gpurun_out/s3s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DIAG_KERNELS=wide DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py 1 4096 256 256 64 > $O/diag_wide.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag_wide.txt; exit 1; }
cat $O/diag_wide.txt
