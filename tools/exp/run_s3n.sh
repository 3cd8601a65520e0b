set -o pipefail
O=gpurun_out/s3n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "int8 or smoke or edge or i8" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
I8_AB=1 DIAG_KERNELS=none DIAG_ROUNDS=7 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
