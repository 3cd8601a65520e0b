set -o pipefail
O=gpurun_out/s3w; mkdir -p $O
export TMPDIR=/tmp
DIAG_KERNELS=i8 DIAG_MODES=0,262144,524288,1048576,2097152 DIAG_ROUNDS=7 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
