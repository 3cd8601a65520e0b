set -o pipefail
O=gpurun_out/s3j; mkdir -p $O
export TMPDIR=/tmp
W8_AB=1 DIAG_KERNELS=w8 DIAG_ROUNDS=7 DIAG_STREAMS=0 timeout -k 10 500 python -u tools/diag_fused.py 1 4096 256 256 64 > $O/diag_w8.txt 2>&1 || { echo "diag w8 failed"; tail -20 $O/diag_w8.txt; exit 1; }
cat $O/diag_w8.txt
