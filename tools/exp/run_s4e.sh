set -o pipefail
O=gpurun_out/s4e; mkdir -p $O
export TMPDIR=/tmp
DIAG_KERNELS=i8 DIAG_MODES=0,64,2048,65536 DIAG_ROUNDS=5 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
