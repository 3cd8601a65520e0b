set -o pipefail
O=gpurun_out/s4f; mkdir -p $O
export TMPDIR=/tmp
DIAG_KERNELS=i8 DIAG_MODES=0,8388608 DIAG_ROUNDS=7 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
