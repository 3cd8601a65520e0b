set -o pipefail
O=gpurun_out/s4a; mkdir -p $O
export TMPDIR=/tmp
DIAG_KERNELS=item DIAG_MODES=0,160,192,224,288 DIAG_ROUNDS=5 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
