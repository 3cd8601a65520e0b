set -o pipefail
O=gpurun_out/s4c; mkdir -p $O
export TMPDIR=/tmp
DIAG_KERNELS=i8 DIAG_MODES=0,4194304,524288 DIAG_ROUNDS=7 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
DIAG_KERNELS=i8 DIAG_MODES=0,4194304,2097152 DIAG_ROUNDS=5 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py 4 8192 256 64 16 > $O/diag_b4.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag_b4.txt; exit 1; }
cat $O/diag_b4.txt
