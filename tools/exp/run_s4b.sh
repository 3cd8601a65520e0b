set -o pipefail
O=gpurun_out/s4b; mkdir -p $O
export TMPDIR=/tmp
DIAG_KERNELS=i8 DIAG_MODES=0,8192,16384,24576,1024 DIAG_ROUNDS=5 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
