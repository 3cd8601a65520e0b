set -o pipefail
O=gpurun_out/s3k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
DIAG_KERNELS=item DIAG_MODES=0,64,96 DIAG_ROUNDS=5 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py > $O/diag_item.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag_item.txt; exit 1; }
cat $O/diag_item.txt
