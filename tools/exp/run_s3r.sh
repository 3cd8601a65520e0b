set -o pipefail
O=gpurun_out/s3r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/pmc_profile.py $O/wf -- --workload cfg4 --output f32 --settle-ms 0 > $O/pmc_wide_f32.txt 2>&1 || { echo "pmc failed"; tail -20 $O/pmc_wide_f32.txt; exit 1; }
cat $O/pmc_wide_f32.txt
DIAG_KERNELS=wide DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 400 python -u tools/diag_fused.py 1 4096 256 256 64 > $O/diag_wide.txt 2>&1 || { echo "diag failed"; tail -20 $O/diag_wide.txt; exit 1; }
cat $O/diag_wide.txt
