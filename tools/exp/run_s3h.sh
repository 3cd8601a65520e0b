set -o pipefail
O=gpurun_out/s3h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/pmc_profile.py $O/w8 -- --workload cfg4 --settle-ms 0 > $O/pmc_w8.txt 2>&1 || { echo "pmc failed"; tail -20 $O/pmc_w8.txt; exit 1; }
cat $O/pmc_w8.txt
timeout -k 10 500 python -u tools/pmc_profile.py $O/i8 -- --settle-ms 0 > $O/pmc_i8.txt 2>&1 || { echo "pmc failed"; tail -20 $O/pmc_i8.txt; exit 1; }
cat $O/pmc_i8.txt
