set -o pipefail
OUT=gpurun_out/r3_af
mkdir -p $OUT
export TMPDIR=/tmp
PMC_KERNEL=w32t timeout -k 10 600 python tools/pmc_profile.py $OUT/pmc -- --workload cfg4 --out-int8 > $OUT/w32t_pmc.txt 2>&1 || { echo "pmc failed"; tail -20 $OUT/w32t_pmc.txt; exit 1; }
cat $OUT/w32t_pmc.txt
