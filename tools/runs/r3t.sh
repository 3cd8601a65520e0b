set -o pipefail
OUT=gpurun_out/r3_t
mkdir -p $OUT
export TMPDIR=/tmp
DIAG_KERNELS=w32t W32T_MODES=300,700,701,704,705,708,709,712,713,715,702 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/os_ablation.txt 2>&1 || { echo diag failed; tail $OUT/os_ablation.txt; exit 1; }
cat $OUT/os_ablation.txt
PMC_KERNEL=i8_os timeout -k 10 600 python tools/pmc_profile.py $OUT/pmc -- --workload cfg4 --out-int8 > $OUT/os_pmc.txt 2>&1 || { echo "pmc failed"; tail -20 $OUT/os_pmc.txt; exit 1; }
cat $OUT/os_pmc.txt
