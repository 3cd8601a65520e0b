set -o pipefail
mkdir -p gpurun_out/r3_i
export TMPDIR=/tmp
DIAG_KERNELS=f8,item DIAG_MODES=0,1,2,4,5,8,128,64,96,256 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 8 4096 256 64 16 > gpurun_out/r3_i/cfg3_f32contract_ablation.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_i/cfg3_f32contract_ablation.txt; exit 1; }
cat gpurun_out/r3_i/cfg3_f32contract_ablation.txt
timeout -k 10 900 python -u tools/pmc_profile.py gpurun_out/r3_i/pmc_cfg4_int8 -- --workload cfg4 > gpurun_out/r3_i/cfg4_int8_w32t_pmc.txt 2>&1 || { echo pmc failed; tail gpurun_out/r3_i/cfg4_int8_w32t_pmc.txt; exit 1; }
cat gpurun_out/r3_i/cfg4_int8_w32t_pmc.txt
echo done
