# GPU box: PMC counters (separate rocprofv3 passes, tools/pmc_profile.py) of the config-4 kernels: the int8
# contraction + generator, and the float32 wide kernel.  Usage: bash tools/gpu_pmc_cfg4.sh <out dir>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
PMC_KERNEL=beamform_fused_i8_w32r timeout -k 10 600 python -u tools/pmc_profile.py "$OUT/w32r" -- --workload cfg4 > "$OUT/w32r_pmc.txt" 2>&1 && \
PMC_KERNEL=q14_table timeout -k 10 600 python -u tools/pmc_profile.py "$OUT/gen" -- --workload cfg4 > "$OUT/gen_pmc.txt" 2>&1 && \
PMC_KERNEL=beamform_fused_wide timeout -k 10 600 python -u tools/pmc_profile.py "$OUT/wide" -- --workload cfg4 --output f32 > "$OUT/wide_pmc.txt" 2>&1
