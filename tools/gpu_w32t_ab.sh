# GPU box: same-process A/B of the config-4 int8 contraction forms (tools/diag_fused.py, diagnostic library).
# Usage: bash tools/gpu_w32t_ab.sh <out file> [modes]
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/w32t_ab.txt}
mkdir -p "$(dirname "$OUT")"
DIAG_KERNELS=w32t W32T_MODES=${2:--1,240,900,920,940,908,928,901,921} DIAG_ROUNDS=${3:-3} \
  timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > "$OUT" 2>&1
