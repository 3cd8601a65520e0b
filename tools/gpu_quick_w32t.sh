# GPU box: quick check of the config-4 int8 contraction forms + the product's config-4 int8 tests.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/quick}
mkdir -p "$OUT"
DIAG_KERNELS=w32t W32T_MODES=240,900,940,920 DIAG_ROUNDS=2 \
  timeout -k 10 200 python -u tools/diag_fused.py 1 4096 256 256 64 > "$OUT/w32t_ab.txt" 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_q14table.py -x -q --timeout 120 --timeout-method thread > "$OUT/q14table.txt" 2>&1
