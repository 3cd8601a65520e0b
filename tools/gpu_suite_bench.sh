# GPU box: the whole GPU test suite, then the default bench (headline + secondaries + rocprof re-run + PMC +
# ceiling + CPU baseline).  Usage: bash tools/gpu_suite_bench.sh <out dir under gpurun_out/>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/run}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 && \
timeout -k 10 600 python -u bench.py --prof-out "$OUT/prof" > "$OUT/bench.json" 2> "$OUT/bench.err"
