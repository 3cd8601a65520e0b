#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel-trace summary.
# Usage (from the repo root, through gpurun):  bash tools/gpu_check.sh [tag] [steps...]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
STAGES=${STAGES:-"smoke pytest bench prof"}
for s in $STAGES; do
  case $s in
    smoke)  timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; } ;;
    pytest) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; } ;;
    bench)  timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; } ;;
    # the profiled run's own JSON line (stdout) is kept next to its rocprof summary: both come from one process
    prof)   timeout -k 10 600 /opt/rocm/bin/rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-pmc --no-secondary --no-ceiling ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof.log || { echo "prof failed"; tail -20 $OUT/prof.log; exit 1; } ;;
  esac
  echo "stage $s ok"
done
[ -f $OUT/bench.json ] && cat $OUT/bench.json; true
