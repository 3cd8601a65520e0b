#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench -> rocprofv3 kernel-trace summary.
# Usage (from the repo root, through gpurun):  bash tools/gpu_check.sh [tag] [steps...]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# stages: smoke, pytest (PYTEST_K: a -k expression; PYTEST_ARGS: more arguments), bench / prof (BENCH_ARGS), diag (DIAG_ENV: the
# environment of tools/diag_fused.py, e.g. 'DIAG_KERNELS=w8 W8_MODES=1000,1001'; DIAG_SHAPE defaults to cfg4), ops
# (tools/bench_ops.py, OPS_ARGS), pmc (tools/pmc_profile.py, BENCH_ARGS), cal (tools/pmc_calibrate.py)
STAGES=${STAGES:-"smoke pytest bench prof"}
for s in $STAGES; do
  case $s in
    smoke)  timeout -k 10 300 python __graft_entry__.py > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; } ;;
    pytest) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; } ;;
    bench)  timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; } ;;
    # the profiled run's own JSON line (stdout) is kept next to its rocprof summary: both come from one process
    diag)   env ${DIAG_ENV} DIAG_STREAMS=${DIAG_STREAMS:-0} timeout -k 10 300 python tools/diag_fused.py ${DIAG_SHAPE:-1 4096 256 256 64} > $OUT/diag.txt 2>&1 || { echo "diag failed"; tail -20 $OUT/diag.txt; exit 1; }; cat $OUT/diag.txt ;;
    ops)    timeout -k 10 400 python tools/bench_ops.py ${OPS_ARGS} > $OUT/ops.jsonl 2> $OUT/ops.err || { echo "ops failed"; tail -20 $OUT/ops.err; exit 1; }; cat $OUT/ops.jsonl ;;
    pmc)    timeout -k 10 600 python tools/pmc_profile.py $OUT/pmc -- ${BENCH_ARGS} > $OUT/pmc.txt 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.txt; exit 1; }; cat $OUT/pmc.txt ;;
    stream) timeout -k 10 300 python tools/bench_stream.py > $OUT/stream.json 2> $OUT/stream.err || { echo "stream failed"; tail -20 $OUT/stream.err; exit 1; }; cat $OUT/stream.json ;;
    cal)    timeout -k 10 300 python tools/pmc_calibrate.py $OUT/cal > $OUT/pmc_calibration.jsonl 2>&1 || { echo "cal failed"; exit 1; }; cat $OUT/pmc_calibration.jsonl ;;
    prof)   timeout -k 10 600 /opt/rocm/bin/rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-pmc --no-secondary --no-ceiling --no-rocprof ${BENCH_ARGS} > $OUT/prof_bench.json 2> $OUT/prof.log || { echo "prof failed"; tail -20 $OUT/prof.log; exit 1; } ;;
  esac
  echo "stage $s ok"
done
[ -f $OUT/bench.json ] && cat $OUT/bench.json; true
