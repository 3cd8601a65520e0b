#!/bin/bash
# Full evidence round on one GPU box: smoke, GPU tests, headline bench (+PMC, +CPU baseline), rocprof summaries of
# the int8 (headline) and float benches, per-operator table, streaming.  Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
STAGES="smoke pytest bench prof" bash tools/gpu_check.sh $TAG || exit 1
timeout -k 10 600 python bench.py --output f32 --no-cpu-baseline --no-secondary > $OUT/bench_f32.json 2> $OUT/bench_f32.err || { echo "f32 bench failed"; exit 1; }
timeout -k 10 600 /opt/rocm/bin/rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_f32 -o bench -- python3 bench.py --output f32 --no-cpu-baseline --no-pmc --no-secondary > $OUT/prof_f32.log 2>&1 || { echo "f32 prof failed"; exit 1; }
timeout -k 10 600 python tools/bench_ops.py > $OUT/ops.jsonl 2> $OUT/ops.err || { echo "ops failed"; exit 1; }
timeout -k 10 300 python tools/bench_stream.py > $OUT/stream.json 2> $OUT/stream.err || { echo "stream failed"; exit 1; }
echo "round $TAG ok"
cat $OUT/bench.json
