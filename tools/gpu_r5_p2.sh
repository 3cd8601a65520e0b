#!/bin/bash
# GPU box, round 5: the persistent float wide kernel as the product form -- its parity tests, a same-process A/B
# against the slab kernel (diagnostic library), and the config-4 f32 bench line.  Usage: bash tools/gpu_r5_p2.sh <tag>
set -o pipefail
TAG=${1:-r5_p2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  -k "cfg4 or persistent" > $OUT/pytest_fullsize.txt 2>&1 || { tail -30 $OUT/pytest_fullsize.txt; exit 1; }
tail -1 $OUT/pytest_fullsize.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  > $OUT/pytest_parity.txt 2>&1 || { tail -30 $OUT/pytest_parity.txt; exit 1; }
tail -1 $OUT/pytest_parity.txt
DIAG_STREAMS=0 DIAG_KERNELS=wide WIDE_TW=2 DIAG_ROUNDS=7 WIDE_MODES=1000,20104,20008 timeout -k 10 300 \
  python -u tools/diag_fused.py 1 4096 256 256 64 > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
timeout -k 10 300 python -u bench.py --workload cfg4 --output f32 --no-cpu-baseline --no-pmc --no-secondary \
  > $OUT/bench_cfg4_f32.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo "run $TAG ok"
