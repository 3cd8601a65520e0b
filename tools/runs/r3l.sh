set -o pipefail
mkdir -p gpurun_out/r3_l
export TMPDIR=/tmp
DIAG_KERNELS=f8,item DIAG_MODES=0,64,1 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 8 4096 256 64 16 > gpurun_out/r3_l/f8.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_l/f8.txt; exit 1; }
cat gpurun_out/r3_l/f8.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_l/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_l/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3_l/pytest_gpu.log
timeout -k 10 400 python -u tools/bench_ops.py --only cfg3,cfg4 > gpurun_out/r3_l/ops.jsonl 2>&1 || { echo ops failed; tail gpurun_out/r3_l/ops.jsonl; exit 1; }
cat gpurun_out/r3_l/ops.jsonl
echo done
