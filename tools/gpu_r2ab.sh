# r2: MatrixMultiply table kernels (staging + ring rework): parity subset, ablation, op timings
mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "beamform or matrix or op_sequence or coeff" > gpurun_out/$1/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/$1/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAIL" gpurun_out/$1/pytest.log | head -30; exit $rc; fi
DIAG_KERNELS=table DIAG_STREAMS=0 timeout -k 10 200 python tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/$1/table.txt 2>&1; cat gpurun_out/$1/table.txt
timeout -k 10 200 python tools/bench_ops.py --only cfg4,cfg3 --reps 10 > gpurun_out/$1/ops.jsonl 2>gpurun_out/$1/ops.err; grep -E "matrix|op_seq|coeff|reorder" gpurun_out/$1/ops.jsonl
