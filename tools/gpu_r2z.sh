# r2: f32 wide kernel with 32-sample waves: float parity subset + ablation vs the 64-sample kernel
mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fused or cfg4 or f32" > gpurun_out/$1/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$1/pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAIL" gpurun_out/$1/pytest.log | head -30; exit $rc; fi
DIAG_KERNELS=wide WIDE_TW=2,3 WIDE_MODES=${WIDE_MODES:-0,1,4,5,8} DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 250 python tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/$1/wide.txt 2>&1; cat gpurun_out/$1/wide.txt
