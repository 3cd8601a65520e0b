# r2 32-beam int8 wide kernel: int8 parity subset + w8/w32 ablation timing on cfg4
mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "int8 or cfg4" > gpurun_out/$1/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$1/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAIL" gpurun_out/$1/pytest.log | head -30; exit $rc; fi
W8_MODES=${W8_MODES:-0,1,1000,1001,1002,1003,1004,1008,1009,1013} DIAG_KERNELS=w8 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 200 python tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/$1/w32_ablation.txt 2>&1; cat gpurun_out/$1/w32_ablation.txt
