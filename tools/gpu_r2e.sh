# r2 loader/consumer kernel iteration: parity of the int8 paths + cfg4 ablation timing
mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "int8 or cfg4" > gpurun_out/$1/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$1/pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/$1/pytest.log | head -20; exit $rc; fi
DIAG_KERNELS=lc DIAG_ROUNDS=2 DIAG_STREAMS=0 timeout -k 10 200 python tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/$1/lc_ablation.txt 2>&1; cat gpurun_out/$1/lc_ablation.txt
