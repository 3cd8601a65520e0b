set -o pipefail
mkdir -p gpurun_out/r3_ad
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_q14table.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "q14 or int8 or cfg4" > gpurun_out/r3_ad/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3_ad/pytest.log; exit 1; }
tail -2 gpurun_out/r3_ad/pytest.log
DIAG_KERNELS=w32t W32T_MODES=-1,300 DIAG_ROUNDS=3 DIAG_STREAMS=0 timeout -k 10 200 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_ad/gen.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_ad/gen.txt; exit 1; }
cat gpurun_out/r3_ad/gen.txt
echo done
