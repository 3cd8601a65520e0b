mkdir -p gpurun_out/r4_s
DIAG_KERNELS=wide WIDE_TW=2 WIDE_MODES=1000,0,1064,1128,1001 DIAG_ROUNDS=7 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r4_s/wide_ab.txt 2>&1 || { echo wide failed; exit 1; }
grep wide gpurun_out/r4_s/wide_ab.txt
GEN_AB_WHAT=launch GEN_AB="serial=BF_W32_OVERLAP:1,2 chunks=BF_W32_OVERLAP:2,4 chunks=BF_W32_OVERLAP:4,8 chunks=BF_W32_OVERLAP:8" DIAG_ROUNDS=5 timeout -k 10 300 python -u tools/diag_gen_ab.py > gpurun_out/r4_s/overlap_ab.txt 2>&1 || { echo overlap failed; cat gpurun_out/r4_s/overlap_ab.txt; exit 1; }
cat gpurun_out/r4_s/overlap_ab.txt
DIAG_KERNELS=table TABLE_MODES=500,400,600 DIAG_ROUNDS=5 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r4_s/table_os_ab.txt 2>&1 || { echo table failed; exit 1; }
grep "table" gpurun_out/r4_s/table_os_ab.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_q14table.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/r4_s/pytest.txt 2>&1; tail -3 gpurun_out/r4_s/pytest.txt
