set -o pipefail
mkdir -p gpurun_out/r3_r
export TMPDIR=/tmp
DIAG_KERNELS=wide WIDE_TW=2 WIDE_MODES=0,500,1,501,4,504,508,513 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_r/wide_os_ab.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_r/wide_os_ab.txt; exit 1; }
cat gpurun_out/r3_r/wide_os_ab.txt
echo done
