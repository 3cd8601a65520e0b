set -o pipefail
mkdir -p gpurun_out/r3_q
export TMPDIR=/tmp
DIAG_KERNELS=item,f8 DIAG_MODES=0,16,64,80 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 8 4096 256 64 16 > gpurun_out/r3_q/item_exact_ab.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_q/item_exact_ab.txt; exit 1; }
cat gpurun_out/r3_q/item_exact_ab.txt
DIAG_KERNELS=wide WIDE_PIPE=0,1 WIDE_TW=2 WIDE_MODES=0,1,4 DIAG_STREAMS=0 DIAG_ROUNDS=3 timeout -k 10 300 python -u tools/diag_fused.py 1 4096 256 256 64 > gpurun_out/r3_q/wide_pipe_ab.txt 2>&1 || { echo diag failed; tail gpurun_out/r3_q/wide_pipe_ab.txt; exit 1; }
cat gpurun_out/r3_q/wide_pipe_ab.txt
echo done
