set -o pipefail
mkdir -p gpurun_out/r3_d
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload cfg4 --no-secondary --no-pmc --no-cpu-baseline --no-ceiling --prof-out gpurun_out/r3_d/prof > gpurun_out/r3_d/bench.json 2> gpurun_out/r3_d/bench.err || { echo "bench failed"; tail gpurun_out/r3_d/bench.err; exit 1; }
python tools/kernel_stats.py gpurun_out/r3_d/prof/bench_kernel_trace.csv 2>&1 | tail -5
echo done
