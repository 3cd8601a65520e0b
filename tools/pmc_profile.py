"""Collect PMC counters for the fused kernel in separate rocprofv3 passes (no tracing domains mixed with --pmc)
and print per-dispatch medians.  Run on the GPU box from the repo root:
    python tools/pmc_profile.py [outdir] [-- extra bench.py args]      (PMC_KERNEL: kernel-name filter, "beamform")
The parent process never touches the GPU; each pass runs bench.py under rocprofv3 as a child."""
import csv, glob, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else os.path.join(ROOT, "gpurun_out", "pmc")
extra = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
PASSES = [
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU "
    "SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES",
    "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT "
    "SQ_WAVES",
    "SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL "
    "SQ_LEVEL_WAVES SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT",
    "FETCH_SIZE",
    "WRITE_SIZE",
    "TCC_HIT_sum TCC_MISS_sum",
]
os.makedirs(out, exist_ok=True)
env = dict(os.environ, TMPDIR="/tmp")
vals = {}
for i, p in enumerate(PASSES):
    d = os.path.join(out, f"pass{i}")
    cmd = ["/opt/rocm/bin/rocprofv3", "--pmc", *p.split(), "--output-format", "csv", "-d", d, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-pmc", "--no-secondary",
           "--no-rocprof", "--no-ceiling",
           "--steps", "5", "--warmup", "2", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=ROOT, env=env)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if r.returncode != 0 or not files:
        print(f"pass {i} failed rc={r.returncode}: {r.stderr[-400:]}")
        continue
    per = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            if os.environ.get("PMC_KERNEL", "beamform") not in row.get("Kernel_Name", ""):
                continue
            per.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    for k, v in per.items():
        v.sort()
        vals[k] = v[len(v) // 2]
for k in sorted(vals):
    print(f"{k:32s} {vals[k]:.6g}")
