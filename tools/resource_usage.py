"""Print per-kernel VGPR/AGPR/SGPR/scratch/occupancy for a HIP source (hipcc -Rpass-analysis).
    python tools/resource_usage.py <file.hip> [extra hipcc flags ...]"""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip", "-c", src,
                      "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:],
                     capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    n = re.sub(r"\(.*", "", n.replace("bf::(anonymous namespace)::", "").replace("void ", ""))
    print(f"{n[:90]:90s} V={r.get('VGPRs')} A={r.get('AGPRs')} S={r.get('SGPRs')} scr={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')}")
