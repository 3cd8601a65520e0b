"""Compact trace of memory ops / waits / MFMA / barriers in one kernel of a HIP source's device ISA.
usage: python tools/isa_trace.py <file.hip> <mangled-name-substring> [max_lines]"""
import re, subprocess, sys
src, key = sys.argv[1], sys.argv[2]
maxl = int(sys.argv[3]) if len(sys.argv) > 3 else 400
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip", "-S",
                "--cuda-device-only", src, "-o", "/tmp/_isa.s"], check=True, capture_output=True)
s = open("/tmp/_isa.s").read()
names = [n for n in re.findall(r"^(_Z\w+):", s, re.M) if key in n]
k = names[0]
body = s[s.index(k + ":"):s.index(".Lfunc_end", s.index(k + ":"))].splitlines()
res, prev, cnt, full = [], None, 0, None
for l in body:
    t = l.strip()
    if not t or t.startswith((".", ";")):
        continue
    op = t.split()[0]
    if not (op.startswith(("global_load", "global_store", "s_waitcnt", "s_barrier", "v_mfma", "ds_read", "ds_write",
                           "s_cbranch", "s_branch", "buffer_")) or t.endswith(":")):
        continue
    kk = t if t.endswith(":") or op.startswith("s_waitcnt") else op
    if kk == prev:
        cnt += 1
        continue
    if prev is not None:
        res.append(full + (f"  x{cnt}" if cnt > 1 else ""))
    prev, full, cnt = kk, t[:80], 1
res.append(full + (f"  x{cnt}" if cnt > 1 else ""))
print(k)
print("\n".join(res[:maxl]))
