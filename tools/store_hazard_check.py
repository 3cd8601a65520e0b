"""The store-data hazard of wide vector stores on gfx950: a VALU write to a VGPR that a just-issued dwordx3/x4 store
still reads as data corrupts what that store writes for the last lanes it reads.  hipcc (ROCm 7.2) does not always
keep the two apart: round 5 found a `buffer_store_dwordx4 v[80:83]` followed at once by a write of v83, and the 4th
dword of lanes 12-15 of every row went out wrong in ~1e-5 of the bytes, varying run to run (tools/diag_w32r.py) --
also the signature of round 4's unexplained w64h race.  This scans a source's device ISA for a VALU (or permlane
swap) writing a wide store's data VGPRs within `window` instructions of it.
Also: inline-asm results that reach an MFMA operand unpadded (scan_asm_to_mfma).
usage: python tools/store_hazard_check.py <file.hip> [window] [extra hipcc flags]"""
import re
import subprocess
import sys


def _regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def scan(asm, window=2):
    """(wide stores, [(function, store, offending instruction, distance)]) of a device .s text."""
    fn, lines = None, []
    for line in asm.splitlines():
        t = line.strip()
        m = re.match(r"^(_Z\w+):", t)
        if m:
            fn = m.group(1)
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        lines.append((fn, t))
    total, hits = 0, []
    for i, (fn, t) in enumerate(lines):
        op = t.split()[0]
        if not re.match(r"(buffer|global|flat)_store_dwordx[34]", op):
            continue
        total += 1
        ops = [x.rstrip(",") for x in t.split()[1:]]
        data = _regs(ops[0] if op.startswith("buffer") else ops[1])
        elapsed, j = 0, 1  # wait states between the store and instruction i + j
        while elapsed < window and i + j < len(lines) and lines[i + j][0] == fn:
            n = lines[i + j][1]
            nop = n.split()[0]
            j += 1
            if nop == "s_nop":  # s_nop k is k + 1 wait states (s_nop 0: one, not enough for a 2-state window)
                elapsed += nop_states(n)
                continue
            if nop.startswith("v_") and not nop.startswith("v_mfma"):
                parts = [x.rstrip(",") for x in n.split()[1:]]
                dst = _regs(parts[0]) if parts else set()
                if "swap" in nop and len(parts) > 1:
                    dst |= _regs(parts[1])
                if dst & data:
                    hits.append((fn, t, n, elapsed + 1))
                    break
            elapsed += 1
    return total, hits


def nop_states(line):
    """Wait states of an `s_nop k` line: k + 1."""
    parts = line.split()
    return int(parts[1], 0) + 1 if len(parts) > 1 else 1


def scan_asm_to_mfma(asm, window=2):
    """Inline-asm VGPR results read by an MFMA within `window` instructions after the statement when the statement
    does not end in an s_nop (hipcc pads one state after ;;#ASMEND; a VALU write -> MFMA SrcA/B/C read needs 2):
    [(function, asm instruction, mfma, distance)]."""
    fn, out = None, []
    inside, dst, last, pending = False, set(), "", None
    for line in asm.splitlines():
        t = line.strip()
        m = re.match(r"^(_Z\w+):", t)
        if m:
            fn, pending = m.group(1), None
            continue
        if t.startswith(";;#ASMSTART"):
            inside, dst, last = True, set(), ""
            continue
        if t.startswith(";;#ASMEND"):
            inside = False
            padded = last.startswith("s_nop") and not last.startswith("s_nop 0")
            pending = None if padded or not dst else [dst, 0, last]
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        if inside:
            last = t
            if t.startswith("v_"):
                parts = [x.rstrip(",") for x in t.split()[1:]]
                if parts:
                    dst |= _regs(parts[0])
            continue
        if pending is not None:
            pending[1] += 1
            if t.startswith("s_nop"):
                pending = None
                continue
            if t.startswith("v_mfma"):
                srcs = set()
                for x in [x.rstrip(",") for x in t.split()[2:]]:
                    srcs |= _regs(x)
                if srcs & pending[0]:
                    out.append((fn, pending[2], t, pending[1]))
            if pending[1] >= window:
                pending = None
    return out


def scan_lds_dma_ring(asm, kernel, slot_reads=("ds_read2st64_b64", "ds_read_b64", "ds_read2_b64"), pieces=4,
                      depth=2):
    """the LDS-DMA voltage ring relies on hipcc's vmcnt bookkeeping (its slots are distinct __shared__
    objects).  Replays the vector-memory queue of `kernel`'s main loop (the longest backward branch's body, twice,
    entered with a full ring of `depth` steps x `pieces` DMA pieces in flight): every `s_waitcnt vmcnt(N)` retires the
    oldest entries down to N, in issue order, as the hardware does.  At each slot read at most (depth - 1) x pieces
    DMA pieces may still be outstanding (only the next step's), else the read could see a slot its DMA has not
    written.  Returns (slot reads checked, [(instruction index, DMA pieces outstanding)])."""
    lines, start = [], None
    for line in asm.splitlines():
        t = line.strip()
        if re.match(r"^" + re.escape(kernel) + r":", t):
            start = True
            continue
        if start is None:
            continue
        if t.startswith(".Lfunc_end"):
            break
        if not t or t.startswith(";") or (t.startswith(".") and not t.endswith(":")):
            continue
        lines.append(t.split(";")[0].strip())
    labels = {t[:-1]: i for i, t in enumerate(lines) if re.match(r"^\.LBB\w+:$", t)}
    loops = []
    for i, t in enumerate(lines):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", t)
        if m and labels.get(m.group(1), i + 1) < i:
            loops.append((i - labels[m.group(1)], labels[m.group(1)], i))
    if not loops:
        return 0, []
    _, head, tail = max(loops)
    body = [t for t in lines[head + 1:tail + 1] if not t.endswith(":")]
    queue = ["dma"] * (pieces * depth)
    checked, bad = 0, []
    for rep in range(2):
        for i, t in enumerate(body):
            op = t.split()[0]
            if op.startswith(("buffer_", "global_")) and ("load" in op or "store" in op or "atomic" in op):
                queue.append("dma" if t.endswith(" lds") or " lds " in t else "mem")
            elif op == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", t)
                if m:
                    del queue[:max(0, len(queue) - int(m.group(1)))]
            elif op in slot_reads:
                n = queue.count("dma")
                checked += rep
                if rep and n > (depth - 1) * pieces:
                    bad.append((i, n))
    return checked, bad


def compile_isa(src, flags=()):
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip", "-S",
                        "--cuda-device-only", src, "-o", "-"] + list(flags), capture_output=True, text=True,
                       timeout=600)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-2000:])
    return r.stdout


if __name__ == "__main__":
    window = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    total, hits = scan(compile_isa(sys.argv[1], sys.argv[3:]), window)
    print(f"{total} wide stores, {len(hits)} with a VALU rewriting their data within {window} instructions")
    for fn, t, n, j in hits[:40]:
        name = subprocess.run(["c++filt", fn], capture_output=True, text=True).stdout.strip()[:90]
        print(f"  {name}\n    {t}\n    +{j}: {n}")
