"""Build hygiene of the product kernels (no GPU): every kernel instance libbf.so contains compiles for gfx950 with no
scratch (register spills) and without failed unroll requests.  Runs hipcc on the product sources (device code only,
the Makefile's flags) with -Rpass-analysis=kernel-resource-usage, as tools/resource_usage.py does; the diagnostic
build (BF_DIAG) is not checked."""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dpdk_dc_sand_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
SOURCES = ["bf_coeff.hip", "bf_reorder.hip", "bf_beamform.hip", "bf_fused.hip", "bf_wide.hip", "bf_wide_i8.hip",
           "bf_q14table.hip", "bf_requant.hip", "bf_study.hip"]


def _usage(src):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
           "-x", "hip", "--cuda-device-only", "-c", os.path.join(CSRC, src), "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    kernels, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            kernels.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    warnings = [ln for ln in r.stderr.splitlines() if "warning:" in ln]
    return src, kernels, warnings


@pytest.fixture(scope="module")
def usage():
    if not os.path.exists(HIPCC) or shutil.which("c++filt") is None:
        pytest.skip("hipcc not available")
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        return {src: (k, w) for src, k, w in ex.map(_usage, SOURCES)}


def test_no_scratch_in_any_product_kernel(usage):
    spills = []
    for src, (kernels, _) in usage.items():
        assert kernels, f"no kernels reported for {src}"
        for k in kernels:
            if int(k.get("ScratchSize [bytes/lane]", "0")) != 0:
                name = subprocess.run(["c++filt"], input=k["name"], capture_output=True, text=True).stdout.strip()
                spills.append(f"{src}: {name[:120]} scratch {k['ScratchSize [bytes/lane]']} B/lane, "
                              f"VGPRs {k.get('VGPRs')}")
    assert not spills, "\n".join(spills)


def test_no_compiler_warnings_in_product_sources(usage):
    warnings = [w for _, (_, ws) in usage.items() for w in ws]
    assert not warnings, "\n".join(warnings[:20])


def test_no_wide_store_data_hazard_in_product_kernels():
    """No product kernel lets a VALU rewrite a wide store's data VGPRs right behind the store (tools/
    store_hazard_check.py: the gfx950 store-data hazard hipcc left unguarded once, wrong bytes ~1e-5 of the time)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import store_hazard_check as shc
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        isas = dict(zip(SOURCES, ex.map(lambda s: shc.compile_isa(os.path.join(CSRC, s)), SOURCES)))
    bad = []
    for src, asm in isas.items():
        total, hits = shc.scan(asm, window=2)
        bad += [f"{src}: {fn[:90]}: {st} / {n}" for fn, st, n, _ in hits]
    assert not bad, "\n".join(bad[:20])


def test_no_inline_asm_result_reaches_an_mfma_unpadded():
    """An inline-asm VGPR result read by an MFMA within two instructions of the statement needs the statement to end
    in s_nop 1 (hipcc pads one state after an asm statement; VALU write -> MFMA operand read needs 2): the persistent
    float kernel's uint8 form read a stale fragment in one accumulator without it (tools/store_hazard_check.py)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import store_hazard_check as shc
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        isas = dict(zip(SOURCES, ex.map(lambda s: shc.compile_isa(os.path.join(CSRC, s)), SOURCES)))
    bad = [f"{src}: {fn[:90]}: {a} -> +{n} {m}" for src, asm in isas.items()
           for fn, a, m, n in shc.scan_asm_to_mfma(asm, window=2)]
    assert not bad, "\n".join(bad[:20])


def test_store_hazard_scanner_counts_nop_wait_states():
    """The scanner's window is wait states, not instructions: `s_nop 0` is one state (a VALU right after it still
    hits a 2-state window), `s_nop 1` two."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import store_hazard_check as shc
    head = "_Zk:\n  buffer_store_dwordx4 v[80:83], v1, s[0:3], 0 offen\n"
    assert len(shc.scan(head + "  s_nop 0\n  v_add_u32 v83, v1, v2\n")[1]) == 1
    assert len(shc.scan(head + "  s_nop 1\n  v_add_u32 v83, v1, v2\n")[1]) == 0
    assert len(shc.scan(head + "  s_nop 0\n  s_nop 0\n  v_add_u32 v83, v1, v2\n")[1]) == 0
    assert len(shc.scan(head + "  v_add_u32 v9, v1, v2\n  v_add_u32 v83, v1, v2\n")[1]) == 1
    assert len(shc.scan(head + "  v_add_u32 v9, v1, v2\n  s_nop 0\n  v_add_u32 v83, v1, v2\n")[1]) == 0
    assert len(shc.scan(head + "  v_add_u32 v84, v1, v2\n")[1]) == 0
    assert shc.nop_states("s_nop 0x3") == 4


def test_lds_dma_ring_slot_reads_wait_for_their_dma():
    """the config-4 int8 kernel's voltage ring (w32r) relies on hipcc's vmcnt bookkeeping for its LDS-DMA
    slots.  Replaying the vector-memory queue of its main loop in issue order (tools/store_hazard_check.py
    scan_lds_dma_ring), every slot read finds at most the next step's 4 DMA pieces outstanding -- the DMA that wrote
    the slot being read has retired -- in both instances."""
    import re
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import store_hazard_check as shc
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    asm = shc.compile_isa(os.path.join(CSRC, "bf_wide_i8.hip"))
    kernels = sorted(set(re.findall(r"^(_Z\w*beamform_fused_i8_w32r_kernel\w*):", asm, flags=re.M)))
    assert len(kernels) == 2, kernels
    for k in kernels:
        checked, bad = shc.scan_lds_dma_ring(asm, k, depth=2)
        assert checked == 64, (k, checked)  # 16 steps x 4 two-row reads per channel
        assert not bad, (k, bad[:8])


def test_lds_dma_ring_check_flags_an_early_read():
    """The replay itself: a slot read issued while its own DMA is still counted is flagged; after the right
    s_waitcnt it is not."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import store_hazard_check as shc
    body = ["_Zk:", ".LBB0_1:",
            "buffer_load_dwordx4 v1, s[0:3], s4 offen lds"] * 1 + \
        ["buffer_load_dwordx4 v1, s[0:3], s4 offen lds"] * 3 + \
        ["{wait}", "ds_read2st64_b64 v[2:5], v6 offset1:1", "s_cbranch_scc1 .LBB0_1", ".Lfunc_end0:"]
    early = "\n".join(body).replace("{wait}", "s_waitcnt vmcnt(8)")
    ok = "\n".join(body).replace("{wait}", "s_waitcnt vmcnt(4)")
    assert shc.scan_lds_dma_ring(early, "_Zk", depth=2)[1]
    assert shc.scan_lds_dma_ring(ok, "_Zk", depth=2) == (1, [])
