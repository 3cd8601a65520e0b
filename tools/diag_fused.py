"""Ablation timing of the fused kernel (diagnostic library build/libbf_diag.so) + HBM stream ceilings.

Modes: 1 skip coefficient generation, 2 skip MFMA (cheap VALU reduction instead), 4 skip stores,
8 skip loads (synthetic registers).  Times are HIP-event averages over N launches, 2 rotating buffer sets."""
import ctypes, os, sys
import os as _os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from dpdk_dc_sand_amd import _lib, accel

lib = _lib.load(os.path.join(ROOT, "build", "libbf_diag.so"))
V, I, D, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
lib.bf_diag_fused.argtypes = [I, V, V, V, I, I, I, I, I, I, D, V]
lib.bf_diag_stream.argtypes = [V, V, S, S, I, I, V]
ctx = accel.create_some_context()
q = ctx.create_command_queue()
B, C, T, A, M = [int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (8, 4096, 256, 64, 16))]
nin = B * A * C * T * 4
nout = B * 2 * C * T * 2 * M * 4
bufs = [(accel.DeviceArray(ctx, (nin,), np.uint8), accel.DeviceArray(ctx, (nout,), np.uint8)) for _ in range(2)]
_rng = np.random.default_rng(1)
for xi, yo in bufs:  # random voltages: constant data runs at a higher clock (MI355X_MICROARCH.md) and flatters
    if _os.environ.get("DIAG_CONST", "0") == "1":
        _lib.call("bf_memset", xi.ptr, 7, nin, q.handle)
    else:
        xi.set(q, _rng.integers(0, 256, nin, dtype=np.uint8))
dv = accel.DeviceArray(ctx, (M * A * 4,), np.float32)
_drng = np.random.default_rng(0)
if _os.environ.get("DIAG_DV", "bench") == "tiny":  # near-zero phases: constant (1, 0) phasors, higher clocks
    dv.set(q, _drng.uniform(0, 1e-8, M * A * 4).astype(np.float32))
else:  # the bench's delay model (random phasors: realistic MFMA operand toggling / power)
    _d = np.zeros((M, A, 4), np.float32)
    _d[..., 0] = _drng.uniform(0, 10 / 1712e6, (M, A))
    _d[..., 1] = _drng.uniform(-1e-9, 1e-9, (M, A))
    _d[..., 2] = _drng.uniform(-np.pi, np.pi, (M, A))
    _d[..., 3] = _drng.uniform(-1, 1, (M, A))
    dv.set(q, _d.reshape(-1))
alg = nin + nout


def timeit(fn, n=20):
    for i in range(3):
        fn(i)
    e0, e1 = accel.Event(), accel.Event()
    q.finish(); e0.record(q)
    for i in range(n):
        fn(i)
    e1.record(q); q.finish()
    return e1.time_since(e0) / n


names = {64: "occ 4 bound", 96: "occ 3 bound", 160: "channel-fastest (old)", 192: "batch-fastest", 224: "xcd x batch",
         288: "nt stores (xcd)", 0: "full (fast coef)", 128: "cached loads", 256: "nt stores", 384: "cached loads+nt st",
         16: "full (exact coef)", 1: "no-coef", 2: "no-mfma", 4: "no-store", 8: "no-load",
         3: "no-coef,no-mfma", 5: "no-coef,no-store", 9: "no-coef,no-load", 7: "loads only", 11: "stores only"}
print(f"shape B={B} C={C} T={T} A={A} M={M}: in {nin/2**30:.2f} GiB out {nout/2**30:.2f} GiB")
ROUNDS = int(_os.environ.get("DIAG_ROUNDS", "1"))
if "wide" in _os.environ.get("DIAG_KERNELS", ""):
    lib.bf_diag_wide.argtypes = [I, I, V, V, V, I, I, I, I, I, I, D, V]
    wnames = {0: "full (fast coef)", 1: "no-coef", 2: "no-mfma", 4: "no-store", 8: "no-load", 3: "no-coef,no-mfma",
              5: "no-coef,no-store", 16: "nt stores", 32: "branchy phasor validity", 64: "round-3 polynomial phasors",
              1000: "buffer loads", 1001: "buffer loads, no-coef", 1004: "buffer loads, no-store",
              1064: "buffer loads, round-3 polynomial phasors", 128: "round-3 pair index math",
              1128: "buffer loads, round-3 pair index math", 1256: "buffer loads, prio contraction",
              1512: "buffer loads, prio phasors", 2024: "buffer loads, 16-pair model batches",
              9192: "buffer loads, model loads pipelined, late voltages",
              20004: "persistent 1 wave/SIMD, ring 4", 20008: "persistent 1 wave/SIMD, ring 8",
              20054: "persistent, ring 4, no-store", 20058: "persistent, ring 8, no-store"}
    if _os.environ.get("WIDE_MODES"):
        wnames = {int(m): wnames.get(int(m), str(m)) for m in _os.environ["WIDE_MODES"].split(",")}
    Ctot = int(_os.environ.get("DIAG_CTOT", "32768"))
    ref0 = None  # the first form's beams: every later form (tw) is compared with it too (22: both slabs per workgroup)
    for tw in [int(t) for t in _os.environ.get("WIDE_TW", "2,1").split(",")]:
        ref = None
        full = [m for m in wnames if m % 1000 in (0, 64, 128) or (1000 <= m < 20000 and (m - 1000) & 8192)
                or 20000 <= m < 20050 or m in (20104, 20108)]
        for mode in full:  # float beams of the full forms against mode 0
            assert lib.bf_diag_wide(mode, tw, bufs[0][0].ptr, dv.ptr, bufs[0][1].ptr, B, C, T, A, M, Ctot, 1 / 1712e6,
                                    q.handle) == 0
            y = bufs[0][1].get(q).view(np.float32).astype(np.float64)
            if ref is None:
                ref = y
            if ref0 is None:
                ref0 = y
            print(f"  wide tw={tw} mode {mode:4d} vs mode {min(wnames)}: max |dy| {np.abs(y - ref).max():.3e} "
                  f"(max |y| {np.abs(ref).max():.3e}); vs the first form: max |dy| {np.abs(y - ref0).max():.3e}")
            bad = np.argwhere(np.abs(y - ref).reshape(B, 2, C, T, 2 * M) > 1e-2)
            if len(bad):
                import collections
                bb, pp, cc, tt, col = bad.T
                for nm, v in {"pol": pp, "c%32": cc % 32, "c": cc, "t": tt, "t//64 (wave)": tt // 64,
                              "t%64//4 (tl)": (tt % 64) // 4, "t%4 (i)": tt % 4, "col": col, "beam": col // 2}.items():
                    cnt = collections.Counter(v.tolist())
                    print(f"     {nm:14s} {len(cnt):5d} distinct; top {cnt.most_common(8)}")
        res = {m: [] for m in wnames}
        for r in range(int(_os.environ.get("DIAG_ROUNDS", "1"))):
            for mode in wnames:
                res[mode].append(timeit(lambda i: lib.bf_diag_wide(mode, tw, bufs[i % 2][0].ptr, dv.ptr, bufs[i % 2][1].ptr,
                                                                   B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)))
        for mode in [m for m in wnames if 20100 <= m < 150000 and ((m - 20100) // 10) & 4096]:
            # the persistent kernel's phase stamps (Mode 4096): per-wave s_memtime sums over the output's first bytes
            assert lib.bf_diag_wide(mode, tw, bufs[0][0].ptr, dv.ptr, bufs[0][1].ptr, B, C, T, A, M, Ctot, 1 / 1712e6,
                                    q.handle) == 0
            st = bufs[0][1].get(q).view(np.uint64)[1 << 24:(1 << 24) + 256 * 8 * 4].reshape(-1, 4).astype(np.float64)
            st = st[st[:, 3] > 0]
            tot = st[:, :3].sum(1)
            print(f"  wide stamps mode {mode}: per wave {tot.mean():.0f} clocks over {st[:, 3].mean():.1f} channels: "
                  f"steps {st[:, 0].mean() / tot.mean():.3f}, store issue {st[:, 1].mean() / tot.mean():.3f}, "
                  f"barrier {st[:, 2].mean() / tot.mean():.3f}; per channel steps {st[:, 0].mean() / st[:, 3].mean():.0f}, "
                  f"stores {st[:, 1].mean() / st[:, 3].mean():.0f}, barrier {st[:, 2].mean() / st[:, 3].mean():.0f}")
        for mode in wnames:
            ts = sorted(res[mode])
            print(f"  wide tw={tw} mode {mode:2d} {wnames[mode]:18s} median {ts[len(ts) // 2] * 1e6:8.1f} us  "
                  f"alg {alg / ts[len(ts) // 2] / 1e9:7.1f} GB/s")
if "w32t" in _os.environ.get("DIAG_KERNELS", ""):  # the table-driven 32-beam int8 kernel alone (+ its generator)
    lib.bf_diag_w32_table.argtypes = [I, V, V, V, V, I, I, I, I, I, I, D, V]
    Ctot = int(_os.environ.get("DIAG_CTOT", "32768"))
    tb = accel.DeviceArray(ctx, (B * C * ((M + 31) // 32) * 1024 * 8 + 4096,), np.uint32)
    assert lib.bf_diag_w32_table(-1, bufs[0][0].ptr, dv.ptr, bufs[0][1].ptr, tb.ptr, B, C, T, A, M, Ctot, 1 / 1712e6,
                                 q.handle) == 0
    tnames = {-1: "generator only", 0: "full (early table)", 1: "no table", 4: "no-store", 8: "no-load",
              9: "no table,no-load", 12: "no-store,no-load"}
    base = {m: v for m, v in tnames.items() if m >= 0}
    tnames.update({100 + m: v.replace("early", "late") + (" (late)" if m else "") for m, v in base.items()})
    tnames.update({300 + m: v.replace("early ", "") + " [unrolled NB3]" for m, v in base.items()})
    tnames.update({400 + m: v.replace("early ", "") + " [unrolled NB4]" for m, v in base.items()})
    tnames.update({200 + m: v.replace("early ", "") + " [unrolled NB2: the product form]" for m, v in base.items()})
    tnames.update({220: "full [NB2, 2 ch/WG]", 240: "full [NB2, 8 ch/WG]", 260: "full [NB2, 16 ch/WG]",
                   280: "full [NB2, 8 ch/WG, early table]"})
    tnames.update({500 + m: v + " [unrolled NB3, early table]" for m, v in base.items()})
    # round 4: buffer-resource voltage loads (SGPR row offsets, no per-load VALU addressing) + power-of-two FMA requant
    tnames.update({900 + m: v.replace("early ", "") + " [NB2, 8 ch, buffer loads]" for m, v in base.items()})
    tnames.update({920 + m: v.replace("early ", "") + " [NB3, 8 ch, buffer loads]" for m, v in base.items()})
    tnames.update({940 + m: v.replace("early ", "") + " [NB2, 8 ch, pointer loads, pow2]" for m, v in base.items()})
    # round 4: the next tile's A fragments read while the current tile's MFMAs issue (w32_mfma_pf)
    tnames.update({1532 + m: v.replace("early ", "") + " [NB2, 8 ch, buffer loads, A prefetch]" for m, v in base.items()
                   if m in (0, 1, 4, 8)})
    tnames.update({1564: "full [NB2, 8 ch, buffer loads, nt table loads]", 1628: "full [NB2, 8 ch, buffer loads, nt voltage loads]",
                   1692: "full [NB2, 8 ch, buffer loads, nt table + voltage loads]"})
    # round 5: the LDS-DMA voltage ring over the halved image (beamform_fused_i8_w32r_kernel) + its Mode bits
    tnames.update({2000: "full [w32r: DMA ring, halved image]", 2004: "no-store [w32r]", 2008: "no voltage DMA [w32r]",
                   2012: "no-store,no voltage DMA [w32r]", 2016: "no table [w32r]", 2024: "no table,no voltage DMA [w32r]"})
    tnames.update({1756: "TA test: 16-B loads, wrong beams (spills)"})
    # 700 + m: the output-stationary LDS-DMA kernel (bf_wide_i8os.hip) on the same table; m = its Mode bits
    tnames.update({700 + m: v.replace("early ", "") + " [os, LDS-DMA]" for m, v in base.items() if m in (0, 1, 4, 8, 9, 12)})
    tnames.update({702: "no-mfma [os]", 705: "no table,no-store [os]",
                   713: "no table,no-store,no-load [os]", 715: "skeleton (barriers, LDS reads, VALU) [os]"})
    tnames.update({729: "no table/store/load, no LDS frag reads [os]", 745: "no table/store/load, no barrier [os]",
                   761: "MFMA + epilogue VALU only [os]", 732: "full, no barrier (races) [os]"})
    # 800 + m: the same kernel's 8-wave, one-workgroup-per-CU form (half items, both slabs per workgroup)
    tnames.update({800 + m - 700: v.replace("[os", "[os8") for m, v in list(tnames.items()) if 700 <= m < 800})
    if _os.environ.get("W32T_MODES"):
        tnames = {int(m): tnames.get(int(m), str(m)) for m in _os.environ["W32T_MODES"].split(",")}
    lib.bf_diag_i8_os.argtypes = [I, V, V, V, I, I, I, I, I, V]

    def w32t_call(mode, i):
        if 700 <= mode < 900:
            return lib.bf_diag_i8_os(mode - 700, bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, tb.ptr, B, C, T, A, M, q.handle)
        return lib.bf_diag_w32_table(mode, bufs[i % 2][0].ptr, dv.ptr, bufs[i % 2][1].ptr, tb.ptr, B, C, T, A, M, Ctot,
                                     1 / 1712e6, q.handle)
    for mode in list(tnames):
        if mode >= 0 and w32t_call(mode, 0) != 0:
            print(f"  w32t mode {mode}: launch failed: {lib.bf_last_error().decode(errors='replace')}")
            tnames.pop(mode)
    for alt in (220, 240, 260, 280, 700, 900, 920, 940, 1532, 1564, 1628, 1692, 2000):  # another form's int8 beams, same input and table: bitwise equal
        if alt not in tnames:
            continue
        outs = []
        for mode in (300, alt):
            _lib.call("bf_memset", bufs[0][1].ptr, 0, nout // 4, q.handle)
            assert w32t_call(mode, 0) == 0
            outs.append(bufs[0][1].get(q)[: nout // 4].copy())
        print(f"  mode {alt} vs 300 int8 beams: {'bitwise equal' if np.array_equal(*outs) else 'DIFFERENT'} "
              f"({int((outs[0] != outs[1]).sum())} bytes differ)")
    alg8 = nin + nout // 4
    res = {m: [] for m in tnames}
    for r in range(int(_os.environ.get("DIAG_ROUNDS", "1"))):
        for mode in tnames:
            res[mode].append(timeit(lambda i: w32t_call(mode, i)))
    for mode in tnames:
        ts = sorted(res[mode])
        print(f"  w32t mode {mode:3d} {tnames[mode]:28s} median {ts[len(ts) // 2] * 1e6:8.1f} us  "
              f"alg {alg8 / ts[len(ts) // 2] / 1e9:7.1f} GB/s")
if "w32chunk" in _os.environ.get("DIAG_KERNELS", ""):  # generator + contraction, whole vs channel-chunked launches
    lib.bf_diag_w32_launch.argtypes = [V, V, V, V, I, I, I, I, I, I, D, V]
    Ctot = int(_os.environ.get("DIAG_CTOT", "32768"))
    tb2 = accel.DeviceArray(ctx, (B * C * ((M + 31) // 32) * 1024 * 8 + 4096,), np.uint32)
    # "n": generator + contraction alternated over n channel chunks on one stream; "oN": the generator's N chunks on
    # a second stream beside the contraction chunks (BF_W32_OVERLAP)
    chunks = _os.environ.get("W32_CHUNKS", "1,2,4,8").split(",")

    def set_chunks(n):
        _os.environ["BF_W32_CHUNKS"] = "1" if n.startswith("o") else n
        _os.environ["BF_W32_OVERLAP"] = n[1:] if n.startswith("o") else "1"
    outs, res = {}, {n: [] for n in chunks}
    for n in chunks:
        set_chunks(n)
        _lib.call("bf_memset", bufs[0][1].ptr, 0, nout // 4, q.handle)
        assert lib.bf_diag_w32_launch(bufs[0][0].ptr, dv.ptr, bufs[0][1].ptr, tb2.ptr, B, C, T, A, M, Ctot,
                                      1 / 1712e6, q.handle) == 0
        q.finish()
        outs[n] = bufs[0][1].get(q)[: nout // 4].copy()
    print("  chunked / overlapped == whole launch (int8 beams):",
          all(np.array_equal(outs[chunks[0]], o) for o in outs.values()))
    for r in range(ROUNDS):
        for n in chunks:
            set_chunks(n)
            res[n].append(timeit(lambda i: lib.bf_diag_w32_launch(bufs[i % 2][0].ptr, dv.ptr, bufs[i % 2][1].ptr,
                                                                  tb2.ptr, B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)))
    for n in chunks:
        ts = sorted(res[n])
        kind = f"{n[1:]} chunk(s) overlapped on two streams" if n.startswith("o") else f"{n} channel chunk(s)"
        print(f"  generator + contraction, {kind}: median {ts[len(ts) // 2] * 1e6:8.1f} us")
    _os.environ.pop("BF_W32_CHUNKS")
    _os.environ.pop("BF_W32_OVERLAP")
if "w8" in _os.environ.get("DIAG_KERNELS", ""):
    lib.bf_diag_w8.argtypes = [I, V, V, V, I, I, I, I, I, I, D, V]
    w8names = {0: "full (fast+fixup)", 128: "exact-only coef", 1: "no-coef", 2: "no-mfma", 4: "no-store", 8: "no-load",
               5: "no-coef,no-store", 3: "no-coef,no-mfma", 9: "no-coef,no-load", 13: "no-coef,no-load,no-st",
               19: "slab0 only,no-coef,no-mfma", 35: "nt loads,no-coef,no-mfma", 51: "slab0,nt,no-coef,no-mfma",
               32: "nt loads (full)", 17: "slab0 only,no-coef", 67: "16 ant rows,no-coef,no-mfma",
               83: "16 rows,slab0,no-coef,no-mfma", 259: "xcd-range,no-coef,no-mfma", 275: "xcd-range,slab0,nc,nm",
               256: "xcd-range (full)", 512: "branchy phasors (old)",
               1000: "w32 full", 1001: "w32 no-coef", 1002: "w32 no-mfma", 1003: "w32 no-coef,no-mfma",
               1004: "w32 no-store", 1008: "w32 no-load", 1009: "w32 no-coef,no-load", 1013: "w32 nc,nl,ns",
               1016: "w32 nt stores", 1017: "w32 nt stores, no-coef"}
    if _os.environ.get("W8_MODES"):
        w8names = {int(m): w8names.get(int(m), str(m)) for m in _os.environ["W8_MODES"].split(",")}
    Ctot = int(_os.environ.get("DIAG_CTOT", "32768"))
    alg8 = nin + nout // 4  # int8 beams: 2 B per complex beam sample vs 8 (r2's files used nout // 16: understated)
    res = {m: [] for m in w8names}
    for r in range(int(_os.environ.get("DIAG_ROUNDS", "1"))):
        for mode in w8names:
            res[mode].append(timeit(lambda i: lib.bf_diag_w8(mode, bufs[i % 2][0].ptr, dv.ptr, bufs[i % 2][1].ptr,
                                                             B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)))
    if _os.environ.get("W8_AB"):  # interleaved A/B of the load form (buffer resource vs pointer), full kernel
        ab = {"buffer": [], "pointer": []}
        for r in range(int(_os.environ.get("DIAG_ROUNDS", "1"))):
            for form, val in (("buffer", "1"), ("pointer", "0")):
                _os.environ["BF_W8_BUFFER"] = val
                ab[form].append(timeit(lambda i: lib.bf_diag_w8(0, bufs[i % 2][0].ptr, dv.ptr, bufs[i % 2][1].ptr,
                                                                B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)))
        for form, ts in ab.items():
            ts = sorted(ts)
            print(f"  w8 full, {form:7s} loads  median {ts[len(ts) // 2] * 1e6:8.1f} us  min {ts[0] * 1e6:8.1f} us")
    for mode in w8names:
        ts = sorted(res[mode])
        print(f"  w8 mode {mode:2d} {w8names[mode]:18s} median {ts[len(ts) // 2] * 1e6:8.1f} us  "
              f"alg {alg8 / ts[len(ts) // 2] / 1e9:7.1f} GB/s")
names_i8 = {0: "full (fast+fixup coef, occ 3)", 128: "exact-only coef", 16: "fast coef (inexact)", 1: "no-coef", 2: "no-mfma", 3: "no-coef,no-mfma", 4: "no-store",
            5: "no-coef,no-store", 7: "loads only", 8: "no-load", 64: "occupancy 2", 32: "contig stores(bad)",
            65: "occ 2, no-store", 1024: "serial coef", 2048: "pol order", 3072: "serial+pol order",
            4096: "occ4 (spills)", 7168: "occ4 serial+pol", 6144: "occ4 pol order",
            262144: "batch-fastest order", 524288: "xcd x batch order", 1048576: "xcd range, batch fast", 2097152: "channel-fastest (old)", 4194304: "xcd flat (b, c)", 8388608: "xcd 64-ch blocks", 65536: "prio while loading", 131072: "prio while storing", 8192: "plain stores", 16384: "plain loads", 24576: "plain loads+stores"}
alg_i8 = nin + nout // 4
if _os.environ.get("I8_AB"):  # interleaved A/B: int8 item kernel with uniform-base (A == 64) vs clamped addressing
    ab = {"uniform": [], "clamped": []}
    for r in range(ROUNDS):
        for form, val in (("uniform", "1"), ("clamped", "0")):
            _os.environ["BF_I8_A64"] = val
            ab[form].append(timeit(lambda i: lib.bf_diag_fused(512, bufs[i % 2][0].ptr, dv.ptr, bufs[i % 2][1].ptr,
                                                               B, C, T, A, M, C, 1 / 1712e6, q.handle)))
    for form, ts in ab.items():
        ts = sorted(ts)
        print(f"  i8 full, {form:8s} addressing  median {ts[len(ts) // 2] * 1e6:8.1f} us  min {ts[0] * 1e6:8.1f} us")
names_f8 = {0: "full (f32 contract)", 1: "no-coef", 2: "no-mfma", 4: "no-store", 5: "no-coef,no-store", 8: "no-load",
            128: "cached loads", 64: "occ 4 bound", 96: "occ 3 bound", 16: "exact coef, occ 4", 80: "exact coef",
            65: "occ 4, no-coef", 68: "occ 4, no-store", 69: "occ 4, no-coef,no-store", 72: "occ 4, no-load"}
names_fs = {0: "staged 1 KiB f32 stores", 4: "staged, no-store", 128: "staged, cached loads", 256: "staged, nt stores",
            384: "staged, cached loads, nt st", 192: "staged, cached, occ 3"}
for kbase, kname in ((32, "item"), (512, "i8"), (8192, "f8"), (16384, "fs")):
    if _os.environ.get("DIAG_KERNELS", "item,i8").find(kname) < 0:
        continue
    only = _os.environ.get("DIAG_MODES")
    modes = list(names_i8 if kname == "i8" else names_f8 if kname == "f8" else names_fs if kname == "fs" else names)
    if only:
        modes = [m for m in modes if str(m) in only.split(",")]
    res = {m: [] for m in modes}
    for r in range(ROUNDS):  # interleaved rounds (one process, same data): A/B-safe
        for mode in modes:
            res[mode].append(timeit(lambda i: lib.bf_diag_fused(kbase + mode, bufs[i % 2][0].ptr, dv.ptr,
                                                                bufs[i % 2][1].ptr, B, C, T, A, M, C, 1 / 1712e6,
                                                                q.handle)))
    for mode in modes:
        ts = sorted(res[mode])
        med, mn = ts[len(ts) // 2], ts[0]
        nm, ab = ((names_i8[mode], alg_i8) if kname == "i8" else (names_f8[mode], alg_i8) if kname == "f8"
                  else (names_fs[mode], alg) if kname == "fs" else (names[mode], alg))
        print(f"  {kname} mode {mode:3d} {nm:18s} median {med*1e6:8.1f} us  min {mn*1e6:8.1f} us  "
              f"alg {ab/med/1e9:7.1f} GB/s  ({len(ts)} rounds)")
if _os.environ.get("DIAG_F8_CMP"):  # int8-via-f32 variants against the product order, bitwise (int8 beams)
    outs = {}
    for mode in [int(m) for m in _os.environ["DIAG_F8_CMP"].split(",")]:
        assert lib.bf_diag_fused(8192 + mode, bufs[0][0].ptr, dv.ptr, bufs[0][1].ptr, B, C, T, A, M, C, 1 / 1712e6,
                                 q.handle) == 0
        outs[mode] = bufs[0][1].get(q)[:B * 2 * C * T * 2 * M].copy()
    ref_mode = min(outs)
    for mode, o in outs.items():
        n = int(np.count_nonzero(o != outs[ref_mode]))
        print(f"  f8 mode {mode} vs mode {ref_mode}: {n} of {o.size} int8 beams differ", flush=True)
if _os.environ.get("DIAG_MIX"):  # the int8 path's 4:1 read:write mix, uniformly interleaved
    for grid in (1024, 2048, 4096, 8192, 16384):
        for code, nm in ((200, "nt load+store"), (201, "nt load")):
            t = timeit(lambda i: lib.bf_diag_stream(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, nin, nin // 4, grid, code,
                                                    q.handle))
            print(f"  mix grid {grid:5d} {nm:14s} {t*1e6:8.1f} us  {(nin + nin // 4)/t/1e9:7.1f} GB/s")
if _os.environ.get("DIAG_STREAMS", "1") == "1":
    for grid in (512, 1024, 2048):
        for unroll, uname in ((1, "plain"), (101, "nt-store"), (102, "nt-load"), (103, "nt-both")):
            for (ri, wo, nm) in ((nin, nout, "read+write"), (nin, 0, "read only"), (0, nout, "write only")):
                t = timeit(lambda i: lib.bf_diag_stream(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, ri, wo, grid, unroll,
                                                        q.handle))
                print(f"  stream grid {grid:5d} {uname:8s} {nm:11s} {t*1e6:8.1f} us  {(ri + wo)/t/1e9:7.1f} GB/s")
if _os.environ.get("DIAG_ITEMREAD"):  # the wide kernels' item-major read pattern vs an antenna-major sweep
    lib.bf_diag_item_read.argtypes = [V, V, I, I, I, I, I, V]
    R = T * 4
    t = timeit(lambda i: lib.bf_diag_stream(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, nin, 0, 2048, 102, q.handle))
    print(f"  linear nt-load read-only   {t*1e6:8.1f} us  {nin/t/1e9:7.1f} GB/s")
    for pat, pname in ((0, "item, 1 KiB rows"), (1, "item, w8 4x256 B"), (2, "run, antenna-major")):
        for grid in (256, 512, 1024):
            for ui, u in ((0, 4), (1, 8), (2, 16)):
                t = timeit(lambda i: lib.bf_diag_item_read(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, A, C, R, grid,
                                                           10 * pat + ui, q.handle))
                print(f"  item-read {pname:20s} grid {grid:5d} U {u:2d} {t*1e6:8.1f} us  {nin/t/1e9:7.1f} GB/s")
if "table" in _os.environ.get("DIAG_KERNELS", ""):  # the MatrixMultiply drop-in's ring kernel at 256 ants x 64 beams
    lib.bf_diag_table.argtypes = [I, I, V, V, V, I, I, I, I, I, I, V]
    tnames = {0: "full", 1: "no table staging", 2: "no-mfma", 4: "no-store", 8: "no x loads", 9: "no staging, no x",
              6: "no-mfma,no-store", 7: "staging+x loads only? (no mfma/store, no staging)"}
    xb = accel.DeviceArray(ctx, (B * 2 * C * T * A * 2,), np.uint8)
    wt = accel.DeviceArray(ctx, (B * 2 * C * 2 * A * 2 * M,), np.float32)
    yt = accel.DeviceArray(ctx, (B * 2 * C * T * 2 * M,), np.float32)
    _lib.call("bf_memset", wt.ptr, 0, wt.nbytes if hasattr(wt, "nbytes") else B * 2 * C * 2 * A * 2 * M * 4, q.handle)
    tb = 2 * B * 2 * C * T * A + B * 2 * C * 2 * A * 2 * M * 4 + B * 2 * C * T * 2 * M * 4
    tnames.update({100: "8-byte loads (full)", 108: "8-byte loads, no x loads", 200: "persistent (product)",
                   201: "persistent, no LDS staging", 204: "persistent, no stores", 208: "persistent, no x loads",
                   216: "persistent, no table loads", 217: "persistent, no table at all",
                   220: "persistent, no table loads/stores", 228: "persistent, only MFMA+staging",
                   240: "persistent G4 R8", 268: "persistent G4 R8, only MFMA+staging", 250: "persistent G4 R16",
                   278: "persistent G4 R16, only MFMA+staging", 400: "output-stationary", 404: "os, no stores",
                   408: "os, no x loads", 416: "os, no table loads", 428: "os, only MFMA+staging",
                   500: "os 4 waves", 528: "os 4 waves, only MFMA+staging", 600: "os 8 waves, occupancy 3 (no spill)"})
    if _os.environ.get("TABLE_MODES"):  # e.g. 0,100: interleaved A/B over DIAG_ROUNDS, medians
        tnames = {int(m): tnames.get(int(m), str(m)) for m in _os.environ["TABLE_MODES"].split(",")}
    for nts in [int(v) for v in _os.environ.get("TABLE_NTS", "2,4").split(",")]:
        res = {m: [] for m in tnames}
        for r in range(ROUNDS):
            for mode in tnames:
                res[mode].append(timeit(lambda i: lib.bf_diag_table(mode, nts, xb.ptr, wt.ptr, yt.ptr, B, 2, C, T // 16,
                                                                    A, M, q.handle)))
        for mode, nm in tnames.items():
            t = sorted(res[mode])[len(res[mode]) // 2]
            print(f"  table nts={nts} mode {mode:3d} {nm:26s} {t*1e6:8.1f} us  alg {tb/t/1e9:7.1f} GB/s")
if _os.environ.get("W32_STAMPS"):  # per-wave phase cycles of the 32-beam int8 kernel (s_memtime)
    lib.bf_diag_w32_stamps.argtypes = [V, V, V, V, I, I, I, I, I, I, D, V]
    Ctot = int(_os.environ.get("DIAG_CTOT", "32768"))
    grid = (B * C + 7) // 8 * 8 * ((M + 31) // 32)
    stamps = accel.DeviceArray(ctx, (grid * 4 * 4,), np.uint64)
    for _ in range(3):  # clocks settle
        assert lib.bf_diag_w32_stamps(bufs[0][0].ptr, dv.ptr, bufs[0][1].ptr, stamps.ptr, B, C, T, A, M, Ctot,
                                      1 / 1712e6, q.handle) == 0
    q.finish()
    st = stamps.get(q).reshape(grid, 4, 4).astype(np.float64)
    med = np.median(st.reshape(-1, 4), axis=0)
    mean = st.reshape(-1, 4).mean(axis=0)
    print(f"  w32 stamps (cycles per wave, median / mean over {grid * 4} waves): coefficient phase {med[0]:.0f} / "
          f"{mean[0]:.0f}, contraction {med[1]:.0f} / {mean[1]:.0f}, requant+stores {med[2]:.0f} / {mean[2]:.0f}, "
          f"total {med[3]:.0f} / {mean[3]:.0f}")
