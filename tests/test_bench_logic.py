"""CPU tests of bench.py's bookkeeping and of the timed-region rocprof summary (tools/kernel_stats.py): the real-time
factor against MeerKAT ingest (BeamformerCoefficientTest.cu:422-465), the kernel named for each workload's roofline,
the readable kernel names of the per-step split, and that only the dispatches between a region's two marker
dispatches are summarised (warm-up, clock-settle and contract-check launches excluded)."""
import csv
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import kernel_stats  # noqa: E402


def test_realtime_factor_against_meerkat_ingest():
    wl = bench.WORKLOADS["cfg3"]
    r = bench.realtime(wl, 1, 2475.0)
    need = 64 * 2 * 4096 * (1712e6 / 8192) / 1e9  # 109.57 Gsamples/s for one 4096-channel band
    assert r["ingest_need_Gsamples_s"] == pytest.approx(need, abs=0.01)
    assert r["realtime_factor"] == pytest.approx(2475.0 / need, abs=0.01)
    r8 = bench.realtime(wl, 8, 8 * 2475.0)  # 8 X-engines: 8x the band, 8x the rate
    assert r8["ingest_need_Gsamples_s"] == pytest.approx(8 * need, abs=0.1)
    assert r8["realtime_factor"] == pytest.approx(r["realtime_factor"], abs=0.01)


@pytest.mark.parametrize("workload,out_int8,contract,table,expected", [
    ("cfg3", True, "q14", "on", "beamform_fused_i8_item_kernel"),
    ("cfg3", True, "f32", "on", "beamform_fused_item_kernel"),
    ("cfg3", False, "q14", "on", "beamform_fused_item_kernel"),
    ("cfg2", True, "q14", "on", "beamform_fused_i8_item_kernel"),
    ("cfg4", True, "q14", "on", "beamform_fused_i8_w32r_kernel"),
    ("cfg4", True, "q14", "off", "beamform_fused_i8_w32_kernel"),
    ("cfg4", False, "q14", "on", "beamform_fused_wide_p2_kernel")])
def test_roofline_kernel_per_workload(workload, out_int8, contract, table, expected):
    assert bench.kernel_name(bench.WORKLOADS[workload], out_int8, contract, table) == expected


def test_roofline_kernel_unsigned_config4():
    # uint8 samples keep the register-ring table kernel (the DMA ring kernel is int8-only)
    assert bench.kernel_name(bench.WORKLOADS["cfg4"], True, "q14", "on", signed=False) == \
        "beamform_fused_i8_w32t_kernel"


def test_short_kernel_names():
    assert bench.short_kernel("void bf::(anonymous namespace)::q14_table_kernel<false>"
                              "(bf::(anonymous namespace)::Q14TableArgs)") == "q14_table_kernel<false>"
    assert bench.short_kernel("void bf::beamform_fused_i8_item_kernel<true, 2, true, 0, 3, true>(bf::FusedArgs)") \
        == "beamform_fused_i8_item_kernel<true, 2, true, 0, 3, true>"


def _trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for name, s, e in rows:
            w.writerow([name, s, e])


def test_timed_regions_keep_only_the_bracketed_dispatches(tmp_path):
    mark = "bf::bf_trace_mark_kernel(int)"
    rows = [("warmup_k", 0, 90),                                     # before the first region: excluded
            (mark, 100, 101), ("k_a", 110, 210), ("k_a", 220, 330), ("gen", 335, 345), (mark, 400, 401),
            ("contract_check", 410, 900),                            # between regions: excluded
            (mark, 1000, 1001), ("k_b", 1010, 1060), (mark, 1100, 1101)]
    p = tmp_path / "trace.csv"
    _trace(p, rows)
    regions = kernel_stats.region_stats(str(p))
    assert len(regions) == 2
    assert set(regions[0]) == {"k_a", "gen"} and set(regions[1]) == {"k_b"}
    assert regions[0]["k_a"]["Calls"] == 2 and regions[0]["k_a"]["AverageNs"] == pytest.approx(105.0)
    name, s = kernel_stats.dominant(regions[0])
    assert name == "k_a" and s["TotalDurationNs"] == 210
    assert kernel_stats.dominant(regions[0], "gen")[0] == "gen"
    out = tmp_path / "stats.csv"
    kernel_stats.write_csv(regions, str(out))
    with open(out) as f:
        got = list(csv.DictReader(f))
    assert [(r["Region"], r["Name"]) for r in got] == [("0", "k_a"), ("0", "gen"), ("1", "k_b")]


def test_mfma_block_and_contraction_split():
    """Every line's mfma block: algorithmic ops 8 A M per (b, p, c, t), issued ops two limbs x K = 2A (padded to the
    MFMA depth) x N = 2M (padded to 16); a two-kernel step (config 4's int8 path) also reports the contraction's own
    rates over its rocprof time and the generator's share of the step."""
    wl = bench.WORKLOADS["cfg4"]
    m = bench.mfma_util(wl, True, "q14", 464e-6)
    alg = 8.0 * 256 * 64 * 2 * 4096 * 256 * 1
    assert m["algorithmic"] == pytest.approx(alg / 464e-6 / 1e12, abs=0.1)
    assert m["issued"] == pytest.approx(2 * alg / 464e-6 / 1e12, abs=0.1)  # K, N unpadded here: 2 limbs = 2x
    assert m["peak"] == 5000.0 and m["unit"] == "TOPS"
    sec = {"avg_launch_us": 464.0, "mfma": m}
    bench.mfma_split(sec, {"avg_us": 398.0, "per_step_us_all_kernels": 463.0,
                           "kernels_us_per_step": {"w32t": 398.0, "q14_table_kernel<false>": 65.0}})
    c = sec["mfma"]["contraction_only"]
    assert c["kernel_us"] == 398.0
    assert c["issued"] == pytest.approx(m["issued"] * 464.0 / 398.0, abs=0.2)
    assert sec["mfma"]["generator_share_of_step"] == pytest.approx(65.0 / 463.0, abs=1e-3)
    f = bench.mfma_util(wl, False, "q14", 620e-6)  # float beams: f16 hi/lo on the dense F16 peak
    assert f["peak"] == 2500.0 and f["unit"] == "TFLOP/s"
    one = {"avg_launch_us": 620.0, "mfma": f}
    bench.mfma_split(one, {"avg_us": 620.0})  # one kernel per step: nothing to split
    assert "contraction_only" not in one["mfma"]


def test_pmc_mfma_busy():
    # the persistent f32 kernel's PMC (profiles/r5_f3_cfg4_wide_pmc.txt): 5.37e8 busy cycles over 1024 SIMDs and
    # 9.21e6 GPU-active cycles over 8 XCDs -> 45.5 % busy; no SQ pass -> None
    b = bench.pmc_mfma_busy({"FETCH_SIZE": 1.0, "WRITE_SIZE": 1.0, "SQ_VALU_MFMA_BUSY_CYCLES": 5.37e8,
                             "GRBM_GUI_ACTIVE": 9.21e6}, 589.6e-6)
    assert b["busy_frac"] == pytest.approx(0.4555, abs=1e-4)
    assert b["clock_GHz"] == pytest.approx(1.953, abs=1e-3)
    assert bench.pmc_mfma_busy({"FETCH_SIZE": 1.0, "WRITE_SIZE": 1.0}, 1e-3) is None
    assert bench.pmc_mfma_busy("unavailable", 1e-3) is None


def test_resolve_world_launch_and_mismatch():
    """`--gpus N` without a launcher: this process starts the N ranks; under torch.distributed.run --gpus must equal
    WORLD_SIZE (a mismatch would time a different number of ranks than the command names)."""
    a = bench.parse(["--gpus", "4"])
    assert bench.resolve_world(a, env={}) == (4, True)
    a = bench.parse([])
    assert bench.resolve_world(a, env={}) == (1, False) and a.gpus == 1
    a = bench.parse(["--gpus", "1"])
    assert bench.resolve_world(a, env={}) == (1, False)
    a = bench.parse(["--gpus", "2"])
    assert bench.resolve_world(a, env={"WORLD_SIZE": "2"}) == (2, False)
    a = bench.parse([])
    assert bench.resolve_world(a, env={"WORLD_SIZE": "8"}) == (8, False) and a.gpus == 8
    with pytest.raises(ValueError, match="WORLD_SIZE=2"):
        bench.resolve_world(bench.parse(["--gpus", "8"]), env={"WORLD_SIZE": "2"})
    with pytest.raises(ValueError, match="WORLD_SIZE=1"):
        bench.resolve_world(bench.parse(["--gpus", "2"]), env={"WORLD_SIZE": "1"})
    with pytest.raises(ValueError):
        bench.resolve_world(bench.parse(["--gpus", "0"]), env={})


def _run_bench(args, env_extra=None, timeout=120):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env)


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_its_own_ranks(n):
    """`python bench.py --gpus N` with no launcher (the driver's command form) runs N ranks that meet in the TCP
    rendezvous group: rank 0 reports N ranks, each with its own RANK and LOCAL_RANK (its device)."""
    import json
    r = _run_bench(["--gpus", str(n), "--rank-probe"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["gpus_arg"] == n and out["max_rank"] == n - 1
    assert [(g["rank"], g["local_rank"]) for g in out["ranks"]] == [(i, i) for i in range(n)]
    assert out["ranks_launched_by"] == "bench.py"


def test_bench_launcher_propagates_a_rank_failure():
    """A rank that fails (here: no GPU in this container) fails the launch with its status, and the run ends."""
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-secondary"], timeout=180)
    assert r.returncode != 0
    assert "exited with status" in r.stderr


def test_bench_gpus_mismatch_under_launcher_fails():
    r = _run_bench(["--gpus", "4", "--rank-probe"], env_extra={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_target_block():
    # cfg3 f32 beams on the r5 box: 4.295e9 B against a 759.28 us stream -> 0.707: 0.70 is 0.99 of the stream
    t = bench.target_block(4294983680.0, 759.28)
    assert t["ceiling_frac"] == pytest.approx(0.7071, abs=1e-4) and t["target_reachable"] is True
    assert t["target_needs_frac_of_ceiling"] == pytest.approx(0.70 / 0.7071, abs=1e-3)
    t = bench.target_block(2147483648.0, 428.32)  # a mix whose best stream is below 0.70
    assert t["target_reachable"] is False and t["target_needs_frac_of_ceiling"] > 1


def test_bench_launcher_stops_its_ranks_when_killed():
    """SIGTERM to the launching bench.py (e.g. a driver timeout) reaches its ranks: none outlives it."""
    import json
    import signal
    import subprocess
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rank-probe",
                          "--probe-sleep", "60"], stdout=subprocess.PIPE, text=True, cwd=ROOT, env=env)
    try:
        line = p.stdout.readline()
        pids = [g["pid"] for g in json.loads(line)["ranks"]]
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=30) == 128 + signal.SIGTERM
        deadline = time.monotonic() + 20
        alive = pids
        while alive and time.monotonic() < deadline:
            alive = [q for q in pids if os.path.exists(f"/proc/{q}") and
                     open(f"/proc/{q}/stat").read().split()[2] != "Z"]
            time.sleep(0.1)
        assert not alive, f"ranks {alive} outlived the launcher"
    finally:
        if p.poll() is None:
            p.kill()
