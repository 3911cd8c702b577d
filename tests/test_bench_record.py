"""bench.py's JSON line, assembled on CPU: the N = 1 line the driver reads,
and the N > 1 self-check fields (RCCL ranks, per-rank render and gather
times, slowest rank) gathered over 2 ranks through the torch-free
rendezvous, with a stub in place of the GPU render and the RCCL comm."""
import argparse
import multiprocessing as mp
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))

STATS = {"triangles": 1000036, "nodes": 551000, "build_ms": 45.0}
ROOF = {"bound": "hbm", "achieved": 3700.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.4625, "traffic": None}


def _args(steps=3):
    return argparse.Namespace(scene="c4", width=1920, height=1080, spp=1024, steps=steps, warmup=1, bvh="device")


def test_single_gpu_line_keeps_the_driver_contract():
    import bench

    out = bench.make_record(_args(), 1, 3 * 1.25, STATS, ROOF, None)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in out, k
    assert "ranks" not in out  # the N = 1 line is unchanged
    assert out["n_gpus"] == 1 and out["ms_per_step"] == 1250.0
    assert abs(out["value"] - 1920 * 1080 * 1024 / 1.25 / 1e6) < 0.01
    assert out["metric"] == bench.METRIC


def test_effective_cpus_caps_affinity_by_quota():
    import bench

    assert bench.effective_cpus({"nproc": 256, "affinity": 256, "quota": 16.0}) == 16
    assert bench.effective_cpus({"nproc": 256, "affinity": 256, "quota": 15.5}) == 16
    assert bench.effective_cpus({"nproc": 8, "affinity": 8, "quota": None}) == 8
    assert bench.effective_cpus({"nproc": 256, "affinity": 4, "quota": 16.0}) == 4


def _rank(rank, world, path, q):
    import bench
    import rendezvous

    g = rendezvous.FileGroup(rank, world, path=path, timeout=60)
    # stub timings: rank 1 renders slower, and rank 0 waits for it in the gather
    render_ms = 1000.0 + 100.0 * rank
    gather_ms = 2.0 + (100.0 if rank == 0 else 0.0)
    timed_s = 3 * (render_ms + gather_ms) / 1e3
    rows = g.allgather([timed_s, render_ms, gather_ms])
    per_rank = bench.per_rank_stats(rows, rccl_ranks=world)  # stub comm: ncclCommCount = world
    elapsed = max(r[0] for r in rows)
    out = bench.make_record(_args(), world, elapsed, STATS, ROOF, None, per_rank) if rank == 0 else None
    g.close()
    q.put((rank, out))


def test_multi_gpu_line_carries_per_rank_fields(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, str(tmp_path / "rdzv"), q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    out = got[0]
    assert out["n_gpus"] == 2
    ranks = out["ranks"]
    assert ranks["rccl_ranks"] == 2
    assert ranks["render_ms"] == [1000.0, 1100.0]
    assert ranks["gather_ms"] == [102.0, 2.0]
    assert ranks["slowest_rank"] == 1
    assert abs(ranks["render_imbalance"] - 1.1) < 1e-9
    # value = the whole frame over the slowest rank's timed region
    assert abs(out["ms_per_step"] - 1102.0) < 1e-6
    assert not os.path.exists(tmp_path / "rdzv")


def test_rendezvous_abort_removes_stale_files(tmp_path):
    import rendezvous

    path = str(tmp_path / "g")
    g1 = rendezvous.FileGroup(1, 2, path=path, timeout=0.1)
    g1._put(0, b"x")
    g1.abort()
    assert not any(n.endswith(".1") for n in os.listdir(path))
    g0 = rendezvous.FileGroup(0, 2, path=path, timeout=0.1)
    g0._put(0, b"y")
    g0.abort()
    assert not os.path.exists(path)
    # the default directory carries the launcher's start time as a nonce
    assert rendezvous._start_time(os.getppid()) != "0"


def test_rendezvous_abort_wakes_waiting_ranks(tmp_path):
    """A rank blocked in a collective raises as soon as another rank aborts,
    long before its own timeout."""
    import threading
    import time

    import rendezvous

    path = str(tmp_path / "g")
    waiting = rendezvous.FileGroup(1, 2, path=path, timeout=60.0)
    failing = rendezvous.FileGroup(0, 2, path=path, timeout=60.0)
    seen = {}

    def wait():
        t0 = time.monotonic()
        try:
            waiting.barrier()
        except RuntimeError as e:
            seen["err"] = str(e)
        seen["s"] = time.monotonic() - t0

    th = threading.Thread(target=wait)
    th.start()
    time.sleep(0.2)
    failing.abort()
    th.join(10)
    assert not th.is_alive()
    assert "rank 0 aborted" in seen["err"] and seen["s"] < 5


def test_roofline_bound_comes_from_measured_fractions():
    import bench

    # C3 of round 3: modelled bytes said 0.88 of HBM, the PMC said 0.25 traffic,
    # 0.33 VALU issue and 54 % of wave cycles waiting: latency
    assert bench.roofline_bound(0.25, 0.33, 0.54) == "latency"
    assert bench.roofline_bound(0.25, 0.33, 0.30) == "valu"
    assert bench.roofline_bound(0.70, 0.33, 0.54) == "hbm"
    assert bench.roofline_bound(0.30, 0.62, 0.45) == "valu"
    assert bench.roofline_bound(None, 0.5, 0.5) is None  # unmeasured
    # the CU's scalar unit is a port too (SQ_INSTS_SALU per CU-cycle
    # against the ceiling tools/salu_peak.hip measured). Round 4's PMC files:
    # C4 0.66, C2 0.79 of it, the busiest port of both
    assert bench.roofline_bound(0.313, 0.49, 0.451, 0.66) == "salu"
    assert bench.roofline_bound(0.09, 0.60, 0.197, 0.79) == "salu"
    assert bench.roofline_bound(0.09, 0.60, 0.197, 0.45) == "valu"
    assert bench.roofline_bound(0.25, 0.33, 0.54, 0.40) == "latency"


def test_bound_margins_flag_labels_near_a_threshold():
    """the round-4 C4 line said "latency" with VALU issue at 0.491 and
    waits at 0.451; bound_margins reports the distances and the labels a
    5-point move of one input would give."""
    import bench

    m = bench.bound_margins(0.313, 0.491, 0.451)
    assert m["valu_to_0.5"] == -0.009 and m["wait_to_0.4"] == 0.051
    assert m["close_to"] == ["valu"]
    m = bench.bound_margins(0.09, 0.60, 0.197, 0.79)
    assert m["close_to"] == [] and m["salu_to_0.5"] == 0.29
    assert bench.bound_margins(None, 0.5, 0.5) is None


def _pmc_file(root, build, kernel="render_kernel_lean<false, 6, false, true, false, false, false, false>"):
    import json

    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    pm = {"kernel": "void fs::dev::" + kernel, "code_object_sha256": build, "hbm_bytes_per_sample": 1400.0,
          "valu_insts_per_sample": 300.0, "clock_ghz": 2.4, "valu_lane_util": 0.29, "wait_any_frac": 0.47}
    json.dump(pm, open(os.path.join(root, "profiles", "pmc_c4_1920x1080.json"), "w"))


def test_pmc_replay_only_onto_the_same_build(tmp_path, monkeypatch):
    import bench

    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    kernel = "render_kernel_lean<false, 6, false, true, false, false, false, false>"
    _pmc_file(str(tmp_path), "a" * 64)
    c = {"node_visits": 800, "tri_tests": 100, "small_tri_loads": 10, "object_loads": 5, "segments": 37,
         "samples": 10, "prim_tests": 30}
    args = ("c4", 1920, 1080, 1024, c, 8, [1100.0], kernel, 1, 1024)
    same = bench.make_roofline(*args, build="a" * 64)
    assert same["traffic"] and same["valu"] and same["pmc_replay_refused"] is None
    assert same["bound"] == "latency" and same["bound_source"].startswith("measured")
    assert "valu_busy_rocprof" not in same["valu"]
    other = bench.make_roofline(*args, build="b" * 64)  # same kernel name, another build
    assert other["traffic"] is None and other["valu"] is None
    assert "build" in other["pmc_replay_refused"] and other["bound_source"].startswith("unmeasured")
    assert other["frac_fetch"] == same["frac_fetch"]  # the byte model does not depend on the replay
    # frac is the fraction of the resource bound names, never the byte-model ratio
    busiest = max(same["frac_traffic"], same["valu"]["valu_issue_frac"])  # "latency": the busiest port
    assert abs(same["frac"] - busiest) < 1e-4 and same["frac_of"] in ("hbm", "valu")
    assert abs(same["achieved"] / same["peak"] - same["frac"]) < 1e-3 + 0.05 / same["peak"] and same["frac"] <= 1
    assert other["bound"] == "l2" and other["frac"] == other["frac_fetch_l2"]
    _pmc_file(str(tmp_path), "a" * 64, kernel="render_kernel_lean<false, 6, false, false, false, false, false, false>")
    assert bench.make_roofline(*args, build="a" * 64)["traffic"] is None  # another kernel


def _gather_rank(rank, world, path, q, corrupt):
    import numpy as np

    import bench
    import rendezvous
    import tiles

    W, H, TS = 150, 70, 16
    rng = np.random.default_rng(3)
    full = {"color": rng.random((H, W, 3), dtype=np.float32), "count": rng.integers(1, 9, (H, W)).astype(np.uint32),
            "normal": rng.random((H, W, 3), dtype=np.float32), "depth": rng.random((H, W), dtype=np.float32),
            "material": rng.integers(0, 2**63, (H, W)).astype(np.uint64)}
    own = tiles.owner_map(W, H, world, TS)
    # this rank's frame: its own tiles as rendered; rank 0's also the gathered ones
    mine = {k: np.where((own == rank).reshape(own.shape + (1,) * (v.ndim - 2)), v, 0).astype(v.dtype)
            for k, v in full.items()}
    if rank == 0:
        mine = {k: v.copy() for k, v in full.items()}
        if corrupt:
            mine["color"][own == 1] += np.float32(1e-3)  # one rank's tiles arrive damaged
    g = rendezvous.FileGroup(rank, world, path=path, timeout=60)
    res = bench.gather_check(g, rank, world, lambda k: tiles.pack_words(mine, W, H, k, world, TS).tobytes())
    out = bench.make_record(_args(), world, 1.0, STATS, ROOF, None, res) if rank == 0 else res
    g.close()
    q.put((rank, out))


@pytest.mark.parametrize("corrupt", [False, True])
def test_multi_gpu_line_verifies_the_gathered_frame(tmp_path, corrupt):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_rank, args=(r, world, str(tmp_path / "rdzv"), q, corrupt))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ranks = got[0]["ranks"]
    assert ranks["gather_ok"] is (not corrupt)
    assert ranks["gather_mismatch_ranks"] == ([1] if corrupt else [])
    assert len(ranks["tile_digests"]) == world and got[1] == {}


def _committed_lines():
    import glob
    import json

    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*", "final", "bench_*.json"))):
        yield p, json.load(open(p))


def test_committed_bench_lines_have_physical_fracs():
    """the shipped C3 line read frac 1.0038 (byte model / 8 TB/s).
    Every committed bench line, recomputed with roofline_head from the fields
    it carries (round-5 lines: the byte-model rate was `achieved`), prices a
    real port: 0 < frac <= 1; lines written since carry the same numbers."""
    import bench

    seen = 0
    for path, line in _committed_lines():
        r = line["roofline"]
        fetch = r.get("fetch_gbs", r["achieved"] if r.get("unit") == "GB/s" and "frac_fetch" not in r else None)
        head = bench.roofline_head(fetch, r.get("traffic_gbs"), r.get("valu"))
        assert 0 < head["frac"] <= 1, (path, head)
        assert abs(head["achieved"] / head["peak"] - head["frac"]) < 1e-3, path
        if "frac_fetch" in r:  # written by this bench.py: the line itself agrees
            assert r["frac"] == head["frac"] and r["bound"] == head["bound"], path
            assert 0 < r["frac"] <= 1 and r["frac_fetch_l2"] < 1, path
        seen += 1
    assert seen >= 4
