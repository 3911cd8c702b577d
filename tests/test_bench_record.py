"""bench.py's JSON line, assembled on CPU: the N = 1 line the driver reads,
and the N > 1 self-check fields (RCCL ranks, per-rank render and gather
times, slowest rank) gathered over 2 ranks through the torch-free
rendezvous, with a stub in place of the GPU render and the RCCL comm."""
import argparse
import multiprocessing as mp
import os
import sys

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
