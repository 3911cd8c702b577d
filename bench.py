"""Benchmark: Msamples/s of the path-trace hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

A step is one full render of the workload frame (W x H pixels x spp samples,
the reference's TraceScene called spp times, engine.cpp:253) into a reset
frame; for N > 1 the frame's 64x64 tiles are dealt round-robin to the ranks
and gathered to rank 0 with RCCL (ncclGather over xGMI) inside the step.
Rank 0 prints one JSON line. Scene load/BVH build are outside the timed
region (reported in config).

The GPU processes never import torch: its wheel bundles a second HIP runtime
(libamdhip64) that must not share a process with libfsgpu.so's. The control
plane for N > 1 (RCCL unique id, barriers, the max over ranks) goes through
rendezvous.FileGroup, files in a directory the launcher's ranks share.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "final-stage-path-tracer-2-0_amd")
sys.path.insert(0, PKG)

import fsamd  # noqa: E402
import rendezvous  # noqa: E402
import scenes  # noqa: E402

# The HIP layer (libfsgpu.so + libfshost.so) is loaded here, first.
fsamd.gpu_lib()
fsamd.host_lib()

METRIC = "Msamples/sec (W×H×spp/s) at 1920×1080, 1024spp; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
WORKLOADS = {
    "c4": "~1M-triangle displaced blob + Ceramic/Glass spheres + Metal cuboid in the Cornell room "
          "(BASELINE configs[3] scene; SURVEY §8d C4) at 1920x1080, 1024 spp",
    "c2": "Cornell box + glossy (Ceramic) + glass spheres (BASELINE configs[1]) at 1920x1080, 1024 spp",
    "c3": "~250k-triangle procedural atrium (BASELINE configs[2]) at 1920x1080, 1024 spp",
}
# Algorithmic bytes per unit of work, from the device SoA record
# sizes: BVH node 64 B and triangle 64 B (fs_scene.h DevTri), both per lane;
# an object test 128 B per WAVE (the fields a test reads, at most a cuboid's
# planes + box + kind/material, of the 192-B record; the object loop reads them with scalar
# loads at a wave-uniform index: one load serves the 64 lanes), and so are
# the 64-B triangle records of small meshes (fs_options.small_mesh_tris); per segment
# one material record (76 B) + one normal-table entry (16 B); per sample 12 B
# of radiance.
S_NODE, S_TRI, S_OBJ, S_SEG, S_SAMPLE = 64, 64, 128, 92, 12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--cpu-spp", type=int, default=8, help="spp of the bounded CPU-baseline sample")
    ap.add_argument("--cpu-tile-stride", type=int, default=4, help="CPU sample renders 1/stride of the tiles")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads; 0 = one per hardware thread this process may run on "
                         "(the reference's hardware_concurrency() bands, engine.cpp:174,261-274)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--scene-dir", default=None)
    ap.add_argument("--bvh", default="device", choices=["device", "host"],
                    help="BVH builder of large meshes (fs_upload_scene_ex FS_UPLOAD_GPU_BVH, or host SAH)")
    return ap.parse_args()


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    group = rendezvous.FileGroup(rank, world) if world > 1 else None

    scene_dir = args.scene_dir or os.path.join(tempfile.gettempdir(), f"fs_bench_{os.getuid()}_r{rank}")
    t0 = time.time()
    path = scenes.write(args.scene, os.path.join(scene_dir, args.scene))
    fsamd.reset_main_rng()
    scene = fsamd.HostScene.load(path)
    fsamd.initialize_materials()
    cam = scene.camera(0)
    gen_s = time.time() - t0
    ndev = fsamd.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no HIP device visible")
    device = local_rank if local_rank < ndev else local_rank % ndev  # a launcher may narrow visibility per rank
    r = fsamd.Renderer(device)
    r.upload(scene, gpu_bvh=args.bvh == "device")
    stats = r.scene_stats()
    log(f"rank {rank}: scene {args.scene} written+loaded in {gen_s:.1f}s, BVH {stats}")
    W, H, spp = args.width, args.height, args.spp
    frame = r.frame(W, H)
    params = fsamd.render_params(W, H, spp, tile_offset=rank, tile_stride=world)
    if group:
        uid = group.broadcast(fsamd.Renderer.comm_unique_id() if rank == 0 else None, root=0)
        r.comm_init(world, rank, uid)

    def step():
        frame.reset()
        r.render(cam, frame, spp=spp, tile_offset=rank, tile_stride=world, sync=False)
        if world > 1:
            r.gather(frame, params, root=0)
        r.synchronize()
        return r.last_render_ms()

    for i in range(args.warmup):
        ms = step()
        log(f"rank {rank}: warmup {i} render {ms:.1f} ms")

    def barrier():
        if group:
            group.barrier()

    barrier()
    r.synchronize()
    kernel_ms = []
    t_start = time.perf_counter()
    for i in range(args.steps):
        kernel_ms.append(step())
        log(f"rank {rank}: step {i} render {kernel_ms[-1]:.1f} ms")
    r.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    kernel_name = r.last_kernel()
    launches, launch_spp = r.last_launches()
    if group:
        elapsed = group.max(elapsed)

    # ---- roofline of the trace kernel: algorithmic bytes from a counted launch
    total_samples = W * H * spp * args.steps
    value = total_samples / elapsed / 1e6
    cf = r.frame(W, H)
    cspp = 8
    r.render(cam, cf, spp=cspp, tile_offset=rank, tile_stride=world, counters=True)
    c = r.counters()
    cf.close()
    bytes_per_sample = (S_NODE * c["node_visits"] + S_TRI * (c["tri_tests"] + c["small_tri_loads"])
                        + S_OBJ * c["object_loads"] + S_SEG * c["segments"]) / max(c["samples"], 1) + S_SAMPLE
    avg_launch_s = (sum(kernel_ms) / len(kernel_ms)) / 1e3 / launches
    owned_samples = c["samples"] / cspp * spp  # samples this rank renders per step
    per_launch_bytes = bytes_per_sample * owned_samples / launches
    achieved = per_launch_bytes / avg_launch_s / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{args.scene}_{W}x{H}.json")
    if os.path.exists(pmc):  # PMC passes of tools/gpu_pmc.sh, per sample of the same kernel
        try:
            pm = json.load(open(pmc))
            if kernel_name in pm.get("kernel", "") and pm.get("hbm_bytes_per_sample"):
                traffic = round(pm["hbm_bytes_per_sample"] * owned_samples / launches)
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                # the same launch time against the PMC-measured bytes (FETCH x2 + WRITE per launch)
                "traffic_gbs": round(traffic / avg_launch_s / 1e9, 1) if traffic else None,
                "frac_traffic": round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                "kernel": kernel_name, "avg_launch_ms": round(avg_launch_s * 1e3, 3),
                "launches_per_step": launches, "spp_per_launch": launch_spp,
                "bytes_per_sample": round(bytes_per_sample, 1),
                "segments_per_sample": round(c["segments"] / max(c["samples"], 1), 3),
                "nodes_per_segment": round(c["node_visits"] / max(c["segments"], 1), 2),
                "tris_per_segment": round(c["tri_tests"] / max(c["segments"], 1), 2),
                "object_loads_per_sample": round(c["object_loads"] / max(c["samples"], 1), 3),
                "small_tri_loads_per_sample": round(c["small_tri_loads"] / max(c["samples"], 1), 3),
                "prim_tests_per_sample": round(c["prim_tests"] / max(c["samples"], 1), 3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, scene, cam)

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded procedural scene, per-(pixel,sample) seeded xorshift64*)",
            "config": {"workload": WORKLOADS[args.scene], "scene": args.scene, "width": W, "height": H,
                       "spp": spp, "triangles": stats["triangles"], "bvh_nodes": stats["nodes"],
                       "bvh_build_ms": round(stats["build_ms"], 1), "bvh_builder": args.bvh,
                       "parallelism": f"64x64 tiles round-robin over {world} GPU(s)"
                                      + (" + RCCL ncclGather to rank 0" if world > 1 else "")},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if group:
        group.close()


def host_cpus():
    """nproc, the CPUs this process may run on, and the cgroup CPU quota
    (cpu.max, in CPUs; None if unlimited) of the host that times the baseline."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": nproc, "affinity": aff, "quota": quota}


def cpu_baseline(args, scene, cam):
    """The oracle (CPU port of the reference algorithm, reference octree)
    timed on a bounded tile subset of the same workload."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        t = time.time()
        o = oracle_py.Scene(scene.desc_ptr())
        build = time.time() - t
        stride = args.cpu_tile_stride
        p = fsamd.render_params(args.width, args.height, args.cpu_spp, tile_stride=stride, tile_offset=0)
        hw = host_cpus()
        threads = args.cpu_threads if args.cpu_threads > 0 else hw["affinity"]
        t = time.perf_counter()
        f = o.render(cam, p, threads=threads)
        dt = time.perf_counter() - t
        n = f.stats["samples"]
        o.close()
        cpu_model = ""
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
                "nproc": hw["nproc"], "affinity_cpus": hw["affinity"], "cgroup_cpu_quota": hw["quota"],
                "sample": f"{args.scene} {args.width}x{args.height}, 1/{stride} of the 64x64 tiles, "
                          f"{args.cpu_spp} spp = {n} samples in {dt:.1f}s (octree build {build:.1f}s excluded)",
                "cpu": cpu_model or platform.processor(),
                "calibration": "restatement/reference rate 1.03 on C4 1080p (8 threads, survey container; "
                               "DESIGN §6): the baseline stands for the reference on C4 only"}
    except Exception as e:  # the baseline is reported, never required
        log(f"cpu baseline failed: {e}")
        return None


if __name__ == "__main__":
    main()
