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
import hashlib
import json
import math
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
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2: 4 MiB per XCD, ≈34.5 TB/s aggregate
VALU_LANE_OPS_PEAK = 1024 * 32 * 2.4e9  # 157.3 TF FP32 vector peak / 2 (an FMA is one lane-op)
CUS = 256
# The scalar unit's issue ceiling, SALU instructions per CU-cycle: tools/salu_peak.hip on the
# GPU box (profiles/r05/salu_peak.json): one CU's scalar unit issues at most one instruction
# per cycle (0.97-0.98 over whole kernels with 24-32 waves per CU, launch and tail included;
# one wave alone issues one every 4.7 cycles)
SALU_PEAK_PER_CU_CYCLE = 1.0
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
# one material record (76 B) + one normal-table entry (16 B) + the 4-B c value
# its bounce writes to the path record; per sample the path record's end state
# (16 B) and packed material ids (8 B), which fold_paths reads back.
S_NODE, S_TRI, S_OBJ, S_SEG, S_SAMPLE = 64, 64, 128, 96, 24
# tools/cpu_calibration.py on SURVEY Appendix A's own probe scenes (the C1 room + a UV-sphere blob,
# scenes.write_probe), 8 threads in the build container, against the reference rates and octree
# counts SURVEY records for them
CPU_CALIBRATION = ("oracle vs reference on SURVEY's probe scenes (8 threads, build container, DESIGN §6, "
                   "profiles/r04/cpu_calibration.log): 250k probe rate x1.22 at 3.52 vs 5.02 segments/sample and "
                   "153 vs 137 triangle tests per segment, i.e. x0.96 per triangle test; 1M probe x1.11 at 3.50 vs "
                   "5.05 and 508 vs 451, x0.87 per triangle test; C1's 10.8 vs 15.8 triangle tests per segment is "
                   "mesh grouping: the same geometry with the room's walls and light as one 12-face mesh (one "
                   "Cornell OBJ) gives 16.0 (tools/c1_grouping.py, profiles/r06/c1_grouping.log); the reference "
                   "cannot be built here for a same-machine run")


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


def build_id(so_path=None):
    """Identity of the libfsgpu.so build this process runs: the SHA-256 of its
    gfx950 code object (every kernel's machine code and metadata). A PMC
    summary under profiles/ carries the same digest (tools/pmc_summary.py);
    make_roofline replays one only onto the build it was measured on."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_guard

    so_path = so_path or fsamd.gpu_lib_path()
    try:
        return hashlib.sha256(isa_guard.code_object(so_path)).hexdigest()
    except (OSError, ValueError) as e:
        log(f"build id of {so_path}: {e}")
        return None


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    group = rendezvous.FileGroup(rank, world) if world > 1 else None
    try:
        run(args, rank, world, local_rank, group)
    except BaseException:
        if group:
            group.abort()  # no stale files for a later launch; rank 0 removes the directory
        raise
    if group:
        group.close()


def run(args, rank, world, local_rank, group):
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
    rccl_ranks = None
    if group:
        uid = group.broadcast(fsamd.Renderer.comm_unique_id() if rank == 0 else None, root=0)
        r.comm_init(world, rank, uid)
        rccl_ranks = r.comm_count()

    def step():
        """One step: render (HIP-event time of the trace launches), then for
        N > 1 the RCCL gather, timed on the host from the end of this rank's
        render to the end of the gather (it includes waiting for slower ranks)."""
        frame.reset()
        r.render(cam, frame, spp=spp, tile_offset=rank, tile_stride=world, sync=False)
        g_ms = 0.0
        if world > 1:
            r.synchronize()
            tg = time.perf_counter()
            r.gather(frame, params, root=0)
            r.synchronize()
            g_ms = (time.perf_counter() - tg) * 1e3
        else:
            r.synchronize()
        return r.last_render_ms(), g_ms, r.last_trace_ms()

    for i in range(args.warmup):
        ms, _, _ = step()
        log(f"rank {rank}: warmup {i} render {ms:.1f} ms")

    def barrier():
        if group:
            group.barrier()

    barrier()
    r.synchronize()
    kernel_ms, gather_ms, trace_ms = [], [], []
    t_start = time.perf_counter()
    for i in range(args.steps):
        k_ms, g_ms, t_ms = step()
        kernel_ms.append(k_ms)
        gather_ms.append(g_ms)
        trace_ms.append(t_ms)
        log(f"rank {rank}: step {i} render {k_ms:.1f} ms gather {g_ms:.1f} ms")
    r.synchronize()
    barrier()
    elapsed_local = time.perf_counter() - t_start
    kernel_name = r.last_kernel()
    launches, launch_spp = r.last_launches()
    per_rank = None
    elapsed = elapsed_local
    if group:
        rows = group.allgather([elapsed_local, sum(kernel_ms) / len(kernel_ms), sum(gather_ms) / len(gather_ms)])
        per_rank = per_rank_stats(rows, rccl_ranks)
        elapsed = max(row[0] for row in rows)
        # the last step's gathered frame, checked tile set by tile set (outside the timed region)
        per_rank.update(gather_check(group, rank, world, lambda k: r.pack(
            frame, fsamd.render_params(W, H, spp, tile_offset=k, tile_stride=world)).tobytes()))

    # ---- roofline of the trace kernel: algorithmic bytes from a counted launch
    cf = r.frame(W, H)
    cspp = 8
    r.render(cam, cf, spp=cspp, tile_offset=rank, tile_stride=world, counters=True)
    c = r.counters()
    cf.close()
    roofline = make_roofline(args.scene, W, H, spp, c, cspp, trace_ms, kernel_name, launches, launch_spp,
                             build_id())
    roofline["render_ms_per_step"] = round(sum(kernel_ms) / len(kernel_ms), 3)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, scene, cam)

    if rank == 0:
        out = make_record(args, world, elapsed, stats, roofline, cpu, per_rank)
        print(json.dumps(out), flush=True)


def tile_digest(pack_bytes):
    """Digest of one rank's tile set in the 40-B/pixel exchange format."""
    return hashlib.sha256(pack_bytes).hexdigest()[:16]


def gather_check(group, rank, world, pack_fn):
    """Verifies the gathered frame of an N > 1 step. pack_fn(k) packs tile set
    k (the tiles t with t % world == k, fs_frame_pack's format) from this
    rank's frame: each rank digests its own tiles as it rendered them, the
    digests are allgathered, and rank 0 digests every rank's tiles again
    from the frame the RCCL gather assembled. gather_ok says they all
    match; rank 0 returns the fields, the other ranks an empty dict."""
    own = tile_digest(pack_fn(rank))
    digests = [d.decode() for d in group.allgather_bytes(own.encode())]
    if rank != 0:
        return {}
    root = [tile_digest(pack_fn(k)) for k in range(world)]
    bad = [k for k in range(world) if root[k] != digests[k]]
    return {"gather_ok": not bad, "tile_digests": digests, "gather_mismatch_ranks": bad}


def per_rank_stats(rows, rccl_ranks):
    """The N > 1 self-check fields from every rank's [timed-region s, mean
    render ms, mean gather ms] (rendezvous allgather, rank order): whether a
    loss of scaling is render imbalance or the gather."""
    render = [round(row[1], 2) for row in rows]
    return {"rccl_ranks": rccl_ranks, "render_ms": render, "gather_ms": [round(row[2], 2) for row in rows],
            "timed_s": [round(row[0], 4) for row in rows],
            "slowest_rank": max(range(len(rows)), key=lambda i: rows[i][1]),
            "render_imbalance": round(max(render) / max(min(render), 1e-9), 4)}


def pmc_record(scene, W, H, kernel_name, build):
    """The committed PMC summary of this kernel on this workload (tools/gpu_run.sh
    pmc + tools/pmc_summary.py), or None and the reason: the run replays it,
    it does not measure it, and only onto the build it was measured on (the
    code-object digest both carry; a summary of another build is refused even
    when the kernel's template name is the same)."""
    path = os.path.join("profiles", f"pmc_{scene}_{W}x{H}.json")
    try:
        pm = json.load(open(os.path.join(ROOT, path)))
    except (OSError, ValueError):
        return None, path, "no PMC summary for this workload"
    if kernel_name not in pm.get("kernel", ""):
        return None, path, f"PMC summary is of another kernel ({pm.get('kernel')})"
    if not build or pm.get("code_object_sha256") != build:
        return None, path, (f"PMC summary is of build {str(pm.get('code_object_sha256'))[:12]}, "
                            f"this run is {str(build)[:12]}")
    return pm, path, None


def roofline_bound(frac_traffic, valu_issue_frac, wait_any_frac, salu_issue_frac=None):
    """What bounds the kernel, from MEASURED fractions (the PMC summary of
    this build): the busiest of HBM traffic (against 8 TB/s), VALU issue
    (against one wave64 instruction per 2 SIMD cycles) and scalar-unit issue
    (SALU instructions per CU-cycle against the ceiling tools/salu_peak.hip
    measured, SALU_PEAK_PER_CU_CYCLE); "latency" when none reaches half of
    its peak while waves wait on dependencies for more than 40 % of their
    cycles. Without measurements: None (the line then says "hbm", the
    roofline frac is priced against, and bound_source says it is unmeasured)."""
    if frac_traffic is None or valu_issue_frac is None:
        return None
    fr = {"hbm": frac_traffic, "valu": valu_issue_frac}
    if salu_issue_frac is not None:
        fr["salu"] = salu_issue_frac
    top = max(fr, key=fr.get)
    if fr[top] < 0.5 and (wait_any_frac or 0.0) > 0.4:
        return "latency"
    return top


def bound_margins(frac_traffic, valu_issue_frac, wait_any_frac, salu_issue_frac=None, close=0.05):
    """How firmly roofline_bound decided (a fraction near a
    threshold flips the label on a few % of timing noise): each fraction's
    distance to the 0.5 threshold and the wait share's to 0.4, and
    `close_to`, the other labels roofline_bound gives when any one measured
    input moves by +-close (5 points)."""
    if frac_traffic is None or valu_issue_frac is None:
        return None
    args = [frac_traffic, valu_issue_frac, wait_any_frac, salu_issue_frac]
    names = ["hbm", "valu", "wait", "salu"]
    out = {f"{n}_to_{0.4 if n == 'wait' else 0.5}": round(v - (0.4 if n == "wait" else 0.5), 4)
           for n, v in zip(names, args) if v is not None}
    label = roofline_bound(*args)
    alt = set()
    for i, v in enumerate(args):
        if v is None:
            continue
        for d in (-close, close):
            moved = list(args)
            moved[i] = v + d
            alt.add(roofline_bound(*moved))
    out["close_to"] = sorted(alt - {label, None})
    return out


def roofline_head(fetch_gbs, traffic_gbs, valu):
    """The contract's bound / achieved / peak / unit / frac, with frac the
    fraction of the resource `bound` names (a byte-model volume
    ratio above 1 is no roofline fraction). Measured ports, from the PMC
    replay: HBM traffic (GB/s against 8 TB/s), VALU issue (wave64 VALU
    instructions per second against one per 2 cycles on each of the 1024
    SIMDs at the PMC run's clock) and SALU issue (instructions per second
    against the CU's scalar unit, SALU_PEAK_PER_CU_CYCLE per cycle on 256
    CUs). bound is roofline_bound's label; for "latency" frac is the busiest
    port's fraction (`frac_of` names it). Unmeasured (no PMC summary of this
    build): bound "l2", the byte model's lane fetch volume against the L2
    ceiling."""
    issue = valu.get("valu_issue_frac") if valu else None
    salu = valu.get("salu_issue_frac") if valu else None
    frac_traffic = traffic_gbs / HBM_PEAK_GBS if traffic_gbs is not None else None
    bound = roofline_bound(frac_traffic, issue, valu.get("wait_any_frac") if valu else None, salu)
    if bound is None:
        return {"bound": "l2", "frac_of": "l2_fetch", "measured": False, "achieved": round(fetch_gbs, 1),
                "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": round(fetch_gbs / L2_PEAK_GBS, 4)}
    ports = {"hbm": frac_traffic, "valu": issue, "salu": salu}
    port = bound if bound != "latency" else max((k for k in ports if ports[k] is not None), key=ports.get)
    clock = valu["clock_ghz"]
    if port == "hbm":
        achieved, peak, unit = traffic_gbs, HBM_PEAK_GBS, "GB/s"
        return {"bound": bound, "frac_of": port, "measured": True, "achieved": round(achieved, 1),
                "peak": peak, "unit": unit, "frac": round(frac_traffic, 4)}
    elif port == "valu":
        peak, unit = 1024 * clock / 2, "G wave64 VALU instructions/s"
        achieved = issue * peak
    else:
        peak, unit = CUS * clock * SALU_PEAK_PER_CU_CYCLE, "G SALU instructions/s"
        achieved = salu * peak
    return {"bound": bound, "frac_of": port, "measured": True, "achieved": round(achieved, 1),
            "peak": round(peak, 1), "unit": unit, "frac": round(achieved / peak, 4)}


def make_roofline(scene, W, H, spp, c, cspp, kernel_ms, kernel_name, launches, launch_spp, build=None):
    """kernel_ms: per timed step, the trace kernel's HIP-event time summed over
    its launches (fs_last_trace_ms: the dominant kernel alone, without the
    fold_paths launches that follow each one)."""
    bytes_per_sample = (S_NODE * c["node_visits"] + S_TRI * (c["tri_tests"] + c["small_tri_loads"])
                        + S_OBJ * (c["object_loads"] + c.get("lane_object_loads", 0))
                        + S_SEG * c["segments"]) / max(c["samples"], 1) + S_SAMPLE
    avg_launch_s = (sum(kernel_ms) / len(kernel_ms)) / 1e3 / launches
    owned_samples = c["samples"] / cspp * spp  # samples this rank renders per step
    per_launch_bytes = bytes_per_sample * owned_samples / launches
    achieved = per_launch_bytes / avg_launch_s / 1e9
    hbm_frac = achieved / HBM_PEAK_GBS
    pm, pm_path, refused = pmc_record(scene, W, H, kernel_name, build)
    traffic = None
    valu = None
    src = pm_path + " (same build: replayed per sample onto this run's launch time, not measured by this run)"
    if pm and pm.get("hbm_bytes_per_sample"):
        traffic = round(pm["hbm_bytes_per_sample"] * owned_samples / launches)
    if pm and pm.get("valu_insts_per_sample") and pm.get("clock_ghz"):
        # VALU against the gfx950 peak, replayed per sample from the PMC file onto
        # this run's launch time at the clock the PMC run measured (GRBM_GUI_ACTIVE
        # / 8 / kernel time): issue = wave64 VALU instructions x 2 cycles (the
        # FP32 rate, MI355X_MICROARCH.md: v_fma_f32 wave64 2 cyc) over the 1024
        # SIMDs' cycles; lane-op rate = instructions x active lanes against 1024
        # SIMDs x 32 lanes x 2.4 GHz (157.3 TF FP32 / 2 per FMA)
        samples_launch = owned_samples / launches
        clock = pm["clock_ghz"] * 1e9
        insts = pm["valu_insts_per_sample"] * samples_launch
        issue = insts * 2 / (1024 * clock * avg_launch_s)
        lane_ops = insts * 64 * pm["valu_lane_util"]
        valu = {"valu_issue_frac": round(issue, 4), "valu_lane_util": pm["valu_lane_util"],
                "valu_lane_op_frac": round(lane_ops / avg_launch_s / VALU_LANE_OPS_PEAK, 4),
                "valu_insts_per_sample": pm["valu_insts_per_sample"], "clock_ghz": pm["clock_ghz"],
                "wait_any_frac": pm.get("wait_any_frac"), "source": src}
        if pm.get("salu_insts_per_sample"):
            # the CU's one scalar unit: SALU instructions per CU-cycle, replayed the
            # same way, against the ceiling tools/salu_peak.hip measured
            salu = pm["salu_insts_per_sample"] * samples_launch / (CUS * clock * avg_launch_s)
            valu.update({"salu_insts_per_sample": pm["salu_insts_per_sample"],
                         "salu_per_cu_cycle": round(salu, 4),
                         "salu_issue_frac": round(salu / SALU_PEAK_PER_CU_CYCLE, 4),
                         "salu_peak_per_cu_cycle": SALU_PEAK_PER_CU_CYCLE})
            if pm.get("branch_per_cu_cycle") is not None and pm.get("kernel_ms"):
                valu["branch_per_cu_cycle"] = round(pm["branch_per_cu_cycle"] * pm["kernel_ms"] / (avg_launch_s * 1e3), 4)
        for k in ("mean_waves_per_cu", "occupancy_pct"):  # resident waves: the kernel's, not this run's
            if pm.get(k) is not None:
                valu[k] = pm[k]
    traffic_gbs = traffic / avg_launch_s / 1e9 if traffic else None
    frac_traffic = round(traffic_gbs / HBM_PEAK_GBS, 4) if traffic else None
    fracs = (frac_traffic, valu["valu_issue_frac"] if valu else None, valu["wait_any_frac"] if valu else None,
             valu.get("salu_issue_frac") if valu else None)
    head = roofline_head(achieved, traffic_gbs, valu)
    roof = {**head,
            "bound_source": ("measured: PMC traffic fraction, VALU and SALU issue fractions and wave wait share "
                             "of this build (roofline_bound)") if head["measured"] else
                            f"unmeasured ({refused or 'PMC summary incomplete'}): frac is the byte model's lane "
                            "fetch volume against the L2 ceiling",
            "bound_margins": bound_margins(*fracs),
            # the SURVEY 8d byte model: every lane's node/triangle fetch priced as if it came from
            # HBM; most are L1/L2/MALL hits, so against 8 TB/s it is a volume ratio that may exceed 1
            "fetch_gbs": round(achieved, 1),
            "frac_fetch": round(hbm_frac, 4),
            "frac_fetch_l2": round(achieved / L2_PEAK_GBS, 4),
            "fetch_source": "algorithmic bytes (SURVEY 8d byte model x this run's device counters) per launch / "
                            "the trace kernel's HIP-event launch time (fs_last_trace_ms); frac_fetch against "
                            f"{HBM_PEAK_GBS:.0f} GB/s (may exceed 1), frac_fetch_l2 against the "
                            f"{L2_PEAK_GBS:.0f} GB/s L2 ceiling",
            "traffic": traffic,
            "traffic_source": src if traffic else None,
            # the same launch time against the PMC-measured bytes (FETCH x2 + WRITE per launch)
            "traffic_gbs": round(traffic_gbs, 1) if traffic else None,
            "frac_traffic": frac_traffic,
            "valu": valu,
            "pmc_replay_refused": refused,
            "build": build,
            "kernel": kernel_name, "avg_launch_ms": round(avg_launch_s * 1e3, 3),
            "launches_per_step": launches, "spp_per_launch": launch_spp,
            "bytes_per_sample": round(bytes_per_sample, 1),
            "segments_per_sample": round(c["segments"] / max(c["samples"], 1), 3),
            "nodes_per_segment": round(c["node_visits"] / max(c["segments"], 1), 2),
            "tris_per_segment": round(c["tri_tests"] / max(c["segments"], 1), 2),
            "object_loads_per_sample": round(c["object_loads"] / max(c["samples"], 1), 3),
            "small_tri_loads_per_sample": round(c["small_tri_loads"] / max(c["samples"], 1), 3),
            "prim_tests_per_sample": round(c["prim_tests"] / max(c["samples"], 1), 3)}
    return roof


def make_record(args, world, elapsed, stats, roofline, cpu, per_rank=None):
    W, H, spp = args.width, args.height, args.spp
    value = W * H * spp * args.steps / elapsed / 1e6
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
    if per_rank is not None:
        out["ranks"] = per_rank
    return out


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


def effective_cpus(hw):
    """CPUs the baseline may really use: the affinity set, capped by the cgroup
    quota (a 16-CPU quota on a 256-thread host is 16 CPUs of work)."""
    n = hw["affinity"]
    if hw["quota"]:
        n = min(n, max(1, math.ceil(hw["quota"])))
    return n


def cpu_baseline(args, scene, cam):
    """The oracle (CPU port of the reference algorithm, reference octree)
    timed on a bounded tile subset of the same workload: with one thread per
    CPU the process may use (`value`, `cores`), and, reference-style, with one
    thread per hardware thread of the affinity set (engine.cpp:174,261-274:
    hardware_concurrency() bands; `value_all_threads`)."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py

        t = time.time()
        o = oracle_py.Scene(scene.desc_ptr())
        build = time.time() - t
        stride = args.cpu_tile_stride
        p = fsamd.render_params(args.width, args.height, args.cpu_spp, tile_stride=stride, tile_offset=0)
        hw = host_cpus()
        cores = args.cpu_threads if args.cpu_threads > 0 else effective_cpus(hw)

        def timed(threads):
            t0 = time.perf_counter()
            f = o.render(cam, p, threads=threads)
            return f.stats["samples"], time.perf_counter() - t0

        n, dt = timed(cores)
        all_threads = hw["affinity"]
        n_all, dt_all = (n, dt) if all_threads == cores else timed(all_threads)
        o.close()
        cpu_model = ""
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": cores, "kind": "port",
                "value_all_threads": round(n_all / dt_all / 1e6, 4), "threads_all": all_threads,
                "nproc": hw["nproc"], "affinity_cpus": hw["affinity"], "cgroup_cpu_quota": hw["quota"],
                "sample": f"{args.scene} {args.width}x{args.height}, 1/{stride} of the 64x64 tiles, "
                          f"{args.cpu_spp} spp = {n} samples in {dt:.1f}s on {cores} threads "
                          f"(octree build {build:.1f}s excluded)",
                "cpu": cpu_model or platform.processor(),
                "calibration": CPU_CALIBRATION}
    except Exception as e:  # the baseline is reported, never required
        log(f"cpu baseline failed: {e}")
        return None


if __name__ == "__main__":
    main()
