"""Times the oracle (CPU restatement, reference octree, row-band threads) in
this container on the configurations SURVEY.md §8(d) quotes reference rates
for (8 threads): C1 256x256, C3 and C4 at 1920x1080 (a band of rows)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"), os.path.join(ROOT, "oracle")]
import fsamd  # noqa: E402
import oracle_py  # noqa: E402
import scenes  # noqa: E402

REF = {"c1": 0.73, "p250": 0.180, "c3": 0.180, "c4": 0.067}  # SURVEY.md §8(d) [probe], Msamples/s on 8 threads
threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
which = sys.argv[2].split(",") if len(sys.argv) > 2 else ["c1", "p250", "c3", "c4"]
for name, W, H, spp, stride in (("c1", 256, 256, 8, 1), ("p250", 1920, 1080, 1, 8), ("c3", 1920, 1080, 1, 8),
                                ("c4", 1920, 1080, 1, 16)):
    if name not in which:
        continue
    if name == "p250":
        p = scenes.write_c4(f"/tmp/fs_calib/{name}", nu=500, nv=250)
    else:
        p = scenes.write(name, f"/tmp/fs_calib/{name}")
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    t = time.time()
    o = oracle_py.Scene(s.desc_ptr())
    build = time.time() - t
    prm = fsamd.render_params(W, H, spp, tile_stride=stride)
    t = time.perf_counter()
    f = o.render(s.camera(0), prm, threads=threads)
    dt = time.perf_counter() - t
    rate = f.stats["samples"] / dt / 1e6
    print(f"{name} {W}x{H}: {f.stats['samples']} samples in {dt:.1f}s -> {rate:.3f} Msamples/s "
          f"(reference probe {REF[name]}; ratio {rate / REF[name]:.2f}); octree build {build:.1f}s", flush=True)
    o.close()
