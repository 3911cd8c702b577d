"""Quick GPU check: GPU vs oracle on small renders + 1080p timing per scene.
usage: python tools/gpu_quick.py c1:64x64x16 c4:128x72x4 ... [--time c2,c4]"""
import os
import tempfile
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import fsamd  # noqa: E402
import oracle_py  # noqa: E402
import scenes  # noqa: E402

TMP = os.path.join(tempfile.gettempdir(), "fs_scenes")
_cache = {}


def setup(name):
    if name not in _cache:
        p = scenes.write(name, os.path.join(TMP, name))
        fsamd.reset_main_rng()
        s = fsamd.HostScene.load(p)
        fsamd.initialize_materials()
        r = fsamd.Renderer(0)
        t = time.time()
        r.upload(s)
        print(name, "upload %.2fs" % (time.time() - t), r.scene_stats(), flush=True)
        _cache[name] = (r, s, s.camera(0))
    return _cache[name]


def compare(name, W, H, spp):
    r, s, cam = setup(name)
    f = r.frame(W, H)
    r.render(cam, f, spp=spp, counters=True)
    g = f.read(fsamd.PLANE_COLOR)
    c = r.counters()
    print(name, "counters", c, "segments/sample %.2f nodes/seg %.1f tris/seg %.1f" % (
        c["segments"] / c["samples"], c["node_visits"] / c["segments"], c["tri_tests"] / c["segments"]), flush=True)
    t = time.time()
    o = oracle_py.Scene(s.desc_ptr())
    of = o.render(cam, fsamd.render_params(W, H, spp), threads=16)
    print("  oracle %.2fs" % (time.time() - t), of.stats, flush=True)
    eq = g == of.color
    d = np.abs(g - of.color)
    bad = (d > 1e-3 + 1e-2 * np.abs(of.color)).mean()
    print(f"  {name} {W}x{H}x{spp}: exact {eq.mean()*100:.4f}%  outside-tol {bad*100:.4f}%  max|d| {d.max():.3g}  "
          f"mean gpu {g.mean():.6f} oracle {of.color.mean():.6f}", flush=True)
    print("  count eq", np.array_equal(f.read(fsamd.PLANE_COUNT), of.count),
          "display eq %", (f.read(fsamd.PLANE_DISPLAY) == of.display).mean() * 100,
          "material eq %", (f.read(fsamd.PLANE_MATERIAL) == of.material).mean() * 100, flush=True)


def timing(name, spp=64, W=1920, H=1080):
    r, s, cam = setup(name)
    f = r.frame(W, H)
    r.render(cam, f, spp=2)
    t = time.time()
    r.render(cam, f, spp=spp, sample_base=2)
    dt = time.time() - t
    print(f"TIME {name} {W}x{H}x{spp}: {dt:.3f}s  {W*H*spp/dt/1e6:.1f} Msamples/s  kernel {r.last_render_ms():.1f} ms",
          flush=True)


def main():
    os.makedirs(TMP, exist_ok=True)
    args = sys.argv[1:]
    times = []
    if "--time" in args:
        i = args.index("--time")
        times = args[i + 1].split(",")
        args = args[:i] + args[i + 2:]
    for a in args:
        name, dims = a.split(":")
        W, H, spp = map(int, dims.split("x"))
        compare(name, W, H, spp)
    for name in times:
        timing(name)


if __name__ == "__main__":
    main()
