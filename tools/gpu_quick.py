"""Quick GPU bring-up check: GPU vs oracle on small renders + one timing."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import fsamd  # noqa: E402
import oracle_py  # noqa: E402
import scenes  # noqa: E402


def compare(name, W, H, spp, tmp):
    p = scenes.write(name, os.path.join(tmp, name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    cam = s.camera(0)
    r = fsamd.Renderer(0)
    t = time.time()
    r.upload(s)
    print(name, "upload", time.time() - t, r.scene_stats(), flush=True)
    f = r.frame(W, H)
    r.render(cam, f, spp=spp, counters=True)
    g = f.read(fsamd.PLANE_COLOR)
    print(name, "counters", r.counters(), flush=True)
    o = oracle_py.Scene(s.desc_ptr())
    of = o.render(cam, fsamd.render_params(W, H, spp), threads=16)
    eq = g == of.color
    d = np.abs(g - of.color)
    print(f"{name} {W}x{H}x{spp}: exact {eq.mean()*100:.4f}%  max|d| {d.max():.3g}  "
          f"mean gpu {g.mean():.6f} oracle {of.color.mean():.6f}", flush=True)
    print("  count eq", np.array_equal(f.read(fsamd.PLANE_COUNT), of.count),
          "display eq %", (f.read(fsamd.PLANE_DISPLAY) == of.display).mean() * 100,
          "material eq %", (f.read(fsamd.PLANE_MATERIAL) == of.material).mean() * 100, flush=True)
    return r, s, cam


def main():
    tmp = os.path.join(ROOT, "gpurun_out", "scenes")
    os.makedirs(tmp, exist_ok=True)
    print("devices", fsamd.device_count(), flush=True)
    compare("c1", 64, 64, 16, tmp)
    r, s, cam = compare("c2", 96, 64, 16, tmp)
    f = r.frame(1920, 1080)
    r.render(cam, f, spp=4)
    t = time.time()
    r.render(cam, f, spp=64, sample_base=4)
    dt = time.time() - t
    print(f"c2 1080p x64: {dt:.3f}s  {1920*1080*64/dt/1e6:.1f} Msamples/s  kernel {r.last_render_ms():.1f} ms",
          flush=True)


if __name__ == "__main__":
    main()
