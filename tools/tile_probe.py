"""Render time against the tile size (the unit of XCD placement and of the
multi-GPU partition; measurement aid). usage: python tools/tile_probe.py [spp] [rounds]"""
import os
import tempfile
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import fsamd  # noqa: E402
import numpy as np  # noqa: E402
import scenes  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
W, H = 1920, 1080
for name in ("c4", "c3", "c2"):
    p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    r = fsamd.Renderer(0)
    r.upload(s)
    f = r.frame(W, H)
    cam = s.camera(0)
    sizes = (32, 64, 128)
    res = {t: [] for t in sizes}
    ref = None
    for rd in range(rounds + 1):
        for t in sizes:
            f.reset()
            r.render(cam, f, spp=spp, tile_size=t)
            if rd:
                res[t].append(r.last_render_ms())
            img = f.read(fsamd.PLANE_COLOR)
            if ref is None:
                ref = img
            elif not np.array_equal(img, ref):
                print(f"  !! tile {t} differs", flush=True)
    for t in sizes:
        ms = float(np.median(res[t]))
        print(f"{name} tile {t}: median {ms:.1f} ms  {W * H * spp / ms / 1e3:.1f} Msamples/s", flush=True)
    f.close()
    r.close()
