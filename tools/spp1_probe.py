"""One-sample-per-pixel launches (the reference's TraceScene-per-frame loop)
under a few fs_options, with and without the display-byte readback
(measurement aid). usage: python tools/spp1_probe.py"""
import os
import tempfile, sys, time
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import numpy as np, fsamd, scenes
W, H = 1920, 1080
for name in ["c4", "c2"]:
    p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    r = fsamd.Renderer(0)
    r.upload(s)
    f = r.frame(W, H)
    cam = s.camera(0)
    for v in ["default", "persist=0", "xcd_bands=1", "tile_order=0", "samples_per_block=1"]:
        try:
            r.set_options(**fsamd.options_dict(fsamd.options(**fsamd.parse_variant(v))))
        except Exception as e:
            print(name, v, "ERR", e); continue
        f.reset()
        r.render(cam, f, spp=1)
        ms = []
        for i in range(20):
            r.render(cam, f, spp=1)
            ms.append(r.last_render_ms())
        t0 = time.time()
        for i in range(20):
            r.render(cam, f, spp=1)
            f.read(fsamd.PLANE_DISPLAY)
        wall = (time.time() - t0) / 20 * 1e3
        print(f"{name} {v}: render {np.median(ms):.3f} ms/spp, with display read {wall:.3f} ms/frame", flush=True)
    f.close(); r.close()
