"""A/B of BVH build settings in one process: rebuild + time.
usage: python tools/leaf_ab.py VALUES scenes [spp] [FIELD]   (fs_options field, default bvh_leaf; e.g. bvh_bins)"""
import os
import tempfile
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import numpy as np  # noqa: E402

import fsamd  # noqa: E402
import scenes  # noqa: E402

leaves = sys.argv[1].split(",")
names = sys.argv[2].split(",")
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
env = sys.argv[4] if len(sys.argv) > 4 else "bvh_leaf"
W, H = 1920, 1080
for name in names:
    p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    cam = s.camera(0)
    r = fsamd.Renderer(0)
    f = r.frame(W, H)
    ref = None
    for lf in leaves:
        r.set_options(**{env: int(lf)})
        r.upload(s)
        st = r.scene_stats()
        ms = []
        for k in range(3):
            f.reset()
            r.render(cam, f, spp=spp)
            ms.append(r.last_render_ms())
        img = f.read(fsamd.PLANE_COLOR)
        same = ref is None or np.array_equal(img, ref)
        ref = img if ref is None else ref
        m = float(np.median(ms[1:]))
        print(f"{name} {env}={lf}: nodes {st['nodes']} build {st['build_ms']:.0f} ms  render {m:.1f} ms "
              f"{W*H*spp/m/1e3:.1f} Msamples/s  same-as-first={same}", flush=True)
