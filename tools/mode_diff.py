"""Renders one scene with two kernel modes and prints where the planes differ.
usage: python tools/mode_diff.py scene W H spp modeA modeB"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import numpy as np  # noqa: E402

import fsamd  # noqa: E402
import scenes  # noqa: E402

name, W, H, spp, ma, mb = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5], sys.argv[6]
p = scenes.write(name, os.path.join(ROOT, "gpurun_out", "scenes", name))
fsamd.reset_main_rng()
s = fsamd.HostScene.load(p)
fsamd.initialize_materials()
r = fsamd.Renderer(0)
r.upload(s)
out = {}
for m in (ma, mb):
    os.environ["FS_KERNEL"] = m
    f = r.frame(W, H)
    r.render(s.camera(0), f, spp=spp)
    out[m] = {pl: f.read(pl) for pl in range(6)}
    f.close()
for pl in range(6):
    a, b = out[ma][pl], out[mb][pl]
    if a.ndim == 3:
        bad = (a != b).any(axis=-1)
    else:
        bad = a != b
    ys, xs = np.nonzero(bad)
    print(f"plane {pl}: {bad.sum()} pixels differ", flush=True)
    for y, x in list(zip(ys, xs))[:12]:
        print(f"   ({x},{y}) {ma}={a[y, x]} {mb}={b[y, x]}")
