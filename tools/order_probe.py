"""Upper bound of what a cull bound from later objects could save (measurement
aid): renders C3 with its meshes in the generator's order (stone, floor, wall)
and with the floor and walls first (floor, wall, stone), so the stone walk
runs with the floor's or walls' hit as its t limit. The reordered scene is a
different scene for ties and the mesh-root cull, so only the times compare.
usage: python tools/order_probe.py [spp] [rounds]"""
import os
import tempfile
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import fsamd  # noqa: E402
import numpy as np  # noqa: E402
import scenes  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
W, H = 1920, 1080
d = os.path.join(tempfile.gettempdir(), "fs_scenes", "c3_order")
p = scenes.write("c3", d)
text = open(p).read()
blocks = re.findall(r"mesh\n\{\n  file atrium_(\w+)\.obj\n  material \w+\n\}\n", text)
mesh = {k: re.search(r"mesh\n\{\n  file atrium_%s\.obj\n  material \w+\n\}\n" % k, text).group(0) for k in blocks}
body = text
for k in blocks:
    body = body.replace(mesh[k], "")
reordered = os.path.join(d, "c3_floor_first.scene")
i = body.index("quad\n")
open(reordered, "w").write(body[:i] + mesh["floor"] + mesh["wall"] + mesh["stone"] + body[i:])
res = {}
renderers = {}
for name, path in (("stone_first", p), ("floor_first", reordered)):
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(path)
    fsamd.initialize_materials()
    r = fsamd.Renderer(0)
    r.upload(s)
    f = r.frame(W, H)
    renderers[name] = (s, r, f)
    res[name] = []
for rd in range(rounds + 1):
    for name, (s, r, f) in renderers.items():
        f.reset()
        r.render(s.camera(0), f, spp=spp)
        if rd:
            res[name].append(r.last_render_ms())
for name, ms in res.items():
    m = float(np.median(ms))
    print(f"c3 {name}: median {m:.1f} ms  {W * H * spp / m / 1e3:.1f} Msamples/s", flush=True)
