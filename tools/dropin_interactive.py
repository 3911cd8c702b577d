"""The window loop under camera motion (measurement aid for fs_options.lookahead):
per displayed frame one 1-spp render and one display read, as main.cpp:157-163,
with the camera (a) moving every frame (the frame reset, sample index 0) and
(b) still for 48 frames, then moving once. Prints per-frame wall times
(median, p90, max) and the first frames after the move, for each lookahead
depth given. usage: python tools/dropin_interactive.py [scene] [depths]"""
import math
import os
import statistics
import sys
import tempfile
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import fsamd  # noqa: E402
import scenes  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c4"
depths = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,24").split(",")]
W, H = 1920, 1080
p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
fsamd.reset_main_rng()
s = fsamd.HostScene.load(p)
fsamd.initialize_materials()
base = s.camera(0)
r = fsamd.Renderer(0)
r.upload(s)
f = r.frame(W, H)


def orbit(k):
    """the scene camera turned by k * 0.5 degrees about its target's vertical"""
    o, t = list(base.origin), list(base.target)
    dx, dz = o[0] - t[0], o[2] - t[2]
    a = math.radians(0.5 * k)
    o2 = (t[0] + dx * math.cos(a) - dz * math.sin(a), o[1], t[2] + dx * math.sin(a) + dz * math.cos(a))
    return fsamd.camera(o2, t, fov_y=base.fov_y, aperture=base.aperture_size, focal_depth=base.focal_depth,
                        z_near=base.z_near, z_far=base.z_far, fast_render=bool(base.fast_render))


def frame_ms(cam, k, reset):
    t0 = time.perf_counter()
    if reset:
        f.reset()
    r.render(cam, f, spp=1, sample_base=k)
    f.map(fsamd.PLANE_DISPLAY)
    return (time.perf_counter() - t0) * 1e3


def stats(ms):
    ms = sorted(ms)
    return f"median {statistics.median(ms):7.3f}  p90 {ms[int(0.9 * len(ms))]:7.3f}  max {ms[-1]:7.3f} ms"


for w in depths:
    r.set_options(lookahead=w)
    frame_ms(orbit(0), 0, True)  # warm-up
    moving = [frame_ms(orbit(k), 0, True) for k in range(1, 65)]
    still = [frame_ms(orbit(100), k, k == 0) for k in range(48)]
    after = [frame_ms(orbit(101), 0, True)] + [frame_ms(orbit(101), k, False) for k in range(1, 8)]
    print(f"{name} lookahead {w:2d}: moving every frame: {stats(moving)}", flush=True)
    print(f"{name} lookahead {w:2d}: still: {stats(still[8:])}; the move and the 7 frames after it (ms): "
          + " ".join(f"{x:.2f}" for x in after), flush=True)
f.close()
r.close()
