"""Trace-kernel time of one launch against the samples it holds (measurement
aid for the drop-in loop): for k samples per pixel in ONE
launch (groups = 1, samples_per_block = min(k, 64)) and for k = 1-spp launches
of samples_per_block 1, the median HIP-event time of the trace kernel. A
fixed per-launch cost shows as the intercept of ms against k.
usage: python tools/spp_sweep.py [scenes] [W] [H]"""
import os
import tempfile
import statistics
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import fsamd  # noqa: E402
import scenes  # noqa: E402

names = (sys.argv[1] if len(sys.argv) > 1 else "c4,c2").split(",")
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
for name in names:
    p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    r = fsamd.Renderer(0)
    r.upload(s)
    f = r.frame(W, H)
    cam = s.camera(0)
    r.render(cam, f, spp=4)  # warm-up
    rows = []
    for k, spb, groups in [(1, 1, 1), (2, 2, 1), (4, 4, 1), (8, 8, 1), (16, 16, 1), (32, 32, 1), (64, 64, 1),
                           (64, 16, 4), (256, 16, 16), (16, 1, 16), (64, 1, 64)]:
        r.set_options(**fsamd.options_dict(fsamd.options(samples_per_block=spb, groups=groups)))
        ms = []
        for i in range(7):
            r.render(cam, f, spp=k)
            ms.append(r.last_trace_ms())
        med = statistics.median(ms)
        rows.append((k, spb, groups, med))
        print(f"{name} spp {k:4d} spb {spb:3d} groups {groups:3d}: trace {med:8.3f} ms  {med / k:7.3f} ms/spp  "
              f"{W * H * k / med / 1e3:8.1f} Msamples/s  launches {r.last_launches()[0]}", flush=True)
    f.close()
    r.close()
