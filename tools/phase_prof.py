"""Per-phase wave-cycle split of the lean kernel (needs libfsgpu_prof.so:
make -C final-stage-path-tracer-2-0_amd libfsgpu_prof.so).
usage: python tools/phase_prof.py scenes [spp]"""
import os
import tempfile
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "final-stage-path-tracer-2-0_amd")
os.environ.setdefault("FSAMD_GPU_LIB", os.path.join(PKG, "libfsgpu_prof.so"))
sys.path.insert(0, PKG)
import fsamd  # noqa: E402
import scenes  # noqa: E402

names = sys.argv[1].split(",")
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 32
W, H = 1920, 1080
for name in names:
    p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    r = fsamd.Renderer(0)
    r.upload(s)
    cam = s.camera(0)
    f = r.frame(W, H)
    r.render(cam, f, spp=spp)
    r.counters()
    f.reset()
    print(f"== {name} {W}x{H} {spp} spp", flush=True)
    r.render(cam, f, spp=spp)
    print(f"render {r.last_render_ms():.1f} ms", flush=True)
    r.counters()  # phase line goes to stderr
    f.close()
