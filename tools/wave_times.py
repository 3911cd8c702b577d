"""Wave timeline of the trace kernel (needs libfsgpu_wt.so: make -C
final-stage-path-tracer-2-0_amd libfsgpu_wt.so): per launch, histograms of the
time each wave ends and first finds every block queue empty, and how long
waves run on after that (measurement aid for the 1-spp drop-in launch, VERDICT
r5 item 3). usage: python tools/wave_times.py [scenes] [spp,...]"""
import os
import tempfile
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "final-stage-path-tracer-2-0_amd")
os.environ.setdefault("FSAMD_GPU_LIB", os.path.join(PKG, "libfsgpu_wt.so"))
sys.path.insert(0, PKG)
import fsamd  # noqa: E402
import scenes  # noqa: E402

names = (sys.argv[1] if len(sys.argv) > 1 else "c4,c2").split(",")
spps = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,2,16").split(",")]
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
    for spp in spps:
        r.set_options(**fsamd.options_dict(fsamd.options(samples_per_block=min(spp, 16))))
        for rep in range(3):
            r.render(cam, f, spp=spp)
            r.counters()  # reset
            r.render(cam, f, spp=spp)
            print(f"== {name} {W}x{H} {spp} spp: trace {r.last_trace_ms():.3f} ms", file=sys.stderr, flush=True)
            r.counters()  # the wave line goes to stderr
    f.close()
    r.close()
