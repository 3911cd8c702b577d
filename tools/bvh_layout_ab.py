"""Render speed with the host-built vs the device-built BVH, interleaved.

  python tools/bvh_layout_ab.py [scenes] [spp] [rounds] [variants]

variants: comma list of host|device, each optionally with upload-time env
fs_options settings, e.g. "host,host@node_layout=pairs" (default "host,device").

Two contexts on one GPU hold the same scene, one uploaded with the host SAH
build and one with FS_UPLOAD_GPU_BVH; their renders alternate and every frame
is compared with the first (the trees differ, the frames must not).
"""
import os
import tempfile
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import numpy as np  # noqa: E402

import fsamd  # noqa: E402
import scenes  # noqa: E402


def main():
    names = (sys.argv[1] if len(sys.argv) > 1 else "c4").split(",")
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    variants = (sys.argv[4] if len(sys.argv) > 4 else "host,device").split(",")
    W, H = 1920, 1080
    tmp = os.path.join(tempfile.gettempdir(), "fs_scenes")
    for name in names:
        p = scenes.write(name, os.path.join(tmp, name))
        fsamd.reset_main_rng()
        s = fsamd.HostScene.load(p)
        fsamd.initialize_materials()
        cam = s.camera(0)
        ctx = {}
        for b in variants:
            builder, _, extra = b.partition("@")
            r = fsamd.Renderer(0, **fsamd.parse_variant(extra))
            r.upload(s, gpu_bvh=builder == "device")
            ctx[b] = (r, r.frame(W, H), r.scene_stats())
        res = {b: [] for b in ctx}
        ref = None
        for rd in range(rounds + 1):
            for b, (r, f, _) in ctx.items():
                f.reset()
                r.render(cam, f, spp=spp)
                if rd:
                    res[b].append(r.last_render_ms())
                img = f.read(fsamd.PLANE_COLOR)
                if ref is None:
                    ref = img
                elif not np.array_equal(img, ref):
                    print(f"  !! {b}-built BVH frame differs", flush=True)
        for b, (r, f, st) in ctx.items():
            ms = float(np.median(res[b]))
            print(f"{name} {b} BVH ({st['nodes']} nodes, build {st['build_ms']:.0f} ms): median {ms:.1f} ms "
                  f"{W * H * spp / ms / 1e3:.1f} Msamples/s (min {min(res[b]):.1f})", flush=True)
            f.close()
            r.close()


if __name__ == "__main__":
    main()
