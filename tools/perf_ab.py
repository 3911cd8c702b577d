"""Interleaved A/B of render options (fs_options) in one process.
usage: python tools/perf_ab.py variants scenes [spp] [rounds]
(a variant is default or fields joined by @, e.g. "schedule=parked@xcd_bands=1@park_lanes=8")"""
import os
import tempfile
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import numpy as np  # noqa: E402

import fsamd  # noqa: E402
import scenes  # noqa: E402


BUILD_FIELDS = {"park_min_tris", "gpu_bvh_min_tris", "bvh_leaf", "bvh_bins", "bvh_threads", "node_layout",
                "small_mesh_tris"}


def main():
    variants = sys.argv[1].split(",")
    names = sys.argv[2].split(",")
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    W, H = 1920, 1080
    tmp = os.path.join(tempfile.gettempdir(), "fs_scenes")
    for name in names:
        p = scenes.write(name, os.path.join(tmp, name))
        fsamd.reset_main_rng()
        s = fsamd.HostScene.load(p)
        fsamd.initialize_materials()
        r = fsamd.Renderer(0)
        r.upload(s)
        uploaded = tuple(fsamd.options_dict(fsamd.options())[k] for k in sorted(BUILD_FIELDS))
        cam = s.camera(0)
        f = r.frame(W, H)
        res = {v: [] for v in variants}
        ref = None
        for rd in range(rounds + 1):
            for v in variants:
                od = fsamd.options_dict(fsamd.options(**fsamd.parse_variant(v)))
                r.set_options(**od)
                build = tuple(od[k] for k in sorted(BUILD_FIELDS))
                if build != uploaded:  # scene-build fields are read at upload
                    r.upload(s)
                    uploaded = build
                f.reset()
                r.render(cam, f, spp=spp)
                ms = r.last_render_ms()
                if rd:
                    res[v].append(ms)
                img = f.read(fsamd.PLANE_COLOR)
                if ref is None:
                    ref = img
                elif not np.array_equal(img, ref):
                    print(f"  !! variant {v} output differs from variant {variants[0]}", flush=True)
        if os.environ.get("PERF_AB_HASH"):  # frames of different builds compared across processes
            import hashlib
            print(f"{name} frame md5 {hashlib.md5(ref.tobytes()).hexdigest()}", flush=True)
        for v in variants:
            ms = np.median(res[v])
            print(f"{name} variant {v}: median {ms:.1f} ms  {W*H*spp/ms/1e3:.1f} Msamples/s  (min {min(res[v]):.1f})",
                  flush=True)
        f.close()
        r.close()


if __name__ == "__main__":
    main()
