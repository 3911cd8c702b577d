"""Finds the (pixel, sample) pairs where the GPU frame and the oracle differ.

usage: python tools/flip_hunt.py scene W H spp [out.json] [option variant]

Renders the frame on the GPU and with the oracle, lists the differing pixels,
then re-renders each sample index alone (spp=1, sample_base=k) on the GPU
and compares that pixel's colour with the oracle's trace_sample. Writes the
mismatching (x, y, k) with both colours, normals and depths as JSON.
"""
import json
import os
import tempfile
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import fsamd  # noqa: E402
import oracle_py  # noqa: E402
import scenes  # noqa: E402


def main():
    name, W, H, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    out_path = sys.argv[5] if len(sys.argv) > 5 else os.path.join(ROOT, "gpurun_out", f"flips_{name}.json")
    variant = fsamd.parse_variant(sys.argv[6]) if len(sys.argv) > 6 else {}
    p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    cam = s.camera(0)
    r = fsamd.Renderer(0, **variant)
    r.upload(s)
    f = r.frame(W, H)
    r.render(cam, f, spp=spp)
    g = f.read(fsamd.PLANE_COLOR)
    o = oracle_py.Scene(s.desc_ptr())
    ref = o.render(cam, fsamd.render_params(W, H, spp), threads=16)
    bad = np.argwhere((g != ref.color).any(axis=-1))
    print(f"{name} {W}x{H}x{spp}: {len(bad)} pixels differ", flush=True)
    # every plane of the frame (frame.h:49-92), differing pixels per plane
    planes = {"color": (fsamd.PLANE_COLOR, ref.color), "count": (fsamd.PLANE_COUNT, ref.count),
              "display": (fsamd.PLANE_DISPLAY, ref.display), "normal": (fsamd.PLANE_NORMAL, ref.normal),
              "depth": (fsamd.PLANE_DEPTH, ref.depth), "material": (fsamd.PLANE_MATERIAL, ref.material)}
    per_plane = {}
    for pname, (pid, rv) in planes.items():
        gv = f.read(pid)
        d = gv != rv
        per_plane[pname] = int((d.any(axis=-1) if d.ndim == 3 else d).sum())
    print(f"differing pixels per plane: {json.dumps(per_plane)} of {W * H}", flush=True)
    flips = []
    one = r.frame(W, H)
    per_k = {}
    for y, x in bad[:64]:
        for k in range(spp):
            if k not in per_k:
                one.reset()
                r.render(cam, one, spp=1, sample_base=k)
                per_k[k] = (one.read(fsamd.PLANE_COLOR), one.read(fsamd.PLANE_NORMAL), one.read(fsamd.PLANE_DEPTH))
            gc = per_k[k][0][y, x]
            col, nrm, depth = o.trace_sample(cam, W, H, int(x), int(y), k)[:3]
            if not np.array_equal(gc, col):
                rec = {"x": int(x), "y": int(y), "k": k, "gpu_color": gc.tolist(), "oracle_color": np.asarray(col).tolist(),
                       "gpu_normal": per_k[k][1][y, x].tolist(), "oracle_normal": np.asarray(nrm).tolist(),
                       "gpu_depth": float(per_k[k][2][y, x]), "oracle_depth": float(depth)}
                flips.append(rec)
                print(json.dumps(rec), flush=True)
    json.dump({"scene": name, "W": W, "H": H, "spp": spp, "variant": variant, "pixels": len(bad),
               "differing_pixels_per_plane": per_plane,
               "flips": flips}, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
