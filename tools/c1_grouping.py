"""Why the oracle's C1 triangle-test count (10.8 per segment) is below the
reference probe's 15.8: the C1 geometry
regrouped into meshes four ways, the oracle's (the reference octree's) tests
per segment for each. The reference's mesh-root early-out (mesh.cpp:79-83)
skips a mesh whose box entry lies beyond the best hit, so splitting the room
into small meshes saves tests; one Cornell-room OBJ (walls + light as one
12-face mesh, the two boxes apart) reproduces the probe's figure.
All materials white (segments per sample differ from C1's 5.10).
usage: python tools/c1_grouping.py"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"), os.path.join(ROOT, "oracle")]
import fsamd  # noqa: E402
import oracle_py  # noqa: E402
import scenes  # noqa: E402

NAMES = ["walls", "left", "right", "light", "tall", "short"]  # C1's meshes in object order
GROUPINGS = [("C1 as written (6 meshes)", [[n] for n in NAMES]),
             ("the boxes as one mesh", [["walls"], ["left"], ["right"], ["light"], ["tall", "short"]]),
             ("walls + light as one 12-face mesh, boxes apart", [["walls", "left", "right", "light"], ["tall"], ["short"]]),
             ("one 36-face mesh", [NAMES])]


def main(d="/tmp/fs_c1_grouping"):
    path = scenes.write("c1", os.path.join(d, "c1"))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(path)
    fsamd.initialize_materials()
    o = oracle_py.Scene(s.desc_ptr())
    lib = oracle_py.lib()
    verts, faces = {}, {}
    out = (C.c_float * 3)()
    for k, n in enumerate(NAMES):  # world-space vertices (after the boxes' translation / rotation)
        vs, i = [], 0
        while lib.oracle_mesh_vertex(o.h, k, i, out) == 0:
            vs.append(list(out))
            i += 1
        verts[n] = np.array(vs)
        faces[n] = np.array([ln.split()[1:] for ln in open(os.path.join(d, "c1", f"{n}.obj")) if ln.startswith("f ")],
                            int) - 1
    o.close()
    for label, groups in GROUPINGS:
        gd = os.path.join(d, str(GROUPINGS.index((label, groups))))
        os.makedirs(gd, exist_ok=True)
        text = scenes.BASE_MATERIALS + scenes.CORNELL_CAMERA
        for gi, g in enumerate(groups):
            vs, fs, off = [], [], 0
            for n in g:
                vs.append(verts[n])
                fs.append(faces[n] + off)
                off += len(verts[n])
            scenes._write_obj(os.path.join(gd, f"g{gi}.obj"), np.concatenate(vs), np.concatenate(fs))
            text += f"mesh\n{{\n  file g{gi}.obj\n  material white\n}}\n"
        p = os.path.join(gd, "c1.scene")
        open(p, "w").write(text)
        fsamd.reset_main_rng()
        hs = fsamd.HostScene.load(p)
        fsamd.initialize_materials()
        oo = oracle_py.Scene(hs.desc_ptr())
        st = oo.render(hs.camera(0), fsamd.render_params(256, 256, 8), threads=8).stats
        oo.close()
        print(f"{label}: segments/sample {st['segments'] / st['samples']:.2f}, "
              f"tri tests/segment {st['tri_tests'] / st['segments']:.2f}", flush=True)


if __name__ == "__main__":
    main()
