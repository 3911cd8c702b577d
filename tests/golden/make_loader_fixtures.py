"""Writes tests/golden/loaders.npz: OBJ and EXR inputs and what the
REFERENCE'S OWN vendored loaders return for them (container only).

The outputs come from oracle/_ref/ref_loaders (oracle/ref_loaders.cpp, built
by `make -C oracle ref` from the unmodified tiny_obj_loader.h v1.2.2 and
tiny_exr_loader.h under /root/reference/source/third_party): LoadObj with
triangulate = true as mesh.cpp:177 calls it, and LoadEXR as material.cpp:75
calls it. tests/test_loader_fixtures.py pins the C++ mirror's loaders
(host/fs_host.cpp, host/fs_image.cpp) against them byte for byte. The
fixture holds data only: the input files' bytes and the decoded arrays.

usage: python tests/golden/make_loader_fixtures.py
"""
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
import exrwrite as X  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "ref_loaders")


def obj_cases():
    """OBJ texts: tinyobj's number parser, index forms and its ear clipping."""
    rng = np.random.default_rng(7)
    c = {}
    c["numbers"] = ("v 0.300000086426734924316406251 1.7000001072883605957031251 -2.5e-1\n"
                    "v 1e3 -2.5E-2 +.5\nv 3.4028234e38 -1.17549435e-38 1e-45\n"
                    "v \t 12345678.9\t-0.000000123456789  7\nv 1. -0. .25e+2\n"
                    "v 0.1 0.2 0.3\nv 2.5e-3 1.0000001 9.99999999\n"
                    "f 1 2 3\nf 4 5 6\nf 5 6 7\n")
    verts = [(0, 0), (3, 0), (3, 1), (1, 1), (1, 2), (3, 2), (3, 3), (0, 3)]
    c["concave_c"] = ("".join(f"v {x} {y} 0\n" for x, y in verts) + "vt 0 0\n" +
                      "f " + " ".join(f"{i + 1}/1" for i in range(8)) + "\nf 1 2 3 4\n")
    # an L-shape in the xz plane and a star in yz: other dominant axes
    L = [(0, 0), (2, 0), (2, 1), (1, 1), (1, 3), (0, 3)]
    star = [(np.cos(a) * (1.0 if k % 2 == 0 else 0.4), np.sin(a) * (1.0 if k % 2 == 0 else 0.4))
            for k, a in enumerate(np.linspace(0, 2 * np.pi, 10, endpoint=False))]
    c["axes"] = ("".join(f"v {x} 0.5 {z}\n" for x, z in L) + "".join(f"v 2 {y:.6f} {z:.6f}\n" for y, z in star) +
                 "vn 0 1 0\n" + "f " + " ".join(f"{i + 1}//1" for i in range(6)) + "\n" +
                 "f " + " ".join(str(7 + i) for i in range(10)) + "\n")
    # degenerate polygons: collinear corners, repeated vertices, a zero-area quad
    c["degenerate"] = ("v 0 0 0\nv 1 0 0\nv 2 0 0\nv 3 0 0\nv 0 1 0\nv 1 1 0\n"
                       "f 1 2 3 4\nf 1 2 6 5\nf 1 1 2 6\nf 1 2 2 2 6 5\n")
    # non-planar polygons with texcoords and normals, negative (relative) indices
    pts = rng.normal(size=(40, 3)).round(4)
    txt = "".join(f"v {a} {b} {z}\n" for a, b, z in pts) + "vt 0.5 0.5\nvt 0 1\nvn 0 0 1\nvn 1 0 0\n"
    for k in range(8):
        n = 4 + k % 5
        ids = rng.choice(40, size=n, replace=False) + 1
        txt += "f " + " ".join(f"{i}/{1 + (j % 2)}/{1 + (k % 2)}" for j, i in enumerate(ids)) + "\n"
    txt += "f -1 -2 -3 -4 -5\nf -10/-1 -11/-2 -12/-1\n"
    c["nonplanar"] = txt
    # a ring (regular polygon with a notch) and a long thin sliver polygon
    ring = [(np.cos(a) * r, np.sin(a) * r) for a, r in
            zip(np.linspace(0, 2 * np.pi, 12, endpoint=False), [1, 1, 1, 0.2, 1, 1, 1, 1, 0.2, 1, 1, 1])]
    c["ring_sliver"] = ("".join(f"v {x:.5f} {y:.5f} 0.25\n" for x, y in ring) +
                        "v 0 0 0\nv 10 0.001 0\nv 20 0 0\nv 10 0.002 0\n" +
                        "f " + " ".join(str(i + 1) for i in range(12)) + "\nf 13 14 15 16\n")
    return c


def exr_cases(tmp):
    """EXR files from tests/exrwrite.py: every compression LoadEXR takes,
    scanline and tiled, HALF / FLOAT / UINT channels, alpha, line orders."""
    rng = np.random.default_rng(11)
    out = {}

    def rgb(h, w, kind):
        a = rng.random((3, h, w), dtype=np.float32) * 8 - 2
        return a.astype(np.float16).astype(np.float32) if kind == X.HALF else a

    names = {X.NONE: "none", X.RLE: "rle", X.ZIPS: "zips", X.ZIP: "zip", X.PIZ: "piz"}
    for comp in (X.NONE, X.RLE, X.ZIPS, X.ZIP, X.PIZ):
        for kind, kn in ((X.HALF, "half"), (X.FLOAT, "float")):
            H, W = (37, 21) if comp != X.PIZ else (70, 33)
            r, g, b = rgb(H, W, kind)
            p = os.path.join(tmp, f"{names[comp]}_{kn}.exr")
            X.write(p, [("B", kind, b), ("G", kind, g), ("R", kind, r)], compression=comp, origin=(3, -2))
            out[f"scan_{names[comp]}_{kn}"] = p
        H, W = 19, 23
        r, g, b = rgb(H, W, X.HALF)
        p = os.path.join(tmp, f"tiled_{names[comp]}.exr")
        X.write(p, [("B", X.HALF, b), ("G", X.HALF, g), ("R", X.HALF, r)], compression=comp, tiles=(8, 6))
        out[f"tiled_{names[comp]}"] = p
    H, W = 9, 300
    r = np.zeros((H, W), np.float32)
    r[:, 100:] = 0.5
    a = np.full((H, W), 0.75, np.float32)
    p = os.path.join(tmp, "alpha_rle.exr")
    X.write(p, [("A", X.HALF, a), ("B", X.FLOAT, r * 2), ("G", X.HALF, a * 0.5), ("R", X.FLOAT, r)],
            compression=X.RLE)
    out["alpha_rle"] = p
    r, g, b = rgb(6, 5, X.FLOAT)
    p = os.path.join(tmp, "decreasing.exr")
    X.write(p, [("B", X.FLOAT, b), ("G", X.FLOAT, g), ("R", X.FLOAT, r)], line_order=1)
    out["decreasing"] = p
    u = (rng.integers(0, 1 << 20, size=(3, 8, 8))).astype(np.uint32)
    p = os.path.join(tmp, "uint_zip.exr")
    X.write(p, [("B", X.UINT, u[2]), ("G", X.UINT, u[1]), ("R", X.UINT, u[0])], compression=X.ZIP)
    out["uint_zip"] = p
    p = os.path.join(tmp, "alpha_only.exr")
    X.write(p, [("A", X.FLOAT, rgb(4, 7, X.FLOAT)[0])])
    out["alpha_only"] = p
    return out


def run_obj(path):
    with tempfile.NamedTemporaryFile(suffix=".bin") as f:
        subprocess.run([REF, "obj", path, f.name], check=True)
        b = open(f.name, "rb").read()
    ok, nv, nn, nt, ns = struct.unpack_from("<iIIII", b, 0)
    o = 20
    v = np.frombuffer(b, np.float32, nv, o)
    o += 4 * nv
    n = np.frombuffer(b, np.float32, nn, o)
    o += 4 * nn
    t = np.frombuffer(b, np.float32, nt, o)
    o += 4 * nt
    idx, nfv = [], []
    for _ in range(ns):
        ni, nf = struct.unpack_from("<II", b, o)
        o += 8
        idx.append(np.frombuffer(b, np.int32, 3 * ni, o).reshape(ni, 3))
        o += 12 * ni
        nfv.append(np.frombuffer(b, np.uint32, nf, o))
        o += 4 * nf
    idx = np.concatenate(idx) if idx else np.zeros((0, 3), np.int32)
    nfv = np.concatenate(nfv) if nfv else np.zeros(0, np.uint32)
    return ok, v, n, t, idx, nfv


def run_exr(path):
    with tempfile.NamedTemporaryFile(suffix=".bin") as f:
        subprocess.run([REF, "exr", path, f.name], check=True)
        b = open(f.name, "rb").read()
    rc = struct.unpack_from("<i", b, 0)[0]
    if rc < 0:
        return rc, np.zeros((0, 0, 4), np.float32)
    w, h = struct.unpack_from("<ii", b, 4)
    return rc, np.frombuffer(b, np.float32, w * h * 4, 12).reshape(h, w, 4)


def main():
    if not os.path.exists(REF):
        raise SystemExit(f"{REF} missing: run `make -C oracle ref` (needs /root/reference)")
    arrays = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, text in obj_cases().items():
            p = os.path.join(tmp, name + ".obj")
            open(p, "w").write(text)
            ok, v, n, t, idx, nfv = run_obj(p)
            assert ok == 1 and (nfv == 3).all(), name
            arrays[f"obj/{name}/input"] = np.frombuffer(text.encode(), np.uint8)
            arrays[f"obj/{name}/vertices"] = v
            arrays[f"obj/{name}/normals"] = n
            arrays[f"obj/{name}/texcoords"] = t
            arrays[f"obj/{name}/indices"] = idx  # (vertex, normal, texcoord) per corner, 3 per triangle
        for name, p in exr_cases(tmp).items():
            rc, rgba = run_exr(p)
            arrays[f"exr/{name}/input"] = np.frombuffer(open(p, "rb").read(), np.uint8)
            arrays[f"exr/{name}/rc"] = np.array([rc], np.int32)
            arrays[f"exr/{name}/rgba"] = rgba
    out = os.path.join(HERE, "loaders.npz")
    np.savez_compressed(out, **arrays)
    print(f"wrote {out}: {len([k for k in arrays if k.endswith('/input')])} cases, {os.path.getsize(out)} bytes")


if __name__ == "__main__":
    main()
