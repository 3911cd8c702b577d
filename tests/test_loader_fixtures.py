"""The C++ mirror's loaders against the reference's own (CPU).

tests/golden/loaders.npz holds OBJ and EXR inputs and what the reference's
vendored tinyobjloader 1.2.2 (LoadObj, triangulate = true, mesh.cpp:177)
and tinyexr (LoadEXR, material.cpp:75) return for them, compiled unmodified
from /root/reference into oracle/_ref/ref_loaders by `make -C oracle ref`
(tests/golden/make_loader_fixtures.py). The mirror (host/fs_host.cpp,
host/fs_image.cpp) must return the same bytes: vertex floats bit for bit
(tinyobj's own number parser, not strtof), the same triangles with the
same (vertex, normal, texcoord) indices in the same order (its ear
clipping of concave, degenerate and non-planar polygons), and the same RGBA
floats for every compression, tiling and channel type."""
import os

import numpy as np
import pytest

import fsamd

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "loaders.npz")
DATA = np.load(FIX)
OBJS = sorted({k.split("/")[1] for k in DATA.files if k.startswith("obj/")})
EXRS = sorted({k.split("/")[1] for k in DATA.files if k.startswith("exr/")})


@pytest.mark.parametrize("name", OBJS)
def test_obj_matches_tinyobj(name, tmp_path):
    p = tmp_path / f"{name}.obj"
    p.write_bytes(DATA[f"obj/{name}/input"].tobytes())
    pos, corners = fsamd.load_obj(str(p))
    ref_v = DATA[f"obj/{name}/vertices"].reshape(-1, 3)
    np.testing.assert_array_equal(pos.view(np.uint32), ref_v.view(np.uint32))
    idx = DATA[f"obj/{name}/indices"]  # tinyobj index_t: (vertex, normal, texcoord)
    # the mirror keeps (v, n, t) per corner, 3 corners per triangle, in OBJ order
    np.testing.assert_array_equal(corners.reshape(-1, 3), idx)


@pytest.mark.parametrize("name", EXRS)
def test_exr_matches_tinyexr(name, tmp_path):
    p = tmp_path / f"{name}.exr"
    p.write_bytes(DATA[f"exr/{name}/input"].tobytes())
    rc = int(DATA[f"exr/{name}/rc"][0])
    if rc < 0:
        with pytest.raises(fsamd.FsError):
            fsamd.load_exr(p)
        return
    out = fsamd.load_exr(p)
    ref = DATA[f"exr/{name}/rgba"]
    assert out.shape == ref.shape
    np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_fixture_covers_every_compression_and_layout():
    for c in ("none", "rle", "zips", "zip", "piz"):
        assert f"tiled_{c}" in EXRS
        for k in ("half", "float"):
            assert f"scan_{c}_{k}" in EXRS
    assert {"numbers", "concave_c", "degenerate", "nonplanar", "axes"} <= set(OBJS)
