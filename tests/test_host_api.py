"""The C++ mirror of the reference API (host/fs_host.h): RNG, material ids,
normal table, `.scene` grammar quirks and the OBJ loader. CPU only."""
import ctypes as C
import os

import numpy as np
import pytest

import fsamd
import oracle_py
from conftest import load_scene


def test_host_rng_matches_oracle():
    fsamd.reset_main_rng()
    s = C.c_uint64(521288629)
    for _ in range(100):
        assert fsamd.random_integer() == oracle_py.lib().oracle_random_integer(C.byref(s))
    fsamd.reset_main_rng()
    s = C.c_uint64(521288629)
    for _ in range(100):
        assert np.float32(fsamd.random_float()) == np.float32(oracle_py.lib().oracle_random_float(C.byref(s)))


def test_material_ids_and_table_follow_reference_draw_order(scene_dir):
    # Scene() draws 1 (sky, scene.cpp:143), each material block 1
    # (material.cpp:26); InitializeMaterials then draws the table.
    s = load_scene("c2", scene_dir)
    d = s.desc().contents
    assert d.num_materials == 6  # sky + white, red, light, glossy, glass
    st = C.c_uint64(521288629)
    ids = [oracle_py.lib().oracle_random_integer(C.byref(st)) & 0xFFFFFFFF for _ in range(6)]
    assert [d.materials[i].id for i in range(6)] == ids
    ot = np.zeros((32768, 3), np.float32)
    oracle_py.lib().oracle_normal_table(521288629, 6, 32768, oracle_py.fptr(ot)[1])
    np.testing.assert_array_equal(fsamd.normal_table(), ot)
    kinds = [d.materials[i].kind for i in range(6)]
    assert kinds == [fsamd.MAT_LIGHT, fsamd.MAT_DIFFUSE, fsamd.MAT_DIFFUSE, fsamd.MAT_LIGHT,
                     fsamd.MAT_CERAMIC, fsamd.MAT_GLASS]


def write(tmp, name, text):
    p = os.path.join(tmp, name)
    open(p, "w").write(text)
    return p


def test_scene_grammar_precedence_and_quirks(tmp_path):
    tmp = str(tmp_path)
    write(tmp, "tri.obj", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    text = """# comment line with sphere in it is skipped
material a
{
  color 0.5 0.5 0.5
  emission 0 0 0
  metallic 1
}
material b
{
  color 0.1 0.2 0.3
  metallic 0.4
  roughness 0.2
}
material c
{
  brdf 1
  index 1.2
  texture_scale 2
}
material d
{
  emission 1 2 3 }
  color 9 9 9
material e
{
  metallic 0.25
}
a sky block
{
  material d
}
camera
{
  position 1 2 3
  fov 30
}
mesh
{
  file tri.obj
  material c
  scale 2 2 2
}
cuboid
{
  material e
  position 0 1 0
  width 2
  height 2
  depth 2
}
quad
{
  material a
  position 0 5 0
  normal 0 -1 0
  width 4
  height 4
}
sphere
{
  material b
  position 0 0 0
  radius 1
}
"""
    p = write(tmp, "t.scene", text)
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    d = s.desc().contents
    kinds = {d.materials[i].kind for i in range(d.num_materials)}
    # metallic == 1 -> Mirror; roughness wins over metallic -> Ceramic; brdf 1 -> Liquid;
    # a block ends at the first line containing '}' BEFORE that line is parsed
    # (scene.cpp:267-268): `d` never sees its emission and stays a black Diffuse
    mats = [d.materials[i] for i in range(d.num_materials)]
    by_kind = {m.kind: m for m in mats}
    assert fsamd.MAT_MIRROR in kinds and fsamd.MAT_CERAMIC in kinds and fsamd.MAT_LIQUID in kinds
    assert by_kind[fsamd.MAT_CERAMIC].shininess == np.float32(0.2)
    assert by_kind[fsamd.MAT_LIQUID].index == np.float32(1.2)
    assert by_kind[fsamd.MAT_LIQUID].reflectivity == np.float32(0.1)   # ParseMaterial default
    assert by_kind[fsamd.MAT_METAL].roughness == np.float32(0.25)
    sky = mats[d.sky_material]
    assert sky.kind == fsamd.MAT_DIFFUSE and list(sky.emissive) == [0.0, 0.0, 0.0]
    # `texture_scale 2` also matches " texture %s" (token "_scale"): not a loadable
    # texture, so the material stays untextured, as in material.cpp:68-94
    assert by_kind[fsamd.MAT_LIQUID].texture == -1
    assert s.camera_count() == 1
    cam = s.camera(0)
    assert list(cam.origin) == [1, 2, 3] and cam.fov_y == 30 and cam.aperture_size == np.float32(1.5)
    assert d.num_objects == 4
    obj = [d.objects[i] for i in range(4)]
    assert [o.kind for o in obj] == [fsamd.OBJ_MESH, fsamd.OBJ_CUBOID, fsamd.OBJ_QUAD_ONWH, fsamd.OBJ_SPHERE]
    assert obj[1].rotate == 1  # ParseCuboid always calls Rotate (scene.cpp:452)
    m = d.meshes[0]
    assert m.num_triangles == 1 and list(m.scale) == [2, 2, 2]


def test_object_without_material_is_rejected(tmp_path):
    p = write(str(tmp_path), "n.scene", "sphere\n{\n  position 0 0 0\n  radius 1\n}\n")
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    with pytest.raises(fsamd.FsError, match="no material"):
        s.desc()


def test_missing_scene_file():
    with pytest.raises(fsamd.FsError):
        fsamd.HostScene.load("/nonexistent/x.scene")


def test_obj_loader_formats(tmp_path):
    text = """v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
vt 0 0
vt 1 0
vn 0 0 1
f 1/1/1 2/2/1 3/1/1
f 1//1 3//1 4//1
f -4 -3 -2 -1
"""
    p = write(str(tmp_path), "q.obj", text)
    pos, corners = fsamd.load_obj(p)
    assert pos.shape == (4, 3)
    # triangle, triangle, quad fan-split into two
    assert corners.shape == (4, 9)
    assert list(corners[0]) == [0, 0, 0, 1, 0, 1, 2, 0, 0]  # (v, n, t) per corner
    assert list(corners[1][[0, 1, 2]]) == [0, 0, -1]
    assert list(corners[2][[0, 3, 6]]) == [0, 1, 2] and list(corners[3][[0, 3, 6]]) == [0, 2, 3]


def test_generated_scene_sizes(scene_dir):
    import scenes

    v, f = scenes.blob_mesh(100, 50)
    assert f.shape == (10000, 3) and v.shape == (51 * 100, 3)
    path, ntri = scenes.write_c3(os.path.join(scene_dir, "c3_count"))
    assert abs(ntri - 250_000) / 250_000 < 0.01
    # SURVEY Appendix A's calibration probe: the C1 room (6 meshes + 2 boxes) and one blob, no analytic objects
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(scenes.write_probe(os.path.join(scene_dir, "probe_count"), nu=40, nv=20))
    d = s.desc().contents
    kinds = [d.objects[i].kind for i in range(d.num_objects)]
    assert kinds == [fsamd.OBJ_MESH] * 7
    assert sum(d.meshes[i].num_triangles for i in range(d.num_meshes)) == 40 * 20 * 2 + 36


def test_parallel_bvh_build_is_reproducible(scene_dir, monkeypatch):
    """The BVH build runs subtrees on threads; the uploaded arrays (nodes,
    triangles, normals, objects) must be byte-identical to the sequential
    build (fs_prepare_digest, host only)."""
    import fsamd
    from conftest import load_scene

    s = load_scene("c3", scene_dir)
    digests = set()
    for threads in (1, 2, 16):
        d, nodes, ms = fsamd.prepare_digest(s.desc_ptr(), bvh_threads=threads)
        digests.add((d, nodes))
    assert len(digests) == 1


def test_obj_numbers_follow_tinyobj_parser(tmp_path):
    """tryParseDouble (tiny_obj_loader.h:537-650) is not correctly rounded: it
    accumulates fraction digits in double before the float cast. These two
    strings sit just above a float32 rounding midpoint; tinyobj (and the
    mirror) round them down, a correctly rounded strtof rounds them up."""
    import fsamd

    p = tmp_path / "n.obj"
    p.write_text("v 0.300000086426734924316406251 1.7000001072883605957031251 -2.5e-1\n"
                 "v 1 0 0\nv 0 1 0\nf 1 2 3\n")
    pos, _ = fsamd.load_obj(str(p))
    assert pos[0, 0] == np.float32(0.30000007152557373)
    assert pos[0, 1] == np.float32(1.7000000476837158)
    assert pos[0, 2] == np.float32(-0.25)


def test_obj_polygons_ear_clipped_like_tinyobj(tmp_path):
    """Polygon faces are triangulated by tinyobj's ear clipping
    (tiny_obj_loader.h:1042-1236), not a fan: for this C-shaped octagon a fan
    from vertex 0 would cross the notch. Expected ears worked by hand."""
    import fsamd

    p = tmp_path / "c.obj"
    verts = [(0, 0), (3, 0), (3, 1), (1, 1), (1, 2), (3, 2), (3, 3), (0, 3)]
    p.write_text("".join(f"v {x} {y} 0\n" for x, y in verts) + "vt 0 0\n" +
                 "f " + " ".join(f"{i + 1}/1" for i in range(8)) + "\n" + "f 1 2 3 4\n")
    _, corners = fsamd.load_obj(str(p))
    tris = [tuple(c[0::3]) for c in corners]
    assert tris == [(0, 1, 2), (0, 2, 3), (0, 3, 4), (4, 5, 6), (4, 6, 7), (0, 4, 7),
                    (0, 1, 2), (0, 2, 3)]  # then the convex quad
    assert (corners[:6, 2::3] == 0).all() and (corners[:, 1::3] == -1).all()  # vt kept, no vn
