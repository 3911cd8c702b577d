"""Seeded random scenes against the oracle, every plane bit-exact.

The fixed scenes (C1-C4, the material zoo, the tie scene) pin the kernels on
hand-picked geometry; these draw the geometry: spheres, planes, discs, both
quad kinds and rotated cuboids at random places and sizes, small meshes of
random faces (tested face by face), and a cloud of random triangles large
enough for a BVH walk (with parking forced on one schedule), in the Cornell
room, with every material; with transcendental=True also frosted glass,
sphere-mapped textured spheres, a textured sky and a thin-lens camera (the
fs_libm.h sinf/cosf/atan2f paths). Objects overlap, intersect and nest at random, so
segments start inside boxes, graze faces and tie more often than in the bench
scenes."""
import numpy as np
import pytest

import fsamd
from descbuild import DescBuilder, cornell_room
from test_gpu_parity import assert_parity, gpu_render, oracle_render

pytestmark = pytest.mark.gpu


def random_scene(seed, cloud_tris=3000, crowd=0, textured=False, transcendental=False):
    rng = np.random.default_rng(seed)
    b = DescBuilder()
    white = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.73, 0.73, 0.73))
    red = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.65, 0.05, 0.05))
    light = b.material(fsamd.MAT_LIGHT, emissive=(12, 12, 12))
    u = lambda lo, hi: float(rng.uniform(lo, hi))  # noqa: E731
    col = lambda: tuple(float(x) for x in rng.uniform(0.2, 0.95, 3))  # noqa: E731
    mats = [
        b.material(fsamd.MAT_DIFFUSE, diffuse=col()),
        b.material(fsamd.MAT_METAL, diffuse=col(), roughness=u(0.0, 1.0)),
        b.material(fsamd.MAT_MIRROR, diffuse=col()),
        b.material(fsamd.MAT_GLASS, diffuse=col(), index=u(0.5, 1.6), reflectivity=u(0.0, 0.5)),
        b.material(fsamd.MAT_LIQUID, diffuse=col(), index=u(1.1, 1.6), reflectivity=u(0.0, 0.5)),
        b.material(fsamd.MAT_CERAMIC, diffuse=col(), shininess=u(0.0, 1.0)),
        b.material(fsamd.MAT_GLOW, diffuse=col(), glow=col(), shininess=u(0.0, 1.0)),
        b.material(fsamd.MAT_FOG, diffuse=col(), density=u(0.001, 0.05)),
        b.material(fsamd.MAT_LIGHT, emissive=tuple(3 * x for x in col())),
    ]
    if transcendental:  # frosted glass: the refraction rotated by cosf/sinf of a drawn angle
        mats += [b.material(fsamd.MAT_GLASS, diffuse=col(), index=u(0.5, 1.6), reflectivity=u(0.0, 0.5),
                            frost=u(0.02, 1.0)) for _ in range(2)]
    pick = lambda: mats[int(rng.integers(len(mats)))]  # noqa: E731
    flat = pick  # materials of objects whose texture lookup is bit-exact (planar maps, mesh texcoords)
    if textured:  # diffuse maps of random sizes and scales; spheres (atan2f maps) never take them
        tex = [b.texture(rng.random((int(rng.integers(2, 40)), int(rng.integers(2, 40)), 3)) * u(0.3, 2.0))
               for _ in range(2)]
        tmats = [b.material(fsamd.MAT_DIFFUSE, diffuse=col(), texture=t, texture_scale=u(0.05, 3.0)) for t in tex]
        flat = lambda: tmats[int(rng.integers(2))] if rng.random() < 0.6 else pick()  # noqa: E731
    if textured and transcendental:  # spheres take maps too (atan2f), and the sky
        sphere_pick = lambda: tmats[int(rng.integers(2))] if rng.random() < 0.6 else pick()  # noqa: E731
        b.sky = b.material(fsamd.MAT_LIGHT, emissive=tuple(0.3 * x for x in col()), texture=tex[0],
                           texture_scale=1.0)
    else:
        sphere_pick = pick
    cornell_room(b, white, red, light)
    p = lambda: [u(-8, 8), u(1, 18), u(-8, 8)]  # noqa: E731
    n = lambda: list(rng.normal(size=3))  # noqa: E731
    for _ in range(int(rng.integers(2, 5))):
        b.obj(fsamd.OBJ_SPHERE, sphere_pick(), p() + [u(0.5, 3)])
    if rng.random() < 0.5:
        nv = np.array(n())
        nv /= np.linalg.norm(nv)
        b.obj(fsamd.OBJ_PLANE, flat(), list(nv) + [u(-9, 9)])
    for _ in range(int(rng.integers(1, 3))):
        b.obj(fsamd.OBJ_DISC, flat(), p() + n() + [u(0.5, 4)])
    for _ in range(int(rng.integers(1, 3))):
        b.obj(fsamd.OBJ_QUAD_ONWH, flat(), p() + n() + [u(1, 6), u(1, 6)])
    for _ in range(int(rng.integers(1, 3))):
        b.obj(fsamd.OBJ_QUAD_PUV, flat(), p() + [u(-4, 4) for _ in range(6)])
    for _ in range(int(rng.integers(1, 3))):
        b.obj(fsamd.OBJ_CUBOID, flat(), p() + [u(0.5, 4), u(0.5, 4), u(0.5, 4)] + n() + [u(-3, 3)],
              rotate=int(rng.integers(0, 2)))
    for _ in range(int(rng.integers(2, 4))):  # small meshes: random faces, some sharing an edge
        nf = int(rng.integers(2, 15))
        c = np.array(p())
        v = c + rng.normal(scale=u(0.5, 3), size=(nf + 2, 3))
        faces = [[0, 1, i + 2] if rng.random() < 0.3 else list(rng.choice(nf + 2, 3, replace=False))
                 for i in range(nf)]
        b.mesh(flat(), v.tolist(), faces)
    for j in range(crowd):  # many small analytic objects (the object-octree threshold is 182)
        k = int(rng.integers(4))
        if k == 0:
            b.obj(fsamd.OBJ_SPHERE, pick(), p() + [u(0.2, 0.9)])
        elif k == 1:
            b.obj(fsamd.OBJ_CUBOID, flat(), p() + [u(0.3, 1.2), u(0.3, 1.2), u(0.3, 1.2)] + n() + [u(-3, 3)],
                  rotate=1)
        elif k == 2:
            b.obj(fsamd.OBJ_DISC, flat(), p() + n() + [u(0.3, 1.0)])
        else:
            b.obj(fsamd.OBJ_QUAD_PUV, flat(), p() + [u(-1, 1) for _ in range(6)])
    # a triangle cloud for the BVH walk: small faces around random centres
    c = np.array(p())
    centres = c + rng.normal(scale=3.0, size=(cloud_tris, 1, 3))
    tv = (centres + rng.normal(scale=0.35, size=(cloud_tris, 3, 3))).reshape(-1, 3)
    faces = np.arange(3 * cloud_tris).reshape(-1, 3)
    tc = rng.random((3 * cloud_tris, 2)) * 4.0 - 1.0 if textured else None
    b.mesh(flat(), tv.tolist(), faces.tolist(), rotation=(0, 1, 0, u(-1, 1)), scale=(u(0.7, 1.3),) * 3,
           texcoords=tc, corner_tex=faces if textured else None)
    return b


CAMS = [fsamd.camera((0, 10, -34), (0, 10, 0), fov_y=40, aperture=0.0),
        fsamd.camera((-8, 15, -9), (4, 6, 5), fov_y=70, aperture=0.0)]


@pytest.mark.parametrize("seed", range(16))
def test_random_scene_bit_exact(seed, gpu_renderer):
    """Sixteen seeded scenes, two camera placements (one inside the clutter)."""
    b = random_scene(seed)  # keeps the arrays the description points at alive
    ptr = b.build()
    cam = CAMS[seed % 2]
    out = gpu_render(gpu_renderer, ptr, cam, 80, 60, 8)
    ref = oracle_render(ptr, cam, 80, 60, 8)
    assert_parity(out, ref, exact=True)


@pytest.mark.parametrize("schedule,seed", [("parked", 100), ("parked", 101), ("parked", 102), ("parked", 103),
                                           ("lean", 200), ("lean", 201)])
def test_random_scene_schedules_bit_exact(schedule, seed, gpu_renderer):
    """The parked-walk kernel (C3 and C4's) with parking forced for the
    triangle cloud (park_min_tris = 1), and the lean kernel, on random
    clutter."""
    gpu_renderer.set_options(schedule=schedule, park_min_tris=1)
    b = random_scene(seed)  # keeps the arrays the description points at alive
    ptr = b.build()
    cam = CAMS[seed % 2]
    out = gpu_render(gpu_renderer, ptr, cam, 80, 60, 8)
    ref = oracle_render(ptr, cam, 80, 60, 8)
    assert_parity(out, ref, exact=True)


@pytest.mark.parametrize("optimized,seed", [(True, 300), (True, 301), (False, 302)])
def test_random_crowd_bit_exact(optimized, seed, gpu_renderer):
    """About 200 random objects: optimized, traced through the reference's
    object octree (scene.cpp:11-133, the SOCT kernel), else down the object
    list."""
    b = random_scene(seed, cloud_tris=500, crowd=190)
    ptr = b.build(optimized=optimized)
    cam = CAMS[seed % 2]
    out = gpu_render(gpu_renderer, ptr, cam, 80, 60, 8)
    k = gpu_renderer.last_kernel()
    assert (k[:-1].split(", ")[5] == "true") == optimized, k
    ref = oracle_render(ptr, cam, 80, 60, 8)
    assert_parity(out, ref, exact=True)


@pytest.mark.parametrize("seed", [400, 401, 402])
def test_random_textured_scene_bit_exact(seed, gpu_renderer):
    """Random diffuse maps on planes, discs, quads, cuboids and meshes (planar
    maps and mesh texcoords, material.cpp:108-126): the textured kernel."""
    b = random_scene(seed, cloud_tris=1000, textured=True)
    ptr = b.build()
    cam = CAMS[seed % 2]
    out = gpu_render(gpu_renderer, ptr, cam, 80, 60, 8)
    assert gpu_renderer.last_kernel()[:-1].split(", ")[2] == "true", gpu_renderer.last_kernel()  # TEX
    ref = oracle_render(ptr, cam, 80, 60, 8)
    assert_parity(out, ref, exact=True)


@pytest.mark.parametrize("seed", [500, 501])
def test_random_scene_larger_frame_bit_exact(seed, gpu_renderer):
    """Two random scenes at 256 x 192 x 16 spp (790 k samples each)."""
    b = random_scene(seed)
    ptr = b.build()
    cam = CAMS[seed % 2]
    out = gpu_render(gpu_renderer, ptr, cam, 256, 192, 16)
    ref = oracle_render(ptr, cam, 256, 192, 16)
    assert_parity(out, ref, exact=True)


@pytest.mark.parametrize("seed,textured", [(600, False), (601, True), (602, False), (603, True), (604, True),
                                           (605, False)])
def test_random_scene_with_transcendentals_bit_exact(seed, textured, gpu_renderer):
    """Frosted glass, sphere-mapped spheres, a textured sky and a thin-lens
    camera of random aperture and focal depth: the
    device's sinf/cosf/atan2f are the host C library's bits (fs_libm.h)."""
    rng = np.random.default_rng(seed)
    b = random_scene(seed, cloud_tris=1500, textured=textured, transcendental=True)
    ptr = b.build()
    cam = fsamd.camera((float(rng.uniform(-3, 3)), 10, -34), (0, float(rng.uniform(6, 12)), 0), fov_y=45,
                       aperture=float(rng.uniform(0.1, 2.0)), focal_depth=float(rng.uniform(20, 45)))
    out = gpu_render(gpu_renderer, ptr, cam, 80, 60, 8)
    ref = oracle_render(ptr, cam, 80, 60, 8)
    assert_parity(out, ref, exact=True)
