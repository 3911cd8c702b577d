"""Device BVH build (fs_upload_scene_ex with FS_UPLOAD_GPU_BVH, csrc/fs_bvh_gpu.hip).

The reference builds its mesh octree on the CPU at load time
(mesh.cpp:117-152); SURVEY §8f rank 1 moves the build to the GPU. The BVH only
culls (closest hit by strict `<`, exact ties to the lower face
index), so a device-built tree must give the host-built tree's frames bit for
bit, and both must match the oracle.
"""
import numpy as np
import pytest

import fsamd
import oracle_py
from conftest import load_scene
from descbuild import DescBuilder, cornell_room

pytestmark = pytest.mark.gpu

PLANES = range(6)


def render_planes(r, desc, cam, W, H, spp, gpu_bvh):
    r.upload(desc, gpu_bvh=gpu_bvh)
    stats = r.scene_stats()
    f = r.frame(W, H)
    r.render(cam, f, spp=spp)
    out = {p: f.read(p) for p in PLANES}
    f.close()
    return out, stats


def assert_same(a, b):
    for p in PLANES:
        np.testing.assert_array_equal(a[p], b[p], err_msg=f"plane {p}")


def assert_oracle(out, desc_ptr, cam, W, H, spp):
    o = oracle_py.Scene(desc_ptr)
    ref = o.render(cam, fsamd.render_params(W, H, spp), threads=16)
    o.close()
    np.testing.assert_array_equal(out[fsamd.PLANE_COLOR], ref.color)
    np.testing.assert_array_equal(out[fsamd.PLANE_COUNT], ref.count)
    np.testing.assert_array_equal(out[fsamd.PLANE_DISPLAY], ref.display)
    np.testing.assert_array_equal(out[fsamd.PLANE_MATERIAL], ref.material)


@pytest.mark.parametrize("name,dims,min_tris", [("c4", (1920, 1080, 4), None), ("c3", (480, 270, 8), "1024")])
def test_device_bvh_frames_equal_host_bvh(name, dims, min_tris, scene_dir, gpu_renderer):
    """C4 (one 1 M-face mesh: the default threshold defers it) at full 1080p,
    and C3 with the threshold lowered so every mesh of >= 1024 faces takes the
    device build."""
    if min_tris:
        gpu_renderer.set_options(gpu_bvh_min_tris=int(min_tris))
    W, H, spp = dims
    s = load_scene(name, scene_dir)
    cam = s.camera(0)
    host, hs = render_planes(gpu_renderer, s, cam, W, H, spp, gpu_bvh=False)
    dev, ds = render_planes(gpu_renderer, s, cam, W, H, spp, gpu_bvh=True)
    assert_same(dev, host)
    assert ds["triangles"] == hs["triangles"]
    # binary trees over the same faces with the same leaf bound: similar sizes
    assert 0.8 * hs["nodes"] <= ds["nodes"] <= 1.25 * hs["nodes"], (hs, ds)


def test_device_bvh_c4_matches_oracle(scene_dir, gpu_renderer):
    W, H, spp = 128, 72, 4
    s = load_scene("c4", scene_dir)
    cam = s.camera(0)
    out, _ = render_planes(gpu_renderer, s, cam, W, H, spp, gpu_bvh=True)
    assert_oracle(out, s.desc_ptr(), cam, W, H, spp)


def grid(n, z, jitter=0.0, seed=0):
    """An n x n quad grid (2 n^2 faces) in the plane z, with per-vertex
    normals and texcoords."""
    rng = np.random.default_rng(seed)
    u = np.linspace(-8, 8, n + 1, dtype=np.float32)
    X, Y = np.meshgrid(u, u + 10)
    Z = np.full_like(X, z) + jitter * rng.standard_normal(X.shape).astype(np.float32)
    pos = np.stack([X, Y, Z], -1).reshape(-1, 3)
    idx = np.arange((n + 1) ** 2).reshape(n + 1, n + 1)
    a, b, c, d = idx[:-1, :-1].ravel(), idx[:-1, 1:].ravel(), idx[1:, :-1].ravel(), idx[1:, 1:].ravel()
    faces = np.concatenate([np.stack([a, b, d], -1), np.stack([a, d, c], -1)])
    nrm = np.tile(np.float32([[0.1, 0.2, -1.0]]), (len(pos), 1)) + 0.05 * rng.standard_normal((len(pos), 3)).astype(
        np.float32)
    tex = np.stack([(X.ravel() + 8) / 16, (Y.ravel() - 2) / 16], -1).astype(np.float32)
    return pos, faces, nrm, tex


def test_device_bvh_degenerate_and_attributed_meshes(gpu_renderer):
    """Edge cases of the device build, each against the host build and the
    oracle: 4096 copies of one triangle (every centroid equal: even splits down
    to the leaf bound, ties broken by face index), a coplanar grid (zero
    extent on one axis) carrying vertex normals and texcoords under a diffuse
    map, and a jittered grid with inverted normals behind it."""
    gpu_renderer.set_options(gpu_bvh_min_tris=1024)
    b = DescBuilder()
    white = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.73, 0.73, 0.73))
    red = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.65, 0.05, 0.05))
    light = b.material(fsamd.MAT_LIGHT, emissive=(15, 15, 15))
    tex = b.texture(np.random.default_rng(3).random((16, 24, 3), dtype=np.float32))
    mapped = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.9, 0.9, 0.9), texture=tex, texture_scale=2.0)
    metal = b.material(fsamd.MAT_METAL, diffuse=(0.9, 0.8, 0.6), roughness=0.3)
    cornell_room(b, white, red, light)
    same = np.float32([[-3, 4, 0], [3, 4, 1], [0, 9, 2]])
    b.mesh(metal, same, np.tile(np.int32([[0, 1, 2]]), (4096, 1)), translation=(0, 0, -3))
    pos, faces, nrm, tc = grid(32, 6.0)
    b.mesh(mapped, pos, faces, normals=nrm, corner_normals=faces, texcoords=tc, corner_tex=faces,
           translation=(0.001, 0, 0))
    pos, faces, nrm, _ = grid(40, 8.0, jitter=0.3, seed=1)
    b.mesh(white, pos, faces, normals=nrm, corner_normals=faces, invert=True, translation=(0, 0, 0.5))
    d = b.build()
    cam = fsamd.camera((0, 10, -34), (0, 10, 0), fov_y=40, aperture=0.0)
    W, H, spp = 96, 64, 8
    host, _ = render_planes(gpu_renderer, d, cam, W, H, spp, gpu_bvh=False)
    dev, ds = render_planes(gpu_renderer, d, cam, W, H, spp, gpu_bvh=True)
    assert_same(dev, host)
    assert_oracle(dev, d, cam, W, H, spp)
    assert ds["build_ms"] > 0


def test_upload_flags_validated(gpu_renderer):
    b = DescBuilder()
    white = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.73, 0.73, 0.73))
    light = b.material(fsamd.MAT_LIGHT, emissive=(15, 15, 15))
    cornell_room(b, white, white, light)
    d = b.build()
    lib = fsamd.gpu_lib()
    assert lib.fs_upload_scene_ex(gpu_renderer.ctx, d, 0x80) == -1  # FS_ERR_INVALID


@pytest.mark.parametrize("name,min_tris", [("c4", None), ("c3", 1024)])
def test_device_bvh_build_is_deterministic(name, min_tris, scene_dir, gpu_renderer):
    """The device BVH build partitions by scanned ranks (ties of the median
    split in position order) and numbers nodes by scans over the tasks, not by
    atomic arrival: uploading the same scene three times gives byte-identical
    device arrays (fs_scene_digest) and the same node count."""
    if min_tris:
        gpu_renderer.set_options(gpu_bvh_min_tris=min_tris)
    s = load_scene(name, scene_dir)
    seen = set()
    for _ in range(3):
        gpu_renderer.upload(s, gpu_bvh=True)
        seen.add((gpu_renderer.scene_digest(), gpu_renderer.scene_stats()["nodes"]))
    assert len(seen) == 1, seen
    gpu_renderer.upload(s, gpu_bvh=False)  # the host build is deterministic too, and a different layout
    host = (gpu_renderer.scene_digest(), gpu_renderer.scene_stats()["nodes"])
    gpu_renderer.upload(s, gpu_bvh=False)
    assert (gpu_renderer.scene_digest(), gpu_renderer.scene_stats()["nodes"]) == host
