"""The oracle (CPU restatement of the reference) against the reference's own
recorded outputs (SURVEY.md probes) and the committed golden fixtures."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_py
from conftest import GOLDEN, load_scene

L = oracle_py.lib
F3 = C.c_float * 3


def probes():
    return json.load(open(os.path.join(GOLDEN, "reference_probes.json")))


def test_xorshift_matches_reference_probe():
    s = C.c_uint64(521288629)
    got = [L().oracle_random_integer(C.byref(s)) for _ in range(3)]
    assert [str(v) for v in got] == probes()["xorshift64star_from_521288629"]


def test_random_float_matches_reference_probe():
    s = C.c_uint64(521288629)
    vals = [L().oracle_random_float(C.byref(s)) for _ in range(4)]
    assert np.float32(vals[3]) == np.float32(probes()["random_float_4th_draw"])
    # (float)(r % 0x7FFFFFFF) / 2^31 can reach 1.0 but never exceeds it
    assert all(0.0 <= v <= 1.0 for v in vals)


def test_fast_length_matches_reference_probe():
    # vector3::length() = 1 / inv_sqrt(d) with one Newton step (scalar.h:233-245)
    assert np.float32(L().oracle_fast_sqrt(4.0)) == np.float32(probes()["length_0_0_2"])
    out = (C.c_float * 3)()
    L().oracle_normalize(F3(0, 0, 2), out)
    assert out[2] == np.float32(np.float32(2.0) / np.float32(probes()["length_0_0_2"]))


def test_sphere_known_answer_matches_reference_probe():
    p = probes()["sphere_unit_segment_z"]
    out = (C.c_float * 7)()
    hit = L().oracle_ray_sphere(F3(*p["center"]), p["radius"], F3(*p["start"]), F3(*p["stop"]), out)
    assert hit == 1
    assert np.float32(out[0]) == np.float32(p["param"])
    assert np.float32(out[3]) == np.float32(p["point_z"])


def test_inside_sphere_takes_far_root():
    out = (C.c_float * 7)()
    assert L().oracle_ray_sphere(F3(0, 0, 0), 1.0, F3(0, 0, 0), F3(0, 0, 10), out) == 1
    assert 0.09 < out[0] < 0.11 and out[3] > 0.99


def test_zero_length_ray_never_reports_sphere_hit_info():
    out = (C.c_float * 7)()
    # intersect.cpp:424-426: returns inside/outside without filling hit info
    assert L().oracle_ray_sphere(F3(0, 0, 0), 1.0, F3(0, 0, 0.5), F3(0, 0, 0.5), out) == 1
    assert out[0] == np.float32(2.0)


def test_plane_is_two_sided_and_segment_bounded():
    out = (C.c_float * 7)()
    pl = (C.c_float * 4)(0, 1, 0, -5)  # y = 5
    assert L().oracle_ray_plane(pl, F3(0, 0, 0), F3(0, 10, 0), out) == 1
    assert out[0] == np.float32(0.5) and out[2] == np.float32(5.0)
    assert L().oracle_ray_plane(pl, F3(0, 10, 0), F3(0, 0, 0), out) == 1  # from the back side
    assert L().oracle_ray_plane(pl, F3(0, 0, 0), F3(0, 4, 0), out) == 0  # t > 1
    assert L().oracle_ray_plane(pl, F3(0, 0, 0), F3(10, 0, 0), out) == 0  # parallel


def test_triangle_hits_and_edges():
    out = (C.c_float * 9)()
    p1, p2, p3 = F3(0, 0, 0), F3(1, 0, 0), F3(0, 1, 0)
    assert L().oracle_ray_triangle(p1, p2, p3, F3(0.25, 0.25, -1), F3(0.25, 0.25, 1), out) == 1
    assert out[0] == np.float32(0.5)
    assert L().oracle_ray_triangle(p1, p2, p3, F3(0.75, 0.75, -1), F3(0.75, 0.75, 1), out) == 0
    # zero-length ray: point test uses n.p + 2w (intersect.cpp:45-47); plane through origin
    assert L().oracle_ray_triangle(p1, p2, p3, F3(0.2, 0.2, 0.0), F3(0.2, 0.2, 0.0), out) == 1
    assert out[0] == 0.0


def test_bounds_start_inside_returns_exit_param():
    out = (C.c_float * 4)()
    assert L().oracle_ray_bounds(F3(-1, -1, -1), F3(1, 1, 1), F3(0, 0, 0), F3(0, 0, 4), out) == 1
    assert out[0] == np.float32(0.25)  # exit param: 1 - t of the reversed segment (intersect.cpp:635-649)
    assert L().oracle_ray_bounds(F3(-1, -1, -1), F3(1, 1, 1), F3(0, 0, -4), F3(0, 0, 4), out) == 1
    assert out[0] == np.float32(0.375)
    assert L().oracle_ray_bounds(F3(-1, -1, -1), F3(1, 1, 1), F3(3, 0, -4), F3(3, 0, 4), out) == 0


def test_refract_total_internal_reflection_is_zero():
    out = (C.c_float * 3)()
    L().oracle_refract(F3(0.9, -0.1, 0), F3(0, 1, 0), 1.5, out)
    assert list(out) == [0.0, 0.0, 0.0]


def test_triangle_box_sat():
    assert L().oracle_triangle_box(F3(0, 0, 0), F3(1, 0, 0), F3(0, 1, 0), F3(-1, -1, -1), F3(2, 2, 2)) == 1
    assert L().oracle_triangle_box(F3(0, 0, 0), F3(1, 0, 0), F3(0, 1, 0), F3(5, 5, 5), F3(6, 6, 6)) == 0


def test_rng_golden():
    g = json.load(open(os.path.join(GOLDEN, "rng.json")))
    s = C.c_uint64(g["seed"])
    assert [str(L().oracle_random_integer(C.byref(s))) for _ in range(64)] == g["random_integer"]
    s = C.c_uint64(g["seed"])
    assert [float(np.float32(L().oracle_random_float(C.byref(s)))) for _ in range(16)] == g["random_float"]
    s = C.c_uint64(g["seed"])
    assert [L().oracle_random_integer_range(C.byref(s), 0, 32767) for _ in range(16)] == \
        g["random_integer_range_0_32767"]


@pytest.mark.parametrize("pre", [1, 5, 8])
def test_normal_table_golden(pre):
    g = json.load(open(os.path.join(GOLDEN, "normal_table.json")))[str(pre)]
    t = np.zeros((32768, 3), np.float32)
    L().oracle_normal_table(521288629, pre, 32768, oracle_py.fptr(t)[1])
    assert hashlib.sha256(t.tobytes()).hexdigest() == g["sha256"]
    # rejection sampling + fast-sqrt normalise: lengths within the 1-step Newton error
    n = np.linalg.norm(t.astype(np.float64), axis=1)
    assert np.all(np.abs(n - 1.0) < 2e-3)


@pytest.mark.parametrize("name,dims", [("c1", (32, 32, 8)), ("c2", (48, 32, 8))])
def test_oracle_image_golden(name, dims, scene_dir):
    import fsamd

    W, H, spp = dims
    g = np.load(os.path.join(GOLDEN, f"{name}_{W}x{H}x{spp}.npz"))
    s = load_scene(name, scene_dir)
    o = oracle_py.Scene(s.desc_ptr())
    f = o.render(s.camera(0), fsamd.render_params(W, H, spp), threads=4)
    for plane in ("color", "count", "display", "normal", "depth", "material"):
        np.testing.assert_array_equal(getattr(f, plane), g[plane], err_msg=plane)


def test_oracle_threading_is_deterministic(scene_dir):
    import fsamd

    s = load_scene("c2", scene_dir)
    o = oracle_py.Scene(s.desc_ptr())
    p = fsamd.render_params(40, 24, 4)
    a = o.render(s.camera(0), p, threads=1)
    b = o.render(s.camera(0), p, threads=7)
    np.testing.assert_array_equal(a.color, b.color)
