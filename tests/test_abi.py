"""The C-ABI library loads and exports every symbol include/fs_trace.h
declares; argument validation works without a GPU. No compute calls."""
import ctypes as C
import os
import re

import pytest

import fsamd
from conftest import ROOT


def declared_functions():
    text = open(os.path.join(ROOT, "include", "fs_trace.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(fs_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("fs_create", "fs_upload_scene", "fs_render", "fs_frame_read", "fs_frame_gather", "fs_last_error"):
        assert must in names
    assert len(names) >= 20


def test_every_declared_symbol_is_exported_and_bound():
    lib = fsamd.gpu_lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in fsamd.GPU_SYMBOLS, f"{name} missing from the Python binding"


def test_abi_version_and_errors_without_device():
    lib = fsamd.gpu_lib()
    assert lib.fs_abi_version() == 9
    assert lib.fs_upload_scene(None, None) == -1  # FS_ERR_INVALID
    assert b"null" in lib.fs_last_error()
    assert lib.fs_render(None, None, None, None) == -1
    assert lib.fs_frame_read(None, 0, None, 0) == -1
    assert lib.fs_destroy(None) == 0


def test_options_defaults_and_validation_without_device():
    """fs_options: the documented defaults; invalid settings are refused
    (checked by fs_prepare_digest, which needs no device)."""
    o = fsamd.options()
    d = fsamd.options_dict(o)
    assert d == {"schedule": 0, "park_lanes": 12, "park_min_tris": 1 << 15, "samples_per_block": 16, "groups": 0,
                 "group_major": 0, "tile_order": 1, "xcd_bands": 2, "gpu_bvh_min_tris": 1 << 16, "bvh_leaf": 2,
                 "bvh_bins": 16, "bvh_threads": 0, "node_layout": 0, "build_log": 0, "persist": 1,
                 "small_mesh_tris": 16, "park_lanes_small": 6,
                 "lds_rows": 1, "record_budget_mb": 0, "lookahead": 24}
    assert fsamd.parse_variant("schedule=parked@park_lanes=8") == {"schedule": "parked", "park_lanes": 8}
    assert fsamd.options(schedule="parked").schedule == 2
    lib = fsamd.gpu_lib()
    assert lib.fs_options_default(None) == -1
    assert lib.fs_set_options(None, C.byref(o)) == -1
    d, n = C.c_uint64(), C.c_uint64()
    for bad in ({"bvh_leaf": 0}, {"bvh_leaf": 16}, {"bvh_bins": 65}, {"samples_per_block": 65}, {"schedule": 3}, {"xcd_bands": 3},
                {"persist": 2}, {"small_mesh_tris": 65}, {"park_lanes": 65}, {"lds_rows": 2},
                {"lookahead": 49}):
        ob = fsamd.options(**bad)
        assert lib.fs_prepare_digest(C.c_void_p(1), C.byref(ob), C.byref(d), C.byref(n), None) == -1, bad
    with pytest.raises(fsamd.FsError):
        fsamd.options(no_such_field=1)


def _plan(width, height, spp, budget=0, rec=88, **opt):
    lib = fsamd.gpu_lib()
    p = fsamd.render_params(width, height, spp)
    out = fsamd.fs_render_plan()
    o = fsamd.options(**opt)
    rc = lib.fs_plan_render(C.byref(p), C.byref(o), budget, rec, C.byref(out))
    if rc:
        raise fsamd.FsError(lib.fs_last_error().decode())
    return out


def test_launch_plan_of_the_bench_frame_without_device():
    """C4 at 1080p x 1024 spp under the default 96 GiB budget: one tile part,
    two launches of 32 groups of 16 samples."""
    p = _plan(1920, 1080, 1024)
    assert (p.parts, p.tiles_per_part, p.samples_per_block, p.groups_per_launch, p.launches) == (1, 510, 16, 32, 2)
    assert p.record_bytes_per_launch <= 96 << 30


@pytest.mark.parametrize("w,h,spp,rec,spb", [(16384, 16384, 16, 88, 16), (8192, 8192, 64, 88, 64),
                                             (16384, 16384, 1024, 216, 16), (65536, 32768, 3, 88, 16)])
def test_launch_plan_splits_frames_larger_than_the_budget(w, h, spp, rec, spb):
    """a frame whose one-group launch exceeds the record budget
    renders in tile parts (and, below one tile per part, fewer samples per
    block) instead of failing with FS_ERR_NOMEM; every launch fits."""
    budget = 96 << 30
    p = _plan(w, h, spp, budget, rec, samples_per_block=spb)
    tiles = ((w + 63) // 64) * ((h + 63) // 64)
    assert p.parts > 1 and p.parts * p.tiles_per_part >= tiles > (p.parts - 1) * p.tiles_per_part
    assert p.record_bytes_per_launch <= budget
    assert p.tiles_per_part * 64 * 64 * p.samples_per_block * rec == p.record_bytes_per_launch // p.groups_per_launch


def test_launch_plan_small_budget_without_device():
    """record_budget_mb shrinks launches down to one tile x one sample; below
    that the plan fails with FS_ERR_NOMEM and says why."""
    p = _plan(256, 200, 20, 0, 88, record_budget_mb=1)  # 1 MiB: one 64x64 tile holds 360 KB per sample
    assert (p.tiles_per_part, p.samples_per_block, p.groups_per_launch) == (1, 2, 1)
    assert p.parts == 16 and p.launches == 16 * 10
    p = _plan(256, 200, 20, 0, 88, record_budget_mb=128)
    assert p.parts == 1 and p.samples_per_block == 16
    with pytest.raises(fsamd.FsError, match="below one tile"):
        _plan(256, 200, 20, 100000, 88)


def test_launch_plan_of_fewer_samples_than_a_block_without_device():
    """a 1-spp launch (the drop-in loop's TraceScene) sizes its
    path records to the samples it holds, not to samples_per_block (16)."""
    p = _plan(1920, 1080, 1)
    assert (p.parts, p.samples_per_block, p.groups_per_launch, p.launches) == (1, 1, 1, 1)
    assert p.record_bytes_per_launch == 510 * 64 * 64 * 1 * 88
    p = _plan(1920, 1080, 3)
    assert (p.samples_per_block, p.launches) == (3, 1)
    assert _plan(1920, 1080, 40).samples_per_block == 16


def test_deep_mesh_bvh_fits_the_walk_stack_without_device():
    """the node step writes the walk stack at sp on every trip,
    in bounds because the host builder stops splitting at depth
    kTraversalStack - 1 = 23. A mesh of 200 triangles on a geometric
    progression (every SAH split peels off one face) would build a tree of
    depth ~200 without the guard."""
    import json

    import descbuild

    b = descbuild.DescBuilder()
    m = b.material(fsamd.MAT_DIFFUSE, diffuse=(0.5, 0.5, 0.5))
    pos, faces = [], []
    for i in range(200):
        x = 1.5 ** i
        pos += [[x, 0, 0], [x * 1.01, 1, 0], [x * 1.02, 0, 1]]
        faces.append([3 * i, 3 * i + 1, 3 * i + 2])
    b.mesh(m, pos, faces)
    desc = b.build()
    buf = C.create_string_buffer(1 << 16)
    lib = fsamd.gpu_lib()
    o = fsamd.options()
    assert lib.fs_bvh_quality(desc, C.byref(o), buf, len(buf)) == 0, lib.fs_last_error()
    q = json.loads(buf.value.decode())
    assert len(q) == 1 and q[0]["faces"] == 200
    assert 15 < q[0]["depth"] <= 23  # deep, and within the 24-entry stack


def test_create_fails_cleanly_without_a_gpu():
    if fsamd.device_count() > 0:
        pytest.skip("a HIP device is present")
    h = C.c_void_p()
    rc = fsamd.gpu_lib().fs_create(0, C.byref(h))
    assert rc == -2 and not h.value  # FS_ERR_DEVICE
    assert b"device" in fsamd.gpu_lib().fs_last_error()


def test_host_library_exports():
    lib = fsamd.host_lib()
    for name in fsamd.HOST_SYMBOLS:
        assert hasattr(lib, name)
