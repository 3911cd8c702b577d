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
    assert lib.fs_abi_version() == 7
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
                 "lds_rows": 1}
    assert fsamd.parse_variant("schedule=parked@park_lanes=8") == {"schedule": "parked", "park_lanes": 8}
    assert fsamd.options(schedule="parked").schedule == 2
    lib = fsamd.gpu_lib()
    assert lib.fs_options_default(None) == -1
    assert lib.fs_set_options(None, C.byref(o)) == -1
    d, n = C.c_uint64(), C.c_uint64()
    for bad in ({"bvh_leaf": 0}, {"bvh_leaf": 16}, {"bvh_bins": 65}, {"samples_per_block": 65}, {"schedule": 3}, {"xcd_bands": 3},
                {"persist": 2}, {"small_mesh_tris": 65}, {"park_lanes": 65}, {"lds_rows": 2}):
        ob = fsamd.options(**bad)
        assert lib.fs_prepare_digest(C.c_void_p(1), C.byref(ob), C.byref(d), C.byref(n), None) == -1, bad
    with pytest.raises(fsamd.FsError):
        fsamd.options(no_such_field=1)


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
