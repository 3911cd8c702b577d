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
    assert lib.fs_abi_version() == 1
    assert lib.fs_upload_scene(None, None) == -1  # FS_ERR_INVALID
    assert b"null" in lib.fs_last_error()
    assert lib.fs_render(None, None, None, None) == -1
    assert lib.fs_frame_read(None, 0, None, 0) == -1
    assert lib.fs_destroy(None) == 0


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
