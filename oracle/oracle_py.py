"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of liboracle.so, the plain-C restatement of the reference path
tracer (fs_oracle.h). Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, and only as the checker / timed CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        F = C.POINTER(C.c_float)
        L.oracle_scene_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        L.oracle_scene_destroy.argtypes = [C.c_void_p]
        L.oracle_scene_destroy.restype = None
        L.oracle_mesh_info.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32),
                                       C.POINTER(C.c_uint64), F]
        L.oracle_mesh_vertex.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, F]
        L.oracle_mesh_face_plane.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, F]
        L.oracle_render.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
        L.oracle_trace_sample.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_uint32, C.c_uint32, C.c_uint64, F, F, F,
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        L.oracle_trace_range.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_float, C.c_float, F]
        L.oracle_splitmix64.restype = C.c_uint64
        L.oracle_splitmix64.argtypes = [C.c_uint64]
        L.oracle_pixel_seed.restype = C.c_uint64
        L.oracle_pixel_seed.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.oracle_random_integer.restype = C.c_uint64
        L.oracle_random_integer.argtypes = [C.POINTER(C.c_uint64)]
        L.oracle_random_float.restype = C.c_float
        L.oracle_random_float.argtypes = [C.POINTER(C.c_uint64)]
        L.oracle_random_integer_range.restype = C.c_int64
        L.oracle_random_integer_range.argtypes = [C.POINTER(C.c_uint64), C.c_int32, C.c_int32]
        L.oracle_random_float_range.restype = C.c_float
        L.oracle_random_float_range.argtypes = [C.POINTER(C.c_uint64), C.c_float, C.c_float]
        L.oracle_normal_table.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, F]
        L.oracle_normal_table.restype = None
        L.oracle_inv_sqrt.restype = C.c_float
        L.oracle_inv_sqrt.argtypes = [C.c_float]
        L.oracle_fast_sqrt.restype = C.c_float
        L.oracle_fast_sqrt.argtypes = [C.c_float]
        for n in ("oracle_normalize",):
            getattr(L, n).argtypes = [F, F]
            getattr(L, n).restype = None
        L.oracle_reflect.argtypes = [F, F, F]
        L.oracle_reflect.restype = None
        L.oracle_refract.argtypes = [F, F, C.c_float, F]
        L.oracle_refract.restype = None
        L.oracle_rotate.argtypes = [F, C.c_float, F, F]
        L.oracle_rotate.restype = None
        L.oracle_ray_sphere.argtypes = [F, C.c_float, F, F, F]
        L.oracle_ray_plane.argtypes = [F, F, F, F]
        L.oracle_ray_bounds.argtypes = [F, F, F, F, F]
        L.oracle_ray_triangle.argtypes = [F, F, F, F, F, F]
        L.oracle_triangle_box.argtypes = [F, F, F, F, F]
        _lib = L
    return _lib


def fptr(a):
    a = np.ascontiguousarray(a, np.float32)
    return a, a.ctypes.data_as(C.POINTER(C.c_float))


class OracleFrame(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("color", C.c_void_p),
                ("count", C.c_void_p), ("display", C.c_void_p), ("normal", C.c_void_p),
                ("depth", C.c_void_p), ("material", C.c_void_p)]


class OracleStats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64)]


class Frame:
    """Host DisplayFrame of the oracle (numpy planes, row 0 = bottom)."""

    def __init__(self, width, height):
        self.width, self.height = width, height
        self.color = np.zeros((height, width, 3), np.float32)
        self.count = np.zeros((height, width), np.uint32)
        self.display = np.zeros((height, width, 3), np.uint8)
        self.normal = np.zeros((height, width, 3), np.float32)
        self.depth = np.zeros((height, width), np.float32)
        self.material = np.zeros((height, width), np.uint64)

    def c(self):
        return OracleFrame(self.width, self.height, self.color.ctypes.data, self.count.ctypes.data,
                           self.display.ctypes.data, self.normal.ctypes.data, self.depth.ctypes.data,
                           self.material.ctypes.data)


class Scene:
    def __init__(self, desc_ptr):
        h = C.c_void_p()
        rc = lib().oracle_scene_create(desc_ptr, C.byref(h))
        if rc:
            raise RuntimeError(f"oracle_scene_create failed ({rc})")
        self.h = h
        self._keep = desc_ptr

    def render(self, cam, params, frame=None, threads=1):
        if frame is None:
            frame = Frame(params.width, params.height)
        fc = frame.c()
        st = OracleStats()
        rc = lib().oracle_render(self.h, C.byref(cam), C.byref(params), threads, C.byref(fc), C.byref(st))
        if rc:
            raise RuntimeError(f"oracle_render failed ({rc})")
        frame.stats = {k: getattr(st, k) for k, _ in OracleStats._fields_}
        return frame

    def trace_sample(self, cam, width, height, x, y, sample, seed=0):
        col = (C.c_float * 3)()
        nrm = (C.c_float * 3)()
        dep = C.c_float()
        mid = C.c_uint64()
        rc_ = C.c_uint32()
        lib().oracle_trace_sample(self.h, C.byref(cam), width, height, x, y, sample, seed, col, nrm,
                                  C.byref(dep), C.byref(mid), C.byref(rc_))
        return np.array(col[:], np.float32), np.array(nrm[:], np.float32), dep.value, mid.value, rc_.value

    def trace_range(self, cam, width, height, xy):
        out = []
        for x, y in np.asarray(xy, np.float32).reshape(-1, 2):
            d = C.c_float()
            rc = lib().oracle_trace_range(self.h, C.byref(cam), width, height, C.c_float(x), C.c_float(y), C.byref(d))
            if rc:
                raise RuntimeError(f"oracle_trace_range failed ({rc})")
            out.append(d.value)
        return np.array(out, np.float32)

    def mesh_info(self, m):
        n = C.c_uint32()
        r = C.c_uint64()
        rb = (C.c_float * 6)()
        lib().oracle_mesh_info(self.h, m, C.byref(n), C.byref(r), rb)
        return n.value, r.value, np.array(rb[:], np.float32)

    def close(self):
        if self.h:
            lib().oracle_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
