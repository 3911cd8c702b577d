"""ctypes binding of the MI355X path-trace layer (include/fs_trace.h) and of
the C++ reference-API mirror (host/fs_host.h).

The product path is libfsgpu.so; this module refuses to run without it (no
CPU fallback). Typical use::

    import fsamd
    scene = fsamd.HostScene.load("c2.scene")      # Scene::LoadScene
    fsamd.initialize_materials()                   # InitializeMaterials()
    r = fsamd.Renderer(device=0)
    r.upload(scene)
    frame = r.frame(1920, 1080)
    r.render(scene.camera(0), frame, spp=1024)
    rgb = frame.read(fsamd.PLANE_COLOR)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))

FS_NORMAL_TABLE_SIZE = 32768
PLANE_COLOR, PLANE_COUNT, PLANE_DISPLAY, PLANE_NORMAL, PLANE_DEPTH, PLANE_MATERIAL = range(6)
RENDER_COUNTERS = 1

(MAT_DIFFUSE, MAT_LIGHT, MAT_METAL, MAT_MIRROR, MAT_GLASS, MAT_LIQUID, MAT_CERAMIC, MAT_GLOW,
 MAT_FOG) = range(9)
(OBJ_SPHERE, OBJ_PLANE, OBJ_DISC, OBJ_CUBOID, OBJ_QUAD_ONWH, OBJ_QUAD_PUV, OBJ_MESH) = range(7)


class FsError(RuntimeError):
    pass


# ---- struct mirrors of fs_trace.h -----------------------------------------
class fs_material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("id", C.c_uint32), ("diffuse", C.c_float * 3),
                ("emissive", C.c_float * 3), ("glow", C.c_float * 3), ("roughness", C.c_float),
                ("shininess", C.c_float), ("index", C.c_float), ("reflectivity", C.c_float),
                ("frost", C.c_float), ("density", C.c_float), ("texture", C.c_int32),
                ("texture_scale", C.c_float)]


class fs_object(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("mesh", C.c_int32),
                ("rotate", C.c_int32), ("a", C.c_float * 12)]


class fs_mesh(C.Structure):
    _fields_ = [("positions", C.POINTER(C.c_float)), ("num_positions", C.c_uint32),
                ("normals", C.POINTER(C.c_float)), ("num_normals", C.c_uint32),
                ("texcoords", C.POINTER(C.c_float)), ("num_texcoords", C.c_uint32),
                ("corners", C.POINTER(C.c_int32)), ("num_triangles", C.c_uint32),
                ("invert_normals", C.c_int32), ("translation", C.c_float * 3),
                ("scale", C.c_float * 3), ("rotation", C.c_float * 4)]


class fs_texture(C.Structure):
    _fields_ = [("rgb", C.POINTER(C.c_float)), ("width", C.c_uint32), ("height", C.c_uint32)]


class fs_scene_desc(C.Structure):
    _fields_ = [("materials", C.POINTER(fs_material)), ("num_materials", C.c_uint32),
                ("sky_material", C.c_int32), ("objects", C.POINTER(fs_object)),
                ("num_objects", C.c_uint32), ("meshes", C.POINTER(fs_mesh)),
                ("num_meshes", C.c_uint32), ("textures", C.POINTER(fs_texture)),
                ("num_textures", C.c_uint32), ("normal_table", C.POINTER(C.c_float)), ("flags", C.c_uint32)]


SCENE_OPTIMIZED = 1  # FS_SCENE_OPTIMIZED


class fs_camera(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("target", C.c_float * 3), ("fov_y", C.c_float),
                ("aperture_size", C.c_float), ("focal_depth", C.c_float), ("z_near", C.c_float),
                ("z_far", C.c_float), ("fast_render", C.c_int32)]


class fs_render_params(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32),
                ("sample_base", C.c_uint32), ("seed", C.c_uint64), ("tile_size", C.c_uint32),
                ("tile_offset", C.c_uint32), ("tile_stride", C.c_uint32), ("flags", C.c_uint32)]


class fs_counters(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("prim_tests", C.c_uint64), ("object_loads", C.c_uint64),
                ("small_tri_loads", C.c_uint64), ("lane_object_loads", C.c_uint64)]


class fs_options(C.Structure):
    _fields_ = [("schedule", C.c_int32), ("park_lanes", C.c_uint32), ("park_min_tris", C.c_uint32),
                ("samples_per_block", C.c_uint32), ("groups", C.c_uint32), ("group_major", C.c_uint32),
                ("tile_order", C.c_uint32), ("xcd_bands", C.c_uint32), ("gpu_bvh_min_tris", C.c_uint32),
                ("bvh_leaf", C.c_uint32), ("bvh_bins", C.c_uint32), ("bvh_threads", C.c_uint32),
                ("node_layout", C.c_uint32), ("build_log", C.c_uint32),
                ("persist", C.c_uint32), ("small_mesh_tris", C.c_uint32), ("park_lanes_small", C.c_uint32),
                ("lds_rows", C.c_uint32), ("record_budget_mb", C.c_uint32), ("lookahead", C.c_uint32)]


class fs_render_plan(C.Structure):
    _fields_ = [("parts", C.c_uint32), ("tiles_per_part", C.c_uint32), ("samples_per_block", C.c_uint32),
                ("groups_per_launch", C.c_uint32), ("launches", C.c_uint32),
                ("record_bytes_per_launch", C.c_uint64)]


UPLOAD_GPU_BVH = 1  # FS_UPLOAD_GPU_BVH
SCHEDULES = {"auto": 0, "lean": 1, "parked": 2}  # fs_schedule
NODE_LAYOUTS = {"depth_first": 0, "pairs": 1}

# Exported symbols of include/fs_trace.h, with their ctypes signatures.
_VP = C.c_void_p
GPU_SYMBOLS = {
    "fs_abi_version": ([], C.c_int),
    "fs_last_error": ([], C.c_char_p),
    "fs_device_count": ([C.POINTER(C.c_int)], C.c_int),
    "fs_create": ([C.c_int, C.POINTER(_VP)], C.c_int),
    "fs_destroy": ([_VP], C.c_int),
    "fs_options_default": ([C.POINTER(fs_options)], C.c_int),
    "fs_set_options": ([_VP, C.POINTER(fs_options)], C.c_int),
    "fs_get_options": ([_VP, C.POINTER(fs_options)], C.c_int),
    "fs_upload_scene": ([_VP, _VP], C.c_int),
    "fs_upload_scene_ex": ([_VP, _VP, C.c_uint32], C.c_int),
    "fs_scene_stats": ([_VP, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)], C.c_int),
    "fs_frame_create": ([_VP, C.c_uint32, C.c_uint32, C.POINTER(_VP)], C.c_int),
    "fs_frame_destroy": ([_VP], C.c_int),
    "fs_frame_reset": ([_VP], C.c_int),
    "fs_frame_read": ([_VP, C.c_int, _VP, C.c_size_t], C.c_int),
    "fs_frame_write": ([_VP, C.c_int, _VP, C.c_size_t], C.c_int),
    "fs_frame_map": ([_VP, C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "fs_last_render_lookahead": ([_VP, C.POINTER(C.c_int)], C.c_int),
    "fs_render": ([_VP, C.POINTER(fs_camera), C.POINTER(fs_render_params), _VP], C.c_int),
    "fs_synchronize": ([_VP], C.c_int),
    "fs_read_counters": ([_VP, C.POINTER(fs_counters)], C.c_int),
    "fs_last_render_ms": ([_VP, C.POINTER(C.c_float)], C.c_int),
    "fs_last_trace_ms": ([_VP, C.POINTER(C.c_float)], C.c_int),
    "fs_last_kernel": ([_VP], C.c_char_p),
    "fs_last_render_launches": ([_VP, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)], C.c_int),
    "fs_plan_render": ([C.POINTER(fs_render_params), C.POINTER(fs_options), C.c_uint64, C.c_uint32,
                        C.POINTER(fs_render_plan)], C.c_int),
    "fs_comm_unique_id": ([C.c_char_p], C.c_int),
    "fs_comm_init": ([_VP, C.c_int, C.c_int, C.c_char_p], C.c_int),
    "fs_frame_gather": ([_VP, _VP, C.POINTER(fs_render_params), C.c_int], C.c_int),
    "fs_comm_count": ([_VP, C.POINTER(C.c_int)], C.c_int),
    "fs_bvh_quality": ([_VP, C.POINTER(fs_options), C.c_char_p, C.c_size_t], C.c_int),
    "fs_comm_destroy": ([_VP], C.c_int),
    "fs_frame_pack_bytes": ([C.POINTER(fs_render_params), C.POINTER(C.c_uint64)], C.c_int),
    "fs_frame_pack": ([_VP, _VP, C.POINTER(fs_render_params), _VP, C.c_size_t], C.c_int),
    "fs_frame_unpack": ([_VP, _VP, C.POINTER(fs_render_params), _VP, C.c_size_t], C.c_int),
    "fs_prepare_digest": ([_VP, C.POINTER(fs_options), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                           C.POINTER(C.c_double)], C.c_int),
    "fs_scene_digest": ([_VP, C.POINTER(C.c_uint64)], C.c_int),
    "fs_trace_range": ([_VP, C.POINTER(fs_camera), C.c_uint32, C.c_uint32, _VP, C.c_uint32, _VP], C.c_int),
}
HOST_SYMBOLS = {
    "fsh_last_error": ([], C.c_char_p),
    "fsh_scene_new": ([], _VP),
    "fsh_scene_load": ([C.c_char_p], _VP),
    "fsh_scene_free": ([_VP], None),
    "fsh_scene_describe": ([_VP], C.POINTER(fs_scene_desc)),
    "fsh_scene_camera_count": ([_VP], C.c_int),
    "fsh_scene_camera": ([_VP, C.c_uint32, C.POINTER(fs_camera)], C.c_int),
    "fsh_set_seed": ([C.c_uint64], None),
    "fsh_random_integer": ([], C.c_uint64),
    "fsh_random_float": ([], C.c_float),
    "fsh_initialize_materials": ([], None),
    "fsh_normal_table": ([_VP], C.c_int),
    "fsh_obj_load": ([C.c_char_p], _VP),
    "fsh_obj_info": ([_VP] + [C.POINTER(C.c_uint32)] * 4, C.c_int),
    "fsh_obj_copy": ([_VP, _VP, _VP], C.c_int),
    "fsh_obj_free": ([_VP], None),
    "fsh_load_bitmap": ([C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_uint32),
                         C.POINTER(C.c_uint32), C.POINTER(C.c_size_t)], C.c_int),
    "fsh_load_exr": ([C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_int), C.POINTER(C.c_int)],
                     C.c_int),
    "fsh_free": ([_VP], None),
}

_gpu = None
_host = None


# Entry points added after ABI 4. A measurement build of an earlier round
# (tools/lib_ab.sh A/B against an older libfsgpu.so, selected by
# FSAMD_GPU_LIB) may lack them; the product library always has them.
_OPTIONAL = {"fs_comm_count", "fs_bvh_quality", "fs_plan_render", "fs_frame_map", "fs_last_render_lookahead"}


def _bind(lib, table):
    for name, (args, res) in table.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if name in _OPTIONAL and os.environ.get("FSAMD_GPU_LIB"):
                continue
            raise
        fn.argtypes = args
        fn.restype = res
    return lib


def gpu_lib_path():
    """The libfsgpu.so this process loads: the in-tree product build, or the
    measurement build FSAMD_GPU_LIB names (libfsgpu_prof.so, A/B builds)."""
    return os.environ.get("FSAMD_GPU_LIB") or os.path.join(PKG_DIR, "libfsgpu.so")


def gpu_lib():
    """libfsgpu.so (HIP kernels + C ABI). Raises if it has not been built."""
    global _gpu
    if _gpu is None:
        path = gpu_lib_path()
        if not os.path.exists(path):
            raise FsError(f"{path} missing: run `make -C {PKG_DIR}` (or __graft_entry__.build())")
        _gpu = _bind(C.CDLL(path, mode=C.RTLD_GLOBAL), GPU_SYMBOLS)
    return _gpu


def host_lib():
    global _host
    if _host is None:
        gpu_lib()
        path = os.path.join(PKG_DIR, "libfshost.so")
        if not os.path.exists(path):
            raise FsError(f"{path} missing: run `make -C {PKG_DIR}`")
        _host = _bind(C.CDLL(path, mode=C.RTLD_GLOBAL), HOST_SYMBOLS)
    return _host


def _check(rc, what):
    if rc != 0:
        msg = gpu_lib().fs_last_error().decode(errors="replace")
        raise FsError(f"{what} failed ({rc}): {msg}")


def device_count():
    n = C.c_int(0)
    _check(gpu_lib().fs_device_count(C.byref(n)), "fs_device_count")
    return n.value


# ---- reference-API mirror (host/fs_host.h) ---------------------------------
def set_seed(seed):
    host_lib().fsh_set_seed(seed)


def random_integer():
    return host_lib().fsh_random_integer()


def random_float():
    return host_lib().fsh_random_float()


def reset_main_rng():
    """Main-thread stream back to its static initialiser (random.cpp:6)."""
    set_seed(521288629)


def initialize_materials():
    host_lib().fsh_initialize_materials()


def normal_table():
    out = np.zeros((FS_NORMAL_TABLE_SIZE, 3), np.float32)
    rc = host_lib().fsh_normal_table(out.ctypes.data)
    if rc:
        raise FsError("InitializeMaterials() has not run")
    return out


def camera(origin, target, fov_y=45.0, aperture=1.5, focal_depth=80.0, z_near=1.0, z_far=10000.0,
           fast_render=False):
    """Camera (camera.h:43-63) with the reference defaults (camera.cpp:6-24)."""
    c = fs_camera()
    c.origin[:] = origin
    c.target[:] = target
    c.fov_y, c.aperture_size, c.focal_depth = fov_y, aperture, focal_depth
    c.z_near, c.z_far, c.fast_render = z_near, z_far, int(fast_render)
    return c


class HostScene:
    """base::Scene built by the C++ loader (Scene::LoadScene)."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def load(cls, path):
        h = host_lib().fsh_scene_load(os.fsencode(path))
        if not h:
            raise FsError(f"LoadScene({path}): {host_lib().fsh_last_error().decode()}")
        return cls(h)

    def desc(self):
        d = host_lib().fsh_scene_describe(self.h)
        if not d:
            raise FsError(f"scene describe: {host_lib().fsh_last_error().decode()}")
        return d

    def desc_ptr(self):
        return C.cast(self.desc(), C.c_void_p)

    def camera_count(self):
        return host_lib().fsh_scene_camera_count(self.h)

    def camera(self, i=0):
        c = fs_camera()
        if host_lib().fsh_scene_camera(self.h, i, C.byref(c)):
            raise FsError(f"scene has no camera {i}")
        return c

    def close(self):
        if self.h:
            host_lib().fsh_scene_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_obj(path):
    """Triangle arrays of an OBJ as the C++ loader reads them."""
    lib = host_lib()
    h = lib.fsh_obj_load(os.fsencode(path))
    if not h:
        raise FsError(lib.fsh_last_error().decode())
    n = [C.c_uint32() for _ in range(4)]
    lib.fsh_obj_info(h, *[C.byref(x) for x in n])
    pos = np.zeros((n[0].value, 3), np.float32)
    corners = np.zeros((n[3].value, 9), np.int32)
    lib.fsh_obj_copy(h, pos.ctypes.data, corners.ctypes.data)
    lib.fsh_obj_free(h)
    return pos, corners


# ---- the GPU layer ----------------------------------------------------------
_PLANE_DTYPE = {PLANE_COLOR: (np.float32, 3), PLANE_COUNT: (np.uint32, 1),
                PLANE_DISPLAY: (np.uint8, 3), PLANE_NORMAL: (np.float32, 3),
                PLANE_DEPTH: (np.float32, 1), PLANE_MATERIAL: (np.uint64, 1)}


def render_params(width, height, spp, sample_base=0, seed=0, tile_size=64, tile_offset=0,
                  tile_stride=1, counters=False):
    p = fs_render_params()
    p.width, p.height, p.spp, p.sample_base, p.seed = width, height, spp, sample_base, seed
    p.tile_size, p.tile_offset, p.tile_stride = tile_size, tile_offset, tile_stride
    p.flags = RENDER_COUNTERS if counters else 0
    return p


class Frame:
    """Device-resident DisplayFrame (frame.h:49-92); row 0 is the image bottom."""

    def __init__(self, renderer, width, height):
        self.r = renderer
        self.width, self.height = width, height
        h = C.c_void_p()
        _check(gpu_lib().fs_frame_create(renderer.ctx, width, height, C.byref(h)), "fs_frame_create")
        self.h = h

    def read(self, plane):
        dt, ch = _PLANE_DTYPE[plane]
        shape = (self.height, self.width, ch) if ch > 1 else (self.height, self.width)
        out = np.zeros(shape, dt)
        _check(gpu_lib().fs_frame_read(self.h, plane, out.ctypes.data, out.nbytes), "fs_frame_read")
        return out

    def map(self, plane):
        """fs_frame_map: the plane in the frame's page-locked host buffer (a copy
        of it is returned; the buffer is reused by the next map of the plane)."""
        dt, ch = _PLANE_DTYPE[plane]
        shape = (self.height, self.width, ch) if ch > 1 else (self.height, self.width)
        p = C.c_void_p()
        _check(gpu_lib().fs_frame_map(self.h, plane, C.byref(p)), "fs_frame_map")
        n = int(np.prod(shape)) * np.dtype(dt).itemsize
        return np.frombuffer(C.string_at(p.value, n), dt).reshape(shape).copy()

    def write(self, plane, array):
        dt, _ = _PLANE_DTYPE[plane]
        a = np.ascontiguousarray(array, dtype=dt)
        _check(gpu_lib().fs_frame_write(self.h, plane, a.ctypes.data, a.nbytes), "fs_frame_write")

    def reset(self):
        _check(gpu_lib().fs_frame_reset(self.h), "fs_frame_reset")

    def close(self):
        if self.h:
            gpu_lib().fs_frame_destroy(self.h)
            self.h = None


def options(**kw):
    """fs_options: the defaults (fs_options_default) with fields replaced by
    keyword; schedule and node_layout also take their names."""
    o = fs_options()
    _check(gpu_lib().fs_options_default(C.byref(o)), "fs_options_default")
    names = {k for k, _ in fs_options._fields_}
    for k, v in kw.items():
        if k not in names:
            raise FsError(f"unknown fs_options field {k!r}")
        if k == "schedule" and isinstance(v, str):
            v = SCHEDULES[v]
        if k == "node_layout" and isinstance(v, str):
            v = NODE_LAYOUTS[v]
        setattr(o, k, int(v))
    return o


def options_dict(o):
    return {k: getattr(o, k) for k, _ in fs_options._fields_}


def parse_variant(v):
    """'schedule=lean@park_lanes=8' -> {'schedule': 'lean', 'park_lanes': 8}
    (tools' A/B variant syntax; 'default' -> {})."""
    out = {}
    for kv in v.split("@"):
        if not kv or kv == "default":
            continue
        k, val = kv.split("=", 1)
        out[k] = val if k in ("schedule", "node_layout") else int(val)
    return out


class Renderer:
    """One fs_context (one GPU, one stream)."""

    def __init__(self, device=0, **opts):
        lib = gpu_lib()
        h = C.c_void_p()
        _check(lib.fs_create(device, C.byref(h)), "fs_create")
        self.ctx = h
        self._scene_ref = None
        if opts:
            self.set_options(**opts)

    def set_options(self, **kw):
        """fs_set_options with the given fields changed from the current ones."""
        o = self.get_options()
        for k, v in options_dict(options(**kw)).items():
            if k in kw:
                setattr(o, k, v)
        _check(gpu_lib().fs_set_options(self.ctx, C.byref(o)), "fs_set_options")

    def get_options(self):
        o = fs_options()
        _check(gpu_lib().fs_get_options(self.ctx, C.byref(o)), "fs_get_options")
        return o

    def upload(self, scene, gpu_bvh=False):
        """scene: HostScene, or a ctypes pointer/void* to an fs_scene_desc.
        gpu_bvh: build the BVH of large meshes on the device
        (fs_upload_scene_ex FS_UPLOAD_GPU_BVH) or on the host."""
        ptr = scene.desc_ptr() if isinstance(scene, HostScene) else scene
        flags = UPLOAD_GPU_BVH if gpu_bvh else 0
        _check(gpu_lib().fs_upload_scene_ex(self.ctx, ptr, flags), "fs_upload_scene_ex")
        self._scene_ref = scene

    def scene_stats(self):
        b, u = C.c_double(), C.c_double()
        t, n, m = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(gpu_lib().fs_scene_stats(self.ctx, C.byref(b), C.byref(u), C.byref(t), C.byref(n),
                                        C.byref(m)), "fs_scene_stats")
        return {"build_ms": b.value, "upload_ms": u.value, "triangles": t.value, "nodes": n.value,
                "device_bytes": m.value}

    def scene_digest(self):
        """fs_scene_digest: FNV-1a of every device array of the uploaded scene."""
        d = C.c_uint64()
        _check(gpu_lib().fs_scene_digest(self.ctx, C.byref(d)), "fs_scene_digest")
        return d.value

    def frame(self, width, height):
        return Frame(self, width, height)

    def render(self, cam, frame, spp=1, sample_base=0, seed=0, tile_size=64, tile_offset=0,
               tile_stride=1, counters=False, sync=True):
        p = render_params(frame.width, frame.height, spp, sample_base, seed, tile_size, tile_offset,
                          tile_stride, counters)
        _check(gpu_lib().fs_render(self.ctx, C.byref(cam), C.byref(p), frame.h), "fs_render")
        if sync:
            self.synchronize()
        return p

    def synchronize(self):
        _check(gpu_lib().fs_synchronize(self.ctx), "fs_synchronize")

    def last_render_ms(self):
        ms = C.c_float()
        _check(gpu_lib().fs_last_render_ms(self.ctx, C.byref(ms)), "fs_last_render_ms")
        return ms.value

    def last_trace_ms(self):
        """The trace kernel's share of last_render_ms (its launches, without fold_paths)."""
        ms = C.c_float()
        _check(gpu_lib().fs_last_trace_ms(self.ctx, C.byref(ms)), "fs_last_trace_ms")
        return ms.value

    def last_kernel(self):
        """The trace kernel the last render launched (rocprofv3's name)."""
        return gpu_lib().fs_last_kernel(self.ctx).decode()

    def last_launches(self):
        """(trace-kernel launches, spp of the largest launch) of the last render."""
        n, spp = C.c_uint32(), C.c_uint32()
        _check(gpu_lib().fs_last_render_launches(self.ctx, C.byref(n), C.byref(spp)), "fs_last_render_launches")
        return n.value, spp.value

    def last_lookahead(self):
        """Whether the last render folded a lookahead trace (fs_options.lookahead)."""
        f = C.c_int()
        _check(gpu_lib().fs_last_render_lookahead(self.ctx, C.byref(f)), "fs_last_render_lookahead")
        return bool(f.value)

    def counters(self):
        c = fs_counters()
        _check(gpu_lib().fs_read_counters(self.ctx, C.byref(c)), "fs_read_counters")
        return {k: getattr(c, k) for k, _ in fs_counters._fields_}

    def trace_range(self, cam, width, height, xy):
        """TraceRange (engine.cpp:298-329) for an (n, 2) array of image points."""
        pts = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
        out = np.empty(len(pts), np.float32)
        _check(gpu_lib().fs_trace_range(self.ctx, C.byref(cam), width, height, pts.ctypes.data, len(pts),
                                        out.ctypes.data), "fs_trace_range")
        return out

    # -- RCCL
    @staticmethod
    def comm_unique_id():
        buf = C.create_string_buffer(128)
        _check(gpu_lib().fs_comm_unique_id(buf), "fs_comm_unique_id")
        return buf.raw

    def comm_init(self, nranks, rank, uid):
        _check(gpu_lib().fs_comm_init(self.ctx, nranks, rank, uid), "fs_comm_init")

    def comm_count(self):
        n = C.c_int()
        _check(gpu_lib().fs_comm_count(self.ctx, C.byref(n)), "fs_comm_count")
        return n.value

    def gather(self, frame, params, root=0):
        _check(gpu_lib().fs_frame_gather(self.ctx, frame.h, C.byref(params), root), "fs_frame_gather")

    def pack(self, frame, params):
        """fs_frame_pack: this rank's owned tiles as uint32 words (40 B per pixel)."""
        n = C.c_uint64()
        _check(gpu_lib().fs_frame_pack_bytes(C.byref(params), C.byref(n)), "fs_frame_pack_bytes")
        out = np.zeros(n.value // 4, np.uint32)
        _check(gpu_lib().fs_frame_pack(self.ctx, frame.h, C.byref(params), out.ctypes.data, out.nbytes),
               "fs_frame_pack")
        return out

    def unpack(self, frame, params, packs):
        """fs_frame_unpack: scatters the rank-ordered concatenation of packs."""
        buf = np.ascontiguousarray(np.concatenate(packs), np.uint32)
        _check(gpu_lib().fs_frame_unpack(self.ctx, frame.h, C.byref(params), buf.ctypes.data, buf.nbytes),
               "fs_frame_unpack")

    def close(self):
        if self.ctx:
            gpu_lib().fs_destroy(self.ctx)
            self.ctx = None


def load_bitmap(path):
    """LoadBitmap (bitmap.cpp:40-104) through the host library: (ok, width,
    height, texels) with texels an (n,) float32 array as the loader left it."""
    lib = host_lib()
    buf = C.POINTER(C.c_float)()
    w, h, n = C.c_uint32(), C.c_uint32(), C.c_size_t()
    ok = lib.fsh_load_bitmap(str(path).encode(), C.byref(buf), C.byref(w), C.byref(h), C.byref(n))
    try:
        arr = np.ctypeslib.as_array(buf, shape=(max(n.value, 1),))[:n.value].copy()
    finally:
        lib.fsh_free(buf)
    return bool(ok), w.value, h.value, arr


def load_exr(path):
    """tinyexr LoadEXR restatement: (H, W, 4) float32 RGBA; raises FsError."""
    lib = host_lib()
    buf = C.POINTER(C.c_float)()
    w, h = C.c_int(), C.c_int()
    rc = lib.fsh_load_exr(str(path).encode(), C.byref(buf), C.byref(w), C.byref(h))
    if rc:
        raise FsError(f"LoadEXR failed ({rc}): {lib.fsh_last_error().decode(errors='replace')}")
    try:
        return np.ctypeslib.as_array(buf, shape=(h.value * w.value * 4,)).reshape(h.value, w.value, 4).copy()
    finally:
        lib.fsh_free(buf)


def bvh_quality(desc_ptr, **opts):
    """fs_bvh_quality: per BVH mesh SAH cost, sibling overlap, counts, depth."""
    import json

    buf = C.create_string_buffer(1 << 20)
    o = options(**opts)
    _check(gpu_lib().fs_bvh_quality(desc_ptr, C.byref(o), buf, len(buf)), "fs_bvh_quality")
    return json.loads(buf.value.decode())


def prepare_digest(desc_ptr, **opts):
    """fs_prepare_digest: host-only scene preparation with the build fields
    of fs_options (keywords as options()); (digest, nodes, build_ms)."""
    d, n, ms = C.c_uint64(), C.c_uint64(), C.c_double()
    o = options(**opts)
    _check(gpu_lib().fs_prepare_digest(desc_ptr, C.byref(o), C.byref(d), C.byref(n), C.byref(ms)),
           "fs_prepare_digest")
    return d.value, n.value, ms.value
