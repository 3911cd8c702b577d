"""Builds fs_scene_desc structs directly (for materials/objects the .scene
grammar cannot express: Glow, Fog, discs, planes, PUV quads, inverted normals,
mesh vertex normals). Material ids are drawn from the main-thread stream in
creation order, as Material::Material() does (material.cpp:26)."""
import ctypes as C

import numpy as np

import fsamd


class DescBuilder:
    def __init__(self):
        fsamd.reset_main_rng()
        self.mats = []
        self.objs = []
        self.meshes = []
        self.textures = []
        self._keep = []
        self.sky = self.material(fsamd.MAT_LIGHT, emissive=(0, 0, 0))  # Scene::Scene sky

    def texture(self, rgb):
        """A diffuse map (Texture, material.h:42-52): H x W x 3 floats, rows as loaded."""
        a = np.ascontiguousarray(rgb, np.float32)
        t = fsamd.fs_texture()
        t.rgb = a.ctypes.data_as(C.POINTER(C.c_float))
        t.height, t.width = a.shape[0], a.shape[1]
        self._keep.append(a)
        self.textures.append(t)
        return len(self.textures) - 1

    def material(self, kind, diffuse=(0, 0, 0), emissive=(0, 0, 0), glow=(0, 0, 0), roughness=0.5,
                 shininess=0.0, index=0.75, reflectivity=0.1, frost=0.0, density=0.0, texture=-1,
                 texture_scale=1.0):
        m = fsamd.fs_material()
        m.kind = kind
        m.id = fsamd.random_integer() & 0xFFFFFFFF
        m.diffuse[:] = (1, 1, 1) if kind == fsamd.MAT_LIGHT else diffuse
        m.emissive[:] = emissive
        m.glow[:] = glow
        m.roughness, m.shininess, m.index, m.reflectivity, m.frost = roughness, shininess, index, reflectivity, frost
        m.density = density * 1000.0  # FogMaterial ctor (material.cpp:306)
        m.texture = texture
        m.texture_scale = texture_scale if texture >= 0 else 0.0
        self.mats.append(m)
        return len(self.mats) - 1

    def obj(self, kind, mat, a, rotate=0, mesh=-1):
        o = fsamd.fs_object()
        o.kind, o.material, o.rotate, o.mesh = kind, mat, rotate, mesh
        for i, v in enumerate(a):
            o.a[i] = v
        self.objs.append(o)
        return len(self.objs) - 1

    def mesh(self, mat, positions, faces, normals=None, corner_normals=None, invert=False,
             translation=(0, 0, 0), scale=(1, 1, 1), rotation=(0, 0, 0, 0), texcoords=None, corner_tex=None):
        pos = np.ascontiguousarray(positions, np.float32)
        faces = np.asarray(faces, np.int32)
        corners = np.full((len(faces), 9), -1, np.int32)
        corners[:, 0::3] = faces
        if corner_normals is not None:
            corners[:, 1::3] = np.asarray(corner_normals, np.int32)
        if corner_tex is not None:
            corners[:, 2::3] = np.asarray(corner_tex, np.int32)
        corners = np.ascontiguousarray(corners)
        m = fsamd.fs_mesh()
        m.positions = pos.ctypes.data_as(C.POINTER(C.c_float))
        m.num_positions = len(pos)
        if normals is not None:
            nrm = np.ascontiguousarray(normals, np.float32)
            m.normals = nrm.ctypes.data_as(C.POINTER(C.c_float))
            m.num_normals = len(nrm)
            self._keep.append(nrm)
        if texcoords is not None:
            tc = np.ascontiguousarray(texcoords, np.float32)
            m.texcoords = tc.ctypes.data_as(C.POINTER(C.c_float))
            m.num_texcoords = len(tc)
            self._keep.append(tc)
        m.corners = corners.ctypes.data_as(C.POINTER(C.c_int32))
        m.num_triangles = len(faces)
        m.invert_normals = int(invert)
        m.translation[:] = translation
        m.scale[:] = scale
        m.rotation[:] = rotation
        self._keep += [pos, corners]
        self.meshes.append(m)
        return self.obj(fsamd.OBJ_MESH, mat, [], mesh=len(self.meshes) - 1)

    def build(self, optimized=False):
        """optimized: Scene::Optimize() ran (FS_SCENE_OPTIMIZED): scenes of
        >= 182 objects are traced through the object octree."""
        fsamd.initialize_materials()
        self.table = fsamd.normal_table()
        d = fsamd.fs_scene_desc()
        self._mats = (fsamd.fs_material * len(self.mats))(*self.mats)
        self._objs = (fsamd.fs_object * max(1, len(self.objs)))(*self.objs)
        self._meshes = (fsamd.fs_mesh * max(1, len(self.meshes)))(*self.meshes)
        d.materials = C.cast(self._mats, C.POINTER(fsamd.fs_material))
        d.num_materials = len(self.mats)
        d.sky_material = self.sky
        d.objects = C.cast(self._objs, C.POINTER(fsamd.fs_object))
        d.num_objects = len(self.objs)
        d.meshes = C.cast(self._meshes, C.POINTER(fsamd.fs_mesh))
        d.num_meshes = len(self.meshes)
        if self.textures:
            self._texs = (fsamd.fs_texture * len(self.textures))(*self.textures)
            d.textures = C.cast(self._texs, C.POINTER(fsamd.fs_texture))
            d.num_textures = len(self.textures)
        d.normal_table = self.table.ctypes.data_as(C.POINTER(C.c_float))
        d.flags = fsamd.SCENE_OPTIMIZED if optimized else 0
        self.desc = d
        return C.cast(C.pointer(d), C.c_void_p)


def cornell_room(b, white, red, light):
    """Room of quads-as-meshes (mesh.cpp path) + a ceiling light mesh."""
    b.mesh(white, [[-10, 0, -10], [10, 0, -10], [10, 0, 10], [-10, 0, 10],
                   [-10, 20, -10], [-10, 20, 10], [10, 20, 10], [10, 20, -10],
                   [-10, 0, 10], [10, 0, 10], [10, 20, 10], [-10, 20, 10]],
           [[0, 1, 2], [0, 2, 3], [4, 5, 6], [4, 6, 7], [8, 9, 10], [8, 10, 11]])
    b.mesh(red, [[-10, 0, -10], [-10, 0, 10], [-10, 20, 10], [-10, 20, -10]], [[0, 1, 2], [0, 2, 3]])
    b.mesh(white, [[10, 0, -10], [10, 20, -10], [10, 20, 10], [10, 0, 10]], [[0, 1, 2], [0, 2, 3]])
    b.mesh(light, [[-3, 19.9, -3], [3, 19.9, -3], [3, 19.9, 3], [-3, 19.9, 3]], [[0, 1, 2], [0, 2, 3]])
