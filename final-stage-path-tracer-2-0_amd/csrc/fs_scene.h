// fs_scene.h — device-side scene layout (SoA records in HBM) and the host
// preparation step that builds it from an fs_scene_desc.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "fs_math.h"
#include "fs_trace.h"

namespace fs {

// Object record, 192 B; read wave-uniformly by the object loop of
// Scene::Trace (scene.cpp:231-233), so it is fetched with scalar loads.
// Meshes at least this large let their BVH walks park under the SUSP
// schedule (fs_device.hip): measured on MI355X, parking pays for the ~1M
// triangle C4 blob (+15%) and loses on the ~250k-triangle C3 atrium (-4%,
// meshes of 60-120k triangles), so only scenes with such a mesh select it.
constexpr uint32_t kParkMinTris = 1u << 15;    // meshes whose walks may park (fs_options default)
constexpr uint32_t kParkLargeTris = 1u << 19;  // parkable meshes from here use park_lanes, below park_lanes_small

struct DevObject {
  int32_t kind;  // fs_object_kind (QUAD_PUV is stored as QUAD_ONWH)
  int32_t mat;
  int32_t i0;    // MESH: BVH root node index
  int32_t i1;    // MESH: 1 if the mesh has vertex normals
  int32_t i2;    // MESH: 1 if the reference would have built a tree (mesh.cpp:119)
  int32_t i3;    // MESH: n > 0 for a small mesh of n triangles (fs_options.small_mesh_tris),
                 // tested face by face from triangle d[6] (bits) on, without a walk
  int32_t i4;    // MESH: 1 if the mesh has texcoords (mesh.cpp:300)
  int32_t i5;    // MESH: walks may park (SUSP schedule): 0 never, 1 under kParkLargeTris triangles, 2 from there
  float d[40];
  // SPHERE  d0-2 center, d3 radius
  // PLANE   d0-3 plane
  // DISC    d0-3 plane, d4-6 origin, d7 radius
  // CUBOID  d0-23 six face planes (volume.cpp:234-247); d24-29 padded box
  //         of the 8 corners (a conservative cull, not a reference test)
  // QUAD    d0-3 plane, d4-6 origin, d7 half width, d8 half height,
  //         d9-11 bitangent, d12-14 tangent
  // MESH    d0-5 reference root bounds (min, max) — mesh.cpp:129-133;
  //         d6 (uint bits) the mesh's first triangle slot (small meshes: their faces)
};
static_assert(sizeof(DevObject) == 192, "DevObject layout");

// BVH2 node, 64 B: both child boxes (SoA over the two children) + child words.
// Child word: bit31 set -> leaf, bits 27..30 = triangle count (<= 15), bits
// 0..26 = first triangle slot; otherwise an inner-node index (31 bits). A
// scene holds at most 2^27 triangles. (First slots relative to each mesh, with
// the mesh's base added per walk, cost C4 5.6 %: the extra live value spilled
// the scene pointers' SGPRs into VGPR lanes read in the node loop.)
struct BvhNode {
  float lo_x[2], hi_x[2];
  float lo_y[2], hi_y[2];
  float lo_z[2], hi_z[2];
  uint32_t child[2];
  uint32_t pad[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode layout");
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kLeafCountShift = 27;
constexpr uint32_t kLeafFirstMask = (1u << kLeafCountShift) - 1;
constexpr uint32_t kMaxLeafCount = 15;
constexpr uint32_t kMaxTriangles = 1u << kLeafCountShift;  // per scene
FS_HD uint32_t leaf_word(uint32_t count, uint32_t first) {
  return kLeafBit | (count << kLeafCountShift) | first;
}
FS_HD uint32_t leaf_count(uint32_t w) { return (w >> kLeafCountShift) & 0xFu; }
#ifndef FS_TRAVERSAL_STACK
#define FS_TRAVERSAL_STACK 24  // A/B builds only (make ab DEFS=-DFS_TRAVERSAL_STACK=22)
#endif
constexpr uint32_t kTraversalStack = FS_TRAVERSAL_STACK;  // BVH depth bound (builder enforces); the LDS stack bounds the waves per CU
constexpr uint32_t kMaxSmallMeshTris = 64;  // fs_options.small_mesh_tris bound

// Triangle record: the operands of the reference test (intersect.cpp:357-419)
// with every ray-independent term precomputed on the host by the same float
// operations: p1, the planar-mapped edges v0 = p2-p1 and v1 = p3-p1 (dominant
// plane axis zeroed, intersect.cpp:96-129), their dot products and
// 1/(d00*d11 - d01*d01) (:168-173), the face plane (mesh.cpp:136-146,
// reversed winding) and the face index (tie-break).
// 64 B: the planar map zeroes one axis, so p1, v0 and v1 keep only the two
// others, (a, b) = (axis == 0 ? y : x, axis == 2 ? y : z); face and axis
// share a word (face | axis << 30).
struct DevTri {
  float plane[4];
  float p1[2];
  float v0[2];
  float v1[2];
  uint32_t face_axis;
  uint32_t mesh_obj;  // mesh index; bit 31 (small meshes): the same plane bits as the previous slot's face
  float d00, d01, d11, inv;
};
static_assert(sizeof(DevTri) == 64, "DevTri layout");
constexpr uint32_t kSamePlaneBit = 0x80000000u;
inline uint32_t tri_face_host(const DevTri& t) { return t.face_axis & 0x3FFFFFFFu; }

// The reference's scene object octree (SceneBvh, scene.cpp:11-133), built
// when Scene::Optimize ran and the scene has >= 182 objects (scene.cpp:216-
// 225). Its root always splits into 8 leaves and no leaf splits again (the
// root's depth limit is kMaxSubdivisionDepth = 2, scene.h:47, and
// SceneBvhNode::Subdivide stops at depth 1 for any object count: DESIGN.md
// §3b). Boxes and split planes are computed with the reference's float ops.
struct DevSceneTree {
  float root_mn[3], root_mx[3];
  float center[3];                    // bounds::query_center of the root
  float split[3][4];                  // split_planes_[0..2] (x, y, z)
  float child_mn[8][3], child_mx[8][3];
  uint32_t first[8], count[8];        // each leaf's object indices in tree_objs
};

// A mesh whose BVH is built on the device (fs_upload_scene_ex with
// FS_UPLOAD_GPU_BVH, fs_bvh_gpu.hip). Its node block (num_tris nodes from
// node_base) and triangle slots (num_tris from tri_base, plus normal and
// texcoord slots) follow the host-built arrays: the upload allocates them
// on the device only (PreparedScene::deferred_nodes / deferred_tris), and
// the face-order inputs wait here.
struct DeferredMesh {
  uint32_t mesh = 0, num_tris = 0, node_base = 0, tri_base = 0;
  std::vector<float> lo, hi;  // 3 floats per face: the primitive box
  std::vector<DevTri> tris;   // face order
  std::vector<float> normals, tex;  // face order, or empty
};

struct PreparedScene {
  std::vector<DevObject> objects;
  std::vector<BvhNode> nodes;
  std::vector<DevTri> tris;
  std::vector<float> tri_normals;  // 12 floats per triangle (n0,n1,n2 + pad) or empty
  std::vector<float> tri_tex;      // 6 floats per triangle (t0,t1,t2) or empty
  std::vector<float> tex_rgb;      // all textures, 3 floats per texel
  std::vector<uint32_t> tex_info;  // 4 per texture: first float, width, height, 0
  std::vector<fs_material> materials;
  std::vector<float> table;        // 4 floats per entry
  int32_t sky = 0;
  uint32_t max_depth = 0;
  double build_ms = 0.0;
  std::vector<DeferredMesh> deferred;  // meshes left for the device build
  uint32_t deferred_nodes = 0, deferred_tris = 0;  // device-only slots after the host arrays
  bool any_normals = false, any_tex = false;       // per-triangle normal / texcoord arrays exist
  bool tree_valid = false;                         // the object octree is built (DevSceneTree)
  DevSceneTree tree{};
  std::vector<uint32_t> tree_objs;                 // leaf object lists, leaf after leaf
};

// The scene-build part of fs_options, validated (out-of-range values take
// the defaults).
struct BuildOptions {
  uint32_t leaf = 2;            // faces per BVH leaf (both builders)
  int bins = 16;                // SAH bins per axis
  uint32_t threads = 0;         // host build threads, 0 = 16
  bool pair_layout = false;     // sibling-pair node layout (host build)
  uint32_t park_min_tris = kParkMinTris;
  uint32_t small_mesh_tris = 16;  // meshes tested face by face (DevObject::i3)
  bool log = false;             // build phases to stderr
  static BuildOptions from(const fs_options* o);  // NULL: the defaults
};

// Restates the object constructors (object.cpp, mesh.cpp:168-275) and builds
// one SAH BVH per mesh. Returns FS_OK or an fs_status with *err set.
// Meshes of at least gpu_bvh_min_tris triangles (0: none) are not built
// here but deferred to the device build (PreparedScene::deferred).
int prepare_scene(const fs_scene_desc* desc, PreparedScene* out, std::string* err, const BuildOptions& opt,
                  uint32_t gpu_bvh_min_tris = 0);

}  // namespace fs
