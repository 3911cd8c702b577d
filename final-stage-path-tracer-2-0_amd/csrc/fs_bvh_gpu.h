// fs_bvh_gpu.h — GPU build of one mesh's BVH2 (fs_bvh_gpu.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "fs_scene.h"

namespace fs {

// Meshes of at least kGpuBvhMinTris faces take the device build under
// FS_UPLOAD_GPU_BVH; kGpuBvhFloor is the smallest mesh the builder accepts
// (phase A needs tasks above its 256-face single-thread cutoff).
constexpr uint32_t kGpuBvhMinTris = 1u << 16;
constexpr uint32_t kGpuBvhFloor = 1024;

// One mesh deferred by prepare_scene(..., gpu_build = true): its primitive
// boxes and its face-order triangle records; the node and triangle ranges
// reserved for it in the scene arrays (num_tris nodes from node_base,
// num_tris triangles from tri_base).
struct GpuBvhJob {
  const float* lo;       // 3 floats per triangle: box minimum
  const float* hi;       // 3 floats per triangle: box maximum
  const DevTri* tris;    // face order
  const float* normals;  // 12 floats per triangle, or null
  const float* tex;      // 6 floats per triangle, or null
  uint32_t num_tris, leaf, node_base, tri_base;
  bool log;  // fs_options.build_log: per-phase wall time to stderr
};

struct GpuBvhResult {
  uint32_t nodes_used = 0, max_depth = 0, levels = 0;
  double build_ms = 0.0;
};

// Builds into d_nodes[node_base ...] and writes the leaf-order triangles,
// normals and texcoords at tri_base. Synchronous on `stream`.
int gpu_build_mesh_bvh(hipStream_t stream, const GpuBvhJob& job, BvhNode* d_nodes, DevTri* d_tris,
                       float* d_tri_normals, float* d_tri_tex, GpuBvhResult* res, std::string* err);

}  // namespace fs
