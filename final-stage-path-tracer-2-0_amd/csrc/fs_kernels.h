// fs_kernels.h — device code of the hot path (one wave64 per workgroup; a
// block of work is one 8x8 pixel micro-tile of a sample group).
//
// Restates, per sample, engine.cpp:59-251 (ray generation, TraceStep),
// scene.cpp:227-249 (closest hit + back-face flip), object.cpp / intersect.cpp
// (primitive tests), material.cpp + normal.cpp (BRDF sampling and shading)
// and frame.cpp:53-85 (running-mean accumulation). The recursion of TraceStep
// is unrolled into a forward pass (the megakernel) that writes each bounce's
// shading scalars and each path's end state to per-sample path records in
// HBM, and a backward pass (fold_paths) that applies Material::Sample in the
// reference's order and folds the samples into the frame, so the float
// rounding matches the recursive reference bit for bit.
#pragma once

#include "fs_scene.h"

namespace fs {

constexpr int kBlock = 64;  // one wave64 per block: stacks are per-lane LDS columns
#ifndef FS_CHUNK
#define FS_CHUNK 64  // the largest samples_per_block (default 16: the task pool runs on across blocks)
#endif
constexpr uint32_t kChunk = FS_CHUNK;  // samples per pixel per block (fs_render splits longer renders)
// Scenes with at most this many materials pack a path's per-bounce material
// ids in two registers (8 bits each); larger ones use a scratch row (MMAT).
constexpr uint32_t kPackedMaterials = 255;
// fs_render sizes sample groups so one launch holds at least this many blocks
// (~43 per wave slot of 256 CUs x 24 waves; C4 1080p x 1024 spp: 2 launches
// of 512 spp, +2.6 % over 4 launches of 256 — a launch ends with a tail of
// about one block's duration).
constexpr uint64_t kGroupTargetBlocks = 262144;
// Persistent launches: sample groups per launch up to this many bytes of
// path records (88 B per sample of an untextured scene; of 288 GB of HBM).
constexpr uint64_t kRecordBytes = 96ull << 30;

struct DevScene {
  const DevObject* __restrict__ objects;
  const BvhNode* __restrict__ nodes;
  const DevTri* __restrict__ tris;
  const float4* __restrict__ tri_normals;
  const fs_material* __restrict__ materials;
  // Per material the fields of the backward pass, 3 float4: (kind bits,
  // diffuse), (roughness, emissive), (glow, texture bits); fold_paths stages
  // them in LDS.
  const float4* __restrict__ umat;
  // Per material Material::Reflection's choice (material.cpp), precomputed
  // on the host: (threshold of its one uniform draw, solid angle A, solid
  // angle B, modes and draw flag as bits; see kReflDraws): mat_reflection.
  const float4* __restrict__ rmat;
  uint32_t num_materials;
  const float4* __restrict__ table;
  const float* __restrict__ tex_rgb;   // all textures, 3 floats per texel
  const uint4* __restrict__ tex_info;  // first float, width, height, 0
  const float2* __restrict__ tri_tex;  // 3 texcoords per triangle (BVH order) or null
  const DevSceneTree* __restrict__ tree;    // the object octree, or null (object-list walk)
  const uint32_t* __restrict__ tree_objs;   // its leaves' object indices
  uint32_t num_objects;
  int32_t sky_tex;  // 1: the sky is a LightMaterial with a map
  int32_t sky;
  float sky_r, sky_g, sky_b;  // Scene::SampleSky value (scene.cpp:157-162), x3 applied
  uint32_t sky_id;
};

// Camera basis computed on the host exactly as engine.cpp:170-197.
struct DevCamera {
  f3 origin, right, up, proj_origin;
  float hpw, hph, width, height;
  float aperture, z_far;
  f4 focal;
  int32_t fast_render;
};

struct DevFrame {
  float* color;
  uint32_t* count;
  uint8_t* display;
  float* normal;
  float* depth;
  uint64_t* material;
  uint32_t width, height;
};

struct DevCounters {
  unsigned long long samples, segments, node_visits, tri_tests, prim_tests, object_loads, small_tri_loads,
      lane_object_loads;
  // Per-wave cycle totals by loop phase; filled only by -DFS_PHASE_PROF
  // builds (libfsgpu_prof.so, a measurement tool, never the product path).
  unsigned long long phase[32];
};

// The path records of one launch, indexed by sample
// q = (the block's record row) x spp x 64 + slot, every per-level array level-major
// ([level][q]: a wave's lanes at one depth store and fold_paths' lanes load
// consecutive samples). The megakernel writes them; fold_paths reads them
// once, runs the backward pass and folds the radiance into the frame.
struct PathRecords {
  float* c;        // [level][q]: c = max(0, n.r)
  float* ds;       // [level][q]: Ceramic/Glow's specular term (written by those bounces only)
  float4* end;     // [q]: the radiance entering level top + 1, and (w, as bits) top + 1 | kRecFogDif
  uint2* mats;     // [q]: the packed 8-bit material ids of levels 0-3 and 4-7 (<= 255 materials)
  uint32_t* mat;   // [level][q]: the material id of every level (MMAT), else null
  float4* tex;     // [level][q]: SampleDiffuse's texel of a textured material (TEX), else null
  uint64_t n;      // samples of the launch (the level stride)
  // fold_paths only: the AOV planes a lookahead launch wrote for the samples
  // it folds (fs_options.lookahead), copied into the frame; null otherwise
  const float* aov_n;
  const float* aov_d;
  const uint64_t* aov_m;
};
// PathRecords::end.w flag: level 0 is Fog and its draw took the diffuse colour
constexpr uint32_t kRecFogDif = 0x100u;
// DevScene::rmat.w bits: mode A (bits 0-3), mode B (bits 4-7), and whether
// the material draws one uniform number first (Glass, Liquid, Ceramic, Glow).
enum ReflMode : uint32_t { kReflScatter = 0, kReflZero = 1, kReflMirror = 2, kReflRefract = 3, kReflFrosted = 4, kReflView = 5 };
constexpr uint32_t kReflDraws = 0x100u;  // rmat.w: the material draws one uniform number first

struct Launch {
  uint32_t tile_size, tiles_x, tile_offset, tile_stride;
  uint32_t sample_base, spp;
  uint32_t susp_thr;        // SUSP schedule: park walks of a mesh of >= kParkLargeTris faces when at most
                            // this many lanes still walk
  uint32_t susp_thr_small;  // the same for the smaller parkable meshes
  uint32_t xcd_bands;  // 1: each XCD (blocks b, b+8, ...) renders one contiguous band of micro-tiles
  // Sample groups: one launch renders `groups` consecutive runs of `spp`
  // samples; block (g, micro-tile) takes samples sample_base + g*spp ...
  // fold_paths folds every group's path records into the frame in sample order (the launch tail and a small multi-GPU share no
  // longer leave CUs idle).
  uint32_t groups;
  uint32_t owned;  // 64x64 tiles this launch renders per group
  uint32_t group_major;  // block order: 0 a tile's groups together, 1 group by group (A/B)
  // Dispatch order of the owned tiles (owned entries of owned-tile indices),
  // or null for index order. Only the order changes: every tile keeps its
  // path records, so frames are identical.
  const uint32_t* tile_order;
  uint64_t seed;
  uint32_t nblocks;  // blocks of the launch: owned tiles x micro-tiles x groups
  uint32_t persist;  // 1: persistent waves pull blocks from per-XCD queues; 0: one wave per block
  // Lookahead launches (one sample per group, each group a later TraceScene
  // call): every group's sample leaves its AOVs, group g in plane g, at
  // pixel offset g x aov_plane (group g = record row / aov_rows). 0: only
  // the last group's last sample writes the frame's AOV planes.
  uint32_t aov_rows, aov_plane;
};

}  // namespace fs
