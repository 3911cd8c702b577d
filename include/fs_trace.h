/*
 * fs_trace.h — C ABI of the MI355X path-trace layer (libfsgpu.so).
 *
 * Drop-in boundary for the reference's per-pixel Monte-Carlo path tracer
 * (ramenhut/final-stage-path-tracer-2-0). The reference entry point this layer
 * replaces is
 *
 *     void base::TraceScene(const Camera&, Scene*, DisplayFrame*,
 *                           ImagePlaneCache* = nullptr);      engine.h:74-75
 *
 * which adds ONE jittered sample per pixel to a running-mean frame
 * (engine.cpp:253-296, frame.cpp:53-85). The repo's C++ mirror of that API
 * (final-stage-path-tracer-2-0_amd/host/fs_host.h) calls the functions below.
 *
 * Conventions: plain C types only; every function returns 0 on success and a
 * negative fs_status on failure (fs_last_error() has the message); no C++
 * exception crosses this boundary; the caller owns every pointer it passes.
 */
#ifndef FS_TRACE_H_
#define FS_TRACE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FS_ABI_VERSION 9
#define FS_NORMAL_TABLE_SIZE 32768u /* material.cpp:17  InitializeMaterials */
#define FS_MAX_TRACE_DEPTH 8u       /* engine.cpp:16   kMaximumTraceDepth */
#define FS_NO_INDEX 0xFFFFFFFFu

typedef enum fs_status {
  FS_OK = 0,
  FS_ERR_INVALID = -1,  /* bad argument / malformed scene */
  FS_ERR_DEVICE = -2,   /* HIP runtime error */
  FS_ERR_NOMEM = -3,    /* allocation failed */
  FS_ERR_STATE = -4,    /* call out of order (e.g. render before upload) */
  FS_ERR_COMM = -5,     /* RCCL error */
  FS_ERR_IO = -6        /* file could not be read */
} fs_status;

/* Material kinds: the nine classes of material.h:54-328. */
typedef enum fs_material_kind {
  FS_MAT_DIFFUSE = 0, /* DiffuseMaterial  material.cpp:55-137  */
  FS_MAT_LIGHT = 1,   /* LightMaterial    material.cpp:28-53   */
  FS_MAT_METAL = 2,   /* MetalMaterial    material.cpp:139-170 */
  FS_MAT_MIRROR = 3,  /* MirrorMaterial   material.cpp:172-190 */
  FS_MAT_GLASS = 4,   /* GlassMaterial    material.cpp:192-221 */
  FS_MAT_LIQUID = 5,  /* LiquidMaterial   material.cpp:223-250 */
  FS_MAT_CERAMIC = 6, /* CeramicMaterial  material.cpp:252-282 */
  FS_MAT_GLOW = 7,    /* GlowMaterial     material.cpp:284-301 */
  FS_MAT_FOG = 8      /* FogMaterial      material.cpp:303-339 */
} fs_material_kind;

/* One material instance, field names follow the reference members. */
typedef struct fs_material {
  int32_t kind;         /* fs_material_kind */
  uint32_t id;          /* Material::material_id_ = random_integer() (material.cpp:26) */
  float diffuse[3];     /* diffuse_ */
  float emissive[3];    /* LightMaterial::emissive_ */
  float glow[3];        /* GlowMaterial::glow_ */
  float roughness;      /* MetalMaterial::roughness_ */
  float shininess;      /* CeramicMaterial::shininess_ */
  float index;          /* Glass/Liquid index_ */
  float reflectivity;   /* Glass/Liquid reflectivity_ */
  float frost;          /* GlassMaterial::frost_ */
  float density;        /* FogMaterial::density_ (already x1000, material.cpp:306) */
  int32_t texture;      /* index into fs_scene_desc.textures, or -1 */
  float texture_scale;  /* texture_scale_ */
} fs_material;

/* Object kinds: the constructors of object.h / mesh.h, arguments verbatim. */
typedef enum fs_object_kind {
  FS_OBJ_SPHERE = 0,   /* SphericalObject(origin, radius)            object.cpp:17 */
  FS_OBJ_PLANE = 1,    /* PlanarObject(plane)                        object.cpp:38 */
  FS_OBJ_DISC = 2,     /* DiscObject(origin, normal, radius)         object.cpp:75 */
  FS_OBJ_CUBOID = 3,   /* CuboidObject(origin, w, h, d) [+Rotate]    object.cpp:115-124 */
  FS_OBJ_QUAD_ONWH = 4,/* QuadObject(origin, normal, width, height)  object.cpp:167 */
  FS_OBJ_QUAD_PUV = 5, /* QuadObject(position, u, v)                 object.cpp:191 */
  FS_OBJ_MESH = 6      /* MeshObject(file, invert, T, S, R)          mesh.cpp:168 */
} fs_object_kind;

/*
 * Constructor arguments, by kind (a[] layout):
 *  SPHERE    a[0..2]=origin a[3]=radius
 *  PLANE     a[0..3]=plane (nx,ny,nz,w)
 *  DISC      a[0..2]=origin a[3..5]=normal a[6]=radius
 *  CUBOID    a[0..2]=origin a[3]=width a[4]=height a[5]=depth;
 *            if rotate!=0: CuboidObject::Rotate(axis=a[6..8], angle=a[9])
 *            (ParseCuboid always calls Rotate, scene.cpp:452)
 *  QUAD_ONWH a[0..2]=origin a[3..5]=normal a[6]=width a[7]=height
 *  QUAD_PUV  a[0..2]=position a[3..5]=u a[6..8]=v
 *  MESH      mesh = index into fs_scene_desc.meshes
 */
typedef struct fs_object {
  int32_t kind;     /* fs_object_kind */
  int32_t material; /* index into fs_scene_desc.materials; must be >= 0 */
  int32_t mesh;     /* FS_OBJ_MESH only */
  int32_t rotate;   /* FS_OBJ_CUBOID only */
  float a[12];
} fs_object;

/*
 * A mesh as tinyobj hands it to MeshObject::MeshObject (mesh.cpp:168-275):
 * raw OBJ attribute arrays plus triangle corner indices in OBJ order. The
 * constructor math (T*R*S bake, normal normalisation/inversion, winding
 * reversal, face planes) is applied by the consumer, exactly as the reference.
 */
typedef struct fs_mesh {
  const float* positions;   /* 3 floats per vertex */
  uint32_t num_positions;
  const float* normals;     /* 3 floats per normal, may be NULL */
  uint32_t num_normals;
  const float* texcoords;   /* 2 floats per texcoord, may be NULL */
  uint32_t num_texcoords;
  /* 9 int32 per triangle: (v0,n0,t0, v1,n1,t1, v2,n2,t2), -1 = absent */
  const int32_t* corners;
  uint32_t num_triangles;
  int32_t invert_normals;
  float translation[3];
  float scale[3];
  float rotation[4];        /* <x,y,z> axis, w angle (radians) */
} fs_mesh;

typedef struct fs_texture {
  const float* rgb; /* width*height*3 floats, row-major */
  uint32_t width;
  uint32_t height;
} fs_texture;

typedef struct fs_scene_desc {
  const fs_material* materials; /* Material instances in creation order */
  uint32_t num_materials;
  int32_t sky_material;         /* index of the sky (Scene::sky_material_) */
  const fs_object* objects;     /* Scene::object_list_ order (scene.cpp:231) */
  uint32_t num_objects;
  const fs_mesh* meshes;
  uint32_t num_meshes;
  const fs_texture* textures;
  uint32_t num_textures;
  /* normal_sphere table (normal.cpp:9-27), FS_NORMAL_TABLE_SIZE x 3 floats */
  const float* normal_table;
  uint32_t flags;               /* FS_SCENE_* */
} fs_scene_desc;

/* Scene::Optimize() ran after the last object was added (LoadScene always
 * calls it, scene.cpp:530; AddXObject clears it, scene.cpp:165-214). With it,
 * a scene of >= 182 objects is traced through the reference's object octree
 * (SceneBvh, scene.cpp:11-133, 216-236), as the reference does; without it,
 * or with fewer objects, through the object list. */
#define FS_SCENE_OPTIMIZED 1u

/* Camera POD, camera.h:43-63. */
typedef struct fs_camera {
  float origin[3];
  float target[3];
  float fov_y;         /* degrees */
  float aperture_size; /* > 0 enables the thin lens (engine.cpp:221) */
  float focal_depth;
  float z_near;
  float z_far;
  int32_t fast_render; /* engine.cpp:68-70 */
} fs_camera;

/*
 * One render call = `spp` consecutive calls of the reference TraceScene on the
 * pixels this rank owns. Sample k (k = sample_base .. sample_base+spp-1) of
 * pixel (x, y) draws from the xorshift64* stream seeded with
 *     splitmix64(((uint64)(y*width + x) << 20) ^ k ^ seed) | 1
 * (per-(pixel,sample) seeding replaces the reference's clock seed,
 * engine.cpp:179, so renders are reproducible and shardable). Row y = 0 is the
 * bottom of the image, as in the reference frame (engine.cpp:215).
 *
 * Ownership: the frame is cut into tile_size x tile_size tiles numbered
 * row-major; this call renders tiles t with t % tile_stride == tile_offset.
 */
typedef struct fs_render_params {
  uint32_t width;
  uint32_t height;
  uint32_t spp;
  uint32_t sample_base;
  uint64_t seed;
  uint32_t tile_size;   /* 0 -> 64 */
  uint32_t tile_offset; /* rank */
  uint32_t tile_stride; /* world size (0 -> 1) */
  uint32_t flags;       /* FS_RENDER_* */
} fs_render_params;

#define FS_RENDER_COUNTERS 1u /* accumulate traversal counters (slower) */

/* Device-resident DisplayFrame (frame.h:49-92), row y=0 at the bottom. */
typedef enum fs_frame_plane {
  FS_PLANE_COLOR = 0,    /* float32 x3  render_target_ (running mean) */
  FS_PLANE_COUNT = 1,    /* uint32      count_buffer_ */
  FS_PLANE_DISPLAY = 2,  /* uint8 x3    display_buffer_ (gamma 2.2) */
  FS_PLANE_NORMAL = 3,   /* float32 x3  normal_buffer_ */
  FS_PLANE_DEPTH = 4,    /* float32     depth_buffer_ */
  FS_PLANE_MATERIAL = 5  /* uint64      material_id_buffer_ */
} fs_frame_plane;

/* Traversal / work counters (FS_RENDER_COUNTERS). */
typedef struct fs_counters {
  uint64_t samples;
  uint64_t segments;    /* ray segments traced (closest-hit queries) */
  uint64_t node_visits; /* BVH nodes whose boxes were tested */
  uint64_t tri_tests;   /* ray/triangle tests */
  uint64_t prim_tests;  /* analytic object tests (per lane) */
  uint64_t object_loads; /* object records read: wave-uniform scalar loads, one per
                            wave per object visit of a closest-hit query */
  uint64_t small_tri_loads; /* triangle records of small meshes (fs_options.small_mesh_tris),
                               wave-uniform loads, once per wave; their per-lane tests are
                               not in tri_tests */
  uint64_t lane_object_loads; /* object records read at a per-lane index (the object
                                  octree of an optimised scene, scene.cpp:216-236): vector
                                  loads, once per lane */
} fs_counters;

typedef struct fs_context fs_context;
typedef struct fs_frame fs_frame;

/*
 * Tuning options of a context (no reference counterpart: the reference has
 * one CPU schedule). Every schedule and setting renders identical frames;
 * they change speed only. The library reads no environment
 * variables: a context uses fs_options_default() until fs_set_options.
 */
typedef enum fs_schedule {
  FS_SCHEDULE_AUTO = 0,   /* PARKED when the scene has a mesh of >= park_min_tris
                             triangles and no texture, else LEAN */
  FS_SCHEDULE_LEAN = 1,   /* path-regeneration megakernel, pooled (pixel, sample) tasks */
  FS_SCHEDULE_PARKED = 2  /* LEAN + BVH walks of large meshes park when few lanes walk */
} fs_schedule;

#define FS_NODE_LAYOUT_DEPTH_FIRST 0u
#define FS_NODE_LAYOUT_PAIRS 1u

typedef struct fs_options {
  int32_t schedule;            /* fs_schedule (AUTO) */
  uint32_t park_lanes;         /* PARKED: park when at most this many lanes still walk a mesh of
                                  >= 2^19 triangles (12) */
  uint32_t park_min_tris;      /* meshes whose walks may park (32768); read at upload */
  uint32_t samples_per_block;  /* 1..64 samples of a block's 8x8 pixels per launch group (16) */
  uint32_t groups;             /* sample groups per launch (0). 0 = automatic: with persist = 1
                                  as many groups as the path-record budget allows (88 B per
                                  sample of a launch, 216 B textured; at most 96 GiB and at
                                  most half the free device memory: C4 at 1080p x 1024 spp is
                                  two launches of 512 spp); with persist = 0 enough groups for
                                  >= 262144 blocks per launch */
  uint32_t group_major;        /* block order: 0 a tile's groups together (0), 1 group by group */
  uint32_t tile_order;         /* 1 centre-first dispatch of owned tiles (1), 0 index order */
  uint32_t xcd_bands;          /* 2 whole 64x64 tiles per XCD (2), 1 one band per XCD, 0 none */
  uint32_t gpu_bvh_min_tris;   /* FS_UPLOAD_GPU_BVH: meshes this large build on the device
                                  (65536; never below 1024) */
  uint32_t bvh_leaf;           /* faces per BVH leaf, 1..15 (2) */
  uint32_t bvh_bins;           /* SAH bins per axis, 2..64 (16) */
  uint32_t bvh_threads;        /* host BVH build threads, 0 = 16 (0) */
  uint32_t node_layout;        /* FS_NODE_LAYOUT_* of host-built trees (DEPTH_FIRST) */
  uint32_t build_log;          /* 1: scene build phases to stderr (0) */
  uint32_t persist;            /* 1 persistent waves pulling blocks from per-XCD queues (1),
                                  0 one wave per block */
  uint32_t small_mesh_tris;    /* host-built meshes of at most this many triangles are tested
                                  face by face with wave-uniform loads, no BVH walk (16; 0 off,
                                  max 64); read at upload */
  uint32_t park_lanes_small;   /* PARKED: park_lanes for parkable meshes under 2^19 triangles (6) */
  uint32_t lds_rows;           /* 1: scenes without BVH walks (every mesh small, no texture) run
                                  the NOWALK kernel: no walk stack, 8 waves per SIMD (1); 0 the
                                  LEAN kernel. (The name dates from ABI 5, when that kernel also
                                  kept its shading rows in LDS.) */
  uint32_t record_budget_mb;   /* path-record bytes one launch may hold, in MiB (0: 96 GiB, and
                                  never more than half the free device memory). A frame whose
                                  one-group launch exceeds it renders in parts of its owned tiles
                                  and, below one tile per part, in launches of fewer samples per
                                  block: frames are identical (ABI 8) */
  uint32_t lookahead;          /* w calls, 0..48 (24): a render of at most 4 spp over the whole
                                  frame (tile_stride 1, no counters) that continues the previous
                                  render (same camera, scene, options and parameters, sample_base
                                  = the previous one's + spp) or folded a lookahead itself also
                                  traces, in the background on streams of their own, the samples
                                  the next w calls would add (sample_base + spp, + 2 spp, ...),
                                  in launches of 1, 2, 4, ... calls up to min(16, max(1, w / 3))
                                  each, with fewer waves per SIMD than the trace kernel holds so
                                  that the caller's folds run beside them; a later fs_render with
                                  the same camera, scene, options and parameters and one of those
                                  sample_bases folds its path records instead of tracing, and any
                                  other render discards them (their launches stop taking work).
                                  The reference's window loop (one TraceScene per displayed
                                  frame, main.cpp:157-163) then keeps the GPU busy while the host
                                  reads each frame; a camera that moves every frame starts no
                                  background work. Frames are identical; 0 off (ABI 9) */
} fs_options;

/* ---- context ---------------------------------------------------------- */
int fs_abi_version(void);
const char* fs_last_error(void);                  /* thread-local message */
int fs_device_count(int* count);
int fs_create(int device, fs_context** out);
int fs_destroy(fs_context* ctx);
int fs_options_default(fs_options* out);
/* Applies to later uploads (build fields) and renders (the rest). */
int fs_set_options(fs_context* ctx, const fs_options* opt);
int fs_get_options(fs_context* ctx, fs_options* out);

/* Copies the scene, builds per-mesh BVHs on the host and uploads SoA arrays.
 * Replaces any scene previously uploaded to ctx. */
int fs_upload_scene(fs_context* ctx, const fs_scene_desc* desc);
/* fs_upload_scene with options. FS_UPLOAD_GPU_BVH builds the BVH of every
 * mesh of >= 65536 triangles on the device (binned SAH, same tree rules as
 * the host build; the frames are identical). fs_upload_scene
 * is flags = 0. Replaces the reference's load-time octree build,
 * mesh.cpp:117-152. */
#define FS_UPLOAD_GPU_BVH 1u
int fs_upload_scene_ex(fs_context* ctx, const fs_scene_desc* desc, uint32_t flags);
/* Scene build (host preparation + any device BVH build) and upload time of
 * the last upload, in ms. */
int fs_scene_stats(fs_context* ctx, double* build_ms, double* upload_ms,
                   uint64_t* num_triangles, uint64_t* num_nodes,
                   uint64_t* device_bytes);

/* ---- frames ----------------------------------------------------------- */
int fs_frame_create(fs_context* ctx, uint32_t width, uint32_t height,
                    fs_frame** out);
int fs_frame_destroy(fs_frame* frame);
int fs_frame_reset(fs_frame* frame);              /* DisplayFrame::Reset */
/* Copies one plane (all pixels) to host memory of the plane's byte size. */
int fs_frame_read(fs_frame* frame, int plane, void* host_dst, size_t bytes);
/* Copies one plane to a page-locked host buffer the frame owns and sets
 * *host to it: valid until the next fs_frame_map of that plane or
 * fs_frame_destroy. DisplayFrame::GetDisplayBuffer (frame.h) returns it
 * (ABI 9: PCIe at pinned speed, no copy into pageable memory). */
int fs_frame_map(fs_frame* frame, int plane, const void** host);
/* Overwrites one plane from host memory (resume / test setup). */
int fs_frame_write(fs_frame* frame, int plane, const void* host_src,
                   size_t bytes);

/* ---- the hot path ------------------------------------------------------ */
/* Adds params->spp samples per owned pixel into frame; asynchronous on the
 * context stream; fs_synchronize() waits (for the frame; a background
 * lookahead trace, fs_options.lookahead, runs on). counters may be NULL. */
int fs_render(fs_context* ctx, const fs_camera* camera,
              const fs_render_params* params, fs_frame* frame);
int fs_synchronize(fs_context* ctx);
int fs_read_counters(fs_context* ctx, fs_counters* out); /* and zero them */
/* Device time of the last fs_render in ms (HIP events around all of it: the
 * trace-kernel launches and the fold_paths launches after them). */
int fs_last_render_ms(fs_context* ctx, float* ms);
/* The part of it spent in the trace kernel (the forward pass, the dominant
 * kernel; fs_last_kernel names it): the sum of HIP-event times around each of
 * its launches, without the fold_paths launches (ABI 7). Profiling aid, no
 * reference counterpart. */
int fs_last_trace_ms(fs_context* ctx, float* ms);
/* How fs_render cuts a render into launches (host only, no device needed;
 * ABI 8): the owned tiles in `parts` parts of at most `tiles_per_part`
 * consecutive owned tiles, each part's samples in launches of
 * `groups_per_launch` groups of `samples_per_block` samples; `launches` in
 * all, each holding at most `record_bytes_per_launch` bytes of path records.
 * fs_plan_render gives the plan for a record budget of record_budget_bytes
 * (0: opt's record_budget_mb, or 96 GiB), without the device's free-memory
 * cap; record_bytes_per_sample is 88 for an untextured scene of <= 255
 * materials (fs_render adds texels and material ids as the scene needs).
 * Profiling and test aid, no reference counterpart. */
typedef struct fs_render_plan {
  uint32_t parts;
  uint32_t tiles_per_part;
  uint32_t samples_per_block;
  uint32_t groups_per_launch;
  uint32_t launches;
  uint64_t record_bytes_per_launch;
} fs_render_plan;
int fs_plan_render(const fs_render_params* params, const fs_options* opt, uint64_t record_budget_bytes,
                   uint32_t record_bytes_per_sample, fs_render_plan* out);

/* Name of the trace kernel the last fs_render launched, as rocprofv3 lists it
 * (the schedule depends on the scene: see DESIGN.md); "" before any render.
 * Profiling aid, no reference counterpart. */
const char* fs_last_kernel(fs_context* ctx);
/* Launch shape of the last fs_render: the number of trace-kernel launches and
 * the samples per pixel of the largest one (renders are cut into launches of
 * sample groups). Profiling aid, no reference counterpart. */
int fs_last_render_launches(fs_context* ctx, uint32_t* launches, uint32_t* spp_per_launch);
/* 1 when the last fs_render folded a lookahead trace (fs_options.lookahead)
 * instead of tracing, else 0 (ABI 9). Test and profiling aid. */
int fs_last_render_lookahead(fs_context* ctx, int* folded);

/* ---- multi-GPU (RCCL over xGMI) ---------------------------------------- */
#define FS_COMM_ID_BYTES 128
int fs_comm_unique_id(uint8_t id[FS_COMM_ID_BYTES]);
int fs_comm_init(fs_context* ctx, int nranks, int rank,
                 const uint8_t id[FS_COMM_ID_BYTES]);
/* Gathers every rank's owned tiles (per params' tiling) into root's frame. */
int fs_frame_gather(fs_context* ctx, fs_frame* frame,
                    const fs_render_params* params, int root);
/* Ranks of the context's RCCL communicator (ncclCommCount); FS_ERR_STATE
 * before fs_comm_init. Lets a multi-GPU bench line state how many ranks the
 * gather really spanned. */
int fs_comm_count(fs_context* ctx, int* count);
int fs_comm_destroy(fs_context* ctx);

/* The tile exchange of fs_frame_gather without RCCL, through host memory
 * (tests and tools: an N-rank gather emulated on one device). params' tiling
 * is tile_offset = rank, tile_stride = nranks. fs_frame_pack writes the
 * rank's owned tiles (40 B per pixel, fs_frame_pack_bytes per rank);
 * fs_frame_unpack takes nranks packs concatenated in rank order, as
 * ncclGather delivers them, and scatters every rank's but its own
 * (tile_offset) into frame, rebuilding the display bytes. */
int fs_frame_pack_bytes(const fs_render_params* params, uint64_t* bytes);
int fs_frame_pack(fs_context* ctx, fs_frame* frame, const fs_render_params* params, void* host_dst, size_t bytes);
int fs_frame_unpack(fs_context* ctx, fs_frame* frame, const fs_render_params* params, const void* host_src,
                    size_t bytes);

/* Tree quality of every BVH mesh of a host-side preparation with the build
 * fields of opt (NULL: defaults), as JSON: per mesh the SAH cost relative to
 * its root box, the sibling-box overlap per depth level and area-weighted,
 * node / leaf / face counts and depth. Measurement aid, no device needed,
 * no reference counterpart. */
int fs_bvh_quality(const fs_scene_desc* desc, const fs_options* opt, char* out, size_t size);

/* Host only (no device needed): runs the scene preparation of
 * fs_upload_scene (object constructors, host BVH build, with the build
 * fields of opt, NULL = defaults) and returns a 64-bit digest of every array
 * it would upload, the BVH node count and the build time. For build
 * reproducibility checks and load-time measurements. */
int fs_prepare_digest(const fs_scene_desc* desc, const fs_options* opt, uint64_t* digest, uint64_t* num_nodes,
                      double* build_ms);

/* 64-bit digest of every device array of the uploaded scene (objects, BVH
 * nodes, triangles, normals, texcoords, materials, table, textures, object
 * octree), including the device-built BVHs: equal uploads give equal
 * digests (build reproducibility checks). Synchronous. */
int fs_scene_digest(fs_context* ctx, uint64_t* digest);

/* ---- TraceRange (engine.cpp:298-329) ------------------------------------
 * Focus pick: for each of `count` image points (x, y interleaved in xy) of a
 * width x height frame, the distance from camera->origin to the first hit of
 * the jitter-free, aperture-free camera ray through that point, or
 * camera->z_far when nothing is hit. Synchronous; xy and distances are host
 * memory. */
int fs_trace_range(fs_context* ctx, const fs_camera* camera, uint32_t width, uint32_t height,
                   const float* xy, uint32_t count, float* distances);

#ifdef __cplusplus
}
#endif

#endif /* FS_TRACE_H_ */
