/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the reference per-pixel Monte-Carlo path tracer
 * ramenhut/final-stage-path-tracer-2-0 (read-only at /root/reference during
 * development; never shipped). Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker
 * or the timed CPU baseline — never as part of the product path.
 *
 * Parity status: PARTIALLY PINNED. The reference cannot be built in this
 * image without stand-in headers (math/base.h:37-51 needs <windows.h> or
 * <TargetConditionals.h>), and it ships no tests or fixtures. The restatement
 * is pinned against the reference outputs recorded in SURVEY.md (xorshift64*
 * stream, fast-sqrt length, sphere known answer) and by construction
 * otherwise; image-level goldens are generated from this restatement
 * (tests/golden/make_golden.py). See DESIGN.md §Oracle.
 */
#ifndef FS_ORACLE_H_
#define FS_ORACLE_H_

#include <stdint.h>
#include "fs_trace.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

/* Host-side DisplayFrame (frame.h:49-92); caller-owned arrays of W*H pixels. */
typedef struct oracle_frame {
  uint32_t width, height;
  float* color;       /* 3 per pixel, running mean */
  uint32_t* count;
  uint8_t* display;   /* 3 per pixel */
  float* normal;      /* 3 per pixel */
  float* depth;
  uint64_t* material;
} oracle_frame;

typedef struct oracle_stats {
  uint64_t samples, segments, node_visits, tri_tests;
} oracle_stats;

int oracle_scene_create(const fs_scene_desc* desc, oracle_scene** out);
void oracle_scene_destroy(oracle_scene* scene);
/* Octree node count / leaf face references of mesh m (for tests). */
int oracle_mesh_info(const oracle_scene* scene, uint32_t mesh,
                     uint32_t* nodes, uint64_t* face_refs, float* root_bounds6);
/* Baked (post-transform) vertex i of mesh m, and its face plane f. */
int oracle_mesh_vertex(const oracle_scene* scene, uint32_t mesh, uint32_t i,
                       float out[3]);
int oracle_mesh_face_plane(const oracle_scene* scene, uint32_t mesh,
                           uint32_t f, float out[4]);

/* Renders params->spp samples into the owned tiles of frame with `threads`
 * std-thread-like row bands (engine.cpp:174-203). */
int oracle_render(const oracle_scene* scene, const fs_camera* camera,
                  const fs_render_params* params, int threads,
                  oracle_frame* frame, oracle_stats* stats);

/* One sample of one pixel: TracePixel result (colour, normal, depth, id). */
int oracle_trace_sample(const oracle_scene* scene, const fs_camera* camera,
                        uint32_t width, uint32_t height, uint32_t x, uint32_t y,
                        uint32_t sample, uint64_t seed, float color[3],
                        float normal[3], float* depth, uint64_t* material_id,
                        uint32_t* ray_count);

/* TraceRange (engine.cpp:298-329): distance to the first hit of the
 * jitter-free ray through image point (x, y), or camera->z_far. */
int oracle_trace_range(const oracle_scene* scene, const fs_camera* camera,
                       uint32_t width, uint32_t height, float x, float y,
                       float* distance);

/* ---- diagnostics (tests/tools) ------------------------------------------- */
/* The camera ray (engine.cpp:210-244) of sample `sample` of pixel (x, y). */
int oracle_camera_ray(const fs_camera* camera, uint32_t width, uint32_t height, uint32_t x, uint32_t y,
                      uint32_t sample, uint64_t seed, float start[3], float stop[3]);
/* The segments TraceStep traces for one sample: 10 floats each (start,
 * stop, dir, closest-hit param or 2); returns their number (<= max). */
int oracle_trace_path(const oracle_scene* scene, const fs_camera* camera, uint32_t width, uint32_t height,
                      uint32_t x, uint32_t y, uint32_t sample, uint64_t seed, float* segs, uint32_t max);
/* Object `obj`'s closest hit on the segment (start, stop, dir) with param
 * pre-seeded by `best` (Object::Trace; meshes through the octree, or over
 * every face when brute != 0). Returns 1 on a hit; *face is the mesh face or ~0u. */
int oracle_object_trace(const oracle_scene* scene, uint32_t obj, const float start[3], const float stop[3],
                        const float dir[3], float best, int brute, float* param, uint32_t* face);
/* The octree leaves of mesh `mesh` that list face f (node ids and boxes,
 * up to max); returns how many there are. */
int oracle_face_leaves(const oracle_scene* scene, uint32_t mesh, uint32_t f, uint32_t* leaves, float* boxes,
                       uint32_t max);

/* The scene object octree (SceneBvh): node i's box (min, max), its 8
 * children (-1 for a leaf), its object count and up to max object indices.
 * Returns the number of nodes, 0 when the scene is traced through its list. */
int oracle_scene_tree(const oracle_scene* scene, uint32_t i, float box[6], int32_t children[8], uint32_t* count,
                      uint32_t* objs, uint32_t max);
/* Logs the octree walk's decisions to stderr while on (not thread-safe). */
void oracle_set_walk_log(int on);

/* ---- known-answer helpers ---------------------------------------------- */
uint64_t oracle_splitmix64(uint64_t x);
uint64_t oracle_pixel_seed(uint64_t pixel, uint64_t sample, uint64_t seed);
uint64_t oracle_random_integer(uint64_t* state);
float oracle_random_float(uint64_t* state);
int64_t oracle_random_integer_range(uint64_t* state, int32_t lo, int32_t hi);
float oracle_random_float_range(uint64_t* state, float lo, float hi);
/* normal_sphere::initialize after `predraws` draws of the stream seeded with
 * `seed` (521288629 in the reference, random.cpp:6). out: count*3 floats. */
void oracle_normal_table(uint64_t seed, uint32_t predraws, uint32_t count,
                         float* out);
float oracle_inv_sqrt(float f);
float oracle_fast_sqrt(float f);
void oracle_normalize(const float v[3], float out[3]);
void oracle_reflect(const float v[3], const float n[3], float out[3]);
void oracle_refract(const float v[3], const float n[3], float index,
                    float out[3]);
void oracle_rotate(const float v[3], float angle, const float axis[3],
                   float out[3]);
/* out: param, point[3], normal[3]; return 1 on hit. */
int oracle_ray_sphere(const float c[3], float r, const float start[3],
                      const float stop[3], float out[7]);
int oracle_ray_plane(const float p[4], const float start[3],
                     const float stop[3], float out[7]);
int oracle_ray_bounds(const float bmin[3], const float bmax[3],
                      const float start[3], const float stop[3], float out[4]);
/* out: param, point[3], normal[3], u, v */
int oracle_ray_triangle(const float p1[3], const float p2[3], const float p3[3],
                        const float start[3], const float stop[3],
                        float out[9]);
int oracle_triangle_box(const float p1[3], const float p2[3],
                        const float p3[3], const float bmin[3],
                        const float bmax[3]);

#ifdef __cplusplus
}
#endif
#endif /* FS_ORACLE_H_ */
