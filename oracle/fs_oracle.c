/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see fs_oracle.h for the rules).
 *
 * Plain-C restatement of the reference per-pixel path tracer. Every function
 * cites the reference file:line it restates (paths relative to the reference
 * repository root, `source/`). Floating-point expressions keep the reference's
 * operand order and its float/double promotions: build with
 * -O2 -ffp-contract=off and no -ffast-math (the x86-64 SSE2 baseline has no
 * FMA, matching the reference's g++ -O2 build recorded in SURVEY.md §8c).
 */
#include "fs_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* math/base.h:80-83 */
#define REF_PI (3.14159262f)
#define REF_INFINITY (1.0e15f)
#define REF_EPSILON (1.0e-5f)
#define REF_MAX_INT32 (0x7FFFFFFF)

#define K_TRACE_DEPTH 8u          /* engine.cpp:16 */
#define K_STEP_OFFSET 0.03f       /* engine.cpp:17 */
#define K_DIFFUSE_CONTRIB 0.001f  /* material.cpp:12 */
#define K_ROUGHNESS_THR 0.95f     /* material.cpp:13 */
#define K_MESH_LEAF 16u           /* mesh.cpp:15 */
#define K_MESH_DEPTH 4u           /* mesh.cpp:16 */

/* ------------------------------------------------------------------------ */
/* vector3 (math/vector3.h)                                                   */
/* ------------------------------------------------------------------------ */
typedef struct v3 { float x, y, z; } v3;
typedef struct v4 { float x, y, z, w; } v4;

static inline v3 mk3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 mk4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 add3(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }  /* vector3.h:354 */
static inline v3 sub3(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }  /* vector3.h:350 */
static inline v3 mul3(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }  /* vector3.h:366 */
static inline v3 scl3(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }     /* vector3.h:374 */
static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  /* vector3.h:292 */
static inline v3 cross3(v3 a, v3 b) {                                             /* vector3.h:193-201 */
  return mk3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}

/* scalar.h:233-245: Quake inverse sqrt with ONE Newton step; sqrtf = 1/that. */
static inline float inv_sqrt_ref(float f) {
  float half = 0.5f * f;
  int32_t i;
  memcpy(&i, &f, 4);
  i = 0x5f3759df - (i >> 1);
  memcpy(&f, &i, 4);
  f = f * (1.5f - half * f * f);
  return f;
}
static inline float fsqrt(float f) { return 1.0f / inv_sqrt_ref(f); }
static inline float len3(v3 a) { return fsqrt(dot3(a, a)); }                       /* vector3.h:301 */
static inline v3 norm3(v3 a) {                                                    /* vector3.h:181-191 */
  float l = len3(a);
  if (l == 0.0) l = 1.0f;
  return mk3(a.x / l, a.y / l, a.z / l);
}
static inline v3 reflect3(v3 v, v3 n) {                                           /* vector3.h:208-211 */
  return sub3(v, scl3(n, dot3(n, v) * (1.0f + 1.0f)));
}
static inline v3 refract3(v3 v, v3 n, float index) {                              /* vector3.h:213-222 */
  float n_dot_v = -dot3(v, n);
  float sin2 = (float)((double)(index * index) * (1.0 - (double)(n_dot_v * n_dot_v)));
  if (sin2 >= 1.0) return mk3(0, 0, 0);
  v3 r = add3(scl3(v, index), scl3(n, index * n_dot_v - fsqrt((float)(1.0 - (double)sin2))));
  return norm3(r);
}
static inline float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline v3 rotate3(v3 v, float angle, v3 ax) {                              /* vector3.h:315-333 */
  float c = (float)cosf(angle);
  float s = (float)sinf(angle);
  float a0 = ax.x, a1 = ax.y, a2 = ax.z;
  float o0, o1, o2;
  o0 = (c + (1 - c) * a0 * a0) * v.x;
  o0 += ((1 - c) * a0 * a1 - a2 * s) * v.y;
  o0 += ((1 - c) * a0 * a2 + a1 * s) * v.z;
  o1 = ((1 - c) * a0 * a1 + a2 * s) * v.x;
  o1 += (c + (1 - c) * a1 * a1) * v.y;
  o1 += ((1 - c) * a1 * a2 - a0 * s) * v.z;
  o2 = ((1 - c) * a0 * a2 - a1 * s) * v.x;
  o2 += ((1 - c) * a1 * a2 + a0 * s) * v.y;
  o2 += (c + (1 - c) * a2 * a2) * v.z;
  return mk3(o0, o1, o2);
}
/* scalar.h:337-346 */
static inline int cmp_eps(float a, float b, float ep) { return a > (b - ep) && a < (b + ep); }

/* plane.h:68-84, normal.h:67-79 */
static inline float plane_dist(v4 p, v3 pt) { return p.x * pt.x + p.y * pt.y + p.z * pt.z + p.w; }
static inline v4 plane_np(v3 n, v3 p) { return mk4(n.x, n.y, n.z, -dot3(n, p)); }
static inline v3 calc_normal(v3 a, v3 b, v3 c) { return norm3(cross3(sub3(b, a), sub3(c, a))); }
static inline v4 plane_3p(v3 a, v3 b, v3 c) { return plane_np(calc_normal(a, b, c), a); }

/* ------------------------------------------------------------------------ */
/* RNG (math/random.cpp) and per-(pixel,sample) seeding                       */
/* ------------------------------------------------------------------------ */
uint64_t oracle_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t oracle_pixel_seed(uint64_t pixel, uint64_t sample, uint64_t seed) {
  return oracle_splitmix64((pixel << 20) ^ sample ^ seed) | 1ull;
}
/* random.cpp:14-23 xorshift64* (Marsaglia / Vigna) */
uint64_t oracle_random_integer(uint64_t* s) {
  uint64_t x = *s;
  x ^= x << 12;
  x ^= x >> 25;
  x ^= x << 27;
  *s = x;
  return x * 0x2545F4914F6CDD1Dull;
}
/* random.cpp:25-27: (float)(r % 0x7FFFFFFF) / (float)0x7FFFFFFF (= 2^31f) */
float oracle_random_float(uint64_t* s) {
  return ((float)(oracle_random_integer(s) % (uint64_t)REF_MAX_INT32)) / (float)REF_MAX_INT32;
}
/* random.cpp:29-39 */
int64_t oracle_random_integer_range(uint64_t* s, int32_t imin, int32_t imax) {
  if (imax < imin) return 0;
  if (imin == imax) return imin;
  uint32_t span = (uint32_t)(imax - imin) + 1;
  return ((int32_t)imin + (int64_t)(oracle_random_integer(s) % span));
}
/* random.cpp:41-49 */
float oracle_random_float_range(uint64_t* s, float imin, float imax) {
  if (imax < imin) return 0.0f;
  return imin + oracle_random_float(s) * (imax - imin);
}

/* normal.cpp:9-27. vector3(rfr(), rfr(), rfr()) is evaluated right to left by
 * g++: z is drawn first, then y, then x. */
void oracle_normal_table(uint64_t seed, uint32_t predraws, uint32_t count, float* out) {
  uint64_t s = seed;
  for (uint32_t i = 0; i < predraws; i++) oracle_random_integer(&s);
  for (uint32_t i = 0; i < count; i++) {
    v3 a = mk3(10, 10, 10);
    while (len3(a) > 1.0) {
      float z = oracle_random_float_range(&s, -1.0f, 1.0f);
      float y = oracle_random_float_range(&s, -1.0f, 1.0f);
      float x = oracle_random_float_range(&s, -1.0f, 1.0f);
      a = mk3(x, y, z);
    }
    a = norm3(a);
    out[3 * i + 0] = a.x;
    out[3 * i + 1] = a.y;
    out[3 * i + 2] = a.z;
  }
}

/* ------------------------------------------------------------------------ */
/* ray / collision / bounds (math/trace.*, math/volume.*, math/intersect.cpp) */
/* ------------------------------------------------------------------------ */
typedef struct ray_t { v3 start, stop, dir; } ray_t;
static inline ray_t mkray(v3 s, v3 e) { ray_t r; r.start = s; r.stop = e; r.dir = sub3(e, s); return r; } /* trace.cpp:6-10 */
static inline int zero_len(const ray_t* r) { return cmp_eps(len3(r->dir), 0.0f, REF_EPSILON); }           /* trace.cpp:16 */

typedef struct coll_t { float param; v3 point; v3 normal; } coll_t;                                        /* trace.cpp:18-21 */
static inline coll_t no_coll(void) { coll_t c; c.param = 2.0f; c.point = mk3(0, 0, 0); c.normal = mk3(0, 0, 0); return c; }

typedef struct bounds_t { v3 mn, mx; uint32_t count; } bounds_t;
static inline void bounds_clear(bounds_t* b) { b->count = 0; b->mn = mk3(0, 0, 0); b->mx = mk3(0, 0, 0); }  /* volume.cpp:130-135 */
static void bounds_add(bounds_t* b, v3 p) {                                                                 /* volume.cpp:162-191 */
  if (b->count == 0) { b->mn = p; b->mx = p; b->count = 1; return; }
  b->count++;
  if (p.x > b->mx.x) b->mx.x = p.x;
  if (p.y > b->mx.y) b->mx.y = p.y;
  if (p.z > b->mx.z) b->mx.z = p.z;
  if (p.x < b->mn.x) b->mn.x = p.x;
  if (p.y < b->mn.y) b->mn.y = p.y;
  if (p.z < b->mn.z) b->mn.z = p.z;
}
static inline v3 bounds_center(const bounds_t* b) { return scl3(add3(b->mn, b->mx), 0.5f); }              /* volume.cpp:119-121 */

static inline int point_in_bounds(const bounds_t* b, v3 p) {                                               /* intersect.cpp:16-24 */
  return p.x >= b->mn.x && p.x <= b->mx.x && p.y >= b->mn.y && p.y <= b->mx.y && p.z >= b->mn.z && p.z <= b->mx.z;
}

/* intersect.cpp:656-745 (live code :728-744): two-sided, t in [0,1]; writes only on hit. */
static inline int ray_plane(v4 p, const ray_t* r, coll_t* h) {
  float ts = (p.x * r->dir.x + p.y * r->dir.y + p.z * r->dir.z);
  if (!cmp_eps(ts, 0.0f, REF_EPSILON)) {
    float ns = (float)((double)(p.x * r->start.x + p.y * r->start.y + p.z * r->start.z + p.w) * -1.0);
    float t = ns / ts;
    if (t >= 0 && t <= 1) {
      h->param = t;
      h->point = add3(r->start, scl3(r->dir, t));
      h->normal = mk3(p.x, p.y, p.z);
      return 1;
    }
  }
  return 0;
}

/* intersect.cpp:421-488 */
static int ray_sphere(v3 c, float radius, const ray_t* r, coll_t* h) {
  if (zero_len(r)) return len3(sub3(r->start, c)) <= radius; /* no hit info written (:424-426) */
  v3 o = sub3(r->start, c);
  float a = dot3(r->dir, r->dir);
  float b = 2 * (dot3(o, r->dir));
  float cc = dot3(o, o) - radius * radius;
  float d = b * b - 4 * a * cc;
  float t = 0;
  if (d < 0) return 0;
  if (len3(o) <= radius) t = (-b + fsqrt(d)) / (2 * a);
  else t = (-b - fsqrt(d)) / (2 * a);
  if (t < 0 || t > 1) return 0;
  v3 hp = add3(r->start, scl3(r->dir, t));
  h->param = t;
  h->point = hp;
  h->normal = norm3(sub3(hp, c));
  return 1;
}

/* intersect.cpp:490-529 */
static int ray_slab(float start, float vec, float smin, float smax, float* pn, float* pf) {
  if (cmp_eps(vec, 0.0f, REF_EPSILON)) {
    if (start < smin || start > smax) return 0;
    return 1;
  }
  float t1 = (smin - start) / vec;
  float t2 = (smax - start) / vec;
  if (t1 > t2) { float tt = t1; t1 = t2; t2 = tt; }
  if (t1 > (*pn)) (*pn) = t1;
  if (t2 < (*pf)) (*pf) = t2;
  return 1;
}
/* intersect.cpp:531-597 (the returned normal is never read on the path) */
static int ray_bounds_worker(const bounds_t* b, v3 s, v3 e, coll_t* h) {
  v3 v = sub3(e, s);
  float fnear = -REF_INFINITY, ffar = REF_INFINITY;
  if (!ray_slab(s.x, v.x, b->mn.x, b->mx.x, &fnear, &ffar)) return 0;
  if (!ray_slab(s.y, v.y, b->mn.y, b->mx.y, &fnear, &ffar)) return 0;
  if (!ray_slab(s.z, v.z, b->mn.z, b->mx.z, &fnear, &ffar)) return 0;
  if (fnear > ffar) return 0;
  if (ffar < 0 || fnear < 0 || fnear > 1) return 0;
  h->param = fnear;
  h->point = add3(s, scl3(v, fnear));
  return 1;
}
/* intersect.cpp:599-654 */
static int ray_bounds(const bounds_t* b, const ray_t* r, coll_t* h) {
  if (zero_len(r)) {
    if (point_in_bounds(b, r->start)) { h->param = 0.0f; h->point = r->start; h->normal = mk3(0, 0, 0); return 1; }
    return 0;
  }
  if (point_in_bounds(b, r->start) && point_in_bounds(b, r->stop)) {
    h->param = 0.0f; h->point = r->start; h->normal = mk3(0, 0, 0);
    return 1;
  }
  if (point_in_bounds(b, r->start)) {
    if (ray_bounds_worker(b, r->stop, r->start, h)) { h->param = 1.0f - h->param; return 1; }
    return 0;
  }
  return ray_bounds_worker(b, r->start, r->stop, h);
}

/* intersect.cpp:96-129 */
static void planar_map(v3* v0, v3* v1, v3* vp, v4 p) {
  float ax = fabsf(p.x), ay = fabsf(p.y), az = fabsf(p.z);
  if (ax >= ay) {
    if (ax >= az) v0->x = v1->x = vp->x = 0;
    else v0->z = v1->z = vp->z = 0;
  } else {
    if (ay >= az) v0->y = v1->y = vp->y = 0;
    else v0->z = v1->z = vp->z = 0;
  }
}
/* intersect.cpp:146-177 */
static void bary_coeff(v3 v0, v3 v1, v3 vp, float* u, float* v) {
  float d00 = dot3(v0, v0), d01 = dot3(v0, v1), d02 = dot3(v0, vp);
  float d11 = dot3(v1, v1), d12 = dot3(v1, vp);
  float inv = 1 / (d00 * d11 - d01 * d01);
  *u = (d11 * d02 - d01 * d12) * inv;
  *v = (d00 * d12 - d01 * d02) * inv;
}
/* intersect.cpp:45-47: plane.dot(vector4(pt)) promotes pt with w = 1
 * (vector4.cpp:40-47), so the live test is n.p + w + w. */
static inline int point_in_plane(v4 p, v3 pt) {
  float d4 = p.x * pt.x + p.y * pt.y + p.z * pt.z + p.w * 1.0f;
  return cmp_eps(d4 + p.w, 0.0f, REF_EPSILON);
}
/* intersect.cpp:320-346 */
static int point_in_tri(v3 p1, v3 p2, v3 p3, v4 p, v3 pt, float* bu, float* bv) {
  if (!point_in_plane(p, pt)) return 0;
  v3 v0 = sub3(p2, p1), v1 = sub3(p3, p1), vp = sub3(pt, p1);
  float u = 0, v = 0;
  planar_map(&v0, &v1, &vp, p);
  bary_coeff(v0, v1, vp, &u, &v);
  if ((u >= 0) && (v >= 0) && (u + v <= 1)) { *bu = u; *bv = v; return 1; }
  return 0;
}
/* intersect.cpp:357-419 */
static int ray_tri(v3 p1, v3 p2, v3 p3, v4 p, const ray_t* r, coll_t* h, float* bu, float* bv) {
  if (zero_len(r)) {
    if (point_in_tri(p1, p2, p3, p, r->start, bu, bv)) {
      h->param = 0.0f; h->normal = mk3(p.x, p.y, p.z); h->point = r->start;
      return 1;
    }
    return 0;
  }
  coll_t ph = no_coll();
  if (!ray_plane(p, r, &ph)) return 0;
  if (ph.param < 0 || ph.param > 1) return 0;
  v3 v0 = sub3(p2, p1), v1 = sub3(p3, p1), vp = sub3(ph.point, p1);
  float u = 0, v = 0;
  planar_map(&v0, &v1, &vp, p);
  bary_coeff(v0, v1, vp, &u, &v);
  if ((u >= 0) && (v >= 0) && (u + v <= 1)) { *h = ph; *bu = u; *bv = v; return 1; }
  return 0;
}

/* intersect.cpp:209-226 */
static int bounds_vs_plane(const v3* bv, v4 p) {
  uint32_t count = 0;
  for (int i = 0; i < 8; i++) {
    float d = plane_dist(p, bv[i]);
    if (cmp_eps(d, 0.0f, REF_EPSILON)) return 1;
    count += (d > 0.0f);
  }
  return (count != 0 && count != 8);
}
/* intersect.cpp:228-311 (Akenine-Moller SAT, as written) */
static int tri_vs_bounds(v3 p1, v3 p2, v3 p3, const bounds_t* b) {
  static const v3 bn[3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  v3 bv[8];
  for (int i = 0; i < 8; i++) {
    int xm = (i & 1), ym = ((i >> 1) & 1), zm = ((i >> 2) & 1);
    bv[i] = mk3(b->mn.x * (!xm) + b->mx.x * (xm), b->mn.y * (!ym) + b->mx.y * (ym), b->mn.z * (!zm) + b->mx.z * (zm));
  }
  v3 tv[3] = {p1, p2, p3};
  v3 te[3] = {sub3(p1, p2), sub3(p2, p3), sub3(p3, p1)};
  v4 tp = plane_3p(p1, p2, p3);
  if (!bounds_vs_plane(bv, tp)) return 0;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      v3 axis = cross3(te[i], bn[j]);
      float tmin = 9999999.0f, tmax = -tmin;
      for (int k = 0; k < 3; k++) {
        float pl = dot3(tv[k], axis);
        if (pl < tmin) tmin = pl;
        if (pl > tmax) tmax = pl;
      }
      float bmin = 9999999.0f, bmax = -bmin;
      for (int k = 0; k < 8; k++) {
        float pl = dot3(bv[k], axis);
        if (pl < bmin) bmin = pl;
        if (pl > bmax) bmax = pl;
      }
      if (bmax < tmin || bmin > tmax) return 0;
    }
  return 1;
}

/* ------------------------------------------------------------------------ */
/* Mesh + octree (mesh.cpp, bvh.h)                                            */
/* ------------------------------------------------------------------------ */
typedef struct oface { uint32_t vi[3], ni[3], ti[3]; v4 plane; } oface;    /* mesh.h:63-74 */
typedef struct onode {
  bounds_t aabb;
  uint32_t depth;
  int leaf;
  v4 split[3];
  int32_t child[8];
  uint32_t* faces;
  uint32_t nfaces, cap;
} onode;
typedef struct omesh {
  v3* verts; uint32_t nv;
  v3* normals; uint32_t nn;
  float* tex; uint32_t nt;
  oface* faces; uint32_t nf;
  bounds_t aabb;            /* MeshObject::aabb_ */
  onode* nodes; uint32_t nnodes, capnodes;
  int has_tree;
} omesh;
typedef struct mcoll_t { float param; v3 point; v3 normal; uint32_t face; float bu, bv; } mcoll_t; /* mesh.h:46-61 */

static uint32_t new_node(omesh* m) {
  if (m->nnodes == m->capnodes) {
    m->capnodes = m->capnodes ? 2 * m->capnodes : 64;
    m->nodes = (onode*)realloc(m->nodes, sizeof(onode) * m->capnodes);
  }
  onode* n = &m->nodes[m->nnodes];
  memset(n, 0, sizeof(*n));
  n->leaf = 1;
  for (int i = 0; i < 8; i++) n->child[i] = -1;
  return m->nnodes++;
}
static void node_add_face(onode* n, uint32_t f) {
  if (n->nfaces == n->cap) { n->cap = n->cap ? 2 * n->cap : 16; n->faces = (uint32_t*)realloc(n->faces, 4 * n->cap); }
  n->faces[n->nfaces++] = f;
}

/* bvh.h:108-137 */
static void configure_children(omesh* m, uint32_t ni) {
  v3 mn = m->nodes[ni].aabb.mn;
  v3 center = bounds_center(&m->nodes[ni].aabb);
  v3 hx = sub3(mk3(center.x, mn.y, mn.z), mn);
  v3 hy = sub3(mk3(mn.x, center.y, mn.z), mn);
  v3 hz = sub3(mk3(mn.x, mn.y, center.z), mn);
  v3 span = add3(add3(hx, hy), hz);
  m->nodes[ni].split[0] = plane_np(mk3(1, 0, 0), center);
  m->nodes[ni].split[1] = plane_np(mk3(0, 1, 0), center);
  m->nodes[ni].split[2] = plane_np(mk3(0, 0, 1), center);
  for (int i = 0; i < 8; i++) {
    uint32_t c = new_node(m); /* may realloc m->nodes */
    onode* parent = &m->nodes[ni];
    m->nodes[c].depth = parent->depth + 1;
    parent->child[i] = (int32_t)c;
    v3 nmin = add3(add3(add3(mn, scl3(hx, (float)(i % 2))), scl3(hy, (float)(i >> 2))), scl3(hz, (float)((i % 4) >> 1)));
    v3 nmax = add3(nmin, span);
    bounds_t nb; bounds_clear(&nb);
    bounds_add(&nb, nmin);
    bounds_add(&nb, nmax);
    m->nodes[c].aabb = nb;
  }
  m->nodes[ni].leaf = 0;
}
/* mesh.cpp:39-76 */
static void subdivide(omesh* m, uint32_t ni) {
  if (m->nodes[ni].depth >= K_MESH_DEPTH) return;
  if (m->nodes[ni].nfaces > K_MESH_LEAF) {
    configure_children(m, ni);
    for (uint32_t j = 0; j < m->nodes[ni].nfaces; j++) {
      uint32_t f = m->nodes[ni].faces[j];
      const oface* face = &m->faces[f];
      v3 v0 = m->verts[face->vi[0]], v1 = m->verts[face->vi[1]], v2 = m->verts[face->vi[2]];
      for (int i = 0; i < 8; i++) {
        onode* c = &m->nodes[m->nodes[ni].child[i]];
        if (tri_vs_bounds(v0, v1, v2, &c->aabb)) node_add_face(c, f);
      }
    }
    free(m->nodes[ni].faces);
    m->nodes[ni].faces = NULL;
    m->nodes[ni].nfaces = m->nodes[ni].cap = 0;
    for (int j = 0; j < 8; j++) subdivide(m, (uint32_t)m->nodes[ni].child[j]);
  }
}

/* bvh.h:144-152: child index bit0 = x, bit1 = z, bit2 = y */
static inline uint32_t closest_child(const onode* n, v3 p) {
  v3 d = sub3(p, bounds_center(&n->aabb));
  uint32_t xt = d.x >= 0.0f, yt = d.y >= 0.0f, zt = d.z >= 0.0f;
  return (xt | (zt << 1) | (yt << 2)) & 0xFF;
}

typedef struct tstats { uint64_t nodes, tris, segs; } tstats;
static int mesh_node_trace(const omesh* m, uint32_t ni, const ray_t* r, mcoll_t* h, tstats* st);

/* Diagnostics: when set, the octree walk logs its decisions to stderr. */
static int g_walk_log = 0;
void oracle_set_walk_log(int on) { g_walk_log = on; }

/* bvh.h:154-231 */
static int trace_internal(const omesh* m, uint32_t ni, coll_t node_hit, const ray_t* r, mcoll_t* h, tstats* st) {
  const onode* n = &m->nodes[ni];
  int result = 0, xh, yh, zh;
  uint32_t cn;
  ray_t it = *r;
  coll_t xi = no_coll(), yi = no_coll(), zi = no_coll();
  if (!point_in_bounds(&n->aabb, r->start)) {
    it.start = node_hit.point;
    cn = closest_child(n, node_hit.point);
    xh = ray_plane(n->split[0], &it, &xi);
    yh = ray_plane(n->split[1], &it, &yi);
    zh = ray_plane(n->split[2], &it, &zi);
  } else {
    cn = closest_child(n, r->start);
    xh = ray_plane(n->split[0], r, &xi);
    yh = ray_plane(n->split[1], r, &yi);
    zh = ray_plane(n->split[2], r, &zi);
    if (!xh && !yh && !zh) return mesh_node_trace(m, (uint32_t)n->child[cn], r, h, st);
  }
  if (g_walk_log)
    fprintf(stderr, "internal %u depth %u start_in=%d cn=%u x(%d %.9g) y(%d %.9g) z(%d %.9g)\n", ni, n->depth,
            point_in_bounds(&n->aabb, r->start), cn, xh, xi.param, yh, yi.param, zh, zi.param);
  for (uint32_t i = 0; i < 4; i++) {
    if (mesh_node_trace(m, (uint32_t)n->child[cn], r, h, st)) {
      result = 1;
      if (point_in_bounds(&m->nodes[n->child[cn]].aabb, h->point)) break;
    }
    if (xh && xi.param < yi.param && xi.param < zi.param) {
      cn ^= 0x1; xh = 0; it.start = xi.point; xi.param = REF_INFINITY;
    } else if (yh && yi.param < zi.param && yi.param < xi.param) {
      cn ^= 0x4; yh = 0; it.start = yi.point; yi.param = REF_INFINITY;
    } else if (zh && zi.param < yi.param && zi.param < xi.param) {
      cn ^= 0x2; zh = 0; it.start = zi.point; zi.param = REF_INFINITY;
    } else {
      break;
    }
    if (!point_in_bounds(&n->aabb, it.start)) break;
  }
  return result;
}

/* mesh.cpp:78-115 */
static int mesh_node_trace(const omesh* m, uint32_t ni, const ray_t* r, mcoll_t* h, tstats* st) {
  const onode* n = &m->nodes[ni];
  coll_t nh = no_coll();
  if (st) st->nodes++;
  if (!ray_bounds(&n->aabb, r, &nh) || nh.param > h->param) {
    if (g_walk_log)
      fprintf(stderr, "  node %u culled (param %.9g best %.9g start_in %d)\n", ni, nh.param, h->param,
              point_in_bounds(&n->aabb, r->start));
    return 0;
  }
  if (g_walk_log)
    fprintf(stderr, "  node %u visit leaf=%d nfaces=%u param %.9g box [%g %g %g]-[%g %g %g]\n", ni, n->leaf,
            n->nfaces, nh.param, n->aabb.mn.x, n->aabb.mn.y, n->aabb.mn.z, n->aabb.mx.x, n->aabb.mx.y, n->aabb.mx.z);
  int result = 0;
  if (n->leaf) {
    for (uint32_t i = 0; i < n->nfaces; i++) {
      coll_t th = no_coll();
      float bu = 0, bv = 0;
      uint32_t f = n->faces[i];
      const oface* face = &m->faces[f];
      if (st) st->tris++;
      if (ray_tri(m->verts[face->vi[0]], m->verts[face->vi[1]], m->verts[face->vi[2]], face->plane, r, &th, &bu, &bv)) {
        if (th.param < h->param) {
          h->param = th.param; h->point = th.point; h->normal = th.normal;
          h->face = f; h->bu = bu; h->bv = bv;
          result = 1;
        }
      }
    }
  } else {
    return trace_internal(m, ni, nh, r, h, st);
  }
  return result;
}

/* matrix4 (math/matrix4.h): column-major m[16] */
typedef struct m4 { float m[16]; } m4;
static m4 m4_identity(void) { m4 r; memset(&r, 0, sizeof(r)); r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1; return r; } /* :240-246 */
static m4 m4_mul(const m4* a, const m4* b) {                                                                       /* :529-546 */
  m4 o;
  for (int k = 0; k < 16; k++) {
    int r = k % 4, c = k / 4;
    o.m[k] = 0.0;
    for (int i = 0; i < 4; i++) o.m[k] += a->m[r + (i * 4)] * b->m[(c * 4) + i];
  }
  return o;
}
static m4 m4_rotation(float rad, v3 axis) {                                                                        /* :270-301 */
  float c = cosf(rad), s = sinf(rad), t = 1.0f - c;
  v3 a = norm3(axis);
  float x = a.x, y = a.y, z = a.z;
  m4 o;
  o.m[0] = t * x * x + c;  o.m[4] = t * x * y - s * z;  o.m[8] = t * x * z + s * y;   o.m[12] = 0.0f;
  o.m[1] = t * x * y + s * z;  o.m[5] = t * y * y + c;  o.m[9] = t * y * z - s * x;   o.m[13] = 0.0f;
  o.m[2] = t * x * z - s * y;  o.m[6] = t * y * z + s * x;  o.m[10] = t * z * z + c;  o.m[14] = 0.0f;
  o.m[3] = 0.0f; o.m[7] = 0.0f; o.m[11] = 0.0f; o.m[15] = 1.0f;
  return o;
}
static v3 m4_apply(const m4* M, v3 v) {                                                                            /* :552-557, w = 1 */
  const float* m = M->m;
  float w = 1.0f;
  return mk3(v.x * m[0] + v.y * m[4] + v.z * m[8] + w * m[12],
             v.x * m[1] + v.y * m[5] + v.z * m[9] + w * m[13],
             v.x * m[2] + v.y * m[6] + v.z * m[10] + w * m[14]);
}

/* MeshObject::MeshObject (mesh.cpp:168-275) + MeshBvh::BuildBvh (:117-152) */
static int mesh_build(omesh* m, const fs_mesh* d) {
  memset(m, 0, sizeof(*m));
  bounds_clear(&m->aabb);
  int need = 0;
  m4 T = m4_identity(), S = m4_identity(), R = m4_identity();
  if (d->translation[0] || d->translation[1] || d->translation[2]) {
    need = 1;
    T.m[12] = d->translation[0]; T.m[13] = d->translation[1]; T.m[14] = d->translation[2];
  }
  if (d->scale[0] || d->scale[1] || d->scale[2]) {
    need = 1;
    S.m[0] = d->scale[0]; S.m[5] = d->scale[1]; S.m[10] = d->scale[2];
  }
  if (d->rotation[0] || d->rotation[1] || d->rotation[2]) {
    need = 1;
    R = m4_rotation(d->rotation[3], mk3(d->rotation[0], d->rotation[1], d->rotation[2]));
  }
  if (need) { /* vertices_ is only filled when a transform is needed (mesh.cpp:211-221) */
    m4 TR = m4_mul(&T, &R);
    m4 M = m4_mul(&TR, &S);
    m->nv = d->num_positions;
    m->verts = (v3*)malloc(sizeof(v3) * (m->nv ? m->nv : 1));
    for (uint32_t i = 0; i < m->nv; i++) {
      v3 v = mk3(d->positions[3 * i], d->positions[3 * i + 1], d->positions[3 * i + 2]);
      v = m4_apply(&M, v);
      bounds_add(&m->aabb, v);
      m->verts[i] = v;
    }
  }
  m->nn = d->normals ? d->num_normals : 0;
  m->normals = (v3*)malloc(sizeof(v3) * (m->nn ? m->nn : 1));
  for (uint32_t i = 0; i < m->nn; i++) {
    v3 n = norm3(mk3(d->normals[3 * i], d->normals[3 * i + 1], d->normals[3 * i + 2]));
    if (d->invert_normals) n = scl3(n, (float)-1.0);
    m->normals[i] = n;
  }
  m->nt = d->texcoords ? d->num_texcoords : 0;
  m->tex = (float*)malloc(sizeof(float) * 2 * (m->nt ? m->nt : 1));
  if (m->nt) memcpy(m->tex, d->texcoords, sizeof(float) * 2 * m->nt);
  m->nf = d->num_triangles;
  m->faces = (oface*)malloc(sizeof(oface) * (m->nf ? m->nf : 1));
  for (uint32_t f = 0; f < m->nf; f++) {
    const int32_t* c = d->corners + 9 * f;
    oface* o = &m->faces[f];
    /* winding reversed (mesh.cpp:250-260) */
    for (int k = 0; k < 3; k++) {
      o->vi[k] = (uint32_t)c[3 * (2 - k) + 0];
      o->ni[k] = (uint32_t)c[3 * (2 - k) + 1];
      o->ti[k] = (uint32_t)c[3 * (2 - k) + 2];
      if (o->vi[k] >= d->num_positions) return FS_ERR_INVALID;
      if (m->nn && o->ni[k] >= m->nn) return FS_ERR_INVALID; /* .at() would throw (mesh.cpp:292) */
      if (m->nt && o->ti[k] >= m->nt) return FS_ERR_INVALID;
    }
    o->plane = mk4(0, 0, 0, 0);
  }
  /* BuildBvh: nothing is built without vertices or faces (mesh.cpp:119-121) */
  if (!m->nv || !m->nf) return 0;
  uint32_t root = new_node(m);
  bounds_t rb; bounds_clear(&rb);
  for (uint32_t i = 0; i < m->nv; i++) bounds_add(&rb, m->verts[i]);
  m->nodes[root].aabb = rb;
  for (uint32_t f = 0; f < m->nf; f++) {
    oface* o = &m->faces[f];
    if (o->plane.x == 0 && o->plane.y == 0 && o->plane.z == 0 && o->plane.w == 0) {
      v3 p0 = m->verts[o->vi[0]], p1 = m->verts[o->vi[1]], p2 = m->verts[o->vi[2]];
      v3 n = calc_normal(p0, p1, p2);
      o->plane = plane_np(n, p0);
    }
    node_add_face(&m->nodes[root], f);
  }
  subdivide(m, root);
  m->has_tree = 1;
  return 0;
}
static void mesh_free(omesh* m) {
  for (uint32_t i = 0; i < m->nnodes; i++) free(m->nodes[i].faces);
  free(m->nodes); free(m->verts); free(m->normals); free(m->tex); free(m->faces);
}

/* ------------------------------------------------------------------------ */
/* Scene objects (object.cpp) and Scene::Trace (scene.cpp:227-249)            */
/* ------------------------------------------------------------------------ */
typedef struct oobj {
  int kind, mat;
  v3 origin; float radius;          /* sphere, disc */
  v4 plane;                         /* plane, disc, quad */
  float hw, hh; v3 bitan, tan;      /* quad */
  v3 cverts[8]; v4 cplanes[6];      /* cuboid */
  int mesh;
  bounds_t bb;                      /* Object::GetBounds() (object.cpp, mesh.cpp:218) */
} oobj;

/* ObjectCollision (object.h:47-61); surface_texcoords default to vector2()
 * = (0,0) (vector2.cpp:8-11) and are only written by an improving object. */
typedef struct ocoll { float param; v3 point; v3 normal; int mat; int internal; float tu, tv; } ocoll;

typedef struct otex { float* rgb; uint32_t w, h; } otex; /* Texture (material.h:42-52) */

/* SceneBvhNode (scene.cpp:11-103): an object octree over the object list. */
typedef struct snode {
  bounds_t aabb;
  uint32_t depth, max_depth;
  int leaf;
  v4 split[3];
  int32_t child[8];
  uint32_t* objs;
  uint32_t nobjs, cap;
} snode;

struct oracle_scene {
  fs_material* mats; uint32_t nmats;
  int sky;
  oobj* objs; uint32_t nobjs;
  omesh* meshes; uint32_t nmeshes;
  v3* table; uint32_t ntable;
  otex* texs; uint32_t ntex;
  int tree_valid;                   /* Scene::is_tree_valid_ (scene.cpp:216-225) */
  snode* snodes; uint32_t nsnodes, capsnodes;
};

/* planar_map_texcoords (intersect.cpp:769-778) */
static inline void planar_map_tc(v3 p, v3 n, float* u, float* v) {
  if (n.x > n.y && n.x > n.z) { *u = p.y; *v = p.z; return; }
  if (n.y > n.x && n.y > n.z) { *u = p.x; *v = p.z; return; }
  *u = p.x; *v = p.y;
}
/* sphere_map_texcoords (intersect.cpp:780-784): the float atan2 overload,
 * BASE_PI is a float (base.h:80), the +0.5 / *0.5 / 1.0- terms are double. */
static inline void sphere_map(v3 n, float* u, float* v) {
  float uu = (float)((double)(atan2f(n.x, n.z) / (2 * REF_PI)) + 0.5);
  float vv = (float)((double)n.y * 0.5 + 0.5);
  *u = uu;
  *v = (float)(1.0 - (double)vv);
}
/* float -> uint32 as x86-64 compilers lower it (cvttss2si to 64 bits, low
 * half kept); NaN and |f| >= 2^63 give 0. */
static inline uint32_t f2u32_x64(float f) {
  if (!(f > -9.2233715e18f && f < 9.2233715e18f)) return 0;
  return (uint32_t)(uint64_t)(int64_t)f;
}
/* DiffuseMaterial::SampleDiffuse (material.cpp:108-126) */
static v3 sample_diffuse(const oracle_scene* sc, const fs_material* m, float tu, float tv) {
  v3 d = mk3(m->diffuse[0], m->diffuse[1], m->diffuse[2]);
  if (m->texture < 0) return d;
  const otex* t = &sc->texs[m->texture];
  if (!t->w || !t->h) return d;
  float fx = (tu * m->texture_scale * (float)t->w + 0.5f) - 1;
  float fy = (tv * m->texture_scale * (float)t->h + 0.5f) - 1;
  uint32_t x = f2u32_x64(fx), y = f2u32_x64(fy);
  x %= t->w;
  y %= t->h;
  uint32_t off = y * t->w * 3 + x * 3;
  return mk3(t->rgb[off], t->rgb[off + 1], t->rgb[off + 2]);
}

/* cube::operator=(bounds) + compute_planes (volume.cpp:234-247, 262-283) */
static void cube_planes(oobj* o) {
  v3* v = o->cverts;
  o->cplanes[0] = plane_3p(v[0], v[1], v[2]);
  o->cplanes[1] = plane_3p(v[6], v[5], v[4]);
  o->cplanes[2] = plane_3p(v[5], v[6], v[2]);
  o->cplanes[3] = plane_3p(v[7], v[4], v[0]);
  o->cplanes[4] = plane_3p(v[4], v[5], v[1]);
  o->cplanes[5] = plane_3p(v[6], v[7], v[3]);
}
static void cube_from_bounds(oobj* o, const bounds_t* b) {
  v3 a = b->mn, c = b->mx;
  o->cverts[0] = a;
  o->cverts[1] = mk3(c.x, a.y, a.z);
  o->cverts[2] = mk3(c.x, a.y, c.z);
  o->cverts[3] = mk3(a.x, a.y, c.z);
  o->cverts[4] = mk3(a.x, c.y, a.z);
  o->cverts[5] = mk3(c.x, c.y, a.z);
  o->cverts[6] = mk3(c.x, c.y, c.z);
  o->cverts[7] = mk3(a.x, c.y, c.z);
  cube_planes(o);
}

static int build_object(oobj* o, const fs_object* d) {
  memset(o, 0, sizeof(*o));
  o->kind = d->kind;
  o->mat = d->material;
  const float* a = d->a;
  switch (d->kind) {
    case FS_OBJ_SPHERE: /* object.cpp:17-21 */
      o->origin = mk3(a[0], a[1], a[2]); o->radius = a[3];
      break;
    case FS_OBJ_PLANE: /* object.cpp:38-57 */
      o->plane = mk4(a[0], a[1], a[2], a[3]);
      break;
    case FS_OBJ_DISC: /* object.cpp:75-95: the normal is not normalised */
      o->origin = mk3(a[0], a[1], a[2]);
      o->plane = plane_np(mk3(a[3], a[4], a[5]), o->origin);
      o->radius = a[6];
      break;
    case FS_OBJ_CUBOID: { /* object.cpp:115-124, volume.cpp:434-445 */
      v3 org = mk3(a[0], a[1], a[2]);
      v3 half = mk3((float)(a[3] * 0.5), (float)(a[4] * 0.5), (float)(a[5] * 0.5));
      bounds_t b; bounds_clear(&b);
      bounds_add(&b, sub3(org, half));
      bounds_add(&b, add3(org, half));
      cube_from_bounds(o, &b);
      if (d->rotate) {
        v3 axis = mk3(a[6], a[7], a[8]);
        float angle = a[9];
        bounds_t cb; bounds_clear(&cb);
        bounds_t aabb = b; /* cube::aabb_ = rhs */
        v3 center = bounds_center(&aabb);
        for (int i = 0; i < 8; i++) {
          v3 t = sub3(o->cverts[i], center);
          o->cverts[i] = add3(rotate3(t, angle, axis), center);
          bounds_add(&cb, o->cverts[i]);
        }
        cube_planes(o);
      }
      break;
    }
    case FS_OBJ_QUAD_ONWH: { /* object.cpp:167-189 */
      v3 nrm = norm3(mk3(a[3], a[4], a[5]));
      o->origin = mk3(a[0], a[1], a[2]);
      o->plane = plane_np(nrm, o->origin);
      o->hw = (float)(a[6] * 0.5);
      o->hh = (float)(a[7] * 0.5);
      o->bitan = cross3(nrm, mk3(0, 1, 0));
      o->tan = cross3(nrm, o->bitan);
      break;
    }
    case FS_OBJ_QUAD_PUV: { /* object.cpp:191-211 */
      v3 pos = mk3(a[0], a[1], a[2]), u = mk3(a[3], a[4], a[5]), v = mk3(a[6], a[7], a[8]);
      v3 nrm = norm3(cross3(u, v));
      o->plane = plane_np(nrm, pos);
      o->origin = add3(add3(pos, scl3(u, (float)0.5)), scl3(v, (float)0.5));
      o->hw = (float)(len3(u) * 0.5);
      o->hh = (float)(len3(v) * 0.5);
      o->bitan = norm3(u);
      o->tan = norm3(v);
      break;
    }
    case FS_OBJ_MESH:
      o->mesh = d->mesh;
      break;
    default:
      return FS_ERR_INVALID;
  }
  return 0;
}

/* Object::GetBounds() as each constructor accumulates it (object.cpp:17-21,
 * 38-57, 75-95, 115-124 + volume.cpp:434-445, 167-211; mesh.cpp:218). Bounds
 * are min/max accumulators, so only the points matter, not their order. */
static void object_bounds(oobj* o, const fs_object* d, const oracle_scene* sc) {
  const float* a = d->a;
  bounds_t* b = &o->bb;
  bounds_clear(b);
  const v3 up = mk3(0, 1, 0);
  const float eps = REF_EPSILON;
  switch (d->kind) {
    case FS_OBJ_SPHERE: {
      v3 rr = mk3(o->radius, o->radius, o->radius);
      bounds_add(b, add3(o->origin, rr));
      bounds_add(b, sub3(o->origin, rr));
      break;
    }
    case FS_OBJ_PLANE: {
      v3 n = mk3(a[0], a[1], a[2]);
      float distance = -a[3];
      v3 pop = scl3(n, distance);
      v3 right = cross3(n, up), forward = cross3(n, right);
      bounds_add(b, add3(pop, scl3(right, 1000.0f)));
      bounds_add(b, sub3(pop, scl3(right, 1000.0f)));
      bounds_add(b, add3(pop, scl3(forward, 1000.0f)));
      bounds_add(b, sub3(pop, scl3(forward, 1000.0f)));
      bounds_add(b, add3(pop, scl3(n, eps)));
      bounds_add(b, sub3(pop, scl3(n, eps)));
      break;
    }
    case FS_OBJ_DISC: {
      v3 n = mk3(a[3], a[4], a[5]);
      v3 right = cross3(n, up), forward = cross3(n, right);
      bounds_add(b, add3(o->origin, scl3(right, o->radius)));
      bounds_add(b, sub3(o->origin, scl3(right, o->radius)));
      bounds_add(b, add3(o->origin, scl3(forward, o->radius)));
      bounds_add(b, sub3(o->origin, scl3(forward, o->radius)));
      bounds_add(b, add3(o->origin, scl3(n, eps)));
      bounds_add(b, sub3(o->origin, scl3(n, eps)));
      break;
    }
    case FS_OBJ_CUBOID: /* cube::query_bounds(): the box, or its rotated corners (cube::rotate) */
      for (int i = 0; i < 8; i++) bounds_add(b, o->cverts[i]);
      break;
    case FS_OBJ_QUAD_ONWH: {
      v3 n = mk3(a[3], a[4], a[5]); /* the raw normal argument (object.cpp:187-188) */
      bounds_add(b, add3(o->origin, scl3(o->bitan, o->hw)));
      bounds_add(b, sub3(o->origin, scl3(o->bitan, o->hw)));
      bounds_add(b, add3(o->origin, scl3(o->tan, o->hh)));
      bounds_add(b, sub3(o->origin, scl3(o->tan, o->hh)));
      bounds_add(b, add3(o->origin, scl3(n, eps)));
      bounds_add(b, sub3(o->origin, scl3(n, eps)));
      break;
    }
    case FS_OBJ_QUAD_PUV: {
      v3 n = mk3(o->plane.x, o->plane.y, o->plane.z);
      bounds_add(b, add3(o->origin, scl3(n, eps)));
      bounds_add(b, sub3(o->origin, scl3(n, eps)));
      bounds_add(b, add3(o->origin, scl3(o->bitan, o->hw)));
      bounds_add(b, sub3(o->origin, scl3(o->bitan, o->hw)));
      bounds_add(b, add3(o->origin, scl3(o->tan, o->hh)));
      bounds_add(b, sub3(o->origin, scl3(o->tan, o->hh)));
      break;
    }
    case FS_OBJ_MESH:
      *b = sc->meshes[o->mesh].aabb;
      break;
  }
}

static inline void take(ocoll* h, const coll_t* c, int mat) {
  h->param = c->param; h->point = c->point; h->normal = c->normal; h->mat = mat;
  planar_map_tc(c->point, c->normal, &h->tu, &h->tv);  /* object.cpp:67-68, 106-107, 231-232 */
}

/* Object::Trace implementations (object.cpp:23-237, mesh.cpp:277-322) */
static int object_trace(const oracle_scene* sc, const oobj* o, const ray_t* r, ocoll* h, tstats* st) {
  coll_t t = no_coll();
  switch (o->kind) {
    case FS_OBJ_SPHERE:
      if (ray_sphere(o->origin, o->radius, r, &t) && t.param < h->param) {
        take(h, &t, o->mat);
        sphere_map(t.normal, &h->tu, &h->tv);  /* object.cpp:31 */
        return 1;
      }
      return 0;
    case FS_OBJ_PLANE:
      if (ray_plane(o->plane, r, &t) && t.param < h->param) { take(h, &t, o->mat); return 1; }
      return 0;
    case FS_OBJ_DISC:
      if (ray_plane(o->plane, r, &t)) {
        if (len3(sub3(o->origin, t.point)) <= o->radius && t.param < h->param) { take(h, &t, o->mat); return 1; }
      }
      return 0;
    case FS_OBJ_CUBOID: {
      int det = 0;
      for (uint32_t i = 0; i < 6; i++) {
        coll_t ph = no_coll();
        if (ray_plane(o->cplanes[i], r, &ph)) {
          if (ph.param < h->param) {
            int ok = 1;
            for (uint32_t j = 0; j < 6; j++) {
              if (i / 2 != j / 2) {
                if (plane_dist(o->cplanes[j], ph.point) > 0.0f) { ok = 0; break; }
              }
            }
            if (ok) {
              det = 1;
              take(h, &ph, o->mat);
              h->tu = h->tu * 0.1f;  /* object.cpp:157-158: planar map * 0.1f */
              h->tv = h->tv * 0.1f;
            }
          }
        }
      }
      return det;
    }
    case FS_OBJ_QUAD_ONWH:
    case FS_OBJ_QUAD_PUV:
      if (ray_plane(o->plane, r, &t)) {
        v3 ph = sub3(t.point, o->origin);
        float td = dot3(o->tan, ph);
        float bd = dot3(o->bitan, ph);
        if (fabsf(bd) > o->hw || fabsf(td) > o->hh) return 0;
        if (t.param < h->param) { take(h, &t, o->mat); return 1; }
      }
      return 0;
    case FS_OBJ_MESH: {
      const omesh* m = &sc->meshes[o->mesh];
      if (!m->has_tree) return 0;
      mcoll_t mc;
      mc.param = h->param; mc.point = mk3(0, 0, 0); mc.normal = mk3(0, 0, 0); mc.face = 0xFFFFFFFFu; mc.bu = mc.bv = 0;
      if (mesh_node_trace(m, 0, r, &mc, st)) {
        if (mc.param <= h->param) {
          h->param = mc.param; h->point = mc.point; h->normal = mc.normal; h->mat = o->mat;
          const oface* f = &m->faces[mc.face];
          if (m->nn) { /* triangle_interpolate_barycentric_coeff (intersect.cpp:131-144) */
            v3 n0 = m->normals[f->ni[0]], n1 = m->normals[f->ni[1]], n2 = m->normals[f->ni[2]];
            h->normal = add3(add3(n0, scl3(sub3(n1, n0), mc.bu)), scl3(sub3(n2, n0), mc.bv));
          }
          if (m->nt) { /* mesh.cpp:300-311: vector2 texcoords interpolated as vector3 */
            const float* t0 = &m->tex[2 * f->ti[0]];
            const float* t1 = &m->tex[2 * f->ti[1]];
            const float* t2 = &m->tex[2 * f->ti[2]];
            h->tu = (t0[0] + (t1[0] - t0[0]) * mc.bu) + (t2[0] - t0[0]) * mc.bv;
            h->tv = (t0[1] + (t1[1] - t0[1]) * mc.bu) + (t2[1] - t0[1]) * mc.bv;
          }
          return 1;
        }
      }
      return 0;
    }
  }
  return 0;
}

/* ---- the scene object octree (scene.cpp:11-133, bvh.h:108-231) ---------- */
static uint32_t new_snode(oracle_scene* sc) {
  if (sc->nsnodes == sc->capsnodes) {
    sc->capsnodes = sc->capsnodes ? 2 * sc->capsnodes : 16;
    sc->snodes = (snode*)realloc(sc->snodes, sizeof(snode) * sc->capsnodes);
  }
  snode* n = &sc->snodes[sc->nsnodes];
  memset(n, 0, sizeof(*n));
  n->leaf = 1;
  for (int i = 0; i < 8; i++) n->child[i] = -1;
  return sc->nsnodes++;
}
static void snode_add(snode* n, uint32_t i) {
  if (n->nobjs == n->cap) { n->cap = n->cap ? 2 * n->cap : 16; n->objs = (uint32_t*)realloc(n->objs, 4 * n->cap); }
  n->objs[n->nobjs++] = i;
}
/* bounds::query_volume (volume.cpp:123-126) */
static inline float bounds_volume(const bounds_t* b) {
  return (b->mx.x - b->mn.x) * (b->mx.y - b->mn.y) * (b->mx.z - b->mn.z);
}
/* bounds_intersect_bounds (intersect.cpp:26-43), BASE_PARAM_CHECK on (base.h:102):
 * a box of zero volume intersects nothing. */
static int bounds_vs_bounds(const bounds_t* a, const bounds_t* b) {
  if (0 == bounds_volume(a) || 0 == bounds_volume(b)) return 0;
  v3 ac = bounds_center(a), bc = bounds_center(b);
  v3 ae = sub3(a->mx, ac), be = sub3(b->mx, bc), d = sub3(bc, ac);
  return fabsf(d.x) <= (ae.x + be.x) && fabsf(d.y) <= (ae.y + be.y) && fabsf(d.z) <= (ae.z + be.z);
}
/* bvh.h:108-137 on a scene node */
static void sconfigure_children(oracle_scene* sc, uint32_t ni) {
  v3 mn = sc->snodes[ni].aabb.mn;
  v3 center = bounds_center(&sc->snodes[ni].aabb);
  v3 hx = sub3(mk3(center.x, mn.y, mn.z), mn);
  v3 hy = sub3(mk3(mn.x, center.y, mn.z), mn);
  v3 hz = sub3(mk3(mn.x, mn.y, center.z), mn);
  v3 span = add3(add3(hx, hy), hz);
  sc->snodes[ni].split[0] = plane_np(mk3(1, 0, 0), center);
  sc->snodes[ni].split[1] = plane_np(mk3(0, 1, 0), center);
  sc->snodes[ni].split[2] = plane_np(mk3(0, 0, 1), center);
  for (int i = 0; i < 8; i++) {
    uint32_t c = new_snode(sc); /* may realloc */
    snode* parent = &sc->snodes[ni];
    /* SceneBvhNode(parent) copies neither max_tree_depth_ nor anything but
     * depth/parent/objects (scene.cpp:20-25): the member is left
     * uninitialised, undefined behaviour. Convention here: the child inherits
     * its parent's value (0 or 1 give the same tree: see DESIGN.md §3b). */
    sc->snodes[c].depth = parent->depth + 1;
    sc->snodes[c].max_depth = parent->max_depth;
    parent->child[i] = (int32_t)c;
    v3 nmin = add3(add3(add3(mn, scl3(hx, (float)(i % 2))), scl3(hy, (float)(i >> 2))), scl3(hz, (float)((i % 4) >> 1)));
    v3 nmax = add3(nmin, span);
    bounds_t nb; bounds_clear(&nb);
    bounds_add(&nb, nmin);
    bounds_add(&nb, nmax);
    sc->snodes[c].aabb = nb;
  }
  sc->snodes[ni].leaf = 0;
}
/* SceneBvhNode::Subdivide (scene.cpp:33-74). min() is the two-argument min of
 * the Windows headers: uint32 against double compares and yields a double. */
static void ssubdivide(oracle_scene* sc, uint32_t ni) {
  snode* n = &sc->snodes[ni];
  if (n->depth >= n->max_depth) return;
  double a = (double)(uint32_t)(n->max_depth - n->depth);
  double b = (log((double)n->nobjs) / log(8.0) + 0.5f) - 2.0f;
  double mn = a < b ? a : b;
  if ((double)n->depth >= mn) return;
  if (n->nobjs > 2) { /* kMaxObjectCountPerNode (scene.cpp:9) */
    sconfigure_children(sc, ni);
    n = &sc->snodes[ni];
    for (uint32_t j = 0; j < n->nobjs; j++) {
      uint32_t oi = n->objs[j];
      for (int i = 0; i < 8; i++) {
        snode* c = &sc->snodes[sc->snodes[ni].child[i]];
        if (bounds_vs_bounds(&sc->objs[oi].bb, &c->aabb)) snode_add(c, oi);
      }
    }
    free(sc->snodes[ni].objs);
    sc->snodes[ni].objs = NULL;
    sc->snodes[ni].nobjs = sc->snodes[ni].cap = 0;
    for (int j = 0; j < 8; j++) ssubdivide(sc, (uint32_t)sc->snodes[ni].child[j]);
  }
}
/* Scene::Optimize (scene.cpp:216-225) + SceneBvh::BuildBvh (:105-126). */
static void scene_optimize(oracle_scene* sc) {
  sc->tree_valid = 0;
  int32_t ideal = (int32_t)((log((double)sc->nobjs) / log(8.0) + 0.5) - 2);
  if (!sc->nobjs || ideal <= 0) return;
  uint32_t root = new_snode(sc);
  sc->snodes[root].max_depth = 2; /* SceneBvhNode(data_source) default, kMaxSubdivisionDepth (scene.h:47) */
  bounds_t rb; bounds_clear(&rb);
  for (uint32_t i = 0; i < sc->nobjs; i++) { /* bounds += bounds (volume.cpp:193-224) */
    const bounds_t* ob = &sc->objs[i].bb;
    if (rb.count == 0) { rb.mn = ob->mn; rb.mx = ob->mx; rb.count = 1; continue; }
    rb.count++;
    if (ob->mx.x > rb.mx.x) rb.mx.x = ob->mx.x;
    if (ob->mx.y > rb.mx.y) rb.mx.y = ob->mx.y;
    if (ob->mx.z > rb.mx.z) rb.mx.z = ob->mx.z;
    if (ob->mn.x < rb.mn.x) rb.mn.x = ob->mn.x;
    if (ob->mn.y < rb.mn.y) rb.mn.y = ob->mn.y;
    if (ob->mn.z < rb.mn.z) rb.mn.z = ob->mn.z;
  }
  sc->snodes[root].aabb = rb;
  for (uint32_t i = 0; i < sc->nobjs; i++) snode_add(&sc->snodes[root], i);
  ssubdivide(sc, root);
  sc->tree_valid = 1;
}

static int snode_trace(const oracle_scene* sc, uint32_t ni, const ray_t* r, ocoll* h, tstats* st);
/* bvh.h:154-231 with SceneBvhNode children */
static int strace_internal(const oracle_scene* sc, uint32_t ni, coll_t node_hit, const ray_t* r, ocoll* h,
                           tstats* st) {
  const snode* n = &sc->snodes[ni];
  int result = 0, xh, yh, zh;
  uint32_t cn;
  ray_t it = *r;
  coll_t xi = no_coll(), yi = no_coll(), zi = no_coll();
  if (!point_in_bounds(&n->aabb, r->start)) {
    it.start = node_hit.point;
    v3 d = sub3(node_hit.point, bounds_center(&n->aabb));
    cn = ((d.x >= 0.0f) | ((d.z >= 0.0f) << 1) | ((d.y >= 0.0f) << 2)) & 0xFF;
    xh = ray_plane(n->split[0], &it, &xi);
    yh = ray_plane(n->split[1], &it, &yi);
    zh = ray_plane(n->split[2], &it, &zi);
  } else {
    v3 d = sub3(r->start, bounds_center(&n->aabb));
    cn = ((d.x >= 0.0f) | ((d.z >= 0.0f) << 1) | ((d.y >= 0.0f) << 2)) & 0xFF;
    xh = ray_plane(n->split[0], r, &xi);
    yh = ray_plane(n->split[1], r, &yi);
    zh = ray_plane(n->split[2], r, &zi);
    if (!xh && !yh && !zh) return snode_trace(sc, (uint32_t)n->child[cn], r, h, st);
  }
  for (uint32_t i = 0; i < 4; i++) {
    if (snode_trace(sc, (uint32_t)n->child[cn], r, h, st)) {
      result = 1;
      if (point_in_bounds(&sc->snodes[n->child[cn]].aabb, h->point)) break;
    }
    if (xh && xi.param < yi.param && xi.param < zi.param) {
      cn ^= 0x1; xh = 0; it.start = xi.point; xi.param = REF_INFINITY;
    } else if (yh && yi.param < zi.param && yi.param < xi.param) {
      cn ^= 0x4; yh = 0; it.start = yi.point; yi.param = REF_INFINITY;
    } else if (zh && zi.param < yi.param && zi.param < xi.param) {
      cn ^= 0x2; zh = 0; it.start = zi.point; zi.param = REF_INFINITY;
    } else {
      break;
    }
    if (!point_in_bounds(&n->aabb, it.start)) break;
  }
  return result;
}
/* SceneBvhNode::Trace (scene.cpp:76-103): a leaf traces its objects into ONE
 * fresh ObjectCollision (param 2, texcoords (0,0)) and copies it whole into
 * hit_info each time it beats hit_info's param. */
static int snode_trace(const oracle_scene* sc, uint32_t ni, const ray_t* r, ocoll* h, tstats* st) {
  const snode* n = &sc->snodes[ni];
  coll_t nh = no_coll();
  if (!ray_bounds(&n->aabb, r, &nh) || nh.param > h->param) return 0;
  if (!n->leaf) return strace_internal(sc, ni, nh, r, h, st);
  int result = 0;
  ocoll temp;
  temp.param = 2.0f; temp.point = mk3(0, 0, 0); temp.normal = mk3(0, 0, 0); temp.mat = -1; temp.internal = 0;
  temp.tu = temp.tv = 0.0f;
  for (uint32_t i = 0; i < n->nobjs; i++) {
    if (object_trace(sc, &sc->objs[n->objs[i]], r, &temp, st)) {
      if (temp.param < h->param) {
        *h = temp;
        result = 1;
      }
    }
  }
  return result;
}

static int scene_trace(const oracle_scene* sc, const ray_t* r, ocoll* h, tstats* st) {
  int det = 0;
  h->param = 2.0f; h->point = mk3(0, 0, 0); h->normal = mk3(0, 0, 0); h->mat = -1; h->internal = 0;
  h->tu = h->tv = 0.0f;
  if (sc->tree_valid)
    det = snode_trace(sc, 0, r, h, st); /* SceneBvh::Trace (scene.cpp:128-133) */
  else
    for (uint32_t i = 0; i < sc->nobjs; i++) det |= object_trace(sc, &sc->objs[i], r, h, st);
  v4 cp = plane_np(h->normal, h->point);
  if (plane_dist(cp, r->start) < 0.0) {
    h->normal = scl3(h->normal, (float)-1.0);
    h->internal = 1;
  }
  return det;
}

/* ------------------------------------------------------------------------ */
/* Materials (material.cpp) + normal_sphere (normal.cpp:29-105)               */
/* ------------------------------------------------------------------------ */
static inline v3 table_normal(const oracle_scene* sc, uint64_t* rng) {                  /* normal.cpp:29-34 */
  int64_t i = oracle_random_integer_range(rng, 0, (int32_t)sc->ntable - 1);
  return sc->table[i];
}
static v3 random_reflection(const oracle_scene* sc, v3 inc, v3 n, float solid, uint64_t* rng) { /* normal.cpp:36-62 */
  v3 rd = reflect3(inc, n);
  v3 dd = table_normal(sc, rng);
  if (dot3(dd, n) < 0.0) dd = scl3(dd, -1.0f);
  float interp = solid / REF_PI;
  v3 refl = norm3(add3(scl3(dd, interp), scl3(rd, (float)(1.0 - (double)interp))));
  if (dot3(refl, n) < 0.0) refl = scl3(refl, -1.0f);
  return refl;
}
static v3 random_refraction(const oracle_scene* sc, v3 inc, v3 n, float solid, float index, uint64_t* rng) { /* normal.cpp:64-105 */
  float half = solid / 2.0f;
  float delta = (oracle_random_float_range(rng, -1.0f, 1.0f)) * half;
  v3 refl;
  if (cmp_eps(index, 1.0f, REF_EPSILON)) refl = inc;
  else refl = refract3(inc, n, index);
  refl = norm3(refl);
  v3 axis = table_normal(sc, rng);
  if (dot3(axis, n) < 0.0) axis = scl3(axis, -1.0f);
  if (cmp_eps(solid, REF_PI, REF_EPSILON)) return axis;
  else if (cmp_eps(solid, 0.0f, REF_EPSILON)) return refl;
  return rotate3(refl, delta, axis);
}

static v3 mat_reflection(const oracle_scene* sc, const fs_material* m, v3 view, v3 n, uint64_t* rng) {
  switch (m->kind) {
    case FS_MAT_LIGHT: return mk3(0, 0, 0);                                                 /* material.cpp:38-41 */
    case FS_MAT_DIFFUSE: return random_reflection(sc, view, n, REF_PI, rng);               /* :102-105 */
    case FS_MAT_METAL: return random_reflection(sc, view, n, REF_PI * m->roughness, rng);  /* :155-158 */
    case FS_MAT_MIRROR: return reflect3(view, n);                                           /* :179-182 */
    case FS_MAT_GLASS:                                                                      /* :204-213 */
      if (oracle_random_float(rng) < m->reflectivity) return random_reflection(sc, view, n, REF_PI * m->frost, rng);
      return random_refraction(sc, view, n, REF_PI * m->frost, m->index, rng);
    case FS_MAT_LIQUID:                                                                     /* :234-240 */
      if (oracle_random_float(rng) < m->reflectivity) return reflect3(view, n);
      return refract3(view, n, m->index);
    case FS_MAT_CERAMIC:
    case FS_MAT_GLOW:                                                                       /* :262-270 */
      if (oracle_random_float(rng) < 0.1f) return random_reflection(sc, view, n, 0.0f, rng);
      return random_reflection(sc, view, n, (float)((double)REF_PI * (1.0 - (double)m->shininess)), rng);
    case FS_MAT_FOG: return view;                                                           /* :314-317 */
  }
  return mk3(0, 0, 0);
}
static int mat_will_use_indirect(const fs_material* m, v3 r, v3 n) {
  switch (m->kind) {
    case FS_MAT_LIGHT: return 0;                                                            /* :33-36 */
    case FS_MAT_DIFFUSE: return dot3(r, n) > K_DIFFUSE_CONTRIB;                             /* :97-100 */
    case FS_MAT_METAL: return m->roughness <= K_ROUGHNESS_THR || dot3(r, n) > K_DIFFUSE_CONTRIB; /* :149-153 */
    default: return 1;
  }
}
static inline v3 mat_diffuse(const fs_material* m) { return mk3(m->diffuse[0], m->diffuse[1], m->diffuse[2]); }

/* Material::Sample (material.cpp:43-339). SampleDiffuse is used by Light
 * (textured only), Diffuse, Metal, Ceramic and Glow. */
static v3 mat_sample(const oracle_scene* sc, const fs_material* m, uint32_t depth, v3 sample_pos, v3 view_dir,
                     v3 light_pos, v3 light_dir, v3 light_color, v3 n, float tu, float tv, uint64_t* rng) {
  switch (m->kind) {
    case FS_MAT_LIGHT:
      if (m->texture >= 0 && sc->texs[m->texture].w && sc->texs[m->texture].h) return sample_diffuse(sc, m, tu, tv);
      return mk3(m->emissive[0], m->emissive[1], m->emissive[2]);
    case FS_MAT_DIFFUSE: return scl3(mul3(sample_diffuse(sc, m, tu, tv), light_color), fmaxf(0.0f, dot3(n, light_dir)));
    case FS_MAT_METAL: {
      v3 d = sample_diffuse(sc, m, tu, tv);
      v3 dc = scl3(mul3(d, light_color), fmaxf(0.0f, dot3(n, light_dir)));
      v3 rc = mul3(d, light_color);
      return add3(scl3(dc, m->roughness), scl3(rc, (float)(1.0 - (double)m->roughness)));
    }
    case FS_MAT_MIRROR:
    case FS_MAT_GLASS:
    case FS_MAT_LIQUID: return mul3(light_color, mat_diffuse(m));
    case FS_MAT_CERAMIC:
    case FS_MAT_GLOW: {
      v3 h = norm3(add3(scl3(view_dir, (float)-1.0), light_dir));
      v3 dc = scl3(mul3(sample_diffuse(sc, m, tu, tv), light_color), fmaxf(0.0f, dot3(n, light_dir)));
      float ds = (float)pow((double)dot3(h, n), 50);
      v3 out = add3(scl3(light_color, ds), scl3(dc, (float)(1.0 - (double)ds)));
      if (m->kind == FS_MAT_GLOW) out = add3(out, mk3(m->glow[0], m->glow[1], m->glow[2]));
      return out;
    }
    case FS_MAT_FOG:
      if (0 == depth) {
        float dist = len3(sub3(sample_pos, light_pos));
        float x = (dist * dist) * m->density * 0.00005f;
        float mx = (0.0f < x) ? x : 0.0f;           /* global max template, material.cpp:333 */
        float th = (mx < 0.0f) ? 0.0f : (mx > 1.0f ? 1.0f : mx); /* saturate (scalar.h:183) */
        if (oracle_random_float(rng) < th) return mat_diffuse(m);
      }
      return light_color;
  }
  return mk3(0, 0, 0);
}

/* Scene::SampleSky (scene.cpp:157-162) with the scene.cpp:383 static cast:
 * a non-Light sky dispatches to its own Sample with black light -> 0 (Glow
 * keeps its glow term). A textured Light sky samples its map at the sphere
 * map of the normalised segment direction (engine.cpp:91-92). */
static v3 sample_sky(const oracle_scene* sc, v3 view) {
  const fs_material* m = &sc->mats[sc->sky];
  v3 out = mk3(0, 0, 0);
  if (m->kind == FS_MAT_LIGHT) {
    if (m->texture >= 0 && sc->texs[m->texture].w && sc->texs[m->texture].h) {
      float u, v;
      sphere_map(view, &u, &v);
      out = sample_diffuse(sc, m, u, v);
    } else {
      out = mk3(m->emissive[0], m->emissive[1], m->emissive[2]);
    }
  } else if (m->kind == FS_MAT_GLOW) {
    out = mk3(m->glow[0], m->glow[1], m->glow[2]);
  }
  return scl3(out, (float)3.0);
}

/* ------------------------------------------------------------------------ */
/* TraceStep (engine.cpp:59-159), recursive as in the reference               */
/* ------------------------------------------------------------------------ */
typedef struct tresult { v3 color, normal; float depth; uint64_t material_id; uint64_t ray_count; } tresult; /* frame.h:40-47 */

/* Diagnostics: when set, trace_step records each segment (start, stop, dir,
 * closest-hit param) here (oracle_trace_path; single-threaded use only). */
static float* g_seg_rec = NULL;
static uint32_t g_seg_n = 0, g_seg_max = 0;

static v3 trace_step(const oracle_scene* sc, const fs_camera* cam, const ray_t* r, v3* hit_position, uint32_t depth,
                     tresult* res, uint64_t* rng, tstats* st) {
  if (depth >= K_TRACE_DEPTH) return mk3(0, 0, 0);
  if (cam->fast_render && depth > 1) return mk3(1, 1, 1);
  res->ray_count = depth + 1;
  ocoll ci;
  if (st) st->segs++;
  const int det = scene_trace(sc, r, &ci, st);
  if (g_seg_rec && g_seg_n < g_seg_max) {
    float* q = g_seg_rec + 10 * g_seg_n++;
    q[0] = r->start.x; q[1] = r->start.y; q[2] = r->start.z;
    q[3] = r->stop.x; q[4] = r->stop.y; q[5] = r->stop.z;
    q[6] = r->dir.x; q[7] = r->dir.y; q[8] = r->dir.z;
    q[9] = det ? ci.param : 2.0f;
  }
  if (!det) {
    if (hit_position) *hit_position = r->stop;
    v3 out = sample_sky(sc, norm3(sub3(r->stop, r->start)));
    if (depth == 0) {
      res->color = out;
      res->normal = norm3(r->dir);
      res->material_id = sc->mats[sc->sky].id;
      res->depth = cam->z_far;
    }
    return out;
  }
  if (hit_position) *hit_position = ci.point;
  const fs_material* m = &sc->mats[ci.mat];
  v3 view = norm3(sub3(ci.point, r->start));
  v3 refl = mat_reflection(sc, m, view, ci.normal, rng);
  ray_t rr = mkray(ci.point, add3(ci.point, scl3(refl, cam->z_far)));
  v3 off = scl3(refl, K_STEP_OFFSET);
  rr.start = add3(rr.start, off);
  rr.dir = sub3(rr.dir, off);
  v3 ind_origin = mk3(0, 0, 0), ind = mk3(0, 0, 0);
  if (mat_will_use_indirect(m, refl, ci.normal)) {
    ind = trace_step(sc, cam, &rr, &ind_origin, depth + 1, res, rng, st);
  }
  v3 out = mat_sample(sc, m, depth, ci.point, view, ind_origin, refl, ind, ci.normal, ci.tu, ci.tv, rng);
  if (depth == 0) {
    if (len3(out) > 10.0 && m->kind == FS_MAT_LIGHT) out = scl3(norm3(out), (float)10.0);
    res->color = out;
    res->normal = ci.normal;
    res->material_id = m->id;
    res->depth = len3(sub3(r->start, ci.point));
  }
  return out;
}

/* Camera basis (engine.cpp:170-197), computed once per render. */
typedef struct cambasis {
  float width, height;
  v3 fwd, right, up, proj_origin;
  float hph, hpw;
  v4 focal;
} cambasis;
static void camera_basis(const fs_camera* c, uint32_t W, uint32_t H, cambasis* b) {
  b->width = (float)W;
  b->height = (float)H;
  float aspect = b->width / b->height;
  float fovy = (float)((double)(c->fov_y * REF_PI) / 180.0);
  float fovx = (float)(2.0 * atan(tan((double)fovy * 0.5) * (double)aspect));
  v3 origin = mk3(c->origin[0], c->origin[1], c->origin[2]);
  v3 target = mk3(c->target[0], c->target[1], c->target[2]);
  b->fwd = norm3(sub3(target, origin));
  b->right = norm3(cross3(mk3(0, 1, 0), b->fwd));
  b->up = norm3(cross3(b->fwd, b->right));
  b->hph = tanf(fovy * 0.5f) * c->z_far;
  b->hpw = tanf(fovx * 0.5f) * c->z_far;
  b->proj_origin = add3(origin, scl3(b->fwd, c->z_far));
  b->focal = plane_np(scl3(b->fwd, -1.0f), add3(origin, scl3(b->fwd, c->focal_depth)));
}
/* engine.cpp:210-244 */
static ray_t camera_ray(const fs_camera* c, const cambasis* b, float i, float j, uint64_t* rng) {
  float jx = (float)((double)oracle_random_float(rng) - 0.5);
  float jy = (float)((double)oracle_random_float(rng) - 0.5);
  float xd = (float)((double)b->hpw * ((double)((i + jx) / (b->width - 1)) * 2.0 - 1.0));
  float yd = (float)((double)b->hph * ((double)((j + jy) / (b->height - 1)) * 2.0 - 1.0));
  v3 stop = add3(add3(b->proj_origin, scl3(b->right, xd)), scl3(b->up, yd));
  v3 origin = mk3(c->origin[0], c->origin[1], c->origin[2]);
  ray_t r = mkray(origin, stop);
  if (c->aperture_size > 0.0) {
    coll_t fh = no_coll();
    if (ray_plane(b->focal, &r, &fh)) {
      float ang = (float)((double)oracle_random_float(rng) * 2.0 * (double)REF_PI);
      float mag = fsqrt(oracle_random_float(rng)) * c->aperture_size;
      v3 off = add3(scl3(scl3(b->right, cosf(ang)), mag), scl3(scl3(b->up, sinf(ang)), mag));
      r.start = add3(r.start, off);
      r.stop = add3(r.start, scl3(norm3(sub3(fh.point, r.start)), c->z_far));
      r.dir = sub3(r.stop, r.start);
    }
  }
  return r;
}

static void trace_pixel_sample(const oracle_scene* sc, const fs_camera* c, const cambasis* b, uint32_t W, uint32_t x,
                               uint32_t y, uint32_t s, uint64_t seed, tresult* res, tstats* st) {
  uint64_t rng = oracle_pixel_seed((uint64_t)y * W + x, s, seed);
  ray_t r = camera_ray(c, b, (float)x, (float)y, &rng);
  res->color = mk3(0, 0, 0); res->normal = mk3(0, 0, 0); res->depth = 0.0f; res->material_id = 0; res->ray_count = 0;
  trace_step(sc, c, &r, NULL, 0, res, &rng, st);
}

/* DisplayFrame::WritePixel (frame.cpp:53-85) */
static void write_pixel(oracle_frame* f, const tresult* res, uint32_t x, uint32_t y) {
  size_t p = (size_t)y * f->width + x;
  uint32_t* cnt = &f->count[p];
  float* mean = &f->color[3 * p];
  v3 np = add3(scl3(mk3(mean[0], mean[1], mean[2]), (float)(*cnt)), res->color);
  float dv = (float)(++(*cnt));
  if (!(0 == dv)) np = mk3(np.x / dv, np.y / dv, np.z / dv);
  mean[0] = np.x; mean[1] = np.y; mean[2] = np.z;
  float ch[3] = {np.x, np.y, np.z};
  for (int k = 0; k < 3; k++) {
    float s = ch[k] < 0.0f ? 0.0f : (ch[k] > 1.0f ? 1.0f : ch[k]);
    f->display[3 * p + k] = (uint8_t)(255.0 * pow((double)s, 1.0 / 2.2) + 0.5);
  }
  f->normal[3 * p] = res->normal.x; f->normal[3 * p + 1] = res->normal.y; f->normal[3 * p + 2] = res->normal.z;
  f->depth[p] = res->depth;
  f->material[p] = res->material_id;
}

/* ------------------------------------------------------------------------ */
/* Public API                                                                 */
/* ------------------------------------------------------------------------ */
int oracle_scene_create(const fs_scene_desc* d, oracle_scene** out) {
  if (!d || !out || !d->normal_table || d->num_materials == 0) return FS_ERR_INVALID;
  if (d->sky_material < 0 || (uint32_t)d->sky_material >= d->num_materials) return FS_ERR_INVALID;
  oracle_scene* s = (oracle_scene*)calloc(1, sizeof(oracle_scene));
  s->nmats = d->num_materials;
  s->mats = (fs_material*)malloc(sizeof(fs_material) * s->nmats);
  memcpy(s->mats, d->materials, sizeof(fs_material) * s->nmats);
  s->sky = d->sky_material;
  s->ntable = FS_NORMAL_TABLE_SIZE;
  s->table = (v3*)malloc(sizeof(v3) * s->ntable);
  for (uint32_t i = 0; i < s->ntable; i++)
    s->table[i] = mk3(d->normal_table[3 * i], d->normal_table[3 * i + 1], d->normal_table[3 * i + 2]);
  int rc = 0;
  s->ntex = d->num_textures;
  s->texs = (otex*)calloc(s->ntex ? s->ntex : 1, sizeof(otex));
  for (uint32_t i = 0; i < s->ntex; i++) {
    const fs_texture* t = &d->textures[i];
    size_t n = (size_t)t->width * t->height * 3;
    if (n && !t->rgb) rc = FS_ERR_INVALID;
    s->texs[i].w = t->width;
    s->texs[i].h = t->height;
    s->texs[i].rgb = (float*)malloc(sizeof(float) * (n ? n : 1));
    if (n && t->rgb) memcpy(s->texs[i].rgb, t->rgb, sizeof(float) * n);
  }
  for (uint32_t i = 0; i < s->nmats; i++)
    if (s->mats[i].texture >= 0 && (uint32_t)s->mats[i].texture >= s->ntex) rc = FS_ERR_INVALID;
  s->nmeshes = d->num_meshes;
  s->meshes = (omesh*)calloc(s->nmeshes ? s->nmeshes : 1, sizeof(omesh));
  for (uint32_t i = 0; i < s->nmeshes && !rc; i++) rc = mesh_build(&s->meshes[i], &d->meshes[i]);
  s->nobjs = d->num_objects;
  s->objs = (oobj*)calloc(s->nobjs ? s->nobjs : 1, sizeof(oobj));
  for (uint32_t i = 0; i < s->nobjs && !rc; i++) {
    const fs_object* o = &d->objects[i];
    if (o->material < 0 || (uint32_t)o->material >= s->nmats) rc = FS_ERR_INVALID;
    else if (o->kind == FS_OBJ_MESH && (o->mesh < 0 || (uint32_t)o->mesh >= s->nmeshes)) rc = FS_ERR_INVALID;
    else rc = build_object(&s->objs[i], o);
    if (!rc) object_bounds(&s->objs[i], o, s);
  }
  if (!rc && (d->flags & FS_SCENE_OPTIMIZED)) scene_optimize(s);
  if (rc) { oracle_scene_destroy(s); return rc; }
  *out = s;
  return 0;
}

void oracle_scene_destroy(oracle_scene* s) {
  if (!s) return;
  for (uint32_t i = 0; i < s->nmeshes; i++) mesh_free(&s->meshes[i]);
  for (uint32_t i = 0; i < s->ntex; i++) free(s->texs[i].rgb);
  for (uint32_t i = 0; i < s->nsnodes; i++) free(s->snodes[i].objs);
  free(s->snodes);
  free(s->texs); free(s->meshes); free(s->objs); free(s->mats); free(s->table); free(s);
}

int oracle_mesh_info(const oracle_scene* s, uint32_t mesh, uint32_t* nodes, uint64_t* refs, float* rb) {
  if (!s || mesh >= s->nmeshes) return FS_ERR_INVALID;
  const omesh* m = &s->meshes[mesh];
  uint64_t r = 0;
  for (uint32_t i = 0; i < m->nnodes; i++) r += m->nodes[i].nfaces;
  if (nodes) *nodes = m->nnodes;
  if (refs) *refs = r;
  if (rb && m->nnodes) {
    rb[0] = m->nodes[0].aabb.mn.x; rb[1] = m->nodes[0].aabb.mn.y; rb[2] = m->nodes[0].aabb.mn.z;
    rb[3] = m->nodes[0].aabb.mx.x; rb[4] = m->nodes[0].aabb.mx.y; rb[5] = m->nodes[0].aabb.mx.z;
  }
  return 0;
}
int oracle_mesh_vertex(const oracle_scene* s, uint32_t mesh, uint32_t i, float* out) {
  if (!s || mesh >= s->nmeshes || i >= s->meshes[mesh].nv) return FS_ERR_INVALID;
  v3 v = s->meshes[mesh].verts[i];
  out[0] = v.x; out[1] = v.y; out[2] = v.z;
  return 0;
}
int oracle_mesh_face_plane(const oracle_scene* s, uint32_t mesh, uint32_t f, float* out) {
  if (!s || mesh >= s->nmeshes || f >= s->meshes[mesh].nf) return FS_ERR_INVALID;
  v4 p = s->meshes[mesh].faces[f].plane;
  out[0] = p.x; out[1] = p.y; out[2] = p.z; out[3] = p.w;
  return 0;
}

typedef struct band_job {
  const oracle_scene* sc; const fs_camera* cam; const fs_render_params* prm; const cambasis* b;
  oracle_frame* f; uint32_t y0, y1; tstats st;
} band_job;

static int owns_pixel(const fs_render_params* p, uint32_t x, uint32_t y) {
  uint32_t ts = p->tile_size ? p->tile_size : 64, stride = p->tile_stride ? p->tile_stride : 1;
  uint32_t tiles_x = (p->width + ts - 1) / ts;
  uint32_t t = (y / ts) * tiles_x + (x / ts);
  return (t % stride) == p->tile_offset;
}

/* TraceThreadFunction loop (engine.cpp:205-250) over one band of rows. */
static void* band_worker(void* arg) {
  band_job* j = (band_job*)arg;
  for (uint32_t y = j->y0; y < j->y1; y++)
    for (uint32_t x = 0; x < j->prm->width; x++) {
      if (!owns_pixel(j->prm, x, y)) continue;
      for (uint32_t s = 0; s < j->prm->spp; s++) {
        tresult res;
        trace_pixel_sample(j->sc, j->cam, j->b, j->prm->width, x, y, j->prm->sample_base + s, j->prm->seed, &res, &j->st);
        write_pixel(j->f, &res, x, y);
      }
    }
  return NULL;
}

int oracle_render(const oracle_scene* sc, const fs_camera* cam, const fs_render_params* prm, int threads,
                  oracle_frame* f, oracle_stats* stats) {
  if (!sc || !cam || !prm || !f || f->width != prm->width || f->height != prm->height) return FS_ERR_INVALID;
  if (prm->width < 2 || prm->height < 2) return FS_ERR_INVALID;
  if (threads < 1) threads = 1;
  if ((uint32_t)threads > prm->height) threads = (int)prm->height;
  cambasis b;
  camera_basis(cam, prm->width, prm->height, &b);
  band_job* jobs = (band_job*)calloc((size_t)threads, sizeof(band_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  uint32_t bin = prm->height / (uint32_t)threads; /* engine.cpp:174, last band takes the rest (:200-202) */
  for (int k = 0; k < threads; k++) {
    jobs[k].sc = sc; jobs[k].cam = cam; jobs[k].prm = prm; jobs[k].b = &b; jobs[k].f = f;
    jobs[k].y0 = bin * (uint32_t)k;
    jobs[k].y1 = (k == threads - 1) ? prm->height : bin * (uint32_t)(k + 1);
  }
  for (int k = 1; k < threads; k++) pthread_create(&th[k], NULL, band_worker, &jobs[k]);
  band_worker(&jobs[0]);
  for (int k = 1; k < threads; k++) pthread_join(th[k], NULL);
  if (stats) {
    memset(stats, 0, sizeof(*stats));
    for (int k = 0; k < threads; k++) {
      stats->node_visits += jobs[k].st.nodes;
      stats->tri_tests += jobs[k].st.tris;
      stats->segments += jobs[k].st.segs;
    }
    uint64_t owned = 0;
    for (uint32_t y = 0; y < prm->height; y++)
      for (uint32_t x = 0; x < prm->width; x++) owned += owns_pixel(prm, x, y);
    stats->samples = owned * prm->spp;
  }
  free(jobs); free(th);
  return 0;
}

int oracle_trace_sample(const oracle_scene* sc, const fs_camera* cam, uint32_t W, uint32_t H, uint32_t x, uint32_t y,
                        uint32_t s, uint64_t seed, float color[3], float normal[3], float* depth, uint64_t* mid,
                        uint32_t* ray_count) {
  if (!sc || !cam || W < 2 || H < 2) return FS_ERR_INVALID;
  cambasis b;
  camera_basis(cam, W, H, &b);
  tresult res;
  trace_pixel_sample(sc, cam, &b, W, x, y, s, seed, &res, NULL);
  color[0] = res.color.x; color[1] = res.color.y; color[2] = res.color.z;
  if (normal) { normal[0] = res.normal.x; normal[1] = res.normal.y; normal[2] = res.normal.z; }
  if (depth) *depth = res.depth;
  if (mid) *mid = res.material_id;
  if (ray_count) *ray_count = (uint32_t)res.ray_count;
  return 0;
}

/* TraceRange (engine.cpp:298-329): the jitter-free ray through (x, y). */
int oracle_trace_range(const oracle_scene* sc, const fs_camera* cam, uint32_t W, uint32_t H, float x, float y,
                       float* distance) {
  if (!sc || !cam || !distance || W < 2 || H < 2) return FS_ERR_INVALID;
  cambasis b;
  camera_basis(cam, W, H, &b);
  float xd = (float)((double)b.hpw * ((double)(x / (b.width - 1)) * 2.0 - 1.0));
  float yd = (float)((double)b.hph * ((double)(y / (b.height - 1)) * 2.0 - 1.0));
  v3 origin = mk3(cam->origin[0], cam->origin[1], cam->origin[2]);
  v3 stop = add3(add3(b.proj_origin, scl3(b.right, xd)), scl3(b.up, yd));
  ray_t r = mkray(origin, stop);
  ocoll ci;
  if (!scene_trace(sc, &r, &ci, NULL)) {
    *distance = cam->z_far;
    return 0;
  }
  *distance = len3(sub3(ci.point, origin));
  return 0;
}

/* ---- KAT wrappers ---- */
float oracle_inv_sqrt(float f) { return inv_sqrt_ref(f); }
float oracle_fast_sqrt(float f) { return fsqrt(f); }
void oracle_normalize(const float* v, float* o) { v3 r = norm3(mk3(v[0], v[1], v[2])); o[0] = r.x; o[1] = r.y; o[2] = r.z; }
void oracle_reflect(const float* v, const float* n, float* o) {
  v3 r = reflect3(mk3(v[0], v[1], v[2]), mk3(n[0], n[1], n[2])); o[0] = r.x; o[1] = r.y; o[2] = r.z;
}
void oracle_refract(const float* v, const float* n, float index, float* o) {
  v3 r = refract3(mk3(v[0], v[1], v[2]), mk3(n[0], n[1], n[2]), index); o[0] = r.x; o[1] = r.y; o[2] = r.z;
}
void oracle_rotate(const float* v, float angle, const float* ax, float* o) {
  v3 r = rotate3(mk3(v[0], v[1], v[2]), angle, mk3(ax[0], ax[1], ax[2])); o[0] = r.x; o[1] = r.y; o[2] = r.z;
}
static void put_coll(const coll_t* c, float* out) {
  out[0] = c->param; out[1] = c->point.x; out[2] = c->point.y; out[3] = c->point.z;
  out[4] = c->normal.x; out[5] = c->normal.y; out[6] = c->normal.z;
}
int oracle_ray_sphere(const float* c, float r, const float* s, const float* e, float* out) {
  ray_t ry = mkray(mk3(s[0], s[1], s[2]), mk3(e[0], e[1], e[2]));
  coll_t h = no_coll();
  int hit = ray_sphere(mk3(c[0], c[1], c[2]), r, &ry, &h);
  put_coll(&h, out);
  return hit;
}
int oracle_ray_plane(const float* p, const float* s, const float* e, float* out) {
  ray_t ry = mkray(mk3(s[0], s[1], s[2]), mk3(e[0], e[1], e[2]));
  coll_t h = no_coll();
  int hit = ray_plane(mk4(p[0], p[1], p[2], p[3]), &ry, &h);
  put_coll(&h, out);
  return hit;
}
int oracle_ray_bounds(const float* mn, const float* mx, const float* s, const float* e, float* out) {
  ray_t ry = mkray(mk3(s[0], s[1], s[2]), mk3(e[0], e[1], e[2]));
  bounds_t b; b.mn = mk3(mn[0], mn[1], mn[2]); b.mx = mk3(mx[0], mx[1], mx[2]); b.count = 2;
  coll_t h = no_coll();
  int hit = ray_bounds(&b, &ry, &h);
  out[0] = h.param; out[1] = h.point.x; out[2] = h.point.y; out[3] = h.point.z;
  return hit;
}
int oracle_ray_triangle(const float* p1, const float* p2, const float* p3, const float* s, const float* e, float* out) {
  v3 a = mk3(p1[0], p1[1], p1[2]), b = mk3(p2[0], p2[1], p2[2]), c = mk3(p3[0], p3[1], p3[2]);
  v4 pl = plane_np(calc_normal(a, b, c), a); /* intersect.cpp:348-355 */
  ray_t ry = mkray(mk3(s[0], s[1], s[2]), mk3(e[0], e[1], e[2]));
  coll_t h = no_coll();
  float u = 0, v = 0;
  int hit = ray_tri(a, b, c, pl, &ry, &h, &u, &v);
  put_coll(&h, out);
  out[7] = u; out[8] = v;
  return hit;
}
int oracle_triangle_box(const float* p1, const float* p2, const float* p3, const float* mn, const float* mx) {
  bounds_t b; b.mn = mk3(mn[0], mn[1], mn[2]); b.mx = mk3(mx[0], mx[1], mx[2]); b.count = 2;
  return tri_vs_bounds(mk3(p1[0], p1[1], p1[2]), mk3(p2[0], p2[1], p2[2]), mk3(p3[0], p3[1], p3[2]), &b);
}

/* ------------------------------------------------------------------------ */
/* Diagnostics (tests/tools): the camera ray of one sample, and one object's  */
/* closest hit on a segment, through the octree or over every face.           */
/* ------------------------------------------------------------------------ */
int oracle_camera_ray(const fs_camera* cam, uint32_t W, uint32_t H, uint32_t x, uint32_t y, uint32_t sample,
                      uint64_t seed, float* start, float* stop) {
  cambasis b;
  camera_basis(cam, W, H, &b);
  uint64_t rng = oracle_pixel_seed((uint64_t)y * W + x, sample, seed);
  ray_t r = camera_ray(cam, &b, (float)x, (float)y, &rng);
  start[0] = r.start.x; start[1] = r.start.y; start[2] = r.start.z;
  stop[0] = r.stop.x; stop[1] = r.stop.y; stop[2] = r.stop.z;
  return 0;
}

int oracle_trace_path(const oracle_scene* sc, const fs_camera* cam, uint32_t W, uint32_t H, uint32_t x, uint32_t y,
                      uint32_t sample, uint64_t seed, float* segs, uint32_t max) {
  cambasis b;
  camera_basis(cam, W, H, &b);
  tresult res;
  g_seg_rec = segs;
  g_seg_n = 0;
  g_seg_max = max;
  trace_pixel_sample(sc, cam, &b, W, x, y, sample, seed, &res, NULL);
  g_seg_rec = NULL;
  return (int)g_seg_n;
}

int oracle_object_trace(const oracle_scene* sc, uint32_t obj, const float* s, const float* e, const float* dir,
                        float best, int brute, float* param, uint32_t* face) {
  if (obj >= sc->nobjs) return FS_ERR_INVALID;
  const oobj* o = &sc->objs[obj];
  ray_t r = mkray(mk3(s[0], s[1], s[2]), mk3(e[0], e[1], e[2]));
  r.dir = mk3(dir[0], dir[1], dir[2]);
  *face = 0xFFFFFFFFu;
  *param = best;
  if (o->kind != FS_OBJ_MESH || !brute) {
    ocoll h;
    memset(&h, 0, sizeof(h));
    h.param = best;
    if (o->kind == FS_OBJ_MESH) {
      const omesh* m = &sc->meshes[o->mesh];
      mcoll_t mc;
      mc.param = best; mc.point = mk3(0, 0, 0); mc.normal = mk3(0, 0, 0); mc.face = 0xFFFFFFFFu; mc.bu = mc.bv = 0;
      if (m->has_tree && mesh_node_trace(m, 0, &r, &mc, NULL)) { *param = mc.param; *face = mc.face; return 1; }
      return 0;
    }
    if (object_trace(sc, o, &r, &h, NULL)) { *param = h.param; return 1; }
    return 0;
  }
  const omesh* m = &sc->meshes[o->mesh];
  int hit = 0;
  for (uint32_t f = 0; f < m->nf; f++) {
    const oface* fc = &m->faces[f];
    coll_t th = no_coll();
    float bu, bv;
    if (ray_tri(m->verts[fc->vi[0]], m->verts[fc->vi[1]], m->verts[fc->vi[2]], fc->plane, &r, &th, &bu, &bv) &&
        th.param < *param) {
      *param = th.param; *face = f; hit = 1;
    }
  }
  return hit;
}

/* Which octree leaves hold face f of mesh m, and the leaf boxes (up to max). */
int oracle_face_leaves(const oracle_scene* sc, uint32_t mesh, uint32_t f, uint32_t* leaves, float* boxes, uint32_t max) {
  if (mesh >= sc->nmeshes) return -1;
  const omesh* m = &sc->meshes[mesh];
  uint32_t n = 0;
  for (uint32_t i = 0; i < m->nnodes; i++) {
    const onode* nd = &m->nodes[i];
    if (!nd->leaf) continue;
    for (uint32_t j = 0; j < nd->nfaces; j++)
      if (nd->faces[j] == f) {
        if (n < max) {
          leaves[n] = i;
          float* b = boxes + 6 * n;
          b[0] = nd->aabb.mn.x; b[1] = nd->aabb.mn.y; b[2] = nd->aabb.mn.z;
          b[3] = nd->aabb.mx.x; b[4] = nd->aabb.mx.y; b[5] = nd->aabb.mx.z;
        }
        n++;
      }
  }
  return (int)n;
}

/* The scene object octree (tests/tools): node i's box, leaf flag, children
 * and object list (up to max). Returns the node count (0: no tree). */
int oracle_scene_tree(const oracle_scene* sc, uint32_t i, float* box, int32_t* children, uint32_t* count,
                      uint32_t* objs, uint32_t max) {
  if (!sc->tree_valid) return 0;
  if (i < sc->nsnodes) {
    const snode* n = &sc->snodes[i];
    box[0] = n->aabb.mn.x; box[1] = n->aabb.mn.y; box[2] = n->aabb.mn.z;
    box[3] = n->aabb.mx.x; box[4] = n->aabb.mx.y; box[5] = n->aabb.mx.z;
    for (int k = 0; k < 8; k++) children[k] = n->leaf ? -1 : n->child[k];
    *count = n->nobjs;
    for (uint32_t k = 0; k < n->nobjs && k < max; k++) objs[k] = n->objs[k];
  }
  return (int)sc->nsnodes;
}
