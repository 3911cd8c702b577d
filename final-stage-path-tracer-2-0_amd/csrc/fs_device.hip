// fs_device.hip — gfx950 kernels of the path-trace hot path + the C ABI.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (bit parity with
// the reference needs unfused float ops; the BVH slab test, which only
// culls, uses explicit fmaf).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <algorithm>
#include <vector>

#include "fs_bvh_gpu.h"
#include "fs_kernels.h"
#include "fs_libm.h"
#include "fs_scene.h"
#include "fs_trace.h"

// Round 4 pruned the compile-time A/B switches of rounds 1-3 to the settings
// that ship (each one's measurement is in DESIGN_HISTORY.md §5 and §9): leaves tested
// one triangle per wave trip, no wave priority in the walks, slab constants
// once per segment, the integer-min exit clamp, the mesh-root cull as
// straight-line masks with error-bound margins and a straight-line exact path,
// object heads as one scalar load. The backward pass then left the megakernel
// for fold_paths over per-sample path records (DESIGN_HISTORY.md §10b). The only
// remaining switch is FS_PHASE_PROF (the profiling build, libfsgpu_prof.so).

namespace fs {
namespace dev {

struct Ray {
  f3 start, stop, dir;
};


// |dir| = 1 / inv_sqrt(dot(dir, dir)) (Quake, one Newton step: within 0.2 %
// of the true root for a finite positive argument) against kEpsilon = 1e-5:
// every dot in [1e-9, 1e30] gives |dir| >= 3.1e-5, so only the rest (zero,
// tiny, huge, infinite or NaN; an infinite dot makes inv_sqrt -inf and
// |dir| -0, zero-length) takes the reference's division.
__device__ __forceinline__ bool zero_len(const Ray& r) {  // trace.cpp:16
  const float d = dot(r.dir, r.dir);
  bool zl = false;
  if (!(d >= 1e-9f && d <= 1e30f)) zl = cmp_eps(fsqrt(d), 0.0f, kEpsilon);
  return zl;
}

// intersect.cpp:728-744 — two-sided plane test, t in [0,1].
__device__ __forceinline__ bool ray_plane(f4 p, const Ray& r, float& t, f3& point) {
  float ts = (p.x * r.dir.x + p.y * r.dir.y + p.z * r.dir.z);
  if (!cmp_eps(ts, 0.0f, kEpsilon)) {
    float ns = -(p.x * r.start.x + p.y * r.start.y + p.z * r.start.z + p.w);  // (...) * -1.0
    float tt = ns / ts;
    if (tt >= 0 && tt <= 1) {
      t = tt;
      point = r.start + r.dir * tt;
      return true;
    }
  }
  return false;
}

// intersect.cpp:421-488 (the zero-length branch never reports a hit through
// SphericalObject::Trace, object.cpp:23-36, so callers skip it).
__device__ __forceinline__ bool ray_sphere(f3 c, float radius, const Ray& r, float& t, f3& p, f3& n) {
  f3 o = r.start - c;
  float a = dot(r.dir, r.dir);
  float b = 2 * (dot(o, r.dir));
  float cc = dot(o, o) - radius * radius;
  float d = b * b - 4 * a * cc;
  if (d < 0) return false;
  float tt;
  if (length(o) <= radius)
    tt = (-b + fsqrt(d)) / (2 * a);
  else
    tt = (-b - fsqrt(d)) / (2 * a);
  if (tt < 0 || tt > 1) return false;
  t = tt;
  p = r.start + r.dir * tt;
  n = normalize(p - c);
  return true;
}

// intersect.cpp:490-529
__device__ __forceinline__ bool ref_slab(float s, float v, float mn, float mx, float& pn, float& pf) {
  if (cmp_eps(v, 0.0f, kEpsilon)) return !(s < mn || s > mx);
  float t1 = (mn - s) / v;
  float t2 = (mx - s) / v;
  if (t1 > t2) {
    float tt = t1;
    t1 = t2;
    t2 = tt;
  }
  if (t1 > pn) pn = t1;
  if (t2 < pf) pf = t2;
  return true;
}
// intersect.cpp:531-597 (only the parameter is consumed)
__device__ __forceinline__ bool ref_bounds_worker(f3 mn, f3 mx, f3 s, f3 e, float& param) {
  f3 v = e - s;
  float fnear = -kInfinity, ffar = kInfinity;
  // One slab per iteration, not unrolled: the three IEEE divisions stay
  // sequential and do not inflate the register footprint of the caller.
#pragma unroll 1
  for (int a = 0; a < 3; a++) {
    float sa = a == 0 ? s.x : (a == 1 ? s.y : s.z);
    float va = a == 0 ? v.x : (a == 1 ? v.y : v.z);
    float lo = a == 0 ? mn.x : (a == 1 ? mn.y : mn.z);
    float hi = a == 0 ? mx.x : (a == 1 ? mx.y : mx.z);
    if (!ref_slab(sa, va, lo, hi, fnear, ffar)) return false;
  }
  if (fnear > ffar) return false;
  if (ffar < 0 || fnear < 0 || fnear > 1) return false;
  param = fnear;
  return true;
}
__device__ __forceinline__ bool in_bounds(f3 mn, f3 mx, f3 p) {  // intersect.cpp:16-24
  return p.x >= mn.x && p.x <= mx.x && p.y >= mn.y && p.y <= mx.y && p.z >= mn.z && p.z <= mx.z;
}
// intersect.cpp:599-654
__device__ __forceinline__ bool ref_ray_bounds(f3 mn, f3 mx, const Ray& r, bool zl, float& param) {
  if (zl) {
    if (in_bounds(mn, mx, r.start)) {
      param = 0.0f;
      return true;
    }
    return false;
  }
  bool si = in_bounds(mn, mx, r.start);
  if (si && in_bounds(mn, mx, r.stop)) {
    param = 0.0f;
    return true;
  }
  // Reversed segment when the start is inside (:635-649); selected per
  // component so both cases share one worker instance.
  f3 a = mk3(si ? r.stop.x : r.start.x, si ? r.stop.y : r.start.y, si ? r.stop.z : r.start.z);
  f3 b = mk3(si ? r.start.x : r.stop.x, si ? r.start.y : r.stop.y, si ? r.start.z : r.stop.z);
  if (!ref_bounds_worker(mn, mx, a, b, param)) return false;
  if (si) param = 1.0f - param;
  return true;
}

// ray_intersect_bounds with its collision point (intersect.cpp:599-654): the
// point is start + (stop - start) * t of the (possibly reversed) segment.
__device__ __forceinline__ bool ref_bounds_hit(f3 mn, f3 mx, const Ray& r, bool zl, float& param, f3& point) {
  const bool si = in_bounds(mn, mx, r.start);
  if (zl || (si && in_bounds(mn, mx, r.stop))) {
    if (!si) return false;
    param = 0.0f;
    point = r.start;
    return true;
  }
  const f3 a = si ? r.stop : r.start, b = si ? r.start : r.stop;
  float t;
  if (!ref_bounds_worker(mn, mx, a, b, t)) return false;
  point = a + (b - a) * t;
  param = si ? 1.0f - t : t;
  return true;
}

// Per-ray slab constants of the BVH walks, computed once per segment. A
// zero-length ray (a point test at the leaves) walks with a 1e-20 slope per
// axis: every box that contains the start passes the slab test (entry <= 0 <=
// exit), so the cull stays a superset of the point-in-box test without a
// per-node branch. v_rcp (about 1 ulp) instead of IEEE division: the slab
// test is a conservative cull whose t margins (1e-6 absolute, 2e-6 relative)
// and box padding (4e-5 x scale) dwarf a 1e-7 relative error in the slopes.
struct Slopes {
  float ix, iy, iz, ox, oy, oz;
};
__device__ __forceinline__ Slopes walk_slopes(const Ray& r, bool zl, f3 dir) {
  const float tiny = 1e-20f;
  float dx = fabsf(dir.x) < tiny || zl ? copysignf(tiny, dir.x) : dir.x;
  float dy = fabsf(dir.y) < tiny || zl ? copysignf(tiny, dir.y) : dir.y;
  float dz = fabsf(dir.z) < tiny || zl ? copysignf(tiny, dir.z) : dir.z;
  Slopes sl;
  sl.ix = __builtin_amdgcn_rcpf(dx);
  sl.iy = __builtin_amdgcn_rcpf(dy);
  sl.iz = __builtin_amdgcn_rcpf(dz);
  sl.ox = -r.start.x * sl.ix;
  sl.oy = -r.start.y * sl.iy;
  sl.oz = -r.start.z * sl.iz;
  return sl;
}
__device__ __forceinline__ Slopes walk_slopes(const Ray& r, bool zl) { return walk_slopes(r, zl, r.dir); }
// The object loop's slopes: from the segment stop - start, the
// v of the reference's ray_intersect_bounds (intersect.cpp:531-597), so the
// mesh-root culls reuse them (the reversed segment's slopes are their
// negation, exactly); the walks cull with them as well (dir and stop - start
// differ by rounding only, far inside the walk's margins).
__device__ __forceinline__ Slopes seg_slopes(const Ray& r, bool zl) { return walk_slopes(r, zl, r.stop - r.start); }


// The mesh-root cull of MeshBvhNode::Trace (mesh.cpp:79-83): true when the
// reference would NOT skip the mesh (ray_intersect_bounds hits and its param
// is <= best). Exact by construction: slab times use the segment's v_rcp
// slopes (relative error < 2.4e-7 against the reference's IEEE quotient of the
// same difference), every sign test is exact, and a decision whose operands
// lie within the error bound's margins of its threshold is redone with the
// reference's divisions. The decisions are folded into straight-line masks
// (sure_miss) with one branch to the exact path. The reference's test
// fnear > ffar is max(n_i) > min(f_j); for i == j, n_i <= f_i holds exactly in
// both (the same product sorted, or one product twice for a flat box), so only
// a close cross-slab pair makes it unsure: a flat box (a wall, a quad light)
// hit away from its edges stays certain. A slab parallel to the segment
// (|v_i| < 1e-5, or a zero-length / tiny-substituted axis: a slope of
// magnitude >= 1e5) takes the reference's path.
// seg: the segment's slopes (seg_slopes); the reversed segment's are their
// negation exactly (e - s = -(stop - start)).
__device__ __forceinline__ bool ref_root_visit(f3 mn, f3 mx, const Ray& r, bool zl, float best, const Slopes& seg) {
  const bool si = in_bounds(mn, mx, r.start);
  const bool both = si && in_bounds(mn, mx, r.stop);
  const f3 s = mk3(si ? r.stop.x : r.start.x, si ? r.stop.y : r.start.y, si ? r.stop.z : r.start.z);
  const bool par = fmaxf(fmaxf(fabsf(seg.ix), fabsf(seg.iy)), fabsf(seg.iz)) >= 99990.0f;
  const float rx = si ? -seg.ix : seg.ix, ry = si ? -seg.iy : seg.iy, rz = si ? -seg.iz : seg.iz;
  const float ax = (mn.x - s.x) * rx, bx = (mx.x - s.x) * rx;
  const float ay = (mn.y - s.y) * ry, by = (mx.y - s.y) * ry;
  const float az = (mn.z - s.z) * rz, bz = (mx.z - s.z) * rz;
  const float n0 = fminf(ax, bx), f0 = fmaxf(ax, bx), n1 = fminf(ay, by), f1 = fmaxf(ay, by);
  const float n2 = fminf(az, bz), f2 = fmaxf(az, bz);
  const float fnear = fmaxf(fmaxf(n0, n1), n2), ffar = fminf(fminf(f0, f1), f2);
  // Margins from the error bound: a fast slab time is (lo - s) * rcp(v), the
  // reference's the IEEE quotient of the same difference; v_rcp is within
  // 1 ulp, so the two differ by at most 2.4e-7 |t| (1 ulp + two roundings).
  // fnear, ffar carry the same bound, 1 - fnear adds at most 6e-8 (exact for
  // fnear in [0.5, 2]); the margins below are 4x that.
  auto close = [](float a, float b) { return fabsf(a - b) <= 1e-6f * (fabsf(a) + fabsf(b)); };
  const float tol2 = 1e-6f, tol3 = 1e-6f * fabsf(fnear) + 1e-7f;
  bool u1 = close(fnear, ffar);
  if (u1) u1 = close(n0, f1) || close(n0, f2) || close(n1, f0) || close(n1, f2) || close(n2, f0) || close(n2, f1);
  const bool u2 = fabsf(fnear - 1.0f) <= tol2;
  const float np = si ? 1.0f - fnear : fnear;
  const bool u3 = fabsf(np - best) <= tol3;
  const bool sure_miss = !par && ((ffar < 0) || (fnear < 0) || (!u1 && fnear > ffar) || (!u2 && fnear > 1.0f) ||
                                  (!u3 && np > best));
  bool visit = zl ? si : (both || !sure_miss);
  if (!zl && !both && !sure_miss && (par || u1 || u2 || u3)) {
    // ray_intersect_bounds' worker (intersect.cpp:490-597) on the same
    // segment, straight-line: per slab the entry and exit times as the
    // reference's IEEE quotients ((lo - s) / v and (hi - s) / v, ordered by the
    // sign of v: division by a positive v is monotone, so the reference's
    // swap picks the same operand), a parallel slab (cmp_eps(v, 0)) as no
    // bound or, start outside it, a miss.
    const f3 e = mk3(si ? r.start.x : r.stop.x, si ? r.start.y : r.stop.y, si ? r.start.z : r.stop.z);
    const f3 w = e - s;
    auto entry = [&](float sa, float va, float lo, float hi) { return ((va > 0.0f ? lo : hi) - sa) / va; };
    float en = fmaxf(fmaxf(entry(s.x, w.x, mn.x, mx.x), entry(s.y, w.y, mn.y, mx.y)), entry(s.z, w.z, mn.z, mx.z));
    bool hit;
    if (par || u1) {  // the exit times (and a parallel slab's test) decide too
      bool out = false;
      float ex = kInfinity;
      en = -kInfinity;
      auto slab = [&](float sa, float va, float lo, float hi) {
        const bool p = cmp_eps(va, 0.0f, kEpsilon);
        out |= p && (sa < lo || sa > hi);
        en = p ? en : fmaxf(en, entry(sa, va, lo, hi));
        ex = p ? ex : fminf(ex, ((va > 0.0f ? hi : lo) - sa) / va);
      };
      slab(s.x, w.x, mn.x, mx.x);
      slab(s.y, w.y, mn.y, mx.y);
      slab(s.z, w.z, mn.z, mx.z);
      hit = !out && !(en > ex) && !(ex < 0 || en < 0 || en > 1);
    } else {  // only fnear ~ 1 or param ~ best was unsure: every other test is settled
      hit = !(en > 1);
    }
    const float pe = si ? 1.0f - en : en;
    visit = hit && !(pe > best);
  }
  return visit;
}

// intersect.cpp:96-129 + 146-177: planar map, then barycentrics.
__device__ __forceinline__ void planar_bary(f4 pl, f3 v0, f3 v1, f3 vp, float& u, float& v) {
  float ax = fabsf(pl.x), ay = fabsf(pl.y), az = fabsf(pl.z);
  if (ax >= ay) {
    if (ax >= az) {
      v0.x = v1.x = vp.x = 0;
    } else {
      v0.z = v1.z = vp.z = 0;
    }
  } else {
    if (ay >= az) {
      v0.y = v1.y = vp.y = 0;
    } else {
      v0.z = v1.z = vp.z = 0;
    }
  }
  float d00 = dot(v0, v0), d01 = dot(v0, v1), d02 = dot(v0, vp);
  float d11 = dot(v1, v1), d12 = dot(v1, vp);
  float inv = 1 / (d00 * d11 - d01 * d01);
  u = (d11 * d02 - d01 * d12) * inv;
  v = (d00 * d12 - d01 * d02) * inv;
}

// p1, v0, v1 hold the two components (a, b) the planar map keeps (fs_scene.h).
struct TriData {
  float p1a, p1b, v0a, v0b, v1a, v1b;
  float d00, d01, d11, inv;
  uint32_t axis, face;
  f4 pl;
  bool same_plane;  // small meshes: the previous slot's face has the same plane bits
};
__device__ __forceinline__ TriData unpack_tri(float4 a, float4 b, float4 c, float4 d) {
  TriData t;
  t.pl = mk4(a.x, a.y, a.z, a.w);
  t.p1a = b.x;
  t.p1b = b.y;
  t.v0a = b.z;
  t.v0b = b.w;
  t.v1a = c.x;
  t.v1b = c.y;
  const uint32_t fa = __float_as_uint(c.z);
  t.face = fa & 0x3FFFFFFFu;
  t.axis = fa >> 30;
  t.same_plane = (__float_as_uint(c.w) & kSamePlaneBit) != 0;
  t.d00 = d.x;
  t.d01 = d.y;
  t.d11 = d.z;
  t.inv = d.w;
  return t;
}
__device__ __forceinline__ TriData load_tri(const DevTri* __restrict__ T, uint32_t i) {
  const float4* q = reinterpret_cast<const float4*>(T + i);
  return unpack_tri(q[0], q[1], q[2], q[3]);
}
// A triangle at a wave-uniform index (small meshes): read through the
// constant address space, so the backend uses scalar loads into SGPRs.
typedef const __attribute__((address_space(4))) float* ConstF;
__device__ __forceinline__ TriData load_tri_uniform(const DevTri* T, uint32_t i) {
  ConstF f = (ConstF)(T + i);
  return unpack_tri(make_float4(f[0], f[1], f[2], f[3]), make_float4(f[4], f[5], f[6], f[7]),
                    make_float4(f[8], f[9], f[10], f[11]), make_float4(f[12], f[13], f[14], f[15]));
}
__device__ __forceinline__ uint32_t tri_face(const DevTri* __restrict__ T, uint32_t i) {
  return T[i].face_axis & 0x3FFFFFFFu;
}
// intersect.cpp:146-177 with the triangle-only terms precomputed. The
// reference's 3-term dot products over the planar-mapped vectors carry an
// exact +0 term for the zeroed axis: ((0 + A) + B) for axis x, ((A + 0) + B)
// for y and ((A + B) + 0) for z. All three equal (A + B) + 0 bit for bit: each
// is A + B except that none gives -0 (-0 arises only from -0 + -0, and an
// exact +0 term turns it into +0 in any position; NaN stays NaN), so the
// axis selects no operand order.
__device__ __forceinline__ void bary_pre(const TriData& T, f3 pt, float& u, float& v) {
  const bool az = T.axis == 2;
  const float pa = T.axis == 0 ? pt.y : pt.x, pb = az ? pt.y : pt.z;
  const float va = pa - T.p1a, vb = pb - T.p1b;
  const float d02 = (T.v0a * va + T.v0b * vb) + 0.0f;
  const float d12 = (T.v1a * va + T.v1b * vb) + 0.0f;
  u = (T.d11 * d02 - T.d01 * d12) * T.inv;
  v = (T.d00 * d12 - T.d01 * d02) * T.inv;
}

// intersect.cpp:357-419 (non-zero-length branch)
__device__ __forceinline__ bool ray_tri(const TriData& T, const Ray& r, float& t, f3& p, float& u, float& v) {
  float tt;
  f3 pp;
  if (!ray_plane(T.pl, r, tt, pp)) return false;
  float uu, vv;
  bary_pre(T, pp, uu, vv);
  if ((uu >= 0) && (vv >= 0) && (uu + vv <= 1)) {
    t = tt;
    p = pp;
    u = uu;
    v = vv;
    return true;
  }
  return false;
}
// intersect.cpp:320-346 with point_in_plane's vector4 promotion (:45-47):
// the live test is n.p + w + w.
__device__ __forceinline__ bool point_in_tri(const TriData& T, f3 pt, float& u, float& v) {
  float d4 = T.pl.x * pt.x + T.pl.y * pt.y + T.pl.z * pt.z + T.pl.w * 1.0f;
  if (!cmp_eps(d4 + T.pl.w, 0.0f, kEpsilon)) return false;
  float uu, vv;
  bary_pre(T, pt, uu, vv);
  if ((uu >= 0) && (vv >= 0) && (uu + vv <= 1)) {
    u = uu;
    v = vv;
    return true;
  }
  return false;
}

template <bool COUNT>
struct Tally {
  uint32_t nodes = 0, tris = 0, prims = 0;
  uint32_t objs = 0;  // object records read (wave-uniform loads: counted once per wave)
  uint32_t utris = 0;  // small-mesh triangle records read (wave-uniform loads: once per wave)
  uint32_t lane_objs = 0;  // object records read at a per-lane index (object octree): once per lane
#ifdef FS_PHASE_PROF
  // wave-level loop trips, counted by the first active lane of each trip
  uint32_t node_trips = 0, leaf_trips = 0, lane_nodes = 0, lane_leaves = 0;
#endif
};
#ifdef FS_PHASE_PROF
#define FS_WAVE_TRIP(field)                                                            \
  do {                                                                                 \
    if (threadIdx.x == (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x)) field++; \
  } while (0)
#else
#define FS_WAVE_TRIP(field) \
  do {                      \
  } while (0)
#endif

// normal_sphere (normal.cpp:29-105)
__device__ __forceinline__ f3 table_normal(const DevScene& S, uint64_t& rng) {
  float4 q = S.table[rng_table_index(rng)];
  return mk3(q.x, q.y, q.z);
}
__device__ __forceinline__ f3 random_reflection(const DevScene& S, f3 inc, f3 n, float solid, uint64_t& rng) {
  f3 rd = reflect(inc, n);
  f3 dd = table_normal(S, rng);
  if (dot(dd, n) < 0.0f) dd = dd * -1.0f;
  float interp = solid / kPi;
  f3 refl = normalize(dd * interp + rd * (float)(1.0 - (double)interp));
  if (dot(refl, n) < 0.0f) refl = refl * -1.0f;
  return refl;
}
// TRIG: the host libm's cosf/sinf bits (fs_libm.h); without it ocml's, in
// kernels whose scenes never reach the rotation (no frosted glass) and whose
// registers are then spent as before (the restatement's double constants cost
// C3/C4 1 %, profiles/r06/ab_trig.log).
template <bool TRIG>
__device__ __forceinline__ f3 random_refraction(const DevScene& S, f3 inc, f3 n, float solid, float index,
                                                uint64_t& rng) {
  float half = solid / 2.0f;
  float delta = (rng_float_range(rng, -1.0f, 1.0f)) * half;
  f3 refl = cmp_eps(index, 1.0f, kEpsilon) ? inc : refract(inc, n, index);
  refl = normalize(refl);
  f3 axis = table_normal(S, rng);
  if (dot(axis, n) < 0.0f) axis = axis * -1.0f;
  if (cmp_eps(solid, kPi, kEpsilon)) return axis;
  if (cmp_eps(solid, 0.0f, kEpsilon)) return refl;
  float sn, cs;
  if (TRIG) {
    libm::sincosf(delta, &sn, &cs);  // the host libm's cosf / sinf bits (fs_libm.h)
  } else {
    cs = cosf(delta);
    sn = sinf(delta);
  }
  return rotate(refl, cs, sn, axis);
}

// Ceramic's specular term (float)pow((double)(h.n), 50) (material.cpp:280).
// Computed by repeated squaring in double: within ~1e-15 relative of the
// correctly rounded pow, so the float result is the same except when the
// double lies that close to a float rounding tie (never seen in the tests).
__device__ __forceinline__ float pow50(float xf) {
  double x = xf, x2 = x * x, x4 = x2 * x2, x8 = x4 * x4, x16 = x8 * x8, x32 = x16 * x16;
  return (float)(x32 * x16 * x2);
}

// Material::Reflection (material.cpp:28-339). Each kind either scatters
// around a table normal with its solid angle (Diffuse pi, Metal pi *
// roughness, Glass pi * frost on reflection, Ceramic and Glow 0 or
// pi * (1 - shininess)), mirrors, refracts, refracts frosted, passes the
// view on (Fog) or returns zero (Light); Glass, Liquid, Ceramic and Glow
// first draw one uniform number and pick between two of these. The host
// precomputes per material the threshold of that draw, both choices and
// their solid angles with the reference's float / double operations
// (DevScene::rmat), so the per-lane kind switch is one 16-B load, a draw on
// the lanes whose material draws, and two selects; the lanes of a mixed
// wave then run ONE random_reflection together, with each kind's RNG draws
// in their order.
template <bool TRIG>
__device__ __forceinline__ f3 mat_reflection(const DevScene& S, const fs_material& m, uint32_t mi, f3 view, f3 n,
                                             uint64_t& rng) {
  const float4 rm = S.rmat[mi];
  const uint32_t bits = __float_as_uint(rm.w);
  float u = 0.0f;
  if (bits & kReflDraws) u = rng_float(rng);
  const bool a = u < rm.x;
  const uint32_t mode = a ? (bits & 0xFu) : ((bits >> 4) & 0xFu);
  const float solid = a ? rm.y : rm.z;
  if (mode == kReflScatter) return random_reflection(S, view, n, solid, rng);
  if (mode == kReflMirror) return reflect(view, n);
  if (mode == kReflRefract) return refract(view, n, m.index);
  if (mode == kReflFrosted) return random_refraction<TRIG>(S, view, n, kPi * m.frost, m.index, rng);
  if (mode == kReflView) return view;
  return mk3(0, 0, 0);
}
__device__ __forceinline__ bool mat_will_use(const fs_material& m, f3 r, f3 n) {
  switch (m.kind) {
    case FS_MAT_LIGHT:
      return false;
    case FS_MAT_DIFFUSE:
      return dot(r, n) > kDiffuseContrib;
    case FS_MAT_METAL:
      return m.roughness <= kRoughnessThr || dot(r, n) > kDiffuseContrib;
    default:
      return true;
  }
}

struct Aov {
  f3 normal;
  float depth;
  uint64_t id;
};

// base + a 32-bit byte offset: lets the compiler use the SGPR-base + 32-bit
// VGPR-offset addressing form instead of keeping a 64-bit pointer per lane.
template <class T>
__device__ __forceinline__ T* at_byte(T* base, uint32_t off) {
  using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  return reinterpret_cast<T*>(reinterpret_cast<B*>(base) + off);
}

// The material index of every bounce of a path, for the backward pass. Up to
// 255 materials: 8-bit ids packed in two registers, stored with the path's
// end (PathRecords::mats). More (MMAT): the forward pass stores one u32 per
// bounce in the record's id plane and keeps only level 0's here, so scenes
// with any number of materials render (scene.cpp:251-310 has no limit) and
// the common case keeps its registers.
template <bool MMAT>
struct MatTrail {
  uint32_t lo = 0, hi = 0;
  __device__ __forceinline__ void reset() { lo = hi = 0; }
  __device__ __forceinline__ void set(uint32_t k, uint32_t mi) {
    if (MMAT) {
      if (k == 0) lo = mi;
    } else if (k < 4) {
      lo |= mi << (8 * k);
    } else {
      hi |= mi << (8 * (k - 4));
    }
  }
  __device__ __forceinline__ uint32_t get0() const { return MMAT ? lo : lo & 0xFFu; }
};

// engine.cpp:210-244: jittered ray through the pixel, optional thin lens.
template <bool TRIG>
__device__ __forceinline__ Ray camera_ray(const DevCamera& C, float fx, float fy, uint64_t& rng) {
  float jx = (float)((double)rng_float(rng) - 0.5);
  float jy = (float)((double)rng_float(rng) - 0.5);
  float xd = (float)((double)C.hpw * ((double)((fx + jx) / (C.width - 1)) * 2.0 - 1.0));
  float yd = (float)((double)C.hph * ((double)((fy + jy) / (C.height - 1)) * 2.0 - 1.0));
  f3 stop = C.proj_origin + C.right * xd + C.up * yd;
  Ray r;
  r.start = C.origin;
  r.stop = stop;
  r.dir = stop - C.origin;
  if (C.aperture > 0.0f) {
    float ft;
    f3 fp;
    if (ray_plane(C.focal, r, ft, fp)) {
      float ang = (float)((double)rng_float(rng) * 2.0 * (double)kPi);
      float mag = fsqrt(rng_float(rng)) * C.aperture;
      float sn, cs;
      if (TRIG) {
        libm::sincosf(ang, &sn, &cs);  // the host libm's cosf / sinf bits (fs_libm.h)
      } else {  // never reached: the host picks TRIG kernels for cameras with a lens
        cs = cosf(ang);
        sn = sinf(ang);
      }
      f3 off = C.right * cs * mag + C.up * sn * mag;
      r.start = r.start + off;
      r.stop = r.start + normalize(fp - r.start) * C.z_far;
      r.dir = r.stop - r.start;
    }
  }

  return r;
}

// A path-record store. Records are written once and read back only by
// fold_paths: in the parked-walk kernel non-temporal stores keep them from
// displacing the scene in the L2 (C4 +0.4 %; in the other kernels the
// non-temporal form raised the spills, NOWALK 40 -> 68 B/lane, so they store
// plainly; non-temporal triangle loads lost 8-15 %: leaves are re-read by
// neighbouring rays; profiles/r04/ab_nontemporal.log).
template <bool NT, class T>
__device__ __forceinline__ void rec_store(T* p, T v) {
  if constexpr (NT) {
    if constexpr (sizeof(T) == 16) {
      typedef float v4f __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(*reinterpret_cast<const v4f*>(&v), reinterpret_cast<v4f*>(p));
    } else if constexpr (sizeof(T) == 8) {
      typedef uint32_t v2u __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(*reinterpret_cast<const v2u*>(&v), reinterpret_cast<v2u*>(p));
    } else {
      __builtin_nontemporal_store(v, p);
    }
  } else {
    *p = v;
  }
}

// The path record of sample `slot` (its low bits: s * 64 + 8 * py + px) of
// the block whose record row is `row`.
__device__ __forceinline__ uint64_t rec_index(const Launch& P, uint32_t row, uint32_t slot) {
  return (uint64_t)row * (P.spp * kBlock) + (slot & 0x3FFFFFFFu);
}

// FogMaterial::Sample's draw at level 0 (material.cpp:319-339): true when
// the diffuse colour replaces the incoming light. p0, lp0: the path's first
// two hit points (the second is the segment's end on a miss).
__device__ __forceinline__ bool fog_takes_diffuse(const fs_material& m, f3 p0, f3 lp0, uint64_t& rng) {
  float dist = length(p0 - lp0);
  float x = (dist * dist) * m.density * 0.00005f;
  float mx = (0.0f < x) ? x : 0.0f;
  float th = (mx < 0.0f) ? 0.0f : (mx > 1.0f ? 1.0f : mx);
  return rng_float(rng) < th;
}

// The backward pass of one path (engine.cpp:141-156): Material::Sample of
// levels top .. 0 in the order the TraceStep recursion returns. L enters as
// the radiance of level top + 1; c holds the path's c values (levels
// <= top), M the backward-pass material table (DevScene::umat, in LDS or
// global memory). Levels run unrolled over wave-uniform indices (each lane
// applies the levels <= its top), each kind's operations in the reference's
// order (a per-kind switch: +0.2-0.3 % over one straight-line select
// sequence of every kind, profiles/r04/ab_fold_switch.log):
//   Diffuse  (sd*L)*c                     Metal  ((sd*L)*c)*r + (sd*L)*(1-r)
//   Mirror/Glass/Liquid  L*dif            Ceramic  L*ds + ((sd*L)*c)*(1-ds) (+glow)
//   Light  emissive (its texel when mapped), Fog  L or, at level 0, dif when
//   the forward pass's draw said so (kRecFogDif)
template <bool TEX, bool MMAT, class MatPtr>
__device__ __forceinline__ f3 unwind_path(MatPtr M, const PathRecords& R, uint64_t q, f3 L, int top, bool fog_dif,
                                          uint2 packed, const float (&c)[kMaxDepth]) {
  int32_t kind0 = 0;
#pragma unroll
  for (int k = (int)kMaxDepth - 1; k >= 0; --k) {
    if (k > top) continue;
    const uint32_t id = MMAT ? R.mat[(uint64_t)k * R.n + q]
                             : ((k < 4 ? (packed.x >> (8 * k)) : (packed.y >> (8 * (k - 4)))) & 0xFFu);
    const float4 m0 = M[3 * id], m1 = M[3 * id + 1];
    const int32_t kk = __float_as_int(m0.x);
    const f3 dk = mk3(m0.y, m0.z, m0.w);
    f3 sd = dk;  // SampleDiffuse (material.cpp:108-126)
    bool mapped = false;
    if (TEX) {
      mapped = __float_as_int(M[3 * id + 2].w) >= 0;
      if (mapped) {
        const float4 tx = R.tex[(uint64_t)k * R.n + q];
        sd = mk3(tx.x, tx.y, tx.z);
      }
    }
    f3 out = L;
    switch (kk) {
      case FS_MAT_LIGHT:
        out = (TEX && mapped) ? sd : mk3(m1.y, m1.z, m1.w);
        break;
      case FS_MAT_DIFFUSE:
        out = (sd * L) * c[k];
        break;
      case FS_MAT_METAL: {
        const f3 dc = (sd * L) * c[k];
        const f3 rc = sd * L;
        out = dc * m1.x + rc * (float)(1.0 - (double)m1.x);
        break;
      }
      case FS_MAT_MIRROR:
      case FS_MAT_GLASS:
      case FS_MAT_LIQUID:
        out = L * dk;
        break;
      case FS_MAT_CERAMIC:
      case FS_MAT_GLOW: {
        const float ds = R.ds[(uint64_t)k * R.n + q];
        const f3 dc = (sd * L) * c[k];
        out = L * ds + dc * (float)(1.0 - (double)ds);
        if (kk == FS_MAT_GLOW) {
          const float4 m2 = M[3 * id + 2];
          out = out + mk3(m2.x, m2.y, m2.z);
        }
        break;
      }
      default:
        if (k == 0 && fog_dif) out = dk;
        break;
    }
    L = out;
    if (k == 0) kind0 = kk;
  }
  // engine.cpp:147-151 (level 0's kind)
  if (top >= 0 && length(L) > 10.0f && kind0 == FS_MAT_LIGHT) L = normalize(L) * (float)10.0;
  return L;
}

__device__ __forceinline__ uint8_t gamma8(float c) {  // frame.cpp:67-71
  float s = c < 0.0f ? 0.0f : (c > 1.0f ? 1.0f : c);
  return (uint8_t)(255.0 * pow((double)s, 1.0 / 2.2) + 0.5);
}

// Object records are wave-uniform and never written by a kernel: reading
// them through the constant address space lets the backend use scalar loads
// (SGPRs) instead of vector loads of uniform data (VGPRs).
typedef const __attribute__((address_space(4))) DevObject* ConstObj;
__device__ __forceinline__ ConstObj const_obj(const DevObject* base, uint32_t i) {
  return (ConstObj)(base) + i;
}

// The first 64 B of an object record (kind, material, i0-i5, d0-d7): what the
// object loop reads for meshes, spheres, planes and discs, fetched as one
// scalar load at the top of the object's iteration instead of field by field
// where each is first used (three or four dependent scalar round trips per
// object: C4 +1.4 %).
struct ObjHead {
  int32_t kind, mat, i0, i1, i2, i3, i4, i5;
  float d[8];
};
typedef const __attribute__((address_space(4))) uint32_t* ConstU32;
__device__ __forceinline__ ObjHead load_head(ConstObj o) {
  ConstU32 q = (ConstU32)o;
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; i++) w[i] = q[i];  // adjacent: one s_load_dwordx16
  ObjHead H;
  H.kind = (int32_t)w[0];
  H.mat = (int32_t)w[1];
  H.i0 = (int32_t)w[2];
  H.i1 = (int32_t)w[3];
  H.i2 = (int32_t)w[4];
  H.i3 = (int32_t)w[5];
  H.i4 = (int32_t)w[6];
  H.i5 = (int32_t)w[7];
#pragma unroll
  for (int i = 0; i < 8; i++) H.d[i] = __uint_as_float(w[8 + i]);
  return H;
}

struct MinHit {
  float t, u, v;
  int32_t obj;
  uint32_t prim, point;
  int32_t tc;  // last object that wrote surface_texcoords (-1: still vector2())
};

// A BVH walk parked mid-way (SUSP schedule): the object it belongs to, the
// current node, the parked leaf and the stack depth; the stack entries stay
// in the lane's LDS column and the hit record in its MinHit.
struct WalkSuspend {
  int32_t oi = -1;  // -1: no suspended walk
  uint32_t w = 0, leaf = 0, sp = 0;
};

// The same traversal restructured as while-while with postponed leaves
// (Aila & Laine 2009): a lane that reaches a leaf parks it and keeps walking
// inner nodes until every active lane holds a leaf, then the wave tests the
// parked leaves together. Inner-node and triangle code no longer interleave
// per iteration. The closest hit is a total order on (t, face), so the test
// order does not change the result.
// One face of mesh object oi against the ray: the reference test
// (intersect.cpp:357-419, or the point test of a zero-length ray) and the
// closest-hit update, lower face index first among equal t.
__device__ __forceinline__ void tri_candidate(const DevScene& S, const TriData& T, uint32_t ti, int32_t oi,
                                              const Ray& r, bool zl, MinHit& h) {
  float t = 0.0f, u = 0.0f, v = 0.0f;
  bool hit = false;
  if (!zl) {
    // ray_tri (intersect.cpp:357-419) with ray_plane's two tests as one
    // predicate over a quotient every lane computes (as small_mesh_rays):
    // cmp_eps(ts, 0, eps) is |ts| < eps, a quotient forced to -1 there fails
    // 0 <= q <= 1, which med3(q, 0, 1) == q decides (NaN: false)
    const float ts = (T.pl.x * r.dir.x + T.pl.y * r.dir.y + T.pl.z * r.dir.z);
    const float ns = -(T.pl.x * r.start.x + T.pl.y * r.start.y + T.pl.z * r.start.z + T.pl.w);
    float q = ns / ts;
    asm volatile("" : "+v"(q));
    q = fabsf(ts) < kEpsilon ? -1.0f : q;
    if (__builtin_amdgcn_fmed3f(q, 0.0f, 1.0f) == q) {
      float uu, vv;
      bary_pre(T, r.start + r.dir * q, uu, vv);
      hit = (uu >= 0) && (vv >= 0) && (uu + vv <= 1);
      t = q;
      u = uu;
      v = vv;
    }
  } else {
    hit = point_in_tri(T, r.start, u, v);
    t = 0.0f;
  }
  if (hit) {
    bool better = t < h.t || (t == h.t && h.obj == oi && T.face < tri_face(S.tris, h.prim));
    if (better) {
      h.t = t;
      h.obj = oi;
      h.prim = ti;
      h.u = u;
      h.v = v;
      h.point = zl ? 1u : 0u;
    }
  }
}

template <bool COUNT, int ZLMODE = -1>  // ZLMODE: 0/1 = ray known (non-)zero-length, -1 = runtime zl
__device__ __forceinline__ void test_leaf(const DevScene& S, uint32_t w, int32_t oi, const Ray& r, bool zl_rt, MinHit& h,
                                          Tally<COUNT>& tally) {
  const bool zl = ZLMODE < 0 ? zl_rt : ZLMODE == 1;
  uint32_t cnt = leaf_count(w), first = w & kLeafFirstMask;
  for (uint32_t i = 0; i < cnt; i++) {
    uint32_t ti = first + i;
    TriData T = load_tri(S.tris, ti);
    if (COUNT) tally.tris++;
    tri_candidate(S, T, ti, oi, r, zl, h);
  }
}

// A small mesh (DevObject::i3 = n faces from triangle `first`): every face
// at a wave-uniform index, no BVH walk. The walk's culling is conservative
// and the closest hit is a total order on (t, face), so testing all faces
// gives the walk's hit bit for bit; the faces come in SGPRs, not as
// dependent per-lane node and triangle fetches.
// A face whose plane has the previous face's bits (the two triangles of a
// quad) reuses its plane test: intersect.cpp:728-744 on identical operands.
// One per-lane branch per face: ray_plane's two tests (intersect.cpp:733,
// 737) are one predicate over a quotient every lane computes, and the
// barycentric test with the closest-hit update (intersect.cpp:357-419,
// lower face index first among equal t) runs as selects inside the branch
// that skips planes no lane of the wave hits. Each nested per-lane branch
// cost the CU's one scalar unit an exec-mask save, a branch and a restore
// per face (SALU issue 0.79 per CU-cycle on C2, against a measured ceiling
// of about 1: tools/salu_peak.hip). The tie rule needs the face index of the
// hit this call wrote (h.obj == oi only after a face of this call won:
// objects are traced once per segment), kept in a register instead of
// re-read from the hit's triangle record.
// The closest-hit update of a small-mesh face that passed its plane test:
// the barycentric test (intersect.cpp:146-177) and the (t, face) order, as
// selects. (uu >= 0) && (vv >= 0) && (uu + vv <= 1): uu + vv <= 1 is
// 1 - (uu + vv) >= 0 exactly, a NaN in uu or vv makes w NaN, and w - w is
// NaN for a NaN or infinite w (both fail the test), else +0, which also
// turns a -0 minimum into +0; min3 ignores NaN, the added term restores it.
// The order (t, face) is one 64-bit key (t >= 0 here: its bits order as
// unsigned integers once -0 becomes +0), with the best face 0 unless this
// call wrote h (h.obj == oi only then: objects are traced once per
// segment), so "lower face first among equal t" needs no object compare and
// no load of the best face's record. ONCE (the kernel without walks): h.obj
// and h.point are set once per mesh from a lane mask of the faces that won
// (C2 +1.4 %; C4 -0.6 % in the walking kernels, whose SGPR budget the extra
// mask strains: round 5, profiles/r05/ab_spills.log).
template <bool ONCE>
__device__ __forceinline__ void small_face_hit(const TriData& T, uint32_t ti, int32_t oi, float tt, f3 pp,
                                               uint32_t point, MinHit& h, uint32_t& bface, bool& wrote) {
  float uu, vv;
  bary_pre(T, pp, uu, vv);
  const float w = 1.0f - (uu + vv);
  const float m = fminf(fminf(uu, vv), w) + (w - w);
  const uint64_t key = ((uint64_t)(m >= 0.0f ? __float_as_uint(tt + 0.0f) : 0xFFFFFFFFu) << 32) | T.face;
  const uint64_t best = ((uint64_t)__float_as_uint(h.t + 0.0f) << 32) | bface;
  const bool better = key < best;
  h.t = better ? tt : h.t;
  h.prim = better ? ti : h.prim;
  h.u = better ? uu : h.u;
  h.v = better ? vv : h.v;
  bface = better ? T.face : bface;
  if (ONCE) {
    wrote = wrote || better;
  } else {
    h.obj = better ? oi : h.obj;
    h.point = better ? point : h.point;
  }
}
// The faces of a small mesh for the lanes of non-zero-length rays.
// ray_plane (intersect.cpp:728-744) is a hit when !cmp_eps(ts, 0) and
// 0 <= ns / ts <= 1. cmp_eps(ts, 0, eps) is |ts| < eps (NaN: false in both),
// and a quotient forced to -1 where it holds fails the range test, which
// med3(q, 0, 1) == q decides (NaN: false): one compare, with no lane-mask
// arithmetic on the scalar unit. The quotient is taken on every lane (the
// empty asm keeps the compiler from putting the division behind a branch of
// its own).
template <bool COUNT, bool ONCE>
__device__ __forceinline__ void small_mesh_rays(const DevScene& S, uint32_t first, uint32_t n, int32_t oi,
                                                const Ray& r, MinHit& h, Tally<COUNT>& tally) {
  bool on_plane = false;  // the plane test of the last distinct plane
  bool wrote = false;
  float tt = 0.0f;
  f3 pp = mk3(0, 0, 0);
  uint32_t bface = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t ti = first + i;
    TriData T = load_tri_uniform(S.tris, ti);
    if (COUNT && threadIdx.x == (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x)) tally.utris++;
    if (!T.same_plane || i == 0) {  // wave-uniform
      const float ts = (T.pl.x * r.dir.x + T.pl.y * r.dir.y + T.pl.z * r.dir.z);
      const float ns = -(T.pl.x * r.start.x + T.pl.y * r.start.y + T.pl.z * r.start.z + T.pl.w);
      float q = ns / ts;
      asm volatile("" : "+v"(q));
      q = fabsf(ts) < kEpsilon ? -1.0f : q;
      on_plane = __builtin_amdgcn_fmed3f(q, 0.0f, 1.0f) == q;
      tt = q;
      pp = r.start + r.dir * q;
    }
    if (on_plane) small_face_hit<ONCE>(T, ti, oi, tt, pp, 0u, h, bface, wrote);
  }
  if (ONCE) {
    h.obj = wrote ? oi : h.obj;
    h.point = wrote ? 0u : h.point;
  }
}
// The same for the lanes of zero-length rays (total internal reflection,
// rare): point_in_tri (intersect.cpp:320-346), t = 0 at the segment start.
template <bool COUNT, bool ONCE>
__device__ __forceinline__ void small_mesh_points(const DevScene& S, uint32_t first, uint32_t n, int32_t oi,
                                                  const Ray& r, MinHit& h) {
  uint32_t bface = 0;
  bool wrote = false;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t ti = first + i;
    TriData T = load_tri_uniform(S.tris, ti);
    const float d4 = T.pl.x * r.start.x + T.pl.y * r.start.y + T.pl.z * r.start.z + T.pl.w * 1.0f;
    if (cmp_eps(d4 + T.pl.w, 0.0f, kEpsilon)) small_face_hit<ONCE>(T, ti, oi, 0.0f, r.start, 1u, h, bface, wrote);
  }
  if (ONCE) {
    h.obj = wrote ? oi : h.obj;
    h.point = wrote ? 1u : h.point;
  }
}
// A lane runs the faces of its kind of ray; zero-length rays are tested in a
// second loop that runs only when the wave holds one.
template <bool COUNT, bool ONCE = false>
__device__ __forceinline__ void small_mesh_trace(const DevScene& S, uint32_t first, uint32_t n, int32_t oi,
                                                 const Ray& r, bool zl, MinHit& h, Tally<COUNT>& tally) {
  if (!zl) small_mesh_rays<COUNT, ONCE>(S, first, n, oi, r, h, tally);
  if (__ballot(zl) && zl) small_mesh_points<COUNT, ONCE>(S, first, n, oi, r, h);
}

// SUSP: when at most `thr` lanes are still walking while other live lanes of
// the wave wait, the walkers park (state to *ws) and return true; the wave
// moves on and they resume from *ws in a later iteration (same operations in
// the same order per lane).
template <bool COUNT, bool SUSP = false, int ZLMODE = -1>  // ZLMODE as in test_leaf
__device__ __forceinline__ bool traverse_ww(const DevScene& S, uint32_t root, int32_t oi, const Ray& r, bool zl_rt,
                                            MinHit& h, uint32_t* __restrict__ stk, Tally<COUNT>& tally,
                                            WalkSuspend* ws = nullptr, bool resume = false, uint32_t thr = 0,
                                            uint32_t live = 0, const Slopes* pre = nullptr) {
  const bool zl = ZLMODE < 0 ? zl_rt : ZLMODE == 1;
  constexpr uint32_t kNone = 0x7FFFFFFFu;  // empty-stack sentinel (no leaf bit, never a node index)
  const Slopes sl = pre ? *pre : walk_slopes(r, zl);
  const float ix = sl.ix, iy = sl.iy, iz = sl.iz, ox = sl.ox, oy = sl.oy, oz = sl.oz;
  uint32_t w = root, leaf = 0, sp = 0;
  if (SUSP && resume) {
    w = ws->w;
    leaf = ws->leaf;
    sp = ws->sp;
  }
  float tmax_lim = fminf(h.t, 1.0f) * 1.000002f + 1e-7f;  // h.t only changes in the leaf tests
  bool susp = false;
  while ((w != kNone || leaf) && !(SUSP && susp)) {
    // The node loop. Its exits are wave-uniform (ballots), so the compiler
    // keeps no per-lane exit masks across trips: a lane whose w is an inner
    // node (w < kNone: leaf words have bit 31 set) takes the trip, the others
    // sit it out under one exec-mask region.
    for (;;) {
      const bool inner = w < kNone;
      const uint64_t walking = __ballot(inner);
      if (!walking) break;
      if (inner) {
      const float4* q = reinterpret_cast<const float4*>(S.nodes + w);
      float4 X = q[0], Y = q[1], Z = q[2];
      uint4 Cw = reinterpret_cast<const uint4*>(q)[3];
      // the stack's two top entries, read while the node is in flight (slot 0
      // stands in below the bottom of the stack; its value is not used then)
      const uint32_t top1 = stk[(sp > 0 ? sp - 1 : 0u) * kBlock], top2 = stk[(sp > 1 ? sp - 2 : 0u) * kBlock];
      if (COUNT) tally.nodes++;
#ifdef FS_PHASE_PROF
      FS_WAVE_TRIP(tally.node_trips);
      tally.lane_nodes++;
#endif
      bool h0, h1;
      float t0, t1;
      {
        float a0 = fmaf(X.x, ix, ox), b0 = fmaf(X.z, ix, ox);
        float a1 = fmaf(X.y, ix, ox), b1 = fmaf(X.w, ix, ox);
        float c0 = fmaf(Y.x, iy, oy), e0 = fmaf(Y.z, iy, oy);
        float c1 = fmaf(Y.y, iy, oy), e1 = fmaf(Y.w, iy, oy);
        float g0 = fmaf(Z.x, iz, oz), k0 = fmaf(Z.z, iz, oz);
        float g1 = fmaf(Z.y, iz, oz), k1 = fmaf(Z.w, iz, oz);
        // The exit clamp to the walk's t limit is a signed-integer min on the
        // float bits: the limit is positive, so for finite exits the integer
        // order is the float order, and v_min_f32 would need the loop-carried
        // limit re-canonicalised on every trip (C4 +1 %).
        const int tl = __float_as_int(tmax_lim);
        float n0 = fmaxf(fmaxf(fminf(a0, b0), fminf(c0, e0)), fmaxf(fminf(g0, k0), -1e-6f));
        float f0 = fminf(fminf(fmaxf(a0, b0), fmaxf(c0, e0)), __int_as_float(min(__float_as_int(fmaxf(g0, k0)), tl)));
        float n1 = fmaxf(fmaxf(fminf(a1, b1), fminf(c1, e1)), fmaxf(fminf(g1, k1), -1e-6f));
        float f1 = fminf(fminf(fmaxf(a1, b1), fmaxf(c1, e1)), __int_as_float(min(__float_as_int(fmaxf(g1, k1)), tl)));
        h0 = n0 <= f0;
        h1 = n1 <= f1;
        t0 = n0;
        t1 = n1;
      }
      // The step to the next node as selects, not branches: each per-lane
      // branch of the push / pop / park transitions cost the CU's one scalar
      // unit an exec-mask save, a branch and a restore per node trip, on the
      // critical path of the walking wave (a wave issues one scalar
      // instruction per 4.7 cycles: tools/salu_peak.hip). Both children hit:
      // go to the nearer, push the farther; one hit: go to it; none: pop.
      // A miss enters past every hit (kMissT), so one compare orders them.
      constexpr float kMissT = 3.0e38f;
      const float e0 = h0 ? t0 : kMissT, e1 = h1 ? t1 : kMissT;
      const bool swap = e1 < e0;
      const uint32_t near = swap ? Cw.y : Cw.x, far = swap ? Cw.x : Cw.y;
      const bool any = (swap ? e1 : e0) < kMissT, both = (swap ? e0 : e1) < kMissT;
      // A push only when both are hit (sp + 1 below); else a write above the
      // top. Unconditional, so in bounds only because sp <= this node's depth
      // < kTraversalStack: both builders stop splitting at depth
      // kTraversalStack - 1 (fs_scene.cpp split depth rule, kGuard in
      // fs_bvh_gpu.hip; tests/test_abi.py deep-mesh case).
      static_assert(kTraversalStack >= 2, "the walk stack holds the root's far child");
      stk[sp * kBlock] = far;
      const uint32_t w1 = any ? near : (sp > 0 ? top1 : kNone);
      const uint32_t sp1 = both ? sp + 1 : (any ? sp : (sp > 0 ? sp - 1 : 0u));
      // Park the first leaf and keep walking from the entry under it: far
      // when both were hit, the old top after a one-child step, the one
      // below it after a pop (read before the node arrived, like top1).
      const bool park = (int32_t)(leaf == 0 ? w1 : 0u) < 0;  // a leaf word has bit 31 set
      const uint32_t under = both ? far : (any ? (sp > 0 ? top1 : kNone) : (sp > 1 ? top2 : kNone));
      leaf = park ? w1 : leaf;
      w = park ? under : w1;
      sp = park ? (both ? sp : (sp1 > 0 ? sp1 - 1 : 0u)) : sp1;
      }
      if (__ballot(inner && leaf == 0) == 0) break;  // every walking lane holds a leaf
      // Checked on every node trip: the walkers park as soon as they are few
      // (every 8th trip: C4 -9 %; every 2nd: -2 %; the trips between the drop
      // and the check ran with a nearly idle wave).
      if (SUSP) {
        const uint32_t walkers = (uint32_t)__popcll(walking);
        if (walkers <= thr && walkers < (uint32_t)__builtin_amdgcn_readfirstlane(live)) {
          susp = inner;  // the lanes that took this trip park
          break;
        }
      }
    }
    if (SUSP && susp) break;
    // One triangle per lane per trip, running on through the leaves the walk
    // stopped on (the popped far children may be leaves too), so a lane with
    // 1+2 triangles costs the wave 3 trips, not max-per-leaf 2+2. (Selects for
    // this step and a branch-free triangle test with the (t, face) key, as the
    // node step and the small-mesh faces, measured C4 -3 %, C3 -5 %: round 5,
    // profiles/r05/ab_leafstep.log.)
    while (leaf) {
#ifdef FS_PHASE_PROF
      FS_WAVE_TRIP(tally.leaf_trips);
      tally.lane_leaves++;
#endif
      uint32_t cnt = leaf_count(leaf);
      if (cnt) {
        test_leaf<COUNT, ZLMODE>(S, leaf_word(1, leaf & kLeafFirstMask), oi, r, zl, h, tally);
        cnt--;
      }
      if (cnt) {
        leaf = leaf_word(cnt, (leaf & kLeafFirstMask) + 1u);
      } else if (w & kLeafBit) {  // the walk also stopped on a leaf: test it next
        leaf = w;
        w = sp ? stk[--sp * kBlock] : kNone;
      } else {
        leaf = 0;
      }
    }
    tmax_lim = fminf(h.t, 1.0f) * 1.000002f + 1e-7f;
  }
  if (SUSP && susp) {
    ws->oi = oi;
    ws->w = w;
    ws->leaf = leaf;
    ws->sp = sp;
  }
  return SUSP && susp;
}

// Conservative segment-vs-box cull for analytic objects (not a reference
// test): the slab interval over the segment's slopes (seg_slopes, the ones
// the mesh-root culls and walks use; dir and stop - start differ by rounding
// only) with the BVH traversal's t margins, against a box padded on the host
// (fs_scene.cpp). A segment that can produce a hit with t < best always
// passes. (Slopes of its own from r.dir cost three v_rcp per segment, which
// the compiler hoisted out of the object loop and spilled.)
template <class FloatPtr>
__device__ __forceinline__ bool seg_box_cull(const Slopes& sl, float best, FloatPtr b) {
  float a0 = fmaf(b[0], sl.ix, sl.ox), a1 = fmaf(b[3], sl.ix, sl.ox);
  float c0 = fmaf(b[1], sl.iy, sl.oy), c1 = fmaf(b[4], sl.iy, sl.oy);
  float e0 = fmaf(b[2], sl.iz, sl.oz), e1 = fmaf(b[5], sl.iz, sl.oz);
  float tn = fmaxf(fmaxf(fminf(a0, a1), fminf(c0, c1)), fmaxf(fminf(e0, e1), -1e-6f));
  float tf = fminf(fminf(fmaxf(a0, a1), fmaxf(c0, c1)), fminf(fmaxf(e0, e1), fminf(best, 1.0f) * 1.000002f + 1e-7f));
  return tn <= tf;
}

#ifdef FS_PHASE_PROF
struct PhaseAcc {
  uint64_t cull = 0, trav = 0, prim = 0, small = 0;
  // node trips of this trace call's BVH walks: the sum over meshes of the
  // wave's largest per-lane count (walks one mesh after another, as run) and
  // the wave's largest per-lane sum over meshes (if each lane went on to its
  // next mesh's walk on its own)
  uint64_t seq = 0, chain = 0;
};
#define FS_TICK() __builtin_readcyclecounter()
__device__ __forceinline__ uint32_t prof_wave_max(uint32_t v) {  // over the active lanes
  uint64_t m = __ballot(1);
  uint32_t mx = 0;
  while (m) {
    const int l = __builtin_ctzll(m);
    mx = max(mx, (uint32_t)__builtin_amdgcn_readlane(v, l));
    m &= m - 1;
  }
  return mx;
}
#else
struct PhaseAcc {};
#define FS_TICK() 0ull
#endif

// ---- the scene object octree (SceneBvh, scene.cpp:11-133) -----------------
// One object's Object::Trace into the hit record h (per-lane object index;
// meshes pre-seeded with h.t, mesh.cpp:277-281). Returns true when the
// object wrote h (it then holds the object's hit).
template <bool COUNT, bool TEX>
__device__ __forceinline__ bool object_trace(const DevScene& S, uint32_t oi, const Ray& r, bool zl, MinHit& h,
                                             uint32_t* __restrict__ stk, Tally<COUNT>& tally, const Slopes* slp) {
  const DevObject* __restrict__ o = S.objects + oi;
  const float* d = o->d;
  const int32_t kind = o->kind;
  // per-lane object index (vector loads), counted per lane in its own field:
  // bench.py's byte model weighs object_loads per wave
  if (COUNT) tally.lane_objs++;
  if (kind == FS_OBJ_MESH) {
    if (!o->i2 || !ref_root_visit(mk3(d[0], d[1], d[2]), mk3(d[3], d[4], d[5]), r, zl, h.t, *slp)) return false;
    const int32_t before = h.obj;
    if (o->i3)
      small_mesh_trace<COUNT>(S, __float_as_uint(d[6]), (uint32_t)o->i3, (int32_t)oi, r, zl, h, tally);
    else
      traverse_ww<COUNT>(S, (uint32_t)o->i0, (int32_t)oi, r, zl, h, stk, tally, nullptr, false, 0u, 0u, slp);
    const bool wrote = h.obj == (int32_t)oi && before != (int32_t)oi;
    if (TEX && wrote && o->i4) h.tc = (int32_t)oi;  // mesh.cpp:300-311: only with texcoords
    return wrote;
  }
  if (zl) return false;
  if (COUNT) tally.prims++;
  float t;
  f3 p, n;
  bool hit = false;
  if (kind == FS_OBJ_SPHERE) {
    hit = ray_sphere(mk3(d[0], d[1], d[2]), d[3], r, t, p, n) && t < h.t;
  } else if (kind == FS_OBJ_PLANE) {
    hit = ray_plane(mk4(d[0], d[1], d[2], d[3]), r, t, p) && t < h.t;
  } else if (kind == FS_OBJ_DISC) {
    hit = ray_plane(mk4(d[0], d[1], d[2], d[3]), r, t, p) && length(mk3(d[4], d[5], d[6]) - p) <= d[7] && t < h.t;
  } else if (kind == FS_OBJ_QUAD_ONWH) {
    if (ray_plane(mk4(d[0], d[1], d[2], d[3]), r, t, p)) {
      f3 ph = p - mk3(d[4], d[5], d[6]);
      float td = dot(mk3(d[12], d[13], d[14]), ph);
      float bd = dot(mk3(d[9], d[10], d[11]), ph);
      hit = !(fabsf(bd) > d[7] || fabsf(td) > d[8]) && t < h.t;
    }
  } else if (kind == FS_OBJ_CUBOID) {
    if (seg_box_cull(*slp, h.t, d + 24)) {
      for (uint32_t i = 0; i < 6; i++) {
        float ti;
        if (ray_plane(mk4(d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]), r, ti, p) && ti < h.t) {
          bool ok = true;
          for (uint32_t j = 0; j < 6; j++)
            if (i / 2 != j / 2 && plane_dist(mk4(d[4 * j], d[4 * j + 1], d[4 * j + 2], d[4 * j + 3]), p) > 0.0f) ok = false;
          if (ok) {
            h.t = ti;
            h.obj = (int32_t)oi;
            h.prim = i;
            hit = true;
          }
        }
      }
      if (hit) h.point = 0;
      if (TEX && hit) h.tc = (int32_t)oi;
      return hit;
    }
    return false;
  }
  if (hit) {
    h.t = t;
    h.obj = (int32_t)oi;
    h.point = 0;
    if (TEX) h.tc = (int32_t)oi;  // analytic objects always write texcoords
  }
  return hit;
}

// SceneBvhNode::Trace of leaf c (scene.cpp:76-103): the node test culls by
// the best hit so far; the leaf traces its objects into ONE fresh
// ObjectCollision (param 2, texcoords unset) and copies it whole into h each
// time an object writes it with a param below h's.
template <bool COUNT, bool TEX>
__device__ bool scene_leaf_trace(const DevScene& S, uint32_t c, const Ray& r, bool zl, MinHit& h,
                                 uint32_t* __restrict__ stk, Tally<COUNT>& tally, const Slopes* slp) {
  const DevSceneTree& T = *S.tree;
  float np;
  if (!ref_ray_bounds(mk3(T.child_mn[c][0], T.child_mn[c][1], T.child_mn[c][2]),
                      mk3(T.child_mx[c][0], T.child_mx[c][1], T.child_mx[c][2]), r, zl, np) ||
      np > h.t)
    return false;
  MinHit tmp;
  tmp.t = 2.0f;
  tmp.obj = -1;
  tmp.prim = 0;
  tmp.u = tmp.v = 0.0f;
  tmp.point = 0;
  tmp.tc = -1;
  bool result = false;
  const uint32_t first = T.first[c], cnt = T.count[c];
  for (uint32_t k = 0; k < cnt; k++) {
    if (object_trace<COUNT, TEX>(S, S.tree_objs[first + k], r, zl, tmp, stk, tally, slp) && tmp.t < h.t) {
      h = tmp;
      result = true;
    }
  }
  return result;
}

// Scene::Trace through the object octree: SceneBvhNode::Trace of the root
// (scene.cpp:76-84) and BaseBvhNode::TraceInternal (bvh.h:154-231) over its
// eight leaves, with the reference's plane parameters and tie rules.
template <bool COUNT, bool TEX>
__device__ void scene_trace_tree(const DevScene& S, const Ray& r, MinHit& h, uint32_t* __restrict__ stk,
                                 Tally<COUNT>& tally) {
  h.t = 2.0f;
  h.obj = -1;
  h.prim = 0;
  h.u = h.v = 0.0f;
  h.point = 0;
  h.tc = -1;
  const bool zl = zero_len(r);
  const Slopes sl = seg_slopes(r, zl);  // the mesh-root culls' and the walks' (as the object list's)
  const DevSceneTree& T = *S.tree;
  const f3 rmn = mk3(T.root_mn[0], T.root_mn[1], T.root_mn[2]), rmx = mk3(T.root_mx[0], T.root_mx[1], T.root_mx[2]);
  const f3 ctr = mk3(T.center[0], T.center[1], T.center[2]);
  float rp;
  f3 entry;
  if (!ref_bounds_hit(rmn, rmx, r, zl, rp, entry)) return;  // (h.t = 2 never culls the root)
  const f4 sx = mk4(T.split[0][0], T.split[0][1], T.split[0][2], T.split[0][3]);
  const f4 sy = mk4(T.split[1][0], T.split[1][1], T.split[1][2], T.split[1][3]);
  const f4 sz = mk4(T.split[2][0], T.split[2][1], T.split[2][2], T.split[2][3]);
  float xp = 2.0f, yp = 2.0f, zp = 2.0f;  // collision() params of planes not hit
  f3 xq = mk3(0, 0, 0), yq = xq, zq = xq;
  bool xh, yh, zh;
  uint32_t cn;
  Ray it = r;
  auto closest = [&](f3 q) {  // bvh.h:144-152: bit0 x, bit1 z, bit2 y
    f3 dd = q - ctr;
    return (uint32_t)(dd.x >= 0.0f) | ((uint32_t)(dd.z >= 0.0f) << 1) | ((uint32_t)(dd.y >= 0.0f) << 2);
  };
  if (!in_bounds(rmn, rmx, r.start)) {
    it.start = entry;
    cn = closest(entry);
    xh = ray_plane(sx, it, xp, xq);
    yh = ray_plane(sy, it, yp, yq);
    zh = ray_plane(sz, it, zp, zq);
  } else {
    cn = closest(r.start);
    xh = ray_plane(sx, r, xp, xq);
    yh = ray_plane(sy, r, yp, yq);
    zh = ray_plane(sz, r, zp, zq);
    if (!xh && !yh && !zh) {
      scene_leaf_trace<COUNT, TEX>(S, cn, r, zl, h, stk, tally, &sl);
      return;
    }
  }
  for (uint32_t i = 0; i < 4; i++) {
    if (scene_leaf_trace<COUNT, TEX>(S, cn, r, zl, h, stk, tally, &sl)) {
      const f3 hp = h.point ? r.start : r.start + r.dir * h.t;  // hit_info->point
      if (in_bounds(mk3(T.child_mn[cn][0], T.child_mn[cn][1], T.child_mn[cn][2]),
                    mk3(T.child_mx[cn][0], T.child_mx[cn][1], T.child_mx[cn][2]), hp))
        break;
    }
    if (xh && xp < yp && xp < zp) {
      cn ^= 1u;
      xh = false;
      it.start = xq;
      xp = kInfinity;
    } else if (yh && yp < zp && yp < xp) {
      cn ^= 4u;
      yh = false;
      it.start = yq;
      yp = kInfinity;
    } else if (zh && zp < yp && zp < xp) {
      cn ^= 2u;
      zh = false;
      it.start = zq;
      zp = kInfinity;
    } else {
      break;
    }
    if (!in_bounds(rmn, rmx, it.start)) break;
  }
}

// Scene::Trace's object loop (scene.cpp:227-236) into the lean hit record.
// SUSP: a lane may park inside a mesh walk (*parked = true, state in *ws) and
// resume it in a later call with the same ray: objects before the parked one
// are skipped on resume (already processed), the rest follow in order.
template <bool COUNT, bool TEX = false, bool SUSP = false, bool SOCT = false, bool NOWALK = false>
__device__ __forceinline__ void scene_trace_min(const DevScene& S, const Ray& r, MinHit& h,
                                                uint32_t* __restrict__ stk, Tally<COUNT>& tally,
                                                PhaseAcc& pa, WalkSuspend* ws = nullptr, uint32_t susp_thr = 0,
                                                uint32_t susp_thr_small = 0, bool* parked = nullptr) {
  if (SOCT) {  // Scene::Trace with a valid object tree (scene.cpp:231-236)
    scene_trace_tree<COUNT, TEX>(S, r, h, stk, tally);
    return;
  }
  bool resuming = SUSP && ws->oi >= 0;
  if (!resuming) {
    h.t = 2.0f;
    h.obj = -1;
    h.prim = 0;
    h.u = h.v = 0.0f;
    h.point = 0;
    h.tc = -1;
  }
  bool zl = zero_len(r);
  const uint32_t live = SUSP ? (uint32_t)__popcll(__ballot(1)) : 0u;
  bool park = false;
  const Slopes sl = seg_slopes(r, zl);  // once per segment: the mesh-root culls' and the walks'
#ifdef FS_PHASE_PROF
  const uint32_t nodes_call0 = tally.lane_nodes;
#endif
  for (uint32_t oi_ = 0; oi_ < S.num_objects; ++oi_) {
    const uint32_t oi = __builtin_amdgcn_readfirstlane(oi_);  // uniform by construction
    if (SUSP && (park || (resuming && (uint32_t)ws->oi > oi))) continue;
    ConstObj o = const_obj(S.objects, oi);
    if (COUNT && threadIdx.x == (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x)) tally.objs++;
    const ObjHead H = load_head(o);
    const float* hd = H.d;
    const int32_t kind = H.kind;
    const __attribute__((address_space(4))) float* d = o->d;
    if (kind == FS_OBJ_MESH) {
      if (!H.i2) continue;
      uint64_t t0 = FS_TICK();
      const bool resume_here = SUSP && resuming && (uint32_t)ws->oi == oi;
      bool visit =
          resume_here || ref_root_visit(mk3(hd[0], hd[1], hd[2]), mk3(hd[3], hd[4], hd[5]), r, zl, h.t, sl);
      uint64_t t1 = FS_TICK();
      if (H.i3) {  // a small mesh: its faces, no walk (never parks)
        if (visit)
          small_mesh_trace<COUNT, NOWALK>(S, __float_as_uint(hd[6]), (uint32_t)H.i3, (int32_t)oi, r, zl, h, tally);
#ifdef FS_PHASE_PROF
        {  // the faces are their own phase: neither the cull's nor the walk's
          const uint64_t ts = FS_TICK() - t1;
          pa.small += ts;
          t0 += ts;
          t1 += ts;
        }
#endif
      } else if (NOWALK) {
        // every mesh of the scene is small (chosen at upload): no BVH walk
      } else if (SUSP) {
        // (a separate walk for zero-length rays, moving the per-node zl
        // branch out of the loop, measured 3-4 % slower: code size)
#ifdef FS_PHASE_PROF
        const uint32_t nodes0 = tally.lane_nodes;
#endif
        if (visit)
          park = traverse_ww<COUNT, true>(S, (uint32_t)H.i0, (int32_t)oi, r, zl, h, stk, tally, ws, resume_here,
                                          H.i5 == 2 ? susp_thr : (H.i5 ? susp_thr_small : 0u), live, &sl);
#ifdef FS_PHASE_PROF
        pa.seq += prof_wave_max(tally.lane_nodes - nodes0);
#endif
        if (resume_here) resuming = false;
#ifdef FS_PHASE_PROF
        if (park) {
          pa.cull += t1 - t0;
          pa.trav += FS_TICK() - t1;
        }
#endif
        if (park) continue;
      } else if (visit) {
        traverse_ww<COUNT>(S, (uint32_t)H.i0, (int32_t)oi, r, zl, h, stk, tally, nullptr, false, 0u, 0u, &sl);
      }
      // MeshObject::Trace writes surface_texcoords only when the mesh has
      // texcoords (mesh.cpp:300-311); otherwise the previous writer's stay.
      if (TEX && h.obj == (int32_t)oi && H.i4) h.tc = (int32_t)oi;
#ifdef FS_PHASE_PROF
      uint64_t t2 = FS_TICK();
      pa.cull += t1 - t0;
      pa.trav += t2 - t1;
#else
      (void)t0;
      (void)t1;
#endif
      continue;
    }
#ifdef FS_PHASE_PROF
    uint64_t tp0 = FS_TICK();
#endif
    if (zl) continue;
    if (COUNT) tally.prims++;
    float t;
    f3 p, n;
    if (kind == FS_OBJ_SPHERE) {
      if (ray_sphere(mk3(hd[0], hd[1], hd[2]), hd[3], r, t, p, n) && t < h.t) {
        h.t = t;
        h.obj = (int32_t)oi;
      }
    } else if (kind == FS_OBJ_PLANE) {
      if (ray_plane(mk4(hd[0], hd[1], hd[2], hd[3]), r, t, p) && t < h.t) {
        h.t = t;
        h.obj = (int32_t)oi;
      }
    } else if (kind == FS_OBJ_DISC) {
      if (ray_plane(mk4(hd[0], hd[1], hd[2], hd[3]), r, t, p)) {
        if (length(mk3(hd[4], hd[5], hd[6]) - p) <= hd[7] && t < h.t) {
          h.t = t;
          h.obj = (int32_t)oi;
        }
      }
    } else if (kind == FS_OBJ_QUAD_ONWH) {
      if (ray_plane(mk4(d[0], d[1], d[2], d[3]), r, t, p)) {
        f3 ph = p - mk3(d[4], d[5], d[6]);
        float td = dot(mk3(d[12], d[13], d[14]), ph);
        float bd = dot(mk3(d[9], d[10], d[11]), ph);
        if (!(fabsf(bd) > d[7] || fabsf(td) > d[8]) && t < h.t) {
          h.t = t;
          h.obj = (int32_t)oi;
        }
      }
    } else if (kind == FS_OBJ_CUBOID) {
      if (!seg_box_cull(sl, h.t, d + 24)) continue;
      for (uint32_t i = 0; i < 6; i++) {
        if (ray_plane(mk4(d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]), r, t, p) && t < h.t) {
          bool ok = true;
          for (uint32_t j = 0; j < 6; j++) {
            if (i / 2 != j / 2 && plane_dist(mk4(d[4 * j], d[4 * j + 1], d[4 * j + 2], d[4 * j + 3]), p) > 0.0f) {
              ok = false;
              break;
            }
          }
          if (ok) {
            h.t = t;
            h.obj = (int32_t)oi;
            h.prim = i;
          }
        }
      }
    }
    if (TEX && h.obj == (int32_t)oi) h.tc = (int32_t)oi;  // analytic objects always write texcoords
#ifdef FS_PHASE_PROF
    pa.prim += FS_TICK() - tp0;
#endif
  }
  if (SUSP) {
    if (!park) ws->oi = -1;
    *parked = park;
  }
#ifdef FS_PHASE_PROF
  pa.chain += prof_wave_max(tally.lane_nodes - nodes_call0);
#endif
}

// ---- textures (material.cpp:108-126, intersect.cpp:769-784) -------------
// planar_map_texcoords
__device__ __forceinline__ void planar_tc(f3 p, f3 n, float& u, float& v) {
  if (n.x > n.y && n.x > n.z) {
    u = p.y;
    v = p.z;
  } else if (n.y > n.x && n.y > n.z) {
    u = p.x;
    v = p.z;
  } else {
    u = p.x;
    v = p.y;
  }
}
// sphere_map_texcoords: float atan2 overload, float BASE_PI, double +0.5/*0.5/1.0-.
// atan2f is the host C library's (fs_libm.h restatement), bit for bit.
__device__ __forceinline__ void sphere_tc(f3 n, float& u, float& v) {
  float uu = (float)((double)(libm::atan2f(n.x, n.z) / (2 * kPi)) + 0.5);  // fs_libm.h
  float vv = (float)((double)n.y * 0.5 + 0.5);
  u = uu;
  v = (float)(1.0 - (double)vv);
}
// float -> uint32 as x86-64 compilers lower it: truncate to int64, keep the
// low half; NaN and |f| >= 2^63 give 0.
__device__ __forceinline__ uint32_t f2u32_x64(float f) {
  if (!(f > -9.2233715e18f && f < 9.2233715e18f)) return 0u;
  return (uint32_t)(uint64_t)(int64_t)f;
}
// DiffuseMaterial::SampleDiffuse for a material with a map (texture >= 0).
__device__ __forceinline__ f3 sample_tex(const DevScene& S, const fs_material& m, float tu, float tv) {
  uint4 ti = S.tex_info[m.texture];
  float fx = (tu * m.texture_scale * (float)ti.y + 0.5f) - 1;
  float fy = (tv * m.texture_scale * (float)ti.z + 0.5f) - 1;
  uint32_t x = f2u32_x64(fx) % ti.y, y = f2u32_x64(fy) % ti.z;
  uint32_t off = y * ti.y * 3 + x * 3;
  const float* t = S.tex_rgb + ti.x + off;
  return mk3(t[0], t[1], t[2]);
}

// Texcoords written by object `oi`'s own hit on ray r (when a later mesh
// without texcoords took the hit, the reference keeps these; rare, so the
// object is intersected again here instead of carrying them through the
// traversal).
template <bool COUNT>
__device__ __forceinline__ void stale_texcoords(const DevScene& S, const Ray& r, int32_t oi, uint32_t* __restrict__ stk,
                                             float& tu, float& tv) {
  const DevObject* __restrict__ o = S.objects + oi;
  const float* d = o->d;
  float t;
  f3 p, n;
  tu = tv = 0.0f;
  switch (o->kind) {
    case FS_OBJ_SPHERE:
      if (ray_sphere(mk3(d[0], d[1], d[2]), d[3], r, t, p, n)) sphere_tc(n, tu, tv);
      break;
    case FS_OBJ_PLANE:
    case FS_OBJ_DISC:
    case FS_OBJ_QUAD_ONWH:
      if (ray_plane(mk4(d[0], d[1], d[2], d[3]), r, t, p)) planar_tc(p, mk3(d[0], d[1], d[2]), tu, tv);
      break;
    case FS_OBJ_CUBOID: {
      float best = 2.0f;
      for (uint32_t i = 0; i < 6; i++) {
        if (ray_plane(mk4(d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]), r, t, p) && t < best) {
          bool ok = true;
          for (uint32_t j = 0; j < 6; j++)
            if (i / 2 != j / 2 && plane_dist(mk4(d[4 * j], d[4 * j + 1], d[4 * j + 2], d[4 * j + 3]), p) > 0.0f) ok = false;
          if (ok) {
            best = t;
            planar_tc(p, mk3(d[4 * i], d[4 * i + 1], d[4 * i + 2]), tu, tv);
            tu = tu * 0.1f;
            tv = tv * 0.1f;
          }
        }
      }
      break;
    }
    default: {  // a mesh with texcoords: its own closest face
      MinHit m;
      m.t = 2.0f;
      m.obj = -1;
      m.prim = 0;
      m.u = m.v = 0.0f;
      m.point = 0;
      m.tc = -1;
      Tally<false> tally;
      traverse_ww<false>(S, (uint32_t)o->i0, oi, r, zero_len(r), m, stk, tally);
      if (m.obj == oi) {
        const float2* q = S.tri_tex + 3 * (size_t)m.prim;
        float2 t0 = q[0], t1 = q[1], t2 = q[2];
        tu = (t0.x + (t1.x - t0.x) * m.u) + (t2.x - t0.x) * m.v;
        tv = (t0.y + (t1.y - t0.y) * m.u) + (t2.y - t0.y) * m.v;
      }
      break;
    }
  }
}

// Rebuilds the hit point/normal of a MinHit exactly as the object tests
// produced them (object.cpp, mesh.cpp:289-298) and applies the back-face
// flip of Scene::Trace (scene.cpp:238-247). For a material with a map the
// surface texcoords follow (object.cpp:31-232, mesh.cpp:300-311), from the
// unflipped normal.
template <bool TEX>
__device__ __forceinline__ void rebuild_hit(const DevScene& S, const Ray& r, const MinHit& h, f3& p, f3& n,
                                            int32_t& mat, float& tu, float& tv, uint32_t* __restrict__ stk) {
  const DevObject* __restrict__ o = S.objects + h.obj;
  const float* d = o->d;
  p = h.point ? r.start : r.start + r.dir * h.t;
  int32_t kind = o->kind;
  if (kind == FS_OBJ_MESH) {
    const float4 pl = reinterpret_cast<const float4*>(S.tris + h.prim)[0];  // face plane
    n = mk3(pl.x, pl.y, pl.z);
    if (o->i1) {
      const float4* nq = S.tri_normals + 3 * (size_t)h.prim;
      float4 a = nq[0], b = nq[1], c = nq[2];
      f3 n0 = mk3(a.x, a.y, a.z), n1 = mk3(b.x, b.y, b.z), n2 = mk3(c.x, c.y, c.z);
      n = n0 + (n1 - n0) * h.u + (n2 - n0) * h.v;
    }
  } else if (kind == FS_OBJ_SPHERE) {
    n = normalize(p - mk3(d[0], d[1], d[2]));
  } else if (kind == FS_OBJ_CUBOID) {
    n = mk3(d[4 * h.prim], d[4 * h.prim + 1], d[4 * h.prim + 2]);
  } else {
    n = mk3(d[0], d[1], d[2]);
  }
  mat = o->mat;
  tu = tv = 0.0f;
  if (TEX && S.materials[mat].texture >= 0 && h.tc >= 0) {
    if (h.tc != h.obj) {
      stale_texcoords<false>(S, r, h.tc, stk, tu, tv);
    } else if (kind == FS_OBJ_MESH) {
      const float2* q = S.tri_tex + 3 * (size_t)h.prim;
      float2 t0 = q[0], t1 = q[1], t2 = q[2];
      tu = (t0.x + (t1.x - t0.x) * h.u) + (t2.x - t0.x) * h.v;
      tv = (t0.y + (t1.y - t0.y) * h.u) + (t2.y - t0.y) * h.v;
    } else if (kind == FS_OBJ_SPHERE) {
      sphere_tc(n, tu, tv);
    } else {
      planar_tc(p, n, tu, tv);
      if (kind == FS_OBJ_CUBOID) {
        tu = tu * 0.1f;
        tv = tv * 0.1f;
      }
    }
  }
  f4 cp = plane_np(n, p);
  if (plane_dist(cp, r.start) < 0.0f) n = n * (float)-1.0;
}

// One block of (pixel, sample) tasks: an 8x8 micro-tile of one sample group
// (wave-uniform, lives in SGPRs). Block b of a launch of nblocks decodes as
// a one-shot launch's blockIdx.x = b did: tile-major or group-major order,
// the centre-first tile order, and the XCD placement (block b belongs to
// XCD b & 7, the hardware's round-robin of workgroups over the 8 XCDs).
struct TaskBlock {
  uint32_t x0 = 0, y0 = 0, vx = 0, nvalid = 1;
  uint32_t total = 0, next = 0;  // tasks (in-frame pixels x spp) and the next one to hand out
  uint32_t rad_row = 0;          // record row (group * owned + tile) * micro-tiles + micro-tile
  uint32_t sample0 = 0;          // sample index of the group's first sample
  bool aov = false;              // last group: its last sample leaves the AOV planes
};

__device__ __forceinline__ TaskBlock decode_block(const Launch& P, const DevFrame& F, uint32_t b) {
  const uint32_t micro_per_side = P.tile_size / 8;
  const uint32_t micro_per_tile = micro_per_side * micro_per_side;
  // xcd_bands 2 gives each XCD whole 64x64 tiles, so one L2 serves the rays
  // of a tile; 1 (one band per XCD) is kept for A/B runs.
  if (P.xcd_bands == 1) {
    const uint32_t per = P.nblocks >> 3, rem = P.nblocks & 7u, xcd = b & 7u, k = b >> 3;
    b = xcd < rem ? xcd * (per + 1) + k : rem * (per + 1) + (xcd - rem) * per + k;
  } else if (P.xcd_bands == 2) {  // whole tiles per XCD: tile 8j + x on XCD x
    const uint32_t groups = P.nblocks / (8 * micro_per_tile);  // full groups of 8 tiles
    const uint32_t xcd = b & 7u, k = b >> 3;
    if (k < groups * micro_per_tile) b = ((k / micro_per_tile) * 8 + xcd) * micro_per_tile + k % micro_per_tile;
  }
  // a virtual tile list of owned tiles x groups, tile-major (a tile's groups
  // run together: the resident waves cover few tiles) or, with group_major,
  // group-major
  const uint32_t vtile = b / micro_per_tile, micro = b % micro_per_tile;
  uint32_t t, group;
  if (P.group_major) {
    group = vtile / P.owned;
    t = vtile - group * P.owned;
  } else {
    t = vtile / P.groups;
    group = vtile - t * P.groups;
  }
  if (P.tile_order) t = P.tile_order[t];
  TaskBlock B;
  B.rad_row = (group * P.owned + t) * micro_per_tile + micro;
  const uint32_t tile = P.tile_offset + t * P.tile_stride;
  const uint32_t tx = tile % P.tiles_x, ty = tile / P.tiles_x;
  B.x0 = tx * P.tile_size + (micro % micro_per_side) * 8;
  B.y0 = ty * P.tile_size + (micro / micro_per_side) * 8;
  B.sample0 = P.sample_base + group * P.spp;
  B.aov = group + 1 == P.groups || P.aov_rows != 0;
  B.next = 0;
  if (B.x0 < F.width && B.y0 < F.height) {  // only in-frame pixels are enumerated
    B.vx = min(8u, F.width - B.x0);
    B.nvalid = B.vx * min(8u, F.height - B.y0);
    B.total = B.nvalid * P.spp;
  } else {
    B.vx = 1;
    B.nvalid = 1;
    B.total = 0;
  }
  return B;
}

// A kernel-argument record read through a pointer offset by `zero`, a
// wave-uniform 0 the compiler cannot prove to be 0 (derived from the block
// cursor), so its loads stay at their uses. Read directly, the records the
// persistent loop needs only now and then (the camera basis, the block
// decode, the sky and AOV fields) were hoisted out of the loop and held in
// SGPRs for the whole kernel: about 100 SGPRs spilled into VGPR lanes, and
// reads of spilled scene pointers landed in the BVH node loop.
template <class T>
__device__ __forceinline__ const T& at_use(const T& v, uint32_t zero) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(&v) + zero);
}

constexpr uint32_t kNoBlock = 0xFFFFFFFFu;
constexpr uint32_t kFog0 = 0x40000000u;  // slot bit: the first hit is Fog
constexpr uint32_t kQueueStride = 64;  // work-queue counters 256 B apart

// The wave's next block. One-shot waves (P.persist 0) take block
// blockIdx.x once. Persistent waves pull blocks b = 8i + x from the queue of
// their own XCD x (wave w runs on XCD w & 7), so a block keeps the XCD (and
// L2) the one-shot placement gives it; when that queue is empty they take
// blocks of the other XCDs' queues in turn. One lane performs the atomic.
__device__ __forceinline__ uint32_t fetch_block(const Launch& P, uint32_t* __restrict__ queues, uint32_t& q,
                                                uint32_t& left) {
  if (!P.persist) {
    const uint32_t b = left ? (uint32_t)blockIdx.x : kNoBlock;
    left = 0;
    return b;
  }
  while (left) {
    uint32_t i = 0;
    if (threadIdx.x == (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x)) i = atomicAdd(queues + q * kQueueStride, 1u);
    i = (uint32_t)__builtin_amdgcn_readfirstlane(i);
    const uint64_t b = (uint64_t)i * 8u + q;
    if (b < P.nblocks) return (uint32_t)b;
    q = (q + 1) & 7u;
    left--;
  }
  return kNoBlock;
}

// The path-trace megakernel: the forward pass of every path, with path
// regeneration and a lean register footprint. The closest-hit query keeps
// only (t, object, primitive, u, v); each bounce's shading scalars go to the
// sample's path record and a finished path leaves its end state there
// (PathRecords); fold_paths runs the backward passes afterwards on full
// waves. The Fog anchors live in per-lane scratch rows of the wave; the
// depth-0 AOVs go straight to the frame.
//
// Work: the wave's lanes share one pool of (pixel, sample) tasks. Whenever
// lanes are free (their path ended) they take the next tasks of the wave's
// current block in sample-major order (ballot + mbcnt, no atomics), and
// when the block runs dry the wave fetches the next block and goes on
// handing out its tasks, so lanes never wait for a block's stragglers. With
// P.persist the grid is one wave per wave slot of the chip and the waves
// pull blocks until every queue is empty: the launch tail is one task
// path, not one block. fold_paths folds the records into the frame in
// sample order.
//
// NOWALK (every mesh small): no walk stack and 8 waves per SIMD.
template <bool COUNT, int WAVES, bool TEX = false, bool SUSP = false, bool MMAT = false, bool SOCT = false,
          bool NOWALK = false, bool TRIG = false>
__global__ __launch_bounds__(kBlock, WAVES) void render_kernel_lean(DevScene S, DevCamera C, DevFrame F, Launch P,
                                                                    PathRecords R,
                                                                    float4* __restrict__ anchor_all,
                                                                    uint32_t* __restrict__ queues,
                                                                    DevCounters* __restrict__ counters) {
  __shared__ uint32_t stk_all[NOWALK ? 1 : kTraversalStack * kBlock];
  const uint32_t lane = threadIdx.x % kBlock;
  const uint32_t wid = blockIdx.x;  // this wave's rows
  Tally<COUNT> tally;
  uint32_t* stk = stk_all + lane;
  // The Fog anchor rows of the wave, addressed as wave base (SGPR) + 32-bit lane offset.
  float4* anchor = anchor_all + (size_t)wid * (2 * kBlock);  // [0]: p0.xyz, [1]: lp0.xyz
  const uint32_t a0_off = lane * 16u, a1_off = (kBlock + lane) * 16u;

  TaskBlock cur;  // the block the wave hands out tasks from
  uint32_t queue = blockIdx.x & 7u, queues_left = P.persist ? 8u : 1u;
  uint32_t segments = 0, samples_done = 0;

  // the lane's task: its pixel, sample and record slot
  uint32_t x = 0, y = 0, pix = 0, smp = 0;
  uint32_t rad_row = 0;  // the block's record row: the path record is q = rad_row * spp * 64 + slot's low bits
  // s * kBlock + 8 * py + px; bit 31: this sample leaves the AOVs; bit 30
  // (kFog0): the path's first hit is Fog, so its two anchors are kept
  uint32_t slot = 0;
  uint64_t rng = 0;
  Ray r;
  uint32_t depth = 0;
  MatTrail<MMAT> mats;
  int top = -1;
  bool fresh = true;
  MinHit h;         // persists across iterations while a walk is parked (SUSP)
  WalkSuspend ws;
#ifdef FS_WAVE_TIMES
  // measurement build (libfsgpu_wt.so): when the wave starts, first finds
  // every queue empty and ends (s_memrealtime, 100 MHz), iterations after that
  const uint64_t wt_start = __builtin_amdgcn_s_memrealtime();
  uint64_t wt_drain = 0, wt_iters = 0, wt_drain_iter = 0;
  if (lane == 0) atomicMax(&counters->phase[31], ~wt_start);  // ~ the earliest start
#endif
#ifdef FS_PHASE_PROF
  uint64_t ph[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t seqc[2] = {0, 0};  // PhaseAcc::seq / chain summed over this wave's trace calls
  // lane activity per iteration (wave-uniform sums): lanes tracing, shading, unwinding; unwind level trips
  uint64_t act[4] = {0, 0, 0, 0};
  uint64_t tk = __builtin_readcyclecounter(), t_begin = tk;
#define FS_PHASE(i)                                 \
  do {                                              \
    uint64_t now_ = __builtin_readcyclecounter();   \
    ph[i] += now_ - tk;                             \
    tk = now_;                                      \
  } while (0)
#else
#define FS_PHASE(i) \
  do {              \
  } while (0)
#endif
  for (;;) {
    FS_PHASE(0);
    {
      // Hand the free lanes their next tasks, in lane order, from the
      // current block and, when it runs dry, from the blocks fetched after
      // it. Every update of `cur` is wave-uniform; the loop has no early
      // exits other than the final break of lanes left without work.
      const uint64_t m = __ballot(fresh);
      const uint32_t nfree = (uint32_t)__popcll(m);
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      bool got = false;
      uint32_t served = 0;
      while (served < nfree) {
        if (cur.next >= cur.total) {
          const uint32_t z = cur.sample0 >> 31;  // 0 (sample indices stay below 2^20)
          const uint32_t b = fetch_block(at_use(P, z), queues, queue, queues_left);
#ifdef FS_WAVE_TIMES
          if (b == kNoBlock && !wt_drain) {
            wt_drain = __builtin_amdgcn_s_memrealtime();
            wt_drain_iter = wt_iters;
          }
#endif
          if (b == kNoBlock) break;
          cur = decode_block(at_use(P, z), at_use(F, z), b);
        } else {
          const uint32_t take = min(nfree - served, cur.total - cur.next);
          if (fresh && rank - served < take) {
            const uint32_t task = cur.next + (rank - served);
            uint32_t s, px, py;
            if (cur.nvalid == 64) {  // a whole 8x8 micro-tile (wave-uniform): shifts, not divisions
              s = task >> 6;
              px = task & 7u;
              py = (task >> 3) & 7u;
            } else {  // a micro-tile cut by the frame edge
              s = task / cur.nvalid;
              const uint32_t k = task - s * cur.nvalid;
              px = k % cur.vx;
              py = k / cur.vx;
            }
            x = cur.x0 + px;
            y = cur.y0 + py;
            pix = y * at_use(F, cur.sample0 >> 31).width + x;
            smp = cur.sample0 + s;
            rad_row = cur.rad_row;
            slot = (s * kBlock + py * 8 + px) | ((cur.aov && s == P.spp - 1) ? 0x80000000u : 0u);
            got = true;
          }
          cur.next += take;
          served += take;
        }
      }
      if (fresh && !got) break;  // every queue is empty: this lane is done
    }
    if (fresh) {
      rng = pixel_seed(pix, smp, at_use(P, cur.sample0 >> 31).seed);
      r = camera_ray<TRIG>(at_use(C, cur.sample0 >> 31), (float)x, (float)y, rng);
      depth = 0;
      mats.reset();
      top = -1;
      fresh = false;
    }
    FS_PHASE(1);
    const bool aov = (slot >> 31) != 0;
    bool done = false;
    f3 L = mk3(0, 0, 0);
    if (depth >= kMaxDepth) {
      done = true;
    } else if (C.fast_render && depth > 1) {
      L = mk3(1, 1, 1);
      done = true;
    } else {
      if (!SUSP || ws.oi < 0) segments++;
      bool parked = false;
      PhaseAcc pa;
      scene_trace_min<COUNT, TEX, SUSP, SOCT, NOWALK>(S, r, h, stk, tally, pa, &ws, P.susp_thr, P.susp_thr_small,
                                                      &parked);
#ifdef FS_PHASE_PROF
      ph[5] += pa.cull;
      ph[6] += pa.trav;
      ph[7] += pa.prim;
      ph[10] += pa.small;
      seqc[0] += pa.seq;
      seqc[1] += pa.chain;
      act[0] += (uint64_t)__popcll(__ballot(1));
      act[1] += (uint64_t)__popcll(__ballot(!(SUSP && parked) && h.obj >= 0));
#endif
      FS_PHASE(2);
      if (SUSP && parked) {
        // the walk is parked; the lane resumes it next iteration
      } else if (h.obj < 0) {
        if (depth == 1 && (slot & kFog0)) *at_byte(anchor, a1_off) = make_float4(r.stop.x, r.stop.y, r.stop.z, 0);
        const DevScene& Sz = at_use(S, cur.sample0 >> 31);
        L = mk3(Sz.sky_r, Sz.sky_g, Sz.sky_b);
        if (TEX && Sz.sky_tex) {  // textured Light sky: SampleSky (scene.cpp:157-162, engine.cpp:91-92)
          float tu, tv;
          sphere_tc(normalize(r.stop - r.start), tu, tv);
          L = sample_tex(S, S.materials[Sz.sky], tu, tv) * 3.0f;
        }
        if (depth == 0 && aov) {  // the last sample's AOVs remain
          const DevFrame& Fz = at_use(F, cur.sample0 >> 31);
          const Launch& Pz = at_use(P, cur.sample0 >> 31);
          const uint32_t apix = pix + (Pz.aov_rows ? (rad_row / Pz.aov_rows) * Pz.aov_plane : 0u);
          f3 nd = normalize(r.dir);
          at_byte(Fz.normal, apix * 12u)[0] = nd.x;
          at_byte(Fz.normal, apix * 12u)[1] = nd.y;
          at_byte(Fz.normal, apix * 12u)[2] = nd.z;
          *at_byte(Fz.depth, apix * 4u) = at_use(C, cur.sample0 >> 31).z_far;
          *at_byte(Fz.material, apix * 8u) = Sz.sky_id;
        }
        done = true;
      } else {
        f3 p, nn;
        int32_t mi;
        float tu, tv;
        rebuild_hit<TEX>(S, r, h, p, nn, mi, tu, tv, stk);
        if (depth == 1 && (slot & kFog0)) *at_byte(anchor, a1_off) = make_float4(p.x, p.y, p.z, 0);
        const fs_material& m = S.materials[mi];
        const uint64_t q = rec_index(P, rad_row, slot);
        if (TEX && m.texture >= 0) {
          f3 tx = sample_tex(S, m, tu, tv);
          R.tex[depth * R.n + q] = make_float4(tx.x, tx.y, tx.z, 0.0f);
        }
        int32_t kind = m.kind;
        f3 view = normalize(p - r.start);
        f3 refl = mat_reflection<TRIG>(S, m, (uint32_t)mi, view, nn, rng);
        float c = fmaxf(0.0f, dot(nn, refl));
        float ds = 0.0f;
        if (kind == FS_MAT_CERAMIC || kind == FS_MAT_GLOW) {
          f3 hv = normalize(view * (float)-1.0 + refl);
          ds = pow50(dot(hv, nn));
        }
        rec_store<SUSP>(R.c + depth * R.n + q, c);
        if (kind == FS_MAT_CERAMIC || kind == FS_MAT_GLOW) rec_store<SUSP>(R.ds + depth * R.n + q, ds);
        if (MMAT) R.mat[depth * R.n + q] = (uint32_t)mi;
        mats.set(depth, (uint32_t)mi);
        top = (int)depth;
        if (depth == 0 && kind == FS_MAT_FOG) {  // Fog draws with the distance of its two anchors
          *at_byte(anchor, a0_off) = make_float4(p.x, p.y, p.z, 0);
          slot |= kFog0;
        }
        if (depth == 0 && aov) {
          const DevFrame& Fz = at_use(F, cur.sample0 >> 31);
          const Launch& Pz = at_use(P, cur.sample0 >> 31);
          const uint32_t apix = pix + (Pz.aov_rows ? (rad_row / Pz.aov_rows) * Pz.aov_plane : 0u);
          at_byte(Fz.normal, apix * 12u)[0] = nn.x;
          at_byte(Fz.normal, apix * 12u)[1] = nn.y;
          at_byte(Fz.normal, apix * 12u)[2] = nn.z;
          *at_byte(Fz.depth, apix * 4u) = length(r.start - p);
          *at_byte(Fz.material, apix * 8u) = m.id;
        }
        bool use = mat_will_use(m, refl, nn);
        Ray nr;
        nr.start = p;
        nr.stop = p + refl * C.z_far;
        nr.dir = nr.stop - nr.start;
        f3 off = refl * kStepOffset;
        nr.start = nr.start + off;
        nr.dir = nr.dir - off;
        r = nr;
        if (!use)
          done = true;
        else
          depth++;
      }
    }
    FS_PHASE(3);
#ifdef FS_PHASE_PROF
    act[2] += (uint64_t)__popcll(__ballot(done));
    if (done) act[3] += (uint64_t)(top + 1);
#endif
    if (done) {
      // The path's end state: the radiance entering level top + 1, top, and
      // the packed material ids; fold_paths applies the levels.
      uint32_t meta = (uint32_t)(top + 1);
      if (slot & kFog0) {
        // Fog at level 0 (material.cpp:319-339) draws after every level above
        // it has been applied, i.e. after the forward pass's last draw: the
        // draw is taken here and the record keeps its outcome.
        const float4 a = *at_byte(anchor, a0_off), b = *at_byte(anchor, a1_off);
        const fs_material& m0 = S.materials[mats.get0()];
        if (fog_takes_diffuse(m0, mk3(a.x, a.y, a.z), mk3(b.x, b.y, b.z), rng)) meta |= kRecFogDif;
      }
      const uint64_t q = rec_index(P, rad_row, slot);
      rec_store<SUSP>(R.end + q, make_float4(L.x, L.y, L.z, __uint_as_float(meta)));
      if (!MMAT && top >= 0) rec_store<SUSP>(R.mats + q, make_uint2(mats.lo, mats.hi));
      if (COUNT) samples_done++;
      fresh = true;
    }
    FS_PHASE(4);
#ifdef FS_PHASE_PROF
    ph[8]++;
#endif
#ifdef FS_WAVE_TIMES
    wt_iters++;
#endif
  }
#ifdef FS_WAVE_TIMES
  {
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x)) {
      const uint64_t base = ~atomicOr(&counters->phase[31], 0ull);
      const uint64_t bin = 20000;  // 200 us
      if (!wt_drain) wt_drain = t_end;
      const uint64_t be = (t_end - base) / bin, bd = (wt_drain - base) / bin;
      atomicAdd(&counters->phase[be < 13 ? be : 13], 1ull);
      atomicAdd(&counters->phase[14 + (bd < 13 ? bd : 13)], 1ull);
      atomicAdd(&counters->phase[28], (unsigned long long)(t_end - wt_drain));
      atomicMax(&counters->phase[29], (unsigned long long)(t_end - wt_drain));
      atomicAdd(&counters->phase[30], (unsigned long long)(wt_iters - wt_drain_iter));
    }
  }
#endif
#ifdef FS_PHASE_PROF
  ph[9] = __builtin_readcyclecounter() - t_begin;
  if (lane == 0) {
    for (int i = 0; i < 10; i++) atomicAdd(&counters->phase[i], (unsigned long long)ph[i]);
    atomicAdd(&counters->phase[14], (unsigned long long)ph[10]);
    atomicAdd(&counters->phase[16], (unsigned long long)seqc[0]);
    atomicAdd(&counters->phase[17], (unsigned long long)seqc[1]);
    for (int i = 0; i < 3; i++) atomicAdd(&counters->phase[26 + i], (unsigned long long)act[i]);
  }
  atomicAdd(&counters->phase[29], (unsigned long long)act[3]);
  atomicAdd(&counters->phase[10], (unsigned long long)tally.node_trips);
  atomicAdd(&counters->phase[11], (unsigned long long)tally.leaf_trips);
  atomicAdd(&counters->phase[12], (unsigned long long)tally.lane_nodes);
  atomicAdd(&counters->phase[13], (unsigned long long)tally.lane_leaves);
#endif
#undef FS_PHASE
  if (COUNT) {  // every lane's work
    atomicAdd(&counters->samples, (unsigned long long)samples_done);
    atomicAdd(&counters->segments, (unsigned long long)segments);
    atomicAdd(&counters->node_visits, (unsigned long long)tally.nodes);
    atomicAdd(&counters->tri_tests, (unsigned long long)tally.tris);
    atomicAdd(&counters->prim_tests, (unsigned long long)tally.prims);
    atomicAdd(&counters->object_loads, (unsigned long long)tally.objs);
    atomicAdd(&counters->small_tri_loads, (unsigned long long)tally.utris);
    atomicAdd(&counters->lane_object_loads, (unsigned long long)tally.lane_objs);
  }
}

// A lookahead launch's AOV planes of the folded sample, into the frame.
__device__ __forceinline__ void fold_aovs(const DevFrame& F, const PathRecords& R, size_t pix) {
  F.normal[3 * pix] = R.aov_n[3 * pix];
  F.normal[3 * pix + 1] = R.aov_n[3 * pix + 1];
  F.normal[3 * pix + 2] = R.aov_n[3 * pix + 2];
  F.depth[pix] = R.aov_d[pix];
  F.material[pix] = R.aov_m[pix];
}

// The backward passes of a launch and their fold into the frame: block b is
// micro-tile b of group 0 (decode_block's tile-major order without the XCD
// placement or tile order), lane = pixel; group g's records are row
// g * gridDim.x + b. Each pixel runs its samples' backward passes
// (unwind_path) and folds them in sample order (frame.cpp:53-63), so the
// frame is bit-identical to groups x spp consecutive TraceScene calls.
// The loads are pipelined across samples: while sample i is unwound, the c
// values of sample i + 1 (whose end record arrived one sample earlier) and
// the end record and material ids of sample i + 2 are in flight, and the
// material table sits in LDS (LDSM), so a sample waits on no memory round
// trip of its own.
// (LDSM: 48 B of dynamic LDS per material; up to 64 materials, so that LDS
// does not limit the waves per CU).
constexpr uint32_t kFoldLdsMaterials = 64;
template <bool TEX, bool MMAT, bool LDSM>
__global__ __launch_bounds__(kBlock) void fold_paths(DevScene S, DevFrame F, Launch P, PathRecords R) {
  extern __shared__ float4 mat_lds[];
  const uint32_t lane = threadIdx.x, b = blockIdx.x;
  if (LDSM) {
    for (uint32_t i = lane; i < 3 * S.num_materials; i += kBlock) mat_lds[i] = S.umat[i];
    __syncthreads();
  }
  const uint32_t micro_per_side = P.tile_size / 8, micro_per_tile = micro_per_side * micro_per_side;
  const uint32_t owned = b / micro_per_tile, micro = b % micro_per_tile;
  const uint32_t tile = P.tile_offset + owned * P.tile_stride;
  const uint32_t x = (tile % P.tiles_x) * P.tile_size + (micro % micro_per_side) * 8 + (lane & 7);
  const uint32_t y = (tile / P.tiles_x) * P.tile_size + (micro / micro_per_side) * 8 + (lane >> 3);
  if (x >= F.width || y >= F.height) return;
  const size_t pix = (size_t)y * F.width + x;
  f3 mean = mk3(F.color[3 * pix], F.color[3 * pix + 1], F.color[3 * pix + 2]);
  uint32_t n = F.count[pix];
  const uint32_t total = P.groups * P.spp;
  auto rec = [&](uint32_t i) {  // sample i of the pixel: group i / spp, sample i % spp
    const uint32_t g = i / P.spp, k = i - g * P.spp;
    return rec_index(P, g * gridDim.x + b, k * kBlock + lane);
  };
  auto load_c = [&](uint64_t q, int top, float (&c)[kMaxDepth]) {
#pragma unroll
    for (int k = 0; k < (int)kMaxDepth; k++) c[k] = k <= top ? R.c[(uint64_t)k * R.n + q] : 0.0f;
  };
  auto top_of = [](const float4& e) { return (int)(__float_as_uint(e.w) & 0xFFu) - 1; };
  const uint2 none = make_uint2(0u, 0u);
  // sample i (a), i + 1 (b), i + 2 (e2, m2)
  uint64_t qa = rec(0), qb = total > 1 ? rec(1) : qa;
  float4 ea = R.end[qa], eb = R.end[qb];
  uint2 ma = MMAT ? none : R.mats[qa], mb = MMAT ? none : R.mats[qb];
  float ca[kMaxDepth], cb[kMaxDepth];
  load_c(qa, top_of(ea), ca);
  for (uint32_t i = 0; i < total; i++) {
    uint64_t q2 = qb;
    float4 e2 = eb;
    uint2 m2 = mb;
    if (i + 1 < total) load_c(qb, top_of(eb), cb);
    if (i + 2 < total) {
      q2 = rec(i + 2);
      e2 = R.end[q2];
      if (!MMAT) m2 = R.mats[q2];
    }
    const uint32_t meta = __float_as_uint(ea.w);
    f3 L;
    if (LDSM)
      L = unwind_path<TEX, MMAT>(static_cast<const float4*>(mat_lds), R, qa, mk3(ea.x, ea.y, ea.z), top_of(ea),
                                 (meta & kRecFogDif) != 0, ma, ca);
    else
      L = unwind_path<TEX, MMAT>(S.umat, R, qa, mk3(ea.x, ea.y, ea.z), top_of(ea), (meta & kRecFogDif) != 0, ma, ca);
    f3 np = mean * (float)n + L;
    float dv = (float)(++n);
    mean = mk3(np.x / dv, np.y / dv, np.z / dv);
    qa = qb;
    ea = eb;
    ma = mb;
#pragma unroll
    for (int k = 0; k < (int)kMaxDepth; k++) ca[k] = cb[k];
    qb = q2;
    eb = e2;
    mb = m2;
  }
  F.color[3 * pix] = mean.x;
  F.color[3 * pix + 1] = mean.y;
  F.color[3 * pix + 2] = mean.z;
  F.count[pix] = n;
  F.display[3 * pix] = gamma8(mean.x);
  F.display[3 * pix + 1] = gamma8(mean.y);
  F.display[3 * pix + 2] = gamma8(mean.z);
  if (R.aov_n) fold_aovs(F, R, pix);
}

// fold_paths without its cross-sample load pipeline: the fold of a
// lookahead launch's call (one sample per pixel, or a few), which runs while
// the next lookahead launch traces. With fewer registers (45-55 VGPRs against
// fold_paths' 66-80) it fits beside more background trace waves (bg_waves).
// The same backward passes and fold in sample order as fold_paths.
template <bool TEX, bool MMAT, bool LDSM>
__global__ __launch_bounds__(kBlock) void fold_paths_lite(DevScene S, DevFrame F, Launch P, PathRecords R) {
  extern __shared__ float4 mat_lds[];
  const uint32_t lane = threadIdx.x, b = blockIdx.x;
  if (LDSM) {
    for (uint32_t i = lane; i < 3 * S.num_materials; i += kBlock) mat_lds[i] = S.umat[i];
    __syncthreads();
  }
  const uint32_t micro_per_side = P.tile_size / 8, micro_per_tile = micro_per_side * micro_per_side;
  const uint32_t owned = b / micro_per_tile, micro = b % micro_per_tile;
  const uint32_t tile = P.tile_offset + owned * P.tile_stride;
  const uint32_t x = (tile % P.tiles_x) * P.tile_size + (micro % micro_per_side) * 8 + (lane & 7);
  const uint32_t y = (tile / P.tiles_x) * P.tile_size + (micro / micro_per_side) * 8 + (lane >> 3);
  if (x >= F.width || y >= F.height) return;
  const size_t pix = (size_t)y * F.width + x;
  f3 mean = mk3(F.color[3 * pix], F.color[3 * pix + 1], F.color[3 * pix + 2]);
  uint32_t n = F.count[pix];
  const uint32_t total = P.groups * P.spp;
  const uint2 none = make_uint2(0u, 0u);
  for (uint32_t i = 0; i < total; i++) {
    const uint32_t g = i / P.spp, k = i - g * P.spp;
    const uint64_t q = rec_index(P, g * gridDim.x + b, k * kBlock + lane);
    const float4 e = R.end[q];
    const uint2 m = MMAT ? none : R.mats[q];
    const uint32_t meta = __float_as_uint(e.w);
    const int top = (int)(meta & 0xFFu) - 1;
    float c[kMaxDepth];
#pragma unroll
    for (int l = 0; l < (int)kMaxDepth; l++) c[l] = l <= top ? R.c[(uint64_t)l * R.n + q] : 0.0f;
    f3 L;
    if (LDSM)
      L = unwind_path<TEX, MMAT>(static_cast<const float4*>(mat_lds), R, q, mk3(e.x, e.y, e.z), top,
                                 (meta & kRecFogDif) != 0, m, c);
    else
      L = unwind_path<TEX, MMAT>(S.umat, R, q, mk3(e.x, e.y, e.z), top, (meta & kRecFogDif) != 0, m, c);
    f3 np = mean * (float)n + L;
    float dv = (float)(++n);
    mean = mk3(np.x / dv, np.y / dv, np.z / dv);
  }
  F.color[3 * pix] = mean.x;
  F.color[3 * pix + 1] = mean.y;
  F.color[3 * pix + 2] = mean.z;
  F.count[pix] = n;
  F.display[3 * pix] = gamma8(mean.x);
  F.display[3 * pix + 1] = gamma8(mean.y);
  F.display[3 * pix + 2] = gamma8(mean.z);
  if (R.aov_n) fold_aovs(F, R, pix);
}

// fold_paths for launches of few micro-tiles (a rank of a multi-GPU render):
// the same backward passes and fold, with the serial per-pixel loop split
// over lanes. Micro-tile
// b (decode_block's tile-major order without the XCD placement or tile
// order; group g's records are row g * micro-tiles + b) takes 2^fold_log2
// workgroups, and each pixel 2^fold_log2 lanes: lane `sub` of a pixel
// unwinds (unwind_path) samples sub, sub + 2^k, ... and the pixel's first
// lane folds each step's 2^k radiances in sample order (frame.cpp:53-63),
// so the frame is bit-identical to groups x spp consecutive TraceScene
// calls. fs_render picks k > 0 only for launches of few micro-tiles (a rank
// of a multi-GPU render), whose one-lane-per-pixel fold ran 1024 serial
// steps on a quarter-full GPU.
// The loads are pipelined across a lane's samples as in fold_paths. (A
// separate kernel: the split's bookkeeping in fold_paths itself cost it 4-8
// VGPRs, a wave per SIMD, and 0.2-0.5 % on one GPU.)
template <bool TEX, bool MMAT, bool LDSM>
__global__ __launch_bounds__(kBlock) void fold_paths_split(DevScene S, DevFrame F, Launch P, PathRecords R,
                                                           uint32_t fold_log2) {
  extern __shared__ float4 mat_lds[];
  const uint32_t lane = threadIdx.x;
  if (LDSM) {
    for (uint32_t i = lane; i < 3 * S.num_materials; i += kBlock) mat_lds[i] = S.umat[i];
    __syncthreads();
  }
  const uint32_t fk = fold_log2, fl = 1u << fk;  // lanes per pixel
  const uint32_t b = blockIdx.x >> fk, part = blockIdx.x & (fl - 1u), tiles = gridDim.x >> fk;
  const uint32_t sub = lane & (fl - 1u);
  const uint32_t p = part * (kBlock >> fk) + (lane >> fk);  // pixel of the micro-tile
  const uint32_t micro_per_side = P.tile_size / 8, micro_per_tile = micro_per_side * micro_per_side;
  const uint32_t owned = b / micro_per_tile, micro = b % micro_per_tile;
  const uint32_t tile = P.tile_offset + owned * P.tile_stride;
  const uint32_t x = (tile % P.tiles_x) * P.tile_size + (micro % micro_per_side) * 8 + (p & 7);
  const uint32_t y = (tile / P.tiles_x) * P.tile_size + (micro / micro_per_side) * 8 + (p >> 3);
  if (x >= F.width || y >= F.height) return;  // a pixel's lanes leave together
  const size_t pix = (size_t)y * F.width + x;
  f3 mean = mk3(0, 0, 0);
  uint32_t n = 0;
  if (sub == 0) {
    mean = mk3(F.color[3 * pix], F.color[3 * pix + 1], F.color[3 * pix + 2]);
    n = F.count[pix];
  }
  const uint32_t total = P.groups * P.spp;
  auto rec = [&](uint32_t i) {  // sample i of the pixel: group i / spp, sample i % spp
    const uint32_t g = i / P.spp, k = i - g * P.spp;
    return rec_index(P, g * tiles + b, k * kBlock + p);
  };
  auto load_c = [&](uint64_t q, int top, float (&c)[kMaxDepth]) {
#pragma unroll
    for (int k = 0; k < (int)kMaxDepth; k++) c[k] = k <= top ? R.c[(uint64_t)k * R.n + q] : 0.0f;
  };
  auto top_of = [](const float4& e) { return (int)(__float_as_uint(e.w) & 0xFFu) - 1; };
  // this lane's samples i (a), i + fl (b), i + 2 fl (e2, m2); a lane past
  // the last sample keeps a zero record (top -1) that is never folded
  uint32_t i = sub;
  uint64_t qa = 0, qb = 0;
  float4 ea = make_float4(0, 0, 0, 0), eb = make_float4(0, 0, 0, 0);
  uint2 ma = make_uint2(0u, 0u), mb = make_uint2(0u, 0u);
  if (i < total) {
    qa = rec(i);
    ea = R.end[qa];
    if (!MMAT) ma = R.mats[qa];
  }
  if (i + fl < total) {
    qb = rec(i + fl);
    eb = R.end[qb];
    if (!MMAT) mb = R.mats[qb];
  }
  float ca[kMaxDepth], cb[kMaxDepth];
  load_c(qa, top_of(ea), ca);
  for (uint32_t base = 0; base < total; base += fl, i += fl) {  // base: wave-uniform
    uint64_t q2 = qb;
    float4 e2 = eb;
    uint2 m2 = mb;
    load_c(qb, top_of(eb), cb);
    if (i + 2 * fl < total) {
      q2 = rec(i + 2 * fl);
      e2 = R.end[q2];
      if (!MMAT) m2 = R.mats[q2];
    } else {
      e2 = make_float4(0, 0, 0, 0);
    }
    const uint32_t meta = __float_as_uint(ea.w);
    f3 L;
    if (LDSM)
      L = unwind_path<TEX, MMAT>(static_cast<const float4*>(mat_lds), R, qa, mk3(ea.x, ea.y, ea.z), top_of(ea),
                                 (meta & kRecFogDif) != 0, ma, ca);
    else
      L = unwind_path<TEX, MMAT>(S.umat, R, qa, mk3(ea.x, ea.y, ea.z), top_of(ea), (meta & kRecFogDif) != 0, ma, ca);
    const uint32_t here = min(fl, total - base);  // samples of this step
    {
      for (uint32_t s = 0; s < here; s++) {  // the step's samples in order, folded by the pixel's first lane
        const int src = (int)((lane & ~(fl - 1u)) + s);
        const f3 Ls = mk3(__shfl(L.x, src), __shfl(L.y, src), __shfl(L.z, src));
        if (sub == 0) {
          f3 np = mean * (float)n + Ls;
          float dv = (float)(++n);
          mean = mk3(np.x / dv, np.y / dv, np.z / dv);
        }
      }
    }
    qa = qb;
    ea = eb;
    ma = mb;
#pragma unroll
    for (int k = 0; k < (int)kMaxDepth; k++) ca[k] = cb[k];
    qb = q2;
    eb = e2;
    mb = m2;
  }
  if (sub != 0) return;
  F.color[3 * pix] = mean.x;
  F.color[3 * pix + 1] = mean.y;
  F.color[3 * pix + 2] = mean.z;
  F.count[pix] = n;
  F.display[3 * pix] = gamma8(mean.x);
  F.display[3 * pix + 1] = gamma8(mean.y);
  F.display[3 * pix + 2] = gamma8(mean.z);
  if (R.aov_n) fold_aovs(F, R, pix);
}

// TraceRange (engine.cpp:298-329): one query per lane, the camera ray through
// (x, y) without jitter or aperture, Scene::Trace, distance to the hit point.
template <bool SOCT>
__global__ __launch_bounds__(kBlock) void trace_range_kernel(DevScene S, DevCamera C, const float2* __restrict__ xy,
                                                             uint32_t n, float* __restrict__ out) {
  __shared__ uint32_t stk_all[kTraversalStack * kBlock];
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const float2 q = xy[i];
  // engine.cpp:314-320: the jitter-free form of camera_ray's projection
  float xd = (float)((double)C.hpw * ((double)(q.x / (C.width - 1)) * 2.0 - 1.0));
  float yd = (float)((double)C.hph * ((double)(q.y / (C.height - 1)) * 2.0 - 1.0));
  Ray r;
  r.start = C.origin;
  r.stop = C.proj_origin + C.right * xd + C.up * yd;
  r.dir = r.stop - r.start;
  MinHit h;
  Tally<false> tally;
  PhaseAcc pa;
  scene_trace_min<false, false, false, SOCT>(S, r, h, stk_all + threadIdx.x, tally, pa);
  float d = C.z_far;
  if (h.obj >= 0) {
    f3 p = h.point ? r.start : r.start + r.dir * h.t;
    d = length(p - C.origin);
  }
  out[i] = d;
}

// ---- multi-GPU packing: 10 words per pixel (colour, count, normal, depth, id)
constexpr uint32_t kPackWords = 10;

__global__ void pack_tiles(DevFrame F, Launch P, uint32_t owned_max, uint32_t* __restrict__ out) {
  const uint32_t ts = P.tile_size;
  size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t total = (size_t)owned_max * ts * ts;
  if (gid >= total) return;
  uint32_t k = (uint32_t)(gid / (ts * ts)), in = (uint32_t)(gid % (ts * ts));
  uint32_t tile = P.tile_offset + k * P.tile_stride;
  uint32_t* o = out + gid * kPackWords;
  uint32_t tiles_y = (F.height + ts - 1) / ts;
  if (tile >= P.tiles_x * tiles_y) {
    for (uint32_t i = 0; i < kPackWords; i++) o[i] = 0;
    return;
  }
  uint32_t x = (tile % P.tiles_x) * ts + in % ts, y = (tile / P.tiles_x) * ts + in / ts;
  if (x >= F.width || y >= F.height) {
    for (uint32_t i = 0; i < kPackWords; i++) o[i] = 0;
    return;
  }
  size_t p = (size_t)y * F.width + x;
  o[0] = __float_as_uint(F.color[3 * p]);
  o[1] = __float_as_uint(F.color[3 * p + 1]);
  o[2] = __float_as_uint(F.color[3 * p + 2]);
  o[3] = F.count[p];
  o[4] = __float_as_uint(F.normal[3 * p]);
  o[5] = __float_as_uint(F.normal[3 * p + 1]);
  o[6] = __float_as_uint(F.normal[3 * p + 2]);
  o[7] = __float_as_uint(F.depth[p]);
  o[8] = (uint32_t)(F.material[p] & 0xFFFFFFFFull);
  o[9] = (uint32_t)(F.material[p] >> 32);
}

__global__ void unpack_tiles(DevFrame F, Launch P, uint32_t owned_max, uint32_t nranks, uint32_t self,
                             const uint32_t* __restrict__ in) {
  const uint32_t ts = P.tile_size;
  size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t per_rank = (size_t)owned_max * ts * ts;
  if (gid >= per_rank * nranks) return;
  uint32_t rank = (uint32_t)(gid / per_rank);
  if (rank == self) return;
  size_t rem = gid % per_rank;
  uint32_t k = (uint32_t)(rem / (ts * ts)), inpix = (uint32_t)(rem % (ts * ts));
  uint32_t tile = rank + k * nranks;
  uint32_t tiles_y = (F.height + ts - 1) / ts;
  if (tile >= P.tiles_x * tiles_y) return;
  uint32_t x = (tile % P.tiles_x) * ts + inpix % ts, y = (tile / P.tiles_x) * ts + inpix / ts;
  if (x >= F.width || y >= F.height) return;
  size_t p = (size_t)y * F.width + x;
  const uint32_t* w = in + gid * kPackWords;
  float c0 = __uint_as_float(w[0]), c1 = __uint_as_float(w[1]), c2 = __uint_as_float(w[2]);
  F.color[3 * p] = c0;
  F.color[3 * p + 1] = c1;
  F.color[3 * p + 2] = c2;
  F.count[p] = w[3];
  F.normal[3 * p] = __uint_as_float(w[4]);
  F.normal[3 * p + 1] = __uint_as_float(w[5]);
  F.normal[3 * p + 2] = __uint_as_float(w[6]);
  F.depth[p] = __uint_as_float(w[7]);
  F.material[p] = (uint64_t)w[8] | ((uint64_t)w[9] << 32);
  F.display[3 * p] = gamma8(c0);
  F.display[3 * p + 1] = gamma8(c1);
  F.display[3 * p + 2] = gamma8(c2);
}

}  // namespace dev
}  // namespace fs

// ============================================================================
// C ABI
// ============================================================================
using namespace fs;

namespace {

thread_local std::string g_error;

int fail(int code, const std::string& msg) {
  g_error = msg;
  return code;
}

#define FS_HIP(call)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(FS_ERR_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_));       \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// The lookahead of a 1-spp-style render (fs_options.lookahead = w calls):
// the next w calls' samples traced in the background, in launches of
// g = min(16, max(1, w / 3)) calls each (one group per call: a launch of several
// calls amortizes the latency-bound drain of its last paths), each launch in
// a slot of its own (stream, path records, anchor rows, queues, per-call AOV
// planes), so a launch starts while the earlier ones drain. The context
// stream has the device's highest priority and the slots' streams its
// lowest, so the folds (on the critical path of the caller's frame) take
// free wave slots first.
constexpr uint32_t kLookaheadSpp = 4;
constexpr uint32_t kLookaheadMax = 48;  // fs_options.lookahead <= 48
constexpr uint32_t kLookGroupMax = 16;  // calls per lookahead launch
constexpr int kLookSlots = 3;
struct LookKey {  // everything a lookahead trace depends on
  fs_camera camera;
  fs_render_params params;  // sample_base: the first sample it traces
  fs_options opt;
  uint64_t scene_gen;
};
struct Lookahead {
  hipStream_t stream[kLookSlots] = {};
  hipEvent_t traced[kLookSlots] = {}, folded[kLookSlots] = {}, order = nullptr, kev0[kLookSlots] = {},
             kev1[kLookSlots] = {};
  DevBuf rows[kLookSlots], queues[kLookSlots];
  // per call (group) the AOV planes of its last sample (normal, depth,
  // material), which the call's fold copies into the frame
  DevBuf nrm[kLookSlots], dep[kLookSlots], mid[kLookSlots];
  uint32_t groups[kLookSlots] = {};  // calls the slot's launch traced (key.params.sample_base: the first)
  bool pending[kLookSlots] = {};
  bool folded_valid[kLookSlots] = {};  // folded[i] recorded: the last fold that read slot i
  LookKey key[kLookSlots];
  Launch L[kLookSlots];
  PathRecords R[kLookSlots];
  uint64_t used[kLookSlots] = {};  // when the slot was last launched (its reuse order)
  uint64_t tick = 0;
  // the slots of the last two launches, newest first (-1: none): a launch
  // starts only once the launch two before it has finished, so it takes the
  // wave slots the previous launch frees as it drains and never shares the
  // chip with the launch the caller needs next
  int prev[2] = {-1, -1};
  // the last render's key (valid: it could take a lookahead): a render
  // launches lookahead traces only when it continues that one (same key,
  // sample_base = the last one's + spp) or folded a lookahead itself, so a
  // camera that moves every frame starts no background work
  LookKey last;
  bool last_valid = false;
  uint32_t ramp = 0;  // launches since the sequence started (their calls: 1, 2, 4, ... up to g)
  // a discarded slot's queues were set past every block on the context
  // stream (its waves stop taking blocks); the slot's next launch waits for it
  hipEvent_t cancelled[kLookSlots] = {};
  bool cancel_valid[kLookSlots] = {};
  // bg_waves of the last (trace, fold) kernel pair
  const void* bg_trace = nullptr;
  const void* bg_fold = nullptr;
  uint32_t bg_w = 0;
};

}  // namespace

struct fs_context {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> kev;  // (start, end) of each trace-kernel launch of the last render
  bool have_scene = false;
  DevBuf objects, nodes, tris, tri_normals, tri_tex, tex_rgb, tex_info, materials, umat, rmat, table, counters, pack_send,
      tile_order,
      pack_recv, range_io, tree, tree_objs;
  fs_options opt{};  // fs_set_options; fs_options_default() at fs_create
  bool has_textures = false;
  bool has_parking = false;  // a mesh of >= park_min_tris triangles: the PARKED schedule
  bool has_walks = false;    // a mesh with a BVH (not small): the kernel needs the walk stack
  bool many_materials = false;  // > kPackedMaterials: material ids in scratch rows (MMAT kernels)
  bool has_frost = false;  // a Glass of frost != 0: its refraction rotates by cosf/sinf (TRIG kernels)
  const char* last_kernel = "";  // the trace kernel the last fs_render launched
  std::vector<uint32_t> tile_order_host;  // the device tile_order buffer holds this order of ...
  uint64_t tile_order_key[3] = {0, 0, 0};  // ... the tile set (offset, stride, owned; width, height) it was built for
  uint32_t last_launches = 0;    // trace-kernel launches of the last fs_render
  uint32_t last_launch_spp = 0;  // samples per pixel of its largest launch
  DevScene scene{};
  uint32_t num_objects = 0;
  PreparedScene host;
  double upload_ms = 0.0;
  double gpu_bvh_ms = 0.0;                              // device BVH builds of the last upload
  uint64_t gpu_bvh_nodes = 0, gpu_bvh_tris = 0;         // nodes they built / triangles they placed
  float last_ms = 0.0f;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  DevBuf rows;  // the Fog anchor rows and the path records of a render (path_records)
  DevBuf queues;  // per-XCD work-queue counters of the persistent trace kernel
  uint32_t cus = 0;  // compute units: the persistent grid is one wave per wave slot
  uint64_t scene_gen = 0;  // uploads so far (a lookahead is of one upload)
  Lookahead la;
  int last_spec = -1;  // the lookahead slot the last fs_render folded, or -1
};

struct fs_frame {
  fs_context* ctx = nullptr;
  uint32_t width = 0, height = 0;
  DevBuf color, count, display, normal, depth, material;
  void* pinned[FS_PLANE_MATERIAL + 1] = {};  // fs_frame_map's page-locked copies
};

namespace {

int set_device(fs_context* ctx) {
  FS_HIP(hipSetDevice(ctx->device));
  return FS_OK;
}

// Allocates bytes + extra (the extra tail is left for device-side writers)
// and copies `bytes` from the host.
int upload(fs_context* ctx, DevBuf* b, const void* src, size_t bytes, size_t extra = 0) {
  b->release();
  size_t alloc = bytes + extra ? bytes + extra : 16;
  FS_HIP(hipMalloc(&b->p, alloc));
  b->bytes = alloc;
  if (bytes) FS_HIP(hipMemcpyAsync(b->p, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  // The tail (device-built slots a build may leave unused, or the placeholder
  // of an empty array) starts zeroed, so equal uploads are equal bytes.
  if (alloc > bytes) FS_HIP(hipMemsetAsync((char*)b->p + bytes, 0, alloc - bytes, ctx->stream));
  return FS_OK;
}

int ensure(DevBuf* b, size_t bytes) {
  if (b->bytes >= bytes && b->p) return FS_OK;
  b->release();
  FS_HIP(hipMalloc(&b->p, bytes));
  b->bytes = bytes;
  return FS_OK;
}

DevFrame frame_view(fs_frame* f) {
  DevFrame F;
  F.color = (float*)f->color.p;
  F.count = (uint32_t*)f->count.p;
  F.display = (uint8_t*)f->display.p;
  F.normal = (float*)f->normal.p;
  F.depth = (float*)f->depth.p;
  F.material = (uint64_t*)f->material.p;
  F.width = f->width;
  F.height = f->height;
  return F;
}

// engine.cpp:170-197, evaluated on the host with the same libm as the oracle.
DevCamera camera_basis(const fs_camera* c, uint32_t W, uint32_t H) {
  DevCamera b;
  b.width = (float)W;
  b.height = (float)H;
  float aspect = b.width / b.height;
  float fovy = (float)((double)(c->fov_y * kPi) / 180.0);
  float fovx = (float)(2.0 * std::atan(std::tan((double)fovy * 0.5) * (double)aspect));
  f3 origin = mk3(c->origin[0], c->origin[1], c->origin[2]);
  f3 target = mk3(c->target[0], c->target[1], c->target[2]);
  f3 fwd = normalize(target - origin);
  b.origin = origin;
  b.right = normalize(cross(mk3(0, 1, 0), fwd));
  b.up = normalize(cross(fwd, b.right));
  b.hph = tanf(fovy * 0.5f) * c->z_far;
  b.hpw = tanf(fovx * 0.5f) * c->z_far;
  b.proj_origin = origin + fwd * c->z_far;
  b.focal = plane_np(fwd * -1.0f, origin + fwd * c->focal_depth);
  b.aperture = c->aperture_size;
  b.z_far = c->z_far;
  b.fast_render = c->fast_render;
  return b;
}

// Scratch of a render, carved out of one allocation: per wave of the grid,
// the per-lane Fog anchor rows; per sample of the launch, its path record
// (PathRecords: c and Ceramic's term per level, the end state, the material
// ids, and on textured scenes the texel per level).
size_t record_bytes(bool tex, bool mmat) {
  return 8 * kMaxDepth + 16 + (mmat ? 4 * kMaxDepth : 8) + (tex ? 16 * kMaxDepth : 0);
}
size_t rows_bytes(uint64_t wave_lanes, uint64_t samples, bool tex, bool mmat) {
  return (size_t)wave_lanes * 32 + (size_t)samples * record_bytes(tex, mmat) + 6 * 256;  // + alignment
}
int carve_records(DevBuf* rows, uint64_t wave_lanes, uint64_t samples, PathRecords* R, float4** anchors, bool tex,
                  bool mmat);
int path_records(fs_context* ctx, uint64_t wave_lanes, uint64_t samples, PathRecords* R, float4** anchors, bool tex,
                 bool mmat) {
  const size_t bytes = rows_bytes(wave_lanes, samples, tex, mmat);
  // Shrink a buffer more than 4x (and 1 GiB) larger than this render needs:
  // a context that once rendered a long launch does not keep its records.
  if (ctx->rows.bytes > 4 * bytes && ctx->rows.bytes - bytes > (1ull << 30)) ctx->rows.release();
  if (ctx->rows.bytes < bytes) {
    int rc = ensure(&ctx->rows, bytes);
    if (rc) return rc == FS_ERR_DEVICE ? fail(FS_ERR_NOMEM, "path records: " + g_error) : rc;
  }
  return carve_records(&ctx->rows, wave_lanes, samples, R, anchors, tex, mmat);
}
int carve_records(DevBuf* rows, uint64_t wave_lanes, uint64_t samples, PathRecords* R, float4** anchors, bool tex,
                  bool mmat) {
  char* p = (char*)rows->p;
  auto take = [&](size_t n) {
    char* q = p;
    p += (n + 255) & ~(size_t)255;
    return q;
  };
  *R = PathRecords{};
  *anchors = (float4*)take(32ull * wave_lanes);
  R->n = samples;
  R->c = (float*)take(4ull * kMaxDepth * samples);
  R->ds = (float*)take(4ull * kMaxDepth * samples);
  R->end = (float4*)take(16ull * samples);
  R->mats = mmat ? nullptr : (uint2*)take(8ull * samples);
  R->mat = mmat ? (uint32_t*)take(4ull * kMaxDepth * samples) : nullptr;
  R->tex = tex ? (float4*)take(16ull * kMaxDepth * samples) : nullptr;
  if ((size_t)(p - (char*)rows->p) > rows->bytes) return fail(FS_ERR_NOMEM, "path record overflow");
  return FS_OK;
}

// Waits for every lookahead trace of the context and drops them (before the
// scene, the tile order or the context they read is replaced or freed).
void la_quiesce(fs_context* ctx) {
  for (int i = 0; i < kLookSlots; i++) {
    if (ctx->la.stream[i]) (void)hipStreamSynchronize(ctx->la.stream[i]);
    ctx->la.pending[i] = false;
  }
}

size_t plane_bytes(int plane, size_t pixels) {
  switch (plane) {
    case FS_PLANE_COLOR:
    case FS_PLANE_NORMAL:
      return 12 * pixels;
    case FS_PLANE_COUNT:
    case FS_PLANE_DEPTH:
      return 4 * pixels;
    case FS_PLANE_DISPLAY:
      return 3 * pixels;
    case FS_PLANE_MATERIAL:
      return 8 * pixels;
    default:
      return 0;
  }
}
DevBuf* plane_buf(fs_frame* f, int plane) {
  switch (plane) {
    case FS_PLANE_COLOR:
      return &f->color;
    case FS_PLANE_COUNT:
      return &f->count;
    case FS_PLANE_DISPLAY:
      return &f->display;
    case FS_PLANE_NORMAL:
      return &f->normal;
    case FS_PLANE_DEPTH:
      return &f->depth;
    case FS_PLANE_MATERIAL:
      return &f->material;
    default:
      return nullptr;
  }
}

int check_params(const fs_render_params* p, const fs_frame* f, uint32_t* ts, uint32_t* stride) {
  if (!p) return fail(FS_ERR_INVALID, "null render params");
  if (p->width != f->width || p->height != f->height)
    return fail(FS_ERR_INVALID, "render size does not match the frame");
  if (p->width < 2 || p->height < 2) return fail(FS_ERR_INVALID, "frame must be at least 2x2 (engine.cpp:214)");
  *ts = p->tile_size ? p->tile_size : 64;
  *stride = p->tile_stride ? p->tile_stride : 1;
  if (*ts % 8 || *ts > 1024) return fail(FS_ERR_INVALID, "tile_size must be a multiple of 8, <= 1024");
  if (p->tile_offset >= *stride) return fail(FS_ERR_INVALID, "tile_offset must be < tile_stride");
  if ((uint64_t)p->sample_base + p->spp > (1ull << 20))
    return fail(FS_ERR_INVALID, "sample index must stay below 2^20 (seed layout)");
  return FS_OK;
}

// Waves per SIMD (__launch_bounds__) of the three kernel families: the lean
// kernels (6), the parked-walk kernel (6; 5 waves with 96 VGPRs measured
// C4 -6.5 %, 7 waves with a 22-entry stack -9.5 %) and the NOWALK kernel (8:
// no LDS stack, its LDS rows take 4 KiB per wave; 6 waves -4 %, 7 -1.5 %).
#ifndef FS_SUSP_WAVES
#define FS_SUSP_WAVES 6  // A/B builds only (make ab DEFS=-DFS_SUSP_WAVES=7)
#endif
constexpr int kLeanWaves = 6, kSuspWaves = FS_SUSP_WAVES, kNowalkWaves = 8;

#define FS_STR2(x) #x
#define FS_STR(x) FS_STR2(x)

// The instantiations of the lean kernel: <COUNT, waves, TEX, SUSP (parked
// walks), MMAT (material ids in scratch rows), SOCT (object octree), NOWALK>.
// Textured scenes never park. Names as rocprofv3 prints the uncounted ones
// (fs_last_kernel).
typedef void (*LeanFn)(DevScene, DevCamera, DevFrame, Launch, PathRecords, float4*, uint32_t*, DevCounters*);
typedef void (*FoldFn)(DevScene, DevFrame, Launch, PathRecords);
typedef void (*FoldSplitFn)(DevScene, DevFrame, Launch, PathRecords, uint32_t);
template <bool TEX, bool MMAT>
FoldFn pick_fold2(bool lds_materials) {
  return lds_materials ? dev::fold_paths<TEX, MMAT, true> : dev::fold_paths<TEX, MMAT, false>;
}
FoldFn pick_fold(bool tex, bool mmat, bool lds_materials) {
  return tex ? (mmat ? pick_fold2<true, true>(lds_materials) : pick_fold2<true, false>(lds_materials))
             : (mmat ? pick_fold2<false, true>(lds_materials) : pick_fold2<false, false>(lds_materials));
}
template <bool TEX, bool MMAT>
FoldFn pick_fold_lite2(bool lds_materials) {
  return lds_materials ? dev::fold_paths_lite<TEX, MMAT, true> : dev::fold_paths_lite<TEX, MMAT, false>;
}
FoldFn pick_fold_lite(bool tex, bool mmat, bool lds_materials) {
  return tex ? (mmat ? pick_fold_lite2<true, true>(lds_materials) : pick_fold_lite2<true, false>(lds_materials))
             : (mmat ? pick_fold_lite2<false, true>(lds_materials) : pick_fold_lite2<false, false>(lds_materials));
}
template <bool TEX, bool MMAT>
FoldSplitFn pick_fold_split2(bool lds_materials) {
  return lds_materials ? dev::fold_paths_split<TEX, MMAT, true> : dev::fold_paths_split<TEX, MMAT, false>;
}
FoldSplitFn pick_fold_split(bool tex, bool mmat, bool lds_materials) {
  return tex ? (mmat ? pick_fold_split2<true, true>(lds_materials) : pick_fold_split2<true, false>(lds_materials))
             : (mmat ? pick_fold_split2<false, true>(lds_materials) : pick_fold_split2<false, false>(lds_materials));
}
struct LeanKernel {
  LeanFn fn;
  const char* name;
  uint32_t waves;  // waves per SIMD (__launch_bounds__)
};
template <bool TEX, bool SUSP, bool MMAT, bool SOCT = false, bool NOWALK = false, bool TRIG = false>
LeanKernel lean_kernel(bool count) {
  constexpr int W = SUSP ? kSuspWaves : NOWALK ? kNowalkWaves : kLeanWaves;
  static const std::string name = std::string("render_kernel_lean<false, ") + std::to_string(W) + ", " +
                                  (TEX ? "true" : "false") + ", " + (SUSP ? "true" : "false") + ", " +
                                  (MMAT ? "true" : "false") + ", " + (SOCT ? "true" : "false") + ", " +
                                  (NOWALK ? "true" : "false") + ", " + (TRIG ? "true>" : "false>");
  return {count ? (LeanFn)dev::render_kernel_lean<true, W, TEX, SUSP, MMAT, SOCT, NOWALK, TRIG>
                : (LeanFn)dev::render_kernel_lean<false, W, TEX, SUSP, MMAT, SOCT, NOWALK, TRIG>,
          name.c_str(), (uint32_t)W};
}
template <bool TEX, bool SUSP, bool MMAT, bool SOCT = false, bool NOWALK = false>
LeanKernel lean_kernel(bool count, bool trig) {
  return trig ? lean_kernel<TEX, SUSP, MMAT, SOCT, NOWALK, true>(count)
              : lean_kernel<TEX, SUSP, MMAT, SOCT, NOWALK, false>(count);
}
// Scenes traced through the object octree take one instantiation that covers
// textures and any material count (their object loop is per lane anyway).
// Untextured scenes whose meshes are all small (no BVH walk) take the NOWALK
// instantiation: no walk stack, shading rows in LDS. trig: the host libm's
// sinf/cosf for a thin-lens camera or frosted glass (TRIG; textured kernels
// always, for their sphere maps' atan2f too).
LeanKernel pick_kernel(bool count, bool tex, bool parked, bool many_materials, bool object_tree, bool walks,
                       bool trig) {
  if (object_tree) return lean_kernel<true, false, true, true, false, true>(count);
  if (tex)
    return many_materials ? lean_kernel<true, false, true, false, false, true>(count)
                          : lean_kernel<true, false, false, false, false, true>(count);
  if (parked)
    return many_materials ? lean_kernel<false, true, true>(count, trig) : lean_kernel<false, true, false>(count, trig);
  if (!walks)
    return many_materials ? lean_kernel<false, false, true, false, true>(count, trig)
                          : lean_kernel<false, false, false, false, true>(count, trig);
  return many_materials ? lean_kernel<false, false, true>(count, trig) : lean_kernel<false, false, false>(count, trig);
}

bool valid_options(const fs_options* o, std::string* why) {
  if (o->schedule < FS_SCHEDULE_AUTO || o->schedule > FS_SCHEDULE_PARKED) *why = "unknown schedule";
  else if (o->samples_per_block < 1 || o->samples_per_block > kChunk) *why = "samples_per_block must be 1..64";
  else if (o->xcd_bands > 2) *why = "xcd_bands must be 0, 1 or 2";
  else if (o->bvh_leaf < 1 || o->bvh_leaf > kMaxLeafCount) *why = "bvh_leaf must be 1..15";
  else if (o->bvh_bins < 2 || o->bvh_bins > 64) *why = "bvh_bins must be 2..64";
  else if (o->node_layout > FS_NODE_LAYOUT_PAIRS) *why = "unknown node_layout";
  else if (o->persist > 1) *why = "persist must be 0 or 1";
  else if (o->small_mesh_tris > kMaxSmallMeshTris) *why = "small_mesh_tris must be 0..64";
  else if (o->park_lanes > 64 || o->park_lanes_small > 64) *why = "park_lanes must be 0..64";
  else if (o->lds_rows > 1) *why = "lds_rows must be 0 or 1";
  else if (o->lookahead > kLookaheadMax) *why = "lookahead must be 0..48";
  else return true;
  return false;
}

// The record budget of a render: fs_plan_render's explicit bytes, else the
// context's record_budget_mb, else kRecordBytes (96 GiB).
uint64_t record_budget(const fs_options& O, uint64_t explicit_bytes) {
  if (explicit_bytes) return explicit_bytes;
  return O.record_budget_mb ? (uint64_t)O.record_budget_mb << 20 : kRecordBytes;
}

// How a render is cut into launches: the owned tiles in `parts` parts of at
// most `tiles` consecutive owned tiles, each part's samples in launches of G
// groups of `chunk` samples per block. A launch of blocks b holds
// b x G x chunk x 64 path records. Normally one part takes every owned tile
// and only G follows the record budget; a frame whose one-group launch
// exceeds the budget (16K x 16K at 16 spp: 378 GB of records)
// renders in tile parts and, below one tile per part, with fewer samples per
// block. Tiles are disjoint and each pixel still takes its samples in order,
// so the frame is the same.
struct Plan {
  uint32_t chunk = 1, G = 1, tiles = 0, parts = 0;
  // one step smaller after an allocation failure; false when at the minimum
  bool shrink(uint32_t owned) {
    if (G > 1) {
      G = (G + 1) / 2;
    } else if (tiles > 1) {
      tiles = (tiles + 1) / 2;
      parts = (owned + tiles - 1) / tiles;
    } else if (chunk > 1) {
      chunk = (chunk + 1) / 2;
    } else {
      return false;
    }
    return true;
  }
  uint32_t launches(uint32_t spp) const {  // per part: the full groups, then the remainder
    const uint32_t full = spp / chunk;
    return parts * ((full + G - 1) / G + (spp % chunk ? 1u : 0u));
  }
};
int make_plan(uint32_t owned, uint32_t mpt, uint32_t spp, const fs_options& O, uint64_t budget, size_t rec_bytes,
              Plan* out) {
  Plan p;
  // a launch of fewer samples than a block holds sizes its records to spp
  // (the 1-spp drop-in loop: no 16x over-allocation)
  p.chunk = std::min<uint32_t>(O.samples_per_block, std::max<uint32_t>(spp, 1));
  p.tiles = owned;
  const uint64_t cap = budget / rec_bytes;          // path records one launch may hold
  const uint64_t tile_samples = (uint64_t)mpt * kBlock;  // one sample of each pixel of one tile
  if (owned && tile_samples * p.chunk * owned > cap) {
    if (tile_samples > cap)
      return fail(FS_ERR_NOMEM, "path-record budget of " + std::to_string(budget) +
                                    " bytes is below one tile x one sample (" +
                                    std::to_string(tile_samples * rec_bytes) + " bytes)");
    if (tile_samples * p.chunk > cap) p.chunk = (uint32_t)(cap / tile_samples);  // >= 1
    p.tiles = (uint32_t)std::min<uint64_t>(owned, cap / (tile_samples * p.chunk));
  }
  p.parts = owned ? (owned + p.tiles - 1) / p.tiles : 0;
  // Sample groups: a launch renders G runs of `chunk` samples as G x blocks
  // blocks, then fold_paths runs their backward passes and folds them in
  // order. Persistent waves have a launch tail of one task path, so G is as
  // large as the budget allows (C4 at 1080p x 1024 spp: two launches of 512
  // spp). One-shot waves size G so a launch holds >= kGroupTargetBlocks blocks
  // (about 43 per wave slot of the chip), within the budget.
  const uint64_t blocks = (uint64_t)p.tiles * mpt;
  const uint32_t full_chunks = spp / p.chunk;
  if (blocks && full_chunks > 1) {
    const uint64_t fit = std::max<uint64_t>(1, cap / (blocks * p.chunk * kBlock));
    uint64_t want = O.groups    ? (uint64_t)O.groups
                    : O.persist ? fit
                                : std::min<uint64_t>(fit, (kGroupTargetBlocks + blocks - 1) / blocks);
    want = std::max<uint64_t>(1, std::min<uint64_t>({want, full_chunks, ((1ull << 31) - 1) / blocks}));
    const uint32_t nl = (uint32_t)((full_chunks + want - 1) / want);  // launches for the full chunks
    p.G = (full_chunks + nl - 1) / nl;                                 // balanced groups per launch
  }
  *out = p;
  return FS_OK;
}

// Waves per SIMD of a background (lookahead) trace launch: at most the
// kernel's bound, and few enough that kBgFoldWaves waves of the fold kernel
// fit in the SIMD's 512 VGPRs beside them (allocation in blocks of 8): C4 5 of
// 6 trace waves (80 VGPRs) beside 2 fold waves (50 VGPRs) measured 1744 /
// 1852 M samples/s in the window loop (lookahead 12 / 24), 3 beside 4 1703 /
// 1873; C2 6 of 8 (64 VGPRs) 2990 / 3010, 4 3376 / 3419; C3 1166 / 1208 and
// 1198 / 1211 (profiles/r06/ab_bg_waves.log).
constexpr int kBgFoldWaves = 4;
uint32_t bg_waves(LeanFn trace, uint32_t waves, FoldFn fold) {
  hipFuncAttributes t{}, f{};
  if (hipFuncGetAttributes(&t, reinterpret_cast<const void*>(trace)) != hipSuccess ||
      hipFuncGetAttributes(&f, reinterpret_cast<const void*>(fold)) != hipSuccess || t.numRegs <= 0 ||
      f.numRegs <= 0) {
    (void)hipGetLastError();
    return waves;
  }
  const int vt = (t.numRegs + 7) / 8 * 8, vf = (f.numRegs + 7) / 8 * 8;
  return (uint32_t)std::max(1, std::min<int>((int)waves, (512 - kBgFoldWaves * vf) / vt));
}

// Resident waves per CU of a fold kernel with `lds` bytes of dynamic LDS
// (the HIP occupancy query on its compiled resources; 28 if it fails).
uint32_t fold_waves_per_cu(const void* fn, uint32_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds) != hipSuccess || per_cu <= 0) {
    (void)hipGetLastError();
    return 28;
  }
  return (uint32_t)per_cu;
}
template <class Fn>
uint32_t fold_waves_per_cu(Fn fn, uint32_t lds) {
  return fold_waves_per_cu(reinterpret_cast<const void*>(fn), lds);
}

}  // namespace

extern "C" {

int fs_abi_version(void) { return FS_ABI_VERSION; }
const char* fs_last_error(void) { return g_error.c_str(); }

int fs_device_count(int* count) {
  if (!count) return fail(FS_ERR_INVALID, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return FS_OK;
}

int fs_create(int device, fs_context** out) {
  if (!out) return fail(FS_ERR_INVALID, "null out");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(FS_ERR_DEVICE, "no HIP device available");
  if (device < 0 || device >= n) return fail(FS_ERR_INVALID, "device index out of range");
  std::unique_ptr<fs_context> ctx(new fs_context());
  ctx->device = device;
  fs_options_default(&ctx->opt);
  FS_HIP(hipSetDevice(device));
  {  // the highest priority: a fold waiting for wave slots goes before lookahead traces
    int least = 0, greatest = 0;
    FS_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    FS_HIP(hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, greatest));
  }
  FS_HIP(hipEventCreate(&ctx->ev0));
  FS_HIP(hipEventCreate(&ctx->ev1));
  FS_HIP(hipMalloc(&ctx->counters.p, sizeof(DevCounters)));
  ctx->counters.bytes = sizeof(DevCounters);
  FS_HIP(hipMemset(ctx->counters.p, 0, sizeof(DevCounters)));
  int cus = 0;
  FS_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  ctx->cus = cus > 0 ? (uint32_t)cus : 1u;
  FS_HIP(hipMalloc(&ctx->queues.p, 8 * dev::kQueueStride * sizeof(uint32_t)));
  ctx->queues.bytes = 8 * dev::kQueueStride * sizeof(uint32_t);
  *out = ctx.release();
  return FS_OK;
}

int fs_destroy(fs_context* ctx) {
  if (!ctx) return FS_OK;
  (void)hipSetDevice(ctx->device);
  la_quiesce(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  for (int i = 0; i < kLookSlots; i++) {
    Lookahead& A = ctx->la;
    for (DevBuf* b : {&A.rows[i], &A.queues[i], &A.nrm[i], &A.dep[i], &A.mid[i]}) b->release();
    for (hipEvent_t e : {A.traced[i], A.folded[i], A.kev0[i], A.kev1[i], A.cancelled[i]})
      if (e) (void)hipEventDestroy(e);
    if (A.stream[i]) (void)hipStreamDestroy(A.stream[i]);
  }
  if (ctx->la.order) (void)hipEventDestroy(ctx->la.order);
  for (DevBuf* b : {&ctx->objects, &ctx->nodes, &ctx->tris, &ctx->tri_normals, &ctx->tri_tex, &ctx->tree, &ctx->tree_objs,
                    &ctx->tex_rgb, &ctx->tex_info, &ctx->materials, &ctx->umat, &ctx->rmat, &ctx->table, &ctx->range_io,
                    &ctx->counters, &ctx->pack_send, &ctx->pack_recv, &ctx->tile_order, &ctx->queues})
    b->release();
  ctx->rows.release();
  for (hipEvent_t e : ctx->kev) (void)hipEventDestroy(e);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return FS_OK;
}

int fs_options_default(fs_options* o) {
  if (!o) return fail(FS_ERR_INVALID, "null options");
  *o = fs_options{};
  o->schedule = FS_SCHEDULE_AUTO;
  o->park_lanes = 12;       // C4 (1 M-face blob): 12 best on the round-3 build (10: -0.5 %, 14: -0.1 %)
  o->park_lanes_small = 6;  // C3 (38 k and 209 k-face meshes): 4-6 best
  o->park_min_tris = kParkMinTris;
  o->lds_rows = 1;
  o->samples_per_block = 16;  // persistent waves: C4 +0.7 %, C3 +2 %, C2 +3 % over 64 (8 and 4 no better)
  o->groups = 0;
  o->group_major = 0;
  o->tile_order = 1;
  o->xcd_bands = 2;
  o->gpu_bvh_min_tris = kGpuBvhMinTris;
  o->bvh_leaf = 2;
  o->bvh_bins = 16;
  o->bvh_threads = 0;
  o->node_layout = FS_NODE_LAYOUT_DEPTH_FIRST;
  o->build_log = 0;
  o->persist = 1;
  o->small_mesh_tris = 16;
  o->lookahead = 24;
  return FS_OK;
}

int fs_set_options(fs_context* ctx, const fs_options* opt) {
  if (!ctx || !opt) return fail(FS_ERR_INVALID, "null argument");
  std::string why;
  if (!valid_options(opt, &why)) return fail(FS_ERR_INVALID, "fs_set_options: " + why);
  ctx->opt = *opt;
  return FS_OK;
}

int fs_get_options(fs_context* ctx, fs_options* out) {
  if (!ctx || !out) return fail(FS_ERR_INVALID, "null argument");
  *out = ctx->opt;
  return FS_OK;
}

int fs_upload_scene(fs_context* ctx, const fs_scene_desc* desc) { return fs_upload_scene_ex(ctx, desc, 0u); }

int fs_upload_scene_ex(fs_context* ctx, const fs_scene_desc* desc, uint32_t flags) {
  if (!ctx) return fail(FS_ERR_INVALID, "null context");
  if (flags & ~FS_UPLOAD_GPU_BVH) return fail(FS_ERR_INVALID, "unknown upload flags");
  std::string err;
  PreparedScene P;
  // Meshes this large take the device build (fs_bvh_gpu.hip); smaller ones
  // stay on the host, where a tree of a few thousand faces is cheaper to
  // build than the level-synchronous launches. FS_GPU_BVH_MIN_TRIS lowers
  // the threshold (tests), never below the device builder's minimum.
  uint32_t gpu_min = 0;
  if (flags & FS_UPLOAD_GPU_BVH) gpu_min = std::max(ctx->opt.gpu_bvh_min_tris, kGpuBvhFloor);
  const BuildOptions bo = BuildOptions::from(&ctx->opt);
  int rc = prepare_scene(desc, &P, &err, bo, gpu_min);
  if (rc) return fail(rc, err);
  if ((rc = set_device(ctx))) return rc;
  la_quiesce(ctx);  // lookahead traces read the scene this upload replaces
  ctx->scene_gen++;
  auto t0 = std::chrono::steady_clock::now();
  ctx->have_scene = false;
  if ((rc = upload(ctx, &ctx->objects, P.objects.data(), P.objects.size() * sizeof(DevObject)))) return rc;
  if ((rc = upload(ctx, &ctx->nodes, P.nodes.data(), P.nodes.size() * sizeof(BvhNode),
                   (size_t)P.deferred_nodes * sizeof(BvhNode))))
    return rc;
  if ((rc = upload(ctx, &ctx->tris, P.tris.data(), P.tris.size() * sizeof(DevTri),
                   (size_t)P.deferred_tris * sizeof(DevTri))))
    return rc;
  if ((rc = upload(ctx, &ctx->tri_normals, P.tri_normals.data(), P.tri_normals.size() * sizeof(float),
                   P.any_normals ? 48ull * P.deferred_tris : 0)))
    return rc;
  if ((rc = upload(ctx, &ctx->tri_tex, P.tri_tex.data(), P.tri_tex.size() * sizeof(float),
                   P.any_tex ? 24ull * P.deferred_tris : 0)))
    return rc;
  if ((rc = upload(ctx, &ctx->tex_rgb, P.tex_rgb.data(), P.tex_rgb.size() * sizeof(float)))) return rc;
  if ((rc = upload(ctx, &ctx->tex_info, P.tex_info.data(), P.tex_info.size() * sizeof(uint32_t)))) return rc;
  if ((rc = upload(ctx, &ctx->materials, P.materials.data(), P.materials.size() * sizeof(fs_material)))) return rc;
  {  // the backward pass's fields of every material (DevScene::umat)
    auto __int_as_float = [](int32_t v) {
      float f;
      std::memcpy(&f, &v, 4);
      return f;
    };
    std::vector<float4> um(3 * P.materials.size());
    for (size_t i = 0; i < P.materials.size(); i++) {
      const fs_material& m = P.materials[i];
      um[3 * i] = make_float4(__int_as_float(m.kind), m.diffuse[0], m.diffuse[1], m.diffuse[2]);
      um[3 * i + 1] = make_float4(m.roughness, m.emissive[0], m.emissive[1], m.emissive[2]);
      um[3 * i + 2] = make_float4(m.glow[0], m.glow[1], m.glow[2], __int_as_float(m.texture));
    }
    if ((rc = upload(ctx, &ctx->umat, um.data(), um.size() * sizeof(float4)))) return rc;
    // Material::Reflection's choices (DevScene::rmat, mat_reflection), each
    // solid angle with the reference's operations: float pi * roughness and
    // pi * frost (material.cpp:145, 199), double pi * (1 - shininess) to
    // float (material.cpp:259-265); the draw's threshold: reflectivity
    // (Glass, Liquid: material.cpp:197, 228) or 0.1f (Ceramic, Glow:
    // material.cpp:259); a non-drawing kind takes choice A (0 < 1).
    std::vector<float4> rm(P.materials.size());
    for (size_t i = 0; i < P.materials.size(); i++) {
      const fs_material& m = P.materials[i];
      uint32_t a = kReflScatter, b = kReflScatter, draws = 0;
      float thr = 1.0f, sa = kPi, sb = 0.0f;
      switch (m.kind) {
        case FS_MAT_LIGHT: a = kReflZero; break;
        case FS_MAT_DIFFUSE: break;
        case FS_MAT_METAL: sa = kPi * m.roughness; break;
        case FS_MAT_MIRROR: a = kReflMirror; break;
        case FS_MAT_GLASS: draws = kReflDraws; thr = m.reflectivity; sa = kPi * m.frost; b = kReflFrosted; break;
        case FS_MAT_LIQUID: draws = kReflDraws; thr = m.reflectivity; a = kReflMirror; b = kReflRefract; break;
        case FS_MAT_CERAMIC:
        case FS_MAT_GLOW:
          draws = kReflDraws;
          thr = 0.1f;
          sa = 0.0f;
          sb = (float)((double)kPi * (1.0 - (double)m.shininess));
          break;
        default: a = kReflView; break;  // FS_MAT_FOG
      }
      const uint32_t w = a | (b << 4) | draws;
      rm[i] = make_float4(thr, sa, sb, __int_as_float((int32_t)w));
    }
    if ((rc = upload(ctx, &ctx->rmat, rm.data(), rm.size() * sizeof(float4)))) return rc;
  }
  if ((rc = upload(ctx, &ctx->table, P.table.data(), P.table.size() * sizeof(float)))) return rc;
  if ((rc = upload(ctx, &ctx->tree, &P.tree, P.tree_valid ? sizeof(DevSceneTree) : 0))) return rc;
  if ((rc = upload(ctx, &ctx->tree_objs, P.tree_objs.data(), P.tree_objs.size() * sizeof(uint32_t)))) return rc;
  FS_HIP(hipStreamSynchronize(ctx->stream));
  ctx->upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ctx->gpu_bvh_ms = 0.0;
  ctx->gpu_bvh_nodes = 0;
  ctx->gpu_bvh_tris = P.deferred_tris;
  for (DeferredMesh& D : P.deferred) {  // device BVH builds into the reserved blocks
    GpuBvhJob job{};
    job.lo = D.lo.data();
    job.hi = D.hi.data();
    job.tris = D.tris.data();
    job.normals = D.normals.empty() ? nullptr : D.normals.data();
    job.tex = D.tex.empty() ? nullptr : D.tex.data();
    job.num_tris = D.num_tris;
    job.leaf = bo.leaf;
    job.log = bo.log;
    job.node_base = D.node_base;
    job.tri_base = D.tri_base;
    GpuBvhResult res;
    rc = gpu_build_mesh_bvh(ctx->stream, job, (BvhNode*)ctx->nodes.p, (DevTri*)ctx->tris.p, (float*)ctx->tri_normals.p,
                            (float*)ctx->tri_tex.p, &res, &err);
    if (rc) return fail(rc, "mesh " + std::to_string(D.mesh) + ": " + err);
    P.max_depth = std::max(P.max_depth, res.max_depth);
    ctx->gpu_bvh_ms += res.build_ms;
    ctx->gpu_bvh_nodes += res.nodes_used;
    if (bo.log)
      std::fprintf(stderr, "[fs build] mesh %u: %u tris, device bvh %.1f ms (%u levels, %u nodes, depth %u)\n", D.mesh,
                   D.num_tris, res.build_ms, res.levels, res.nodes_used, res.max_depth);
    D = DeferredMesh();  // release the host copies
  }
  DevScene& S = ctx->scene;
  S.objects = (const DevObject*)ctx->objects.p;
  S.nodes = (const BvhNode*)ctx->nodes.p;
  S.tris = (const DevTri*)ctx->tris.p;
  S.tri_normals = (const float4*)ctx->tri_normals.p;
  S.materials = (const fs_material*)ctx->materials.p;
  S.umat = (const float4*)ctx->umat.p;
  S.rmat = (const float4*)ctx->rmat.p;
  S.num_materials = (uint32_t)P.materials.size();
  S.table = (const float4*)ctx->table.p;
  S.tri_tex = (const float2*)ctx->tri_tex.p;
  S.tex_rgb = (const float*)ctx->tex_rgb.p;
  S.tex_info = (const uint4*)ctx->tex_info.p;
  S.tree = P.tree_valid ? (const DevSceneTree*)ctx->tree.p : nullptr;
  S.tree_objs = (const uint32_t*)ctx->tree_objs.p;
  S.num_objects = (uint32_t)P.objects.size();
  S.sky = P.sky;
  // Scene::SampleSky (scene.cpp:157-162): LightMaterial emissive x 3; a
  // non-Light sky dispatches to its own Sample with black light (0, or the
  // glow term of a GlowMaterial) — scene.cpp:383 static_pointer_cast.
  const fs_material& sky = P.materials[P.sky];
  f3 sv = mk3(0, 0, 0);
  if (sky.kind == FS_MAT_LIGHT) sv = mk3(sky.emissive[0], sky.emissive[1], sky.emissive[2]);
  if (sky.kind == FS_MAT_GLOW) sv = mk3(sky.glow[0], sky.glow[1], sky.glow[2]);
  sv = sv * (float)3.0;
  S.sky_r = sv.x;
  S.sky_g = sv.y;
  S.sky_b = sv.z;
  S.sky_id = sky.id;
  S.sky_tex = (sky.kind == FS_MAT_LIGHT && sky.texture >= 0) ? 1 : 0;
  ctx->has_textures = false;
  for (const fs_material& m : P.materials) ctx->has_textures |= m.texture >= 0;
  ctx->has_parking = false;
  ctx->has_walks = false;
  for (const DevObject& o : P.objects) {
    ctx->has_parking |= o.kind == FS_OBJ_MESH && o.i5 != 0;
    ctx->has_walks |= o.kind == FS_OBJ_MESH && o.i2 && !o.i3;
  }
  ctx->many_materials = P.materials.size() > kPackedMaterials;
  ctx->has_frost = false;
  for (const fs_material& m : P.materials) ctx->has_frost |= m.kind == FS_MAT_GLASS && m.frost != 0.0f;
  ctx->num_objects = S.num_objects;
  ctx->host = std::move(P);
  ctx->have_scene = true;
  return FS_OK;
}

int fs_scene_stats(fs_context* ctx, double* build_ms, double* upload_ms, uint64_t* num_triangles,
                   uint64_t* num_nodes, uint64_t* device_bytes) {
  if (!ctx) return fail(FS_ERR_INVALID, "null context");
  if (!ctx->have_scene) return fail(FS_ERR_STATE, "no scene uploaded");
  if (build_ms) *build_ms = ctx->host.build_ms + ctx->gpu_bvh_ms;
  if (upload_ms) *upload_ms = ctx->upload_ms;
  if (num_triangles) *num_triangles = ctx->host.tris.size() + ctx->gpu_bvh_tris;
  if (num_nodes) *num_nodes = ctx->host.nodes.size() + ctx->gpu_bvh_nodes;
  if (device_bytes)
    *device_bytes = ctx->objects.bytes + ctx->nodes.bytes + ctx->tris.bytes + ctx->tri_normals.bytes +
                     ctx->materials.bytes + ctx->table.bytes;
  return FS_OK;
}

int fs_frame_create(fs_context* ctx, uint32_t width, uint32_t height, fs_frame** out) {
  if (!ctx || !out) return fail(FS_ERR_INVALID, "null argument");
  if (width == 0 || height == 0) return fail(FS_ERR_INVALID, "empty frame");
  int rc;
  if ((rc = set_device(ctx))) return rc;
  std::unique_ptr<fs_frame> f(new fs_frame());
  f->ctx = ctx;
  f->width = width;
  f->height = height;
  size_t px = (size_t)width * height;
  for (int pl = FS_PLANE_COLOR; pl <= FS_PLANE_MATERIAL; pl++) {
    DevBuf* b = plane_buf(f.get(), pl);
    FS_HIP(hipMalloc(&b->p, plane_bytes(pl, px)));
    b->bytes = plane_bytes(pl, px);
  }
  fs_frame* raw = f.release();
  rc = fs_frame_reset(raw);
  if (rc) {
    fs_frame_destroy(raw);
    return rc;
  }
  *out = raw;
  return FS_OK;
}

int fs_frame_destroy(fs_frame* f) {
  if (!f) return FS_OK;
  (void)hipSetDevice(f->ctx->device);
  (void)hipStreamSynchronize(f->ctx->stream);
  for (int pl = FS_PLANE_COLOR; pl <= FS_PLANE_MATERIAL; pl++) {
    plane_buf(f, pl)->release();
    if (f->pinned[pl]) (void)hipHostFree(f->pinned[pl]);
  }
  delete f;
  return FS_OK;
}

int fs_frame_map(fs_frame* f, int plane, const void** host) {
  if (!f || !host) return fail(FS_ERR_INVALID, "null argument");
  DevBuf* b = plane_buf(f, plane);
  if (!b) return fail(FS_ERR_INVALID, "unknown plane");
  int rc;
  if ((rc = set_device(f->ctx))) return rc;
  if (!f->pinned[plane]) FS_HIP(hipHostMalloc(&f->pinned[plane], b->bytes, hipHostMallocDefault));
  FS_HIP(hipMemcpyAsync(f->pinned[plane], b->p, b->bytes, hipMemcpyDeviceToHost, f->ctx->stream));
  FS_HIP(hipStreamSynchronize(f->ctx->stream));
  *host = f->pinned[plane];
  return FS_OK;
}

int fs_frame_reset(fs_frame* f) {  // DisplayFrame::Reset (frame.cpp:43-51)
  if (!f) return fail(FS_ERR_INVALID, "null frame");
  int rc;
  if ((rc = set_device(f->ctx))) return rc;
  for (int pl = FS_PLANE_COLOR; pl <= FS_PLANE_MATERIAL; pl++) {
    DevBuf* b = plane_buf(f, pl);
    FS_HIP(hipMemsetAsync(b->p, 0, b->bytes, f->ctx->stream));
  }
  FS_HIP(hipStreamSynchronize(f->ctx->stream));
  return FS_OK;
}

int fs_frame_read(fs_frame* f, int plane, void* dst, size_t bytes) {
  if (!f || !dst) return fail(FS_ERR_INVALID, "null argument");
  DevBuf* b = plane_buf(f, plane);
  if (!b) return fail(FS_ERR_INVALID, "unknown plane");
  if (bytes != b->bytes) return fail(FS_ERR_INVALID, "byte count does not match the plane size");
  int rc;
  if ((rc = set_device(f->ctx))) return rc;
  FS_HIP(hipMemcpyAsync(dst, b->p, bytes, hipMemcpyDeviceToHost, f->ctx->stream));
  FS_HIP(hipStreamSynchronize(f->ctx->stream));
  return FS_OK;
}

int fs_frame_write(fs_frame* f, int plane, const void* src, size_t bytes) {
  if (!f || !src) return fail(FS_ERR_INVALID, "null argument");
  DevBuf* b = plane_buf(f, plane);
  if (!b) return fail(FS_ERR_INVALID, "unknown plane");
  if (bytes != b->bytes) return fail(FS_ERR_INVALID, "byte count does not match the plane size");
  int rc;
  if ((rc = set_device(f->ctx))) return rc;
  FS_HIP(hipMemcpyAsync(b->p, src, bytes, hipMemcpyHostToDevice, f->ctx->stream));
  FS_HIP(hipStreamSynchronize(f->ctx->stream));
  return FS_OK;
}

int fs_render(fs_context* ctx, const fs_camera* camera, const fs_render_params* params, fs_frame* frame) {
  if (!ctx || !camera || !params || !frame) return fail(FS_ERR_INVALID, "null argument");
  if (!ctx->have_scene) return fail(FS_ERR_STATE, "fs_render before fs_upload_scene");
  if (frame->ctx != ctx) return fail(FS_ERR_INVALID, "frame belongs to another context");
  uint32_t ts, stride;
  int rc = check_params(params, frame, &ts, &stride);
  if (rc) return rc;
  if ((rc = set_device(ctx))) return rc;
  Launch L{};
  L.tile_size = ts;
  L.tiles_x = (params->width + ts - 1) / ts;
  uint32_t tiles_y = (params->height + ts - 1) / ts;
  uint32_t tiles = L.tiles_x * tiles_y;
  L.tile_offset = params->tile_offset;
  L.tile_stride = stride;
  L.seed = params->seed;
  const fs_options& O = ctx->opt;
  L.susp_thr = O.park_lanes;
  L.susp_thr_small = O.park_lanes_small;
  // XCD placement: 0 dispatch order, 1 one band per XCD (C4 -25 %: the bands
  // are unbalanced), 2 (default) whole 64x64 tiles per XCD (C4 +1.5 %)
  L.xcd_bands = O.xcd_bands;
  uint32_t owned = params->tile_offset < tiles ? (tiles - params->tile_offset + stride - 1) / stride : 0;
  uint64_t blocks = (uint64_t)owned * (ts / 8) * (ts / 8);
  DevCamera C = camera_basis(camera, params->width, params->height);
  DevFrame F = frame_view(frame);
  bool count = (params->flags & FS_RENDER_COUNTERS) != 0;
  // Schedule (every schedule produces identical frames): LEAN, the
  // path-regeneration megakernel writing path records,
  // while-while traversal and the wave's (pixel, sample) tasks pooled across
  // lanes; PARKED the same with walks of large meshes parked when few lanes
  // still walk. AUTO: PARKED when the scene has a mesh of >= park_min_tris
  // triangles and no texture (the textured instantiation has no parking).
  const bool parked = O.schedule == FS_SCHEDULE_PARKED ||
                      (O.schedule == FS_SCHEDULE_AUTO && ctx->has_parking && !ctx->has_textures && !ctx->scene.tree);
  if (parked && ctx->has_textures) return fail(FS_ERR_INVALID, "the PARKED schedule does not take textured scenes");
  if (parked && ctx->scene.tree)
    return fail(FS_ERR_INVALID, "the PARKED schedule does not take scenes traced through the object octree");
  if (blocks >= (1ull << 31)) return fail(FS_ERR_INVALID, "frame too large (2^31 or more 8x8 blocks)");
  FS_HIP(hipEventRecord(ctx->ev0, ctx->stream));
  const bool tree = ctx->scene.tree != nullptr;
  const bool mm = ctx->many_materials || tree;
  const bool tex_rec = ctx->has_textures || tree;
  const size_t rec_bytes = record_bytes(tex_rec, mm);
  // The path records of a launch: at most the record budget (96 GiB, or
  // fs_options.record_budget_mb) and at most half of the device memory that
  // is free (counting the records this context already holds), so a smaller
  // or shared GPU renders in more, smaller launches instead of failing.
  uint64_t row_budget = record_budget(O, 0);
  const uint32_t mpt = (ts / 8) * (ts / 8);  // micro-tiles per tile
  Plan plan;
  if ((rc = make_plan(owned, mpt, params->spp, O, row_budget, rec_bytes, &plan))) return rc;
  // The free-memory cap is queried only for launches of more than 1 GiB of
  // records (hipMemGetInfo costs the small renders of a window loop a
  // driver round trip per frame).
  if ((uint64_t)plan.tiles * mpt * plan.G * plan.chunk * kBlock * rec_bytes > (1ull << 30)) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
        (free_b + ctx->rows.bytes) / 2 < row_budget) {
      row_budget = (free_b + ctx->rows.bytes) / 2;
      if ((rc = make_plan(owned, mpt, params->spp, O, row_budget, rec_bytes, &plan))) return rc;
    }
  }
  ctx->last_launches = 0;
  ctx->last_launch_spp = 0;
  ctx->last_spec = -1;
  PathRecords rec;
  float4* anchors = nullptr;
  const LeanKernel K = pick_kernel(count, ctx->has_textures, parked, mm, ctx->scene.tree != nullptr,
                                   ctx->has_walks || !O.lds_rows, C.aperture > 0.0f || ctx->has_frost);
  // The persistent grid: one wave per wave slot of the chip (4 SIMDs per CU,
  // K.waves waves per SIMD), never more than the launch has blocks.
  const uint64_t wave_slots = (uint64_t)ctx->cus * 4u * K.waves;
  auto grid_for = [&](uint64_t nb) { return O.persist ? std::min<uint64_t>(wave_slots, nb) : nb; };
  ctx->last_kernel = K.name;
  L.persist = O.persist;
  L.groups = 1;
  L.group_major = O.group_major;
  L.tile_order = nullptr;
  bool order_copied = false;  // the tile order was (re)written on the context stream by this call
  // Longest jobs first: tiles nearer the image centre (where the scenes put
  // their geometry) are dispatched first, so the launch tail runs on cheap
  // edge tiles. Ties keep index order. Only the dispatch order changes: every
  // tile keeps its path records. (A render in several tile parts dispatches
  // each part in index order.)
  if (owned > 1 && O.tile_order && plan.parts == 1) {
    const uint64_t okey[3] = {((uint64_t)L.tile_offset << 32) | L.tile_stride, owned,
                              ((uint64_t)params->width << 32) | params->height};
    std::vector<uint32_t>& ord = ctx->tile_order_host;
    if (!std::equal(okey, okey + 3, ctx->tile_order_key)) {
      la_quiesce(ctx);  // a lookahead may read the old order
      order_copied = true;
      ord.resize(owned);
      std::vector<float> dist(owned);
      const float cx = 0.5f * (float)params->width, cy = 0.5f * (float)params->height;
      for (uint32_t i = 0; i < owned; i++) {
        const uint32_t tile = L.tile_offset + i * L.tile_stride;
        const float x = ((float)(tile % L.tiles_x) + 0.5f) * (float)ts - cx;
        const float y = ((float)(tile / L.tiles_x) + 0.5f) * (float)ts - cy;
        dist[i] = x * x + y * y;
        ord[i] = i;
      }
      std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return dist[a] < dist[b]; });
      if ((rc = ensure(&ctx->tile_order, owned * sizeof(uint32_t)))) return rc;
      FS_HIP(hipMemcpyAsync(ctx->tile_order.p, ord.data(), owned * sizeof(uint32_t), hipMemcpyHostToDevice,
                            ctx->stream));
      std::copy(okey, okey + 3, ctx->tile_order_key);
    }
    L.tile_order = (const uint32_t*)ctx->tile_order.p;
  }
  // Lookahead (fs_options.lookahead): a whole-frame render of at most
  // kLookaheadSpp samples in one launch. A pending lookahead slot that traced
  // exactly this call (as its group g) is folded instead of tracing; slots of
  // later calls of the same sequence stay; every other one is dropped (its
  // stream may still run: it writes only its own slot).
  Lookahead& A = ctx->la;
  // (the per-call AOV planes of a launch must stay within 32-bit byte offsets)
  const bool la_ok = O.lookahead && !count && stride == 1 && params->tile_offset == 0 && O.persist && blocks &&
                     params->spp <= kLookaheadSpp && plan.parts == 1 && plan.G == 1 && plan.chunk == params->spp &&
                     (uint64_t)frame->width * frame->height * 12 < (1ull << 32);
  LookKey key;
  std::memset(&key, 0, sizeof key);
  int hit = -1;
  uint32_t hit_group = 0;
  auto same_sequence = [&](int i) {  // slot i's key but for the first sample
    LookKey k = A.key[i];
    k.params.sample_base = params->sample_base;
    return !std::memcmp(&k, &key, sizeof key);
  };
  if (la_ok) {
    key.camera = *camera;
    key.params = *params;
    key.opt = O;
    key.scene_gen = ctx->scene_gen;
    for (int i = 0; i < kLookSlots; i++) {
      const uint32_t b0 = A.key[i].params.sample_base, k = params->sample_base;
      if (A.pending[i] && k >= b0 && (k - b0) % params->spp == 0 && (k - b0) / params->spp < A.groups[i] &&
          same_sequence(i)) {
        hit = i;
        hit_group = (k - b0) / params->spp;
      }
    }
  }
  for (int i = 0; i < kLookSlots; i++) {
    if (!A.pending[i]) continue;
    const uint64_t end = (uint64_t)A.key[i].params.sample_base + (uint64_t)A.groups[i] * A.key[i].params.spp;
    const bool later = hit >= 0 && end > (uint64_t)params->sample_base + params->spp && same_sequence(i);
    if (later) continue;
    A.pending[i] = false;  // the hit slot too once its last call is folded
    if (i != hit) {
      // Dropped unread: its waves may still trace. Its block queues set past
      // every block (0x7F7F7F7F) end the launch after the paths in flight (a
      // launch still waiting for its start zeroes them first and runs out).
      FS_HIP(hipMemsetAsync(A.queues[i].p, 0x7F, A.queues[i].bytes, ctx->stream));
      if (!A.cancelled[i]) FS_HIP(hipEventCreateWithFlags(&A.cancelled[i], hipEventDisableTiming));
      FS_HIP(hipEventRecord(A.cancelled[i], ctx->stream));
      A.cancel_valid[i] = true;
    }
  }
  if (hit < 0) A.prev[0] = A.prev[1] = -1;  // a new sequence: no launch to queue behind
  // On an allocation failure the launches shrink (groups per launch, then
  // tiles per part, then samples per block, each halved) until the records fit.
  while (blocks && hit < 0) {
    const uint64_t pb = (uint64_t)plan.tiles * mpt;  // blocks of the largest part
    if (!(rc = path_records(ctx, grid_for(pb * plan.G) * kBlock, pb * plan.G * plan.chunk * kBlock, &rec, &anchors,
                            tex_rec, mm)))
      break;
    if (O.groups || !plan.shrink(owned)) return rc;
    (void)hipGetLastError();  // clear the failed hipMalloc's error state
  }
  if (plan.parts != 1) L.tile_order = nullptr;  // shrunk into tile parts: index order
  const bool lm = ctx->scene.num_materials <= dev::kFoldLdsMaterials;
  const uint32_t fold_lds = lm ? 48 * ctx->scene.num_materials : 0;
  const FoldFn fold = pick_fold(tex_rec, mm, lm);
  const FoldSplitFn fold_split = pick_fold_split(tex_rec, mm, lm);
  const FoldFn fold_lite = pick_fold_lite(tex_rec, mm, lm);
  // Lanes per pixel of the fold: 1 while a launch's micro-tiles fill the
  // fold kernel's resident wave slots at least twice over, else 2 or 4 (a
  // rank's share of a multi-GPU frame), so the serial per-pixel loop is split.
  const uint64_t fold_slots = (uint64_t)ctx->cus * fold_waves_per_cu(fold, fold_lds);
  if (hit >= 0) {
    // The lookahead traced exactly these samples as group g of its launch:
    // the fold of group g's records (the record planes from group g's first
    // row, as a one-group launch of this call) after the launch's trace on
    // its stream, copying group g's AOV planes into the frame.
    FS_HIP(hipStreamWaitEvent(ctx->stream, A.traced[hit], 0));
    const size_t px = (size_t)frame->width * frame->height;
    const uint64_t pblocks = (uint64_t)A.L[hit].owned * mpt;
    Launch Lh = A.L[hit];
    Lh.groups = 1;
    Lh.sample_base = params->sample_base;
    Lh.nblocks = (uint32_t)pblocks;
    Lh.aov_rows = Lh.aov_plane = 0;
    PathRecords Rh = A.R[hit];
    const uint64_t off = (uint64_t)hit_group * pblocks * Lh.spp * kBlock;
    Rh.c += off;
    Rh.ds += off;
    Rh.end += off;
    if (Rh.mats) Rh.mats += off;
    if (Rh.mat) Rh.mat += off;
    if (Rh.tex) Rh.tex += off;
    Rh.aov_n = (const float*)A.nrm[hit].p + 3 * px * hit_group;
    Rh.aov_d = (const float*)A.dep[hit].p + px * hit_group;
    Rh.aov_m = (const uint64_t*)A.mid[hit].p + px * hit_group;
    const uint32_t fold_log2 = pblocks >= 2 * fold_slots ? 0u : (pblocks >= fold_slots ? 1u : 2u);
    if (fold_log2 == 0)
      hipLaunchKernelGGL(fold_lite, dim3((uint32_t)pblocks), dim3(kBlock), fold_lds, ctx->stream, ctx->scene, F, Lh,
                         Rh);
    else
      hipLaunchKernelGGL(fold_split, dim3((uint32_t)(pblocks << fold_log2)), dim3(kBlock), fold_lds, ctx->stream,
                         ctx->scene, F, Lh, Rh, fold_log2);
    FS_HIP(hipGetLastError());
    FS_HIP(hipEventRecord(A.folded[hit], ctx->stream));  // the slot's latest reader
    A.folded_valid[hit] = true;
    ctx->last_spec = hit;
    ctx->last_launches = 1;
    ctx->last_launch_spp = Lh.spp;
  }
  for (uint32_t part = 0; part < plan.parts && hit < 0; part++) {
    // part p: the render's owned tiles p * tiles ..., i.e. the frame's tiles
    // tile_offset + (p * tiles + i) * stride
    const uint32_t first = part * plan.tiles;
    L.owned = std::min<uint32_t>(plan.tiles, owned - first);
    L.tile_offset = params->tile_offset + first * stride;
    const uint64_t pblocks = (uint64_t)L.owned * mpt;
    const uint32_t fold_log2 = pblocks >= 2 * fold_slots ? 0u : (pblocks >= fold_slots ? 1u : 2u);
    for (uint32_t done = 0; done < params->spp;) {
      L.sample_base = params->sample_base + done;
      L.spp = std::min(plan.chunk, params->spp - done);
      L.groups = L.spp == plan.chunk ? std::min(plan.G, (params->spp - done) / plan.chunk) : 1u;
      L.nblocks = (uint32_t)(pblocks * L.groups);
      done += L.groups * L.spp;
      const uint32_t grid = (uint32_t)grid_for(L.nblocks);
      if (O.persist) FS_HIP(hipMemsetAsync(ctx->queues.p, 0, ctx->queues.bytes, ctx->stream));
      const size_t ke = 2 * (size_t)ctx->last_launches;
      while (ctx->kev.size() < ke + 2) {
        hipEvent_t e;
        FS_HIP(hipEventCreate(&e));
        ctx->kev.push_back(e);
      }
      FS_HIP(hipEventRecord(ctx->kev[ke], ctx->stream));
      hipLaunchKernelGGL(K.fn, dim3(grid), dim3(kBlock), 0, ctx->stream, ctx->scene, C, F, L, rec, anchors,
                         (uint32_t*)ctx->queues.p, (DevCounters*)ctx->counters.p);
      FS_HIP(hipEventRecord(ctx->kev[ke + 1], ctx->stream));
      // counted once both of its events are recorded (fs_last_trace_ms reads them)
      ctx->last_launches++;
      ctx->last_launch_spp = std::max(ctx->last_launch_spp, L.groups * L.spp);
      if (fold_log2 == 0)
        hipLaunchKernelGGL(fold, dim3((uint32_t)pblocks), dim3(kBlock), fold_lds, ctx->stream, ctx->scene, F, L, rec);
      else
        hipLaunchKernelGGL(fold_split, dim3((uint32_t)(pblocks << fold_log2)), dim3(kBlock), fold_lds, ctx->stream,
                           ctx->scene, F, L, rec, fold_log2);
      FS_HIP(hipGetLastError());
    }
  }
  // The next calls' samples, up to `lookahead` calls ahead, traced now in
  // the background in launches of g calls into free slots, after what the
  // pending slots of this sequence already cover; never past the 2^20-sample
  // seed range.
  bool continues = false;  // this call continues the last one's sequence
  if (la_ok && A.last_valid) {
    LookKey k = A.last;
    k.params.sample_base = params->sample_base;
    continues = (uint64_t)A.last.params.sample_base + A.last.params.spp == params->sample_base &&
                !std::memcmp(&k, &key, sizeof key);
  }
  if (la_ok) A.last = key;
  A.last_valid = la_ok;
  if (la_ok && (hit >= 0 || continues)) {
    // g calls per launch: w / 3, so three slots hold the window; at most
    // kLookGroupMax, and fewer where the per-call AOV planes would pass the
    // 32-bit byte offsets of the trace kernel's AOV stores
    const uint64_t pxl = (uint64_t)frame->width * frame->height;
    const uint32_t spp = params->spp, w = O.lookahead,
                   g = (uint32_t)std::min<uint64_t>({kLookGroupMax, std::max<uint32_t>(1, w / 3),
                                                     ((1ull << 32) - 1) / (12 * pxl)});
    uint64_t cov = (uint64_t)params->sample_base + spp;  // first sample no pending slot traces
    for (int i = 0; i < kLookSlots; i++)
      if (A.pending[i]) cov = std::max<uint64_t>(cov, (uint64_t)A.key[i].params.sample_base + (uint64_t)A.groups[i] * spp);
    const uint64_t want = (uint64_t)params->sample_base + (uint64_t)spp * (1 + w);
    const uint64_t pb = (uint64_t)owned * mpt;
    // Fewer waves per SIMD than the kernel's bound, so that one wave of the
    // fold fits beside them on every SIMD: the caller's next fold (context
    // stream) then runs at once instead of waiting for the launch's waves to
    // leave (persistent waves leave only when the launch's blocks run out).
    if (A.bg_trace != reinterpret_cast<const void*>(K.fn) || A.bg_fold != reinterpret_cast<const void*>(fold_lite)) {
      A.bg_trace = reinterpret_cast<const void*>(K.fn);
      A.bg_fold = reinterpret_cast<const void*>(fold_lite);
      A.bg_w = bg_waves(K.fn, K.waves, fold_lite);
    }
    const uint64_t bg_slots = (uint64_t)ctx->cus * 4u * A.bg_w;
    const size_t px = (size_t)frame->width * frame->height;
    if (hit < 0) A.ramp = 0;  // a sequence starts: its first launches are short
    for (;;) {
      // 1, 2, 4, ... calls per launch up to g, so the first calls of a
      // sequence wait for a short launch rather than a full one
      const uint32_t gl = std::min<uint32_t>(g, 1u << std::min<uint32_t>(A.ramp, 4));
      if (!(cov < want && cov + (uint64_t)gl * spp <= (1ull << 20))) break;
      const uint64_t grid = std::min<uint64_t>(grid_for(pb * gl), bg_slots);
      int s = -1;  // the free slot launched longest ago (its stream's last work is the oldest)
      for (int i = 0; i < kLookSlots; i++)
        if (!A.pending[i] && (s < 0 || A.used[i] < A.used[s])) s = i;
      if (s < 0) break;
      if (!A.stream[s]) {
        int least = 0, greatest = 0;
        FS_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        FS_HIP(hipStreamCreateWithPriority(&A.stream[s], hipStreamNonBlocking, least));
        FS_HIP(hipEventCreateWithFlags(&A.traced[s], hipEventDisableTiming));
        FS_HIP(hipEventCreateWithFlags(&A.folded[s], hipEventDisableTiming));
        FS_HIP(hipEventCreate(&A.kev0[s]));
        FS_HIP(hipEventCreate(&A.kev1[s]));
        if (!A.order) FS_HIP(hipEventCreateWithFlags(&A.order, hipEventDisableTiming));
      }
      // (sized for g calls at once, so the ramp does not reallocate)
      const size_t need = rows_bytes(std::min<uint64_t>(grid_for(pb * g), bg_slots) * kBlock, pb * g * spp * kBlock,
                                     tex_rec, mm);
      if (A.rows[s].bytes < need || A.nrm[s].bytes < 12 * px * g || A.dep[s].bytes < 4 * px * g ||
          A.mid[s].bytes < 8 * px * g || !A.queues[s].p) {
        FS_HIP(hipStreamSynchronize(A.stream[s]));  // its last trace and folds still use the old buffers
        FS_HIP(hipStreamSynchronize(ctx->stream));
        if (ensure(&A.rows[s], need) || ensure(&A.nrm[s], 12 * px * g) || ensure(&A.dep[s], 4 * px * g) ||
            ensure(&A.mid[s], 8 * px * g) || ensure(&A.queues[s], 8 * dev::kQueueStride * sizeof(uint32_t))) {
          (void)hipGetLastError();  // no room: no (further) lookahead for this call
          break;
        }
      }
      if (carve_records(&A.rows[s], grid * kBlock, pb * gl * spp * kBlock, &A.R[s], &anchors, tex_rec, mm)) break;
      Launch Ls = L;
      Ls.owned = owned;
      Ls.tile_offset = 0;
      Ls.sample_base = (uint32_t)cov;
      Ls.spp = spp;
      Ls.groups = gl;
      Ls.nblocks = (uint32_t)(pb * gl);
      Ls.aov_rows = (uint32_t)pb;  // group k's AOVs in plane k
      Ls.aov_plane = (uint32_t)px;
      DevFrame Fs{};  // the trace writes only the AOVs: into the slot's planes
      Fs.width = frame->width;
      Fs.height = frame->height;
      Fs.normal = (float*)A.nrm[s].p;
      Fs.depth = (float*)A.dep[s].p;
      Fs.material = (uint64_t*)A.mid[s].p;
      if (A.folded_valid[s]) FS_HIP(hipStreamWaitEvent(A.stream[s], A.folded[s], 0));  // its records' last reader
      if (order_copied) {
        FS_HIP(hipEventRecord(A.order, ctx->stream));
        FS_HIP(hipStreamWaitEvent(A.stream[s], A.order, 0));
      }
      if (A.prev[1] >= 0 && A.prev[1] != s) FS_HIP(hipStreamWaitEvent(A.stream[s], A.traced[A.prev[1]], 0));
      if (A.cancel_valid[s]) {  // the cancel's write lands before this launch zeroes the queues
        FS_HIP(hipStreamWaitEvent(A.stream[s], A.cancelled[s], 0));
        A.cancel_valid[s] = false;
      }
      FS_HIP(hipMemsetAsync(A.queues[s].p, 0, A.queues[s].bytes, A.stream[s]));
      FS_HIP(hipEventRecord(A.kev0[s], A.stream[s]));
      hipLaunchKernelGGL(K.fn, dim3((uint32_t)grid), dim3(kBlock), 0, A.stream[s], ctx->scene, C, Fs, Ls, A.R[s],
                         anchors, (uint32_t*)A.queues[s].p, (DevCounters*)ctx->counters.p);
      FS_HIP(hipGetLastError());
      FS_HIP(hipEventRecord(A.kev1[s], A.stream[s]));
      FS_HIP(hipEventRecord(A.traced[s], A.stream[s]));
      A.L[s] = Ls;
      A.key[s] = key;
      A.key[s].params.sample_base = Ls.sample_base;
      A.groups[s] = gl;
      A.pending[s] = true;
      A.used[s] = ++A.tick;
      A.prev[1] = A.prev[0];
      A.prev[0] = s;
      A.ramp++;
      cov += (uint64_t)gl * spp;
    }
  }
  FS_HIP(hipEventRecord(ctx->ev1, ctx->stream));
  return FS_OK;
}

int fs_plan_render(const fs_render_params* params, const fs_options* opt, uint64_t record_budget_bytes,
                   uint32_t record_bytes_per_sample, fs_render_plan* out) {
  if (!params || !out) return fail(FS_ERR_INVALID, "null argument");
  fs_options O;
  if (opt) {
    std::string why;
    if (!valid_options(opt, &why)) return fail(FS_ERR_INVALID, "fs_plan_render: " + why);
    O = *opt;
  } else {
    fs_options_default(&O);
  }
  if (!record_bytes_per_sample) return fail(FS_ERR_INVALID, "record_bytes_per_sample must be > 0");
  fs_frame probe;
  probe.width = params->width;
  probe.height = params->height;
  uint32_t ts, stride;
  int rc = check_params(params, &probe, &ts, &stride);
  if (rc) return rc;
  const uint32_t tiles = ((params->width + ts - 1) / ts) * ((params->height + ts - 1) / ts);
  const uint32_t owned = params->tile_offset < tiles ? (tiles - params->tile_offset + stride - 1) / stride : 0;
  const uint32_t mpt = (ts / 8) * (ts / 8);
  Plan p;
  if ((rc = make_plan(owned, mpt, params->spp, O, record_budget(O, record_budget_bytes), record_bytes_per_sample, &p)))
    return rc;
  out->parts = p.parts;
  out->tiles_per_part = p.tiles;
  out->samples_per_block = p.chunk;
  out->groups_per_launch = p.G;
  out->launches = owned ? p.launches(params->spp) : 0;
  out->record_bytes_per_launch = (uint64_t)p.tiles * mpt * p.G * p.chunk * kBlock * record_bytes_per_sample;
  return FS_OK;
}

int fs_synchronize(fs_context* ctx) {
  if (!ctx) return fail(FS_ERR_INVALID, "null context");
  int rc;
  if ((rc = set_device(ctx))) return rc;
  FS_HIP(hipStreamSynchronize(ctx->stream));
  return FS_OK;
}

const char* fs_last_kernel(fs_context* ctx) { return ctx ? ctx->last_kernel : ""; }

int fs_last_render_launches(fs_context* ctx, uint32_t* launches, uint32_t* spp_per_launch) {
  if (!ctx || !launches || !spp_per_launch) return fail(FS_ERR_INVALID, "null argument");
  *launches = ctx->last_launches;
  *spp_per_launch = ctx->last_launch_spp;
  return FS_OK;
}

int fs_last_render_ms(fs_context* ctx, float* ms) {
  if (!ctx || !ms) return fail(FS_ERR_INVALID, "null argument");
  int rc;
  if ((rc = set_device(ctx))) return rc;
  FS_HIP(hipEventSynchronize(ctx->ev1));
  FS_HIP(hipEventElapsedTime(ms, ctx->ev0, ctx->ev1));
  return FS_OK;
}

int fs_last_trace_ms(fs_context* ctx, float* ms) {
  if (!ctx || !ms) return fail(FS_ERR_INVALID, "null argument");
  int rc;
  if ((rc = set_device(ctx))) return rc;
  float sum = 0.0f;
  if (ctx->last_spec >= 0) {  // the last render folded a lookahead: its trace's time
    FS_HIP(hipEventSynchronize(ctx->la.kev1[ctx->last_spec]));
    FS_HIP(hipEventElapsedTime(ms, ctx->la.kev0[ctx->last_spec], ctx->la.kev1[ctx->last_spec]));
    return FS_OK;
  }
  for (uint32_t i = 0; i < ctx->last_launches; i++) {
    float t = 0.0f;
    FS_HIP(hipEventSynchronize(ctx->kev[2 * i + 1]));
    FS_HIP(hipEventElapsedTime(&t, ctx->kev[2 * i], ctx->kev[2 * i + 1]));
    sum += t;
  }
  *ms = sum;
  return FS_OK;
}

int fs_last_render_lookahead(fs_context* ctx, int* folded) {
  if (!ctx || !folded) return fail(FS_ERR_INVALID, "null argument");
  *folded = ctx->last_spec >= 0 ? 1 : 0;
  return FS_OK;
}

int fs_read_counters(fs_context* ctx, fs_counters* out) {
  if (!ctx || !out) return fail(FS_ERR_INVALID, "null argument");
  int rc;
  if ((rc = set_device(ctx))) return rc;
  DevCounters c;
  FS_HIP(hipMemcpyAsync(&c, ctx->counters.p, sizeof(c), hipMemcpyDeviceToHost, ctx->stream));
  FS_HIP(hipMemsetAsync(ctx->counters.p, 0, sizeof(c), ctx->stream));
  FS_HIP(hipStreamSynchronize(ctx->stream));
  out->samples = c.samples;
  out->segments = c.segments;
  out->node_visits = c.node_visits;
  out->tri_tests = c.tri_tests;
  out->prim_tests = c.prim_tests;
  out->object_loads = c.object_loads;
  out->small_tri_loads = c.small_tri_loads;
  out->lane_object_loads = c.lane_object_loads;
#ifdef FS_WAVE_TIMES
  {
    uint64_t waves = 0;
    for (int i = 0; i < 14; i++) waves += c.phase[i];
    std::fprintf(stderr, "[fs waves] %llu waves; end time (200 us bins):", (unsigned long long)waves);
    for (int i = 0; i < 14; i++) std::fprintf(stderr, " %llu", c.phase[i]);
    std::fprintf(stderr, "; first empty queues (200 us bins):");
    for (int i = 14; i < 28; i++) std::fprintf(stderr, " %llu", c.phase[i]);
    std::fprintf(stderr, "; drain after empty queues: mean %.1f us, max %.1f us, %.1f iterations per wave\n",
                 c.phase[28] / 100.0 / (waves ? waves : 1), c.phase[29] / 100.0, (double)c.phase[30] / (waves ? waves : 1));
  }
#endif
#ifdef FS_PHASE_PROF
  std::fprintf(stderr,
               "[fs phase] loop-top %llu fresh %llu trace %llu (root-cull %llu mesh-traversal %llu analytic %llu) "
               "shade %llu unwind %llu - iters %llu total %llu\n",
               c.phase[0], c.phase[1], c.phase[2], c.phase[5], c.phase[6], c.phase[7], c.phase[3], c.phase[4],
               c.phase[8], c.phase[9]);
  std::fprintf(stderr,
               "[fs trips] node loop: %llu wave trips, %llu lane visits (%.1f%% of lanes); leaf loop: %llu wave "
               "trips, %llu lane leaves (%.1f%%)\n",
               c.phase[10], c.phase[12], 100.0 * c.phase[12] / (64.0 * (c.phase[10] ? c.phase[10] : 1)), c.phase[11],
               c.phase[13], 100.0 * c.phase[13] / (64.0 * (c.phase[11] ? c.phase[11] : 1)));
  std::fprintf(stderr,
               "[fs small] small-mesh faces %llu cycles (in trace, apart from root-cull and mesh-traversal); lanes per iteration: tracing %.1f, "
               "shading %.1f, finishing %.1f; unwind levels per finished path %.2f\n",
               c.phase[14], (double)c.phase[26] / (c.phase[8] ? c.phase[8] : 1),
               (double)c.phase[27] / (c.phase[8] ? c.phase[8] : 1), (double)c.phase[28] / (c.phase[8] ? c.phase[8] : 1),
               (double)c.phase[29] / (c.phase[28] ? c.phase[28] : 1));
  std::fprintf(stderr,
               "[fs chain] walk node trips per trace call, summed: meshes one after another (wave max per mesh) %llu, "
               "each lane on to its next mesh at once (wave max of the per-lane sum) %llu\n",
               c.phase[16], c.phase[17]);
#endif
  return FS_OK;
}

int fs_scene_digest(fs_context* ctx, uint64_t* digest) {
  if (!ctx || !digest) return fail(FS_ERR_INVALID, "null argument");
  if (!ctx->have_scene) return fail(FS_ERR_STATE, "no scene uploaded");
  int rc;
  if ((rc = set_device(ctx))) return rc;
  uint64_t h = 1469598103934665603ull;  // FNV-1a over every device array of the scene
  std::vector<uint8_t> buf;
  for (DevBuf* b : {&ctx->objects, &ctx->nodes, &ctx->tris, &ctx->tri_normals, &ctx->tri_tex, &ctx->materials,
                    &ctx->table, &ctx->tex_rgb, &ctx->tex_info, &ctx->tree, &ctx->tree_objs}) {
    buf.resize(b->bytes);
    if (b->bytes) FS_HIP(hipMemcpy(buf.data(), b->p, b->bytes, hipMemcpyDeviceToHost));
    for (uint8_t v : buf) h = (h ^ v) * 1099511628211ull;
    for (int k = 0; k < 8; k++) h = (h ^ ((b->bytes >> (8 * k)) & 0xFF)) * 1099511628211ull;
  }
  *digest = h;
  return FS_OK;
}

int fs_prepare_digest(const fs_scene_desc* desc, const fs_options* opt, uint64_t* digest, uint64_t* num_nodes,
                      double* build_ms) {
  if (!desc || !digest) return fail(FS_ERR_INVALID, "null argument");
  std::string err;
  if (opt && !valid_options(opt, &err)) return fail(FS_ERR_INVALID, "fs_prepare_digest: " + err);
  PreparedScene P;
  int rc = prepare_scene(desc, &P, &err, BuildOptions::from(opt));
  if (rc) return fail(rc, err);
  uint64_t h = 1469598103934665603ull;  // FNV-1a over every uploaded array
  auto mix = [&h](const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  };
  mix(P.objects.data(), P.objects.size() * sizeof(DevObject));
  mix(P.nodes.data(), P.nodes.size() * sizeof(BvhNode));
  mix(P.tris.data(), P.tris.size() * sizeof(DevTri));
  mix(P.tri_normals.data(), P.tri_normals.size() * sizeof(float));
  mix(P.tri_tex.data(), P.tri_tex.size() * sizeof(float));
  mix(P.materials.data(), P.materials.size() * sizeof(fs_material));
  mix(P.tex_rgb.data(), P.tex_rgb.size() * sizeof(float));
  mix(P.tex_info.data(), P.tex_info.size() * sizeof(uint32_t));
  mix(P.table.data(), P.table.size() * sizeof(float));
  if (P.tree_valid) {  // the object octree of an optimised scene (SceneBvh)
    mix(&P.tree, sizeof(P.tree));
    mix(P.tree_objs.data(), P.tree_objs.size() * sizeof(uint32_t));
  }
  *digest = h;
  if (num_nodes) *num_nodes = P.nodes.size();
  if (build_ms) *build_ms = P.build_ms;
  return FS_OK;
}

// Tree quality of every BVH mesh of a host-side preparation (measurement aid,
// no reference counterpart): per mesh the SAH cost relative to its root box
// (inner nodes 1, triangle tests 1 per face: sum over nodes of area/root
// area), the overlap of sibling boxes (area of child0 ∩ child1 over the
// parent's area, mean per depth level and area-weighted total), node, leaf
// and face counts and the depth. Written as JSON into out (size bytes).
int fs_bvh_quality(const fs_scene_desc* desc, const fs_options* opt, char* out, size_t size) {
  if (!desc || !out || !size) return fail(FS_ERR_INVALID, "null argument");
  std::string err;
  if (opt && !valid_options(opt, &err)) return fail(FS_ERR_INVALID, "fs_bvh_quality: " + err);
  PreparedScene P;
  int rc = prepare_scene(desc, &P, &err, BuildOptions::from(opt));
  if (rc) return fail(rc, err);
  struct B3 {
    float lo[3], hi[3];
  };
  auto area = [](const B3& b) {
    float d[3];
    for (int k = 0; k < 3; k++) d[k] = std::max(0.0f, b.hi[k] - b.lo[k]);
    return 2.0 * ((double)d[0] * d[1] + (double)d[1] * d[2] + (double)d[2] * d[0]);
  };
  auto child_box = [&](const BvhNode& n, int c) {
    B3 b;
    b.lo[0] = n.lo_x[c]; b.hi[0] = n.hi_x[c];
    b.lo[1] = n.lo_y[c]; b.hi[1] = n.hi_y[c];
    b.lo[2] = n.lo_z[c]; b.hi[2] = n.hi_z[c];
    return b;
  };
  std::string js = "[";
  for (size_t oi = 0; oi < P.objects.size(); oi++) {
    const DevObject& o = P.objects[oi];
    if (o.kind != FS_OBJ_MESH || !o.i2 || o.i3) continue;  // BVH meshes only
    struct Item {
      uint32_t node, depth;
      B3 box;
    };
    const BvhNode& rn = P.nodes[(uint32_t)o.i0];
    B3 root;
    for (int k = 0; k < 3; k++) {
      B3 a = child_box(rn, 0), b = child_box(rn, 1);
      root.lo[k] = std::min(a.lo[k], b.lo[k]);
      root.hi[k] = std::max(a.hi[k], b.hi[k]);
    }
    const double ar = std::max(area(root), 1e-30);
    double sah = 0.0, ov_w = 0.0;
    uint64_t nodes = 0, leaves = 0, faces = 0;
    uint32_t depth = 0;
    std::vector<double> ov_sum, ov_n;
    std::vector<Item> st{{(uint32_t)o.i0, 0, root}};
    while (!st.empty()) {
      Item it = st.back();
      st.pop_back();
      const BvhNode& n = P.nodes[it.node];
      nodes++;
      depth = std::max(depth, it.depth);
      const double a = area(it.box);
      sah += a / ar;
      B3 c0 = child_box(n, 0), c1 = child_box(n, 1), x;
      for (int k = 0; k < 3; k++) {
        x.lo[k] = std::max(c0.lo[k], c1.lo[k]);
        x.hi[k] = std::min(c0.hi[k], c1.hi[k]);
      }
      bool disjoint = false;
      for (int k = 0; k < 3; k++) disjoint |= x.lo[k] > x.hi[k];
      const double ov = disjoint || a <= 0 ? 0.0 : area(x) / a;
      if (ov_sum.size() <= it.depth) {
        ov_sum.resize(it.depth + 1, 0.0);
        ov_n.resize(it.depth + 1, 0.0);
      }
      ov_sum[it.depth] += ov;
      ov_n[it.depth] += 1.0;
      ov_w += ov * a / ar;
      for (int c = 0; c < 2; c++) {
        const uint32_t w = n.child[c];
        const B3 cb = child_box(n, c);
        if (w & kLeafBit) {
          leaves++;
          faces += leaf_count(w);
          sah += area(cb) / ar * leaf_count(w);
          depth = std::max(depth, it.depth + 1);
        } else {
          st.push_back({w, it.depth + 1, cb});
        }
      }
    }
    char buf[256];
    std::snprintf(buf, sizeof buf,
                  "%s{\"object\": %zu, \"nodes\": %llu, \"leaves\": %llu, \"faces\": %llu, \"depth\": %u, "
                  "\"sah_cost\": %.4f, \"overlap_weighted\": %.4f, \"overlap_per_level\": [",
                  js.size() > 1 ? ", " : "", oi, (unsigned long long)nodes, (unsigned long long)leaves,
                  (unsigned long long)faces, depth, sah, ov_w);
    js += buf;
    for (size_t l = 0; l < ov_sum.size(); l++) {
      std::snprintf(buf, sizeof buf, "%s%.4f", l ? ", " : "", ov_n[l] ? ov_sum[l] / ov_n[l] : 0.0);
      js += buf;
    }
    js += "]}";
  }
  js += "]";
  if (js.size() + 1 > size) return fail(FS_ERR_INVALID, "fs_bvh_quality: output buffer too small");
  std::memcpy(out, js.c_str(), js.size() + 1);
  return FS_OK;
}

int fs_trace_range(fs_context* ctx, const fs_camera* camera, uint32_t width, uint32_t height, const float* xy,
                   uint32_t count, float* distances) {
  if (!ctx || !camera || (count && (!xy || !distances))) return fail(FS_ERR_INVALID, "null argument");
  if (!ctx->have_scene) return fail(FS_ERR_STATE, "fs_trace_range before fs_upload_scene");
  if (width < 2 || height < 2) return fail(FS_ERR_INVALID, "frame must be at least 2x2 (engine.cpp:300-303)");
  if (!count) return FS_OK;
  int rc;
  if ((rc = set_device(ctx))) return rc;
  size_t in_bytes = 8ull * count, bytes = in_bytes + 4ull * count;
  if ((rc = ensure(&ctx->range_io, bytes))) return rc;
  float2* d_xy = (float2*)ctx->range_io.p;
  float* d_out = (float*)((char*)ctx->range_io.p + in_bytes);
  FS_HIP(hipMemcpyAsync(d_xy, xy, in_bytes, hipMemcpyHostToDevice, ctx->stream));
  DevCamera C = camera_basis(camera, width, height);
  if (ctx->scene.tree)
    hipLaunchKernelGGL(dev::trace_range_kernel<true>, dim3((count + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       ctx->stream, ctx->scene, C, d_xy, count, d_out);
  else
    hipLaunchKernelGGL(dev::trace_range_kernel<false>, dim3((count + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       ctx->stream, ctx->scene, C, d_xy, count, d_out);
  FS_HIP(hipGetLastError());
  FS_HIP(hipMemcpyAsync(distances, d_out, 4ull * count, hipMemcpyDeviceToHost, ctx->stream));
  FS_HIP(hipStreamSynchronize(ctx->stream));
  return FS_OK;
}

// ---- RCCL ---------------------------------------------------------------
int fs_comm_unique_id(uint8_t id[FS_COMM_ID_BYTES]) {
  if (!id) return fail(FS_ERR_INVALID, "null id");
  static_assert(sizeof(ncclUniqueId) == FS_COMM_ID_BYTES, "unique id size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(FS_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id, &u, sizeof(u));
  return FS_OK;
}

int fs_comm_init(fs_context* ctx, int nranks, int rank, const uint8_t id[FS_COMM_ID_BYTES]) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(FS_ERR_INVALID, "bad comm arguments");
  int rc;
  if ((rc = set_device(ctx))) return rc;
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  ctx->comm = nullptr;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, u, rank);
  if (r != ncclSuccess) return fail(FS_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  ctx->nranks = nranks;
  ctx->rank = rank;
  return FS_OK;
}

int fs_comm_count(fs_context* ctx, int* count) {
  if (!ctx || !count) return fail(FS_ERR_INVALID, "null argument");
  if (!ctx->comm) return fail(FS_ERR_STATE, "fs_comm_count before fs_comm_init");
  ncclResult_t r = ncclCommCount(ctx->comm, count);
  if (r != ncclSuccess) return fail(FS_ERR_COMM, std::string("ncclCommCount: ") + ncclGetErrorString(r));
  return FS_OK;
}

int fs_comm_destroy(fs_context* ctx) {
  if (!ctx) return fail(FS_ERR_INVALID, "null context");
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  ctx->comm = nullptr;
  ctx->nranks = 1;
  ctx->rank = 0;
  return FS_OK;
}

}  // extern "C"

namespace {

// The tile exchange of a multi-GPU frame: pack_tiles writes a rank's owned
// tiles (tile t of rank r is t = r + k * nranks) as kPackWords words per
// pixel; unpack_tiles scatters nranks such packs, concatenated in rank order
// as ncclGather delivers them, into the root's frame (skipping its own).
struct TileExchange {
  Launch L{};
  uint32_t owned_max = 0;
  size_t pixels = 0;  // per rank
  size_t bytes() const { return pixels * dev::kPackWords * 4; }
};
int tile_exchange(const fs_render_params* params, fs_frame* frame, uint32_t nranks, uint32_t rank, TileExchange* X) {
  uint32_t ts, stride;
  int rc = check_params(params, frame, &ts, &stride);
  if (rc) return rc;
  if (stride != nranks || params->tile_offset != rank)
    return fail(FS_ERR_INVALID, "tiling must be tile_offset=rank, tile_stride=nranks");
  X->L.tile_size = ts;
  X->L.tiles_x = (params->width + ts - 1) / ts;
  X->L.tile_offset = params->tile_offset;
  X->L.tile_stride = stride;
  const uint32_t tiles = X->L.tiles_x * ((params->height + ts - 1) / ts);
  X->owned_max = (tiles + stride - 1) / stride;
  X->pixels = (size_t)X->owned_max * ts * ts;
  return FS_OK;
}
int launch_pack(fs_context* ctx, fs_frame* frame, const TileExchange& X, uint32_t* dst) {
  hipLaunchKernelGGL(dev::pack_tiles, dim3((uint32_t)((X.pixels + 255) / 256)), dim3(256), 0, ctx->stream,
                     frame_view(frame), X.L, X.owned_max, dst);
  FS_HIP(hipGetLastError());
  return FS_OK;
}
int launch_unpack(fs_context* ctx, fs_frame* frame, const TileExchange& X, uint32_t nranks, uint32_t self,
                  const uint32_t* src) {
  const size_t total = X.pixels * nranks;
  hipLaunchKernelGGL(dev::unpack_tiles, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, ctx->stream,
                     frame_view(frame), X.L, X.owned_max, nranks, self, src);
  FS_HIP(hipGetLastError());
  return FS_OK;
}

}  // namespace

extern "C" {

// Packs this rank's owned tiles, ncclGather's them to root over xGMI and
// scatters them into root's frame. One collective per render.
int fs_frame_gather(fs_context* ctx, fs_frame* frame, const fs_render_params* params, int root) {
  if (!ctx || !frame || !params) return fail(FS_ERR_INVALID, "null argument");
  if (!ctx->comm) return fail(FS_ERR_STATE, "fs_frame_gather before fs_comm_init");
  TileExchange X;
  int rc = tile_exchange(params, frame, (uint32_t)ctx->nranks, (uint32_t)ctx->rank, &X);
  if (rc) return rc;
  if (root < 0 || root >= ctx->nranks) return fail(FS_ERR_INVALID, "root out of range");
  if ((rc = set_device(ctx))) return rc;
  if ((rc = ensure(&ctx->pack_send, X.bytes()))) return rc;
  if (ctx->rank == root && (rc = ensure(&ctx->pack_recv, X.bytes() * ctx->nranks))) return rc;
  if ((rc = launch_pack(ctx, frame, X, (uint32_t*)ctx->pack_send.p))) return rc;
  ncclResult_t r = ncclGather(ctx->pack_send.p, ctx->rank == root ? ctx->pack_recv.p : nullptr, X.bytes() / 4,
                              ncclUint32, root, ctx->comm, ctx->stream);
  if (r != ncclSuccess) return fail(FS_ERR_COMM, std::string("ncclGather: ") + ncclGetErrorString(r));
  if (ctx->rank == root &&
      (rc = launch_unpack(ctx, frame, X, (uint32_t)ctx->nranks, (uint32_t)ctx->rank, (const uint32_t*)ctx->pack_recv.p)))
    return rc;
  FS_HIP(hipStreamSynchronize(ctx->stream));
  return FS_OK;
}

int fs_frame_pack_bytes(const fs_render_params* params, uint64_t* bytes) {
  if (!params || !bytes) return fail(FS_ERR_INVALID, "null argument");
  fs_frame probe;
  probe.width = params->width;
  probe.height = params->height;
  TileExchange X;
  int rc = tile_exchange(params, &probe, params->tile_stride ? params->tile_stride : 1, params->tile_offset, &X);
  if (rc) return rc;
  *bytes = X.bytes();
  return FS_OK;
}

int fs_frame_pack(fs_context* ctx, fs_frame* frame, const fs_render_params* params, void* host_dst, size_t bytes) {
  if (!ctx || !frame || !params || !host_dst) return fail(FS_ERR_INVALID, "null argument");
  if (frame->ctx != ctx) return fail(FS_ERR_INVALID, "frame belongs to another context");
  TileExchange X;
  int rc = tile_exchange(params, frame, params->tile_stride ? params->tile_stride : 1, params->tile_offset, &X);
  if (rc) return rc;
  if (bytes != X.bytes()) return fail(FS_ERR_INVALID, "byte count does not match fs_frame_pack_bytes");
  if ((rc = set_device(ctx))) return rc;
  if ((rc = ensure(&ctx->pack_send, X.bytes()))) return rc;
  if ((rc = launch_pack(ctx, frame, X, (uint32_t*)ctx->pack_send.p))) return rc;
  FS_HIP(hipMemcpyAsync(host_dst, ctx->pack_send.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
  FS_HIP(hipStreamSynchronize(ctx->stream));
  return FS_OK;
}

int fs_frame_unpack(fs_context* ctx, fs_frame* frame, const fs_render_params* params, const void* host_src,
                    size_t bytes) {
  if (!ctx || !frame || !params || !host_src) return fail(FS_ERR_INVALID, "null argument");
  if (frame->ctx != ctx) return fail(FS_ERR_INVALID, "frame belongs to another context");
  const uint32_t nranks = params->tile_stride ? params->tile_stride : 1;
  TileExchange X;
  int rc = tile_exchange(params, frame, nranks, params->tile_offset, &X);
  if (rc) return rc;
  if (bytes != X.bytes() * nranks) return fail(FS_ERR_INVALID, "byte count must be nranks x fs_frame_pack_bytes");
  if ((rc = set_device(ctx))) return rc;
  if ((rc = ensure(&ctx->pack_recv, bytes))) return rc;
  FS_HIP(hipMemcpyAsync(ctx->pack_recv.p, host_src, bytes, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = launch_unpack(ctx, frame, X, nranks, params->tile_offset, (const uint32_t*)ctx->pack_recv.p))) return rc;
  FS_HIP(hipStreamSynchronize(ctx->stream));
  return FS_OK;
}

}  // extern "C"
