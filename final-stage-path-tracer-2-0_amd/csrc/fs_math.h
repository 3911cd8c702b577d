// fs_math.h — float vector math of the reference hot path, host + device.
//
// Every routine keeps the reference's operand order and float/double
// promotions so that a gfx950 build with -ffp-contract=off produces the same
// bits as the reference's x86-64 g++ -O2 build. Citations are
// relative to the reference's source/ directory.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FS_HD __host__ __device__ __forceinline__

namespace fs {

constexpr float kPi = 3.14159262f;        // math/base.h:80  BASE_PI
constexpr float kInfinity = 1.0e15f;      // math/base.h:82  BASE_INFINITY
constexpr float kEpsilon = 1.0e-5f;       // math/base.h:83  BASE_EPSILON
constexpr float kStepOffset = 0.03f;      // engine.cpp:17   kTraceStepObjectOffset
constexpr float kDiffuseContrib = 0.001f; // material.cpp:12
constexpr float kRoughnessThr = 0.95f;    // material.cpp:13
constexpr uint32_t kMaxDepth = 8;         // engine.cpp:16

struct f3 {
  float x, y, z;
};
struct f4 {
  float x, y, z, w;
};

FS_HD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
FS_HD f4 mk4(float x, float y, float z, float w) { return f4{x, y, z, w}; }
FS_HD f3 xyz(f4 p) { return f3{p.x, p.y, p.z}; }
FS_HD f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }  // vector3.h:354
FS_HD f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }  // vector3.h:350
FS_HD f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }  // vector3.h:366
FS_HD f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }     // vector3.h:374
FS_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }       // vector3.h:292
FS_HD f3 cross(f3 a, f3 b) {                                                    // vector3.h:193
  return f3{(a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x)};
}

// scalar.h:233-245 — Quake inverse square root, one Newton step.
FS_HD float inv_sqrt(float f) {
  float half = 0.5f * f;
  int32_t i = __builtin_bit_cast(int32_t, f);
  i = 0x5f3759df - (i >> 1);
  f = __builtin_bit_cast(float, i);
  f = f * (1.5f - half * f * f);
  return f;
}
FS_HD float fsqrt(float f) { return 1.0f / inv_sqrt(f); }   // scalar.h:245 base::sqrtf
FS_HD float length(f3 a) { return fsqrt(dot(a, a)); }       // vector3.h:301
FS_HD f3 normalize(f3 a) {                                  // vector3.h:181-191
  float l = length(a);
  if (l == 0.0f) l = 1.0f;
  return f3{a.x / l, a.y / l, a.z / l};
}
FS_HD f3 reflect(f3 v, f3 n) { return v - n * (dot(n, v) * (1.0f + 1.0f)); }  // vector3.h:208
FS_HD f3 refract(f3 v, f3 n, float index) {                                   // vector3.h:213-222
  float n_dot_v = -dot(v, n);
  float sin2 = (float)((double)(index * index) * (1.0 - (double)(n_dot_v * n_dot_v)));
  if (sin2 >= 1.0f) return f3{0.f, 0.f, 0.f};
  f3 r = v * index + n * (index * n_dot_v - fsqrt((float)(1.0 - (double)sin2)));
  return normalize(r);
}
// vector3.h:315-333 (Rodrigues, axis not normalised)
FS_HD f3 rotate(f3 v, float c, float s, f3 ax) {
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
  return f3{o0, o1, o2};
}
FS_HD bool cmp_eps(float a, float b, float ep) { return a > (b - ep) && a < (b + ep); }  // scalar.h:337
FS_HD float plane_dist(f4 p, f3 pt) { return p.x * pt.x + p.y * pt.y + p.z * pt.z + p.w; }  // plane.h:68
FS_HD f4 plane_np(f3 n, f3 p) { return f4{n.x, n.y, n.z, -dot(n, p)}; }                   // plane.h:73
FS_HD f3 calc_normal(f3 a, f3 b, f3 c) { return normalize(cross(b - a, c - a)); }         // normal.h:67
FS_HD f4 plane_3p(f3 a, f3 b, f3 c) { return plane_np(calc_normal(a, b, c), a); }         // plane.h:85

// ---- RNG: xorshift64* (random.cpp:14-49) ---------------------------------
FS_HD uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
FS_HD uint64_t pixel_seed(uint64_t pixel, uint64_t sample, uint64_t seed) {
  return splitmix64((pixel << 20) ^ sample ^ seed) | 1ull;
}
FS_HD uint64_t rng_next(uint64_t& s) {
  uint64_t x = s;
  x ^= x << 12;
  x ^= x >> 25;
  x ^= x << 27;
  s = x;
  return x * 0x2545F4914F6CDD1Dull;
}
// x mod (2^31 - 1) without a 64-bit divide: 2^31 == 1 (mod 2^31 - 1).
FS_HD uint32_t mod_mersenne31(uint64_t x) {
  uint64_t r = (x & 0x7FFFFFFFull) + (x >> 31);   // < 2^34
  r = (r & 0x7FFFFFFFull) + (r >> 31);            // < 2^31 + 8
  r = (r & 0x7FFFFFFFull) + (r >> 31);            // <= 2^31 - 1 + 1
  return (uint32_t)(r >= 0x7FFFFFFFull ? r - 0x7FFFFFFFull : r);
}
// random.cpp:25-27: (float)(r % 0x7FFFFFFF) / (float)0x7FFFFFFF
FS_HD float rng_float(uint64_t& s) { return (float)mod_mersenne31(rng_next(s)) / 2147483648.0f; }
// random.cpp:41-49
FS_HD float rng_float_range(uint64_t& s, float lo, float hi) { return lo + rng_float(s) * (hi - lo); }
// random_integer_range(0, 32767) (random.cpp:29-39) — span 32768
FS_HD uint32_t rng_table_index(uint64_t& s) { return (uint32_t)(rng_next(s) & 32767ull); }

}  // namespace fs
