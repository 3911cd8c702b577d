// fs_libm.h — sinf, cosf and atan2f exactly as the oracle's C library
// computes them, for the device.
//
// The reference calls std::cos / std::sin / atan2f on floats in three places
// of the path: the thin-lens offset (engine.cpp:221-244, the reference's
// default camera has an aperture), the frosted-glass rotation (vector3.h:
// 315-333 via material.cpp random_refraction) and the sphere texture map
// (intersect.cpp:769-784, also the sky texture). The device's own ocml
// routines round differently from the host library in about 0.1 % of the
// arguments, so those paths were held only to a tolerance. These restatements
// give the host library's bits:
//
//  * sinf / cosf: the ARM optimized-routines algorithm (MIT licence; glibc
//    2.28+ flt-32/s_sinf.c, s_cosf.c, sincosf.h, sincosf_data.c): double-
//    precision reduction by pi/2 and two short polynomials, with the fused
//    multiply-adds of the x86-64 FMA build the host's libm dispatches to on
//    an FMA-capable CPU (the build container and the GPU box both). Arguments of at least
//    120 take the table-driven large reduction.
//  * atan2f: the fdlibm float restatement (Sun Microsystems, freely
//    redistributable notice; glibc flt-32/e_atan2f.c + s_atanf.c): plain float
//    arithmetic, unfused.
//
// tests/test_exact_rewrites.py compiles this header on the host with g++ and
// checks it bit for bit against the host's libm: sinf/cosf over EVERY float of
// |x| <= 2*pi (the thin lens draws angles in [0, 2*pi), the frosted rotation
// |delta| <= pi/2) plus a sweep of larger arguments, atan2f over the unit
// normals the sphere map feeds it and the special cases.
#pragma once

#include <math.h>
#include <stdint.h>

#ifndef FS_LIBM_FN
#define FS_LIBM_FN __host__ __device__ __forceinline__
#endif

namespace fs {
namespace libm {

// sincosf_data.c: the polynomial (table 0; table 1, used when bit 1 of the
// quadrant is set, negates every cosine coefficient, which negates the cosine
// polynomial's result exactly) and the reduction constants.
enum : int { kHpiInv, kHpi, kC0, kC1, kC2, kC3, kC4, kS1, kS2, kS3, kPi63, kNumK };
__constant__ constexpr double kSinCos[kNumK] = {
    0x1.45f306dc9c883p+23,  // 2/pi * 2^24
    0x1.921fb54442d18p+0,   // pi/2
    0x1p0,   -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
    -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13,
    0x1.921fb54442d18p-62,  // pi/2 * 2^-63
};

// Constant i, read where it is used: on the device a scalar load at an
// address the compiler cannot see through, so the double constants are not
// hoisted out of the trace kernel's loop into registers (where they were
// spilled to scratch: the parked-walk kernel's scratch rose from 20 to
// 36 B/lane).
FS_LIBM_FN double K(int i) {
  uint32_t z = 0;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
#endif
  return kSinCos[i + (int)z];
}

FS_LIBM_FN uint32_t top12(float x) { return (__builtin_bit_cast(uint32_t, x) >> 20) & 0x7ff; }

// sinf_poly: n even the sine polynomial of x, n odd the cosine polynomial
// (of x2), negated when bit 1 of n is set (table 1)
FS_LIBM_FN float sincos_poly(double x, double x2, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = fma(x2, K(kS3), K(kS2));
    const double x7 = x3 * x2;
    const double s = fma(x3, K(kS1), x);
    return (float)fma(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = fma(x2, K(kC4), K(kC3));
  const double c1 = fma(x2, K(kC1), K(kC0));
  const double x6 = x4 * x2;
  const double c = fma(x4, K(kC2), c1);
  const float r = (float)fma(x6, c2, c);
  return (n & 2) ? -r : r;
}

// reduce_fast: x - n * pi/2 with n the nearest quadrant, |x| < 120
FS_LIBM_FN double reduce_fast(double x, int* np) {
  const double r = x * K(kHpiInv);
  const int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fma(-(double)n, K(kHpi), x);
}

// __inv_pio4[i]: bits 8i .. 8i + 31 of 24 zero bits followed by 2/pi to 192
// bits (0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, ...), taken from the
// bit string by shifts instead of a table, so the device keeps no private array
FS_LIBM_FN uint32_t inv_pio4(uint32_t i) {
  constexpr uint64_t w0 = 0x000000a2f9836e4eull, w1 = 0x441529fc2757d1f5ull, w2 = 0x34ddc0db6295993cull,
                     w3 = 0x439041fe5163abdeull;  // the string as 64-bit words, w3 past the table's last bit
  const uint32_t bit = 8 * i, k = bit >> 6, sh = bit & 63;
  const uint64_t hi = k == 0 ? w0 : k == 1 ? w1 : k == 2 ? w2 : w3;
  const uint64_t lo = k == 0 ? w1 : k == 1 ? w2 : w3;
  const uint64_t v = sh ? (hi << sh) | (lo >> (64 - sh)) : hi;
  return (uint32_t)(v >> 32);
}

// reduce_large: Payne-Hanek with 2/pi to 192 bits (8 new bits per entry)
FS_LIBM_FN double reduce_large(uint32_t xi, int* np) {
  const uint32_t i = (xi >> 26) & 15;
  const int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  uint64_t res0 = (uint32_t)(xi * inv_pio4(i));
  const uint64_t res1 = (uint64_t)xi * inv_pio4(i + 4);
  const uint64_t res2 = (uint64_t)xi * inv_pio4(i + 8);
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  const uint64_t n = (res0 + (1ull << 61)) >> 62;
  res0 -= n << 62;
  *np = (int)n;
  return (double)(int64_t)res0 * K(kPi63);
}

// sign of the sine in quadrants 0..3
FS_LIBM_FN double quadrant_sign(int n) { return (n & 3) == 1 || (n & 3) == 2 ? -1.0 : 1.0; }

// s_sinf.c
FS_LIBM_FN float sinf(float y) {
  double x = y;
  int n;
  if (top12(y) < top12(0x1.921fb6p-1f)) {  // |y| < pi/4
    if (top12(y) < top12(0x1p-12f)) return y;
    return sincos_poly(x, x * x, 0);
  }
  if (top12(y) < top12(120.0f)) {
    x = reduce_fast(x, &n);
    return sincos_poly(x * quadrant_sign(n), x * x, n);
  }
  if (top12(y) < top12(__builtin_inff())) {
    const uint32_t xi = __builtin_bit_cast(uint32_t, y);
    const int sign = (int)(xi >> 31);
    x = reduce_large(xi, &n);
    // the polynomial branch follows n, table 1 (and the sign) n + sign
    return sincos_poly(x * quadrant_sign(n + sign), x * x, (n & 1) | ((n + sign) & 2));
  }
  return y - y;  // NaN for inf and NaN
}

// s_cosf.c
FS_LIBM_FN float cosf(float y) {
  double x = y;
  int n;
  if (top12(y) < top12(0x1.921fb6p-1f)) {
    if (top12(y) < top12(0x1p-12f)) return 1.0f;
    return sincos_poly(x, x * x, 1);
  }
  if (top12(y) < top12(120.0f)) {
    x = reduce_fast(x, &n);
    // n ^ 1 picks the branch; table 1 follows bit 1 of n (which n ^ 1 keeps)
    return sincos_poly(x * quadrant_sign(n), x * x, n ^ 1);
  }
  if (top12(y) < top12(__builtin_inff())) {
    const uint32_t xi = __builtin_bit_cast(uint32_t, y);
    const int sign = (int)(xi >> 31);
    x = reduce_large(xi, &n);
    return sincos_poly(x * quadrant_sign(n + sign), x * x, ((n ^ 1) & 1) | ((n + sign) & 2));
  }
  return y - y;
}

// sinf(y) and cosf(y) together, bit for bit the two calls above (one
// reduction, both polynomials; glibc's s_sincosf.c has the same operations)
FS_LIBM_FN void sincosf(float y, float* sp, float* cp) {
  double x = y;
  int n, ns, nc;
  if (top12(y) < top12(0x1.921fb6p-1f)) {
    if (top12(y) < top12(0x1p-12f)) {
      *sp = y;
      *cp = 1.0f;
      return;
    }
    ns = 0;
    nc = 1;
  } else if (top12(y) < top12(120.0f)) {
    x = reduce_fast(x, &n);
    x = x * quadrant_sign(n);
    ns = n;
    nc = n ^ 1;
  } else if (top12(y) < top12(__builtin_inff())) {
    const uint32_t xi = __builtin_bit_cast(uint32_t, y);
    const int sign = (int)(xi >> 31);
    x = reduce_large(xi, &n);
    x = x * quadrant_sign(n + sign);
    ns = (n & 1) | ((n + sign) & 2);
    nc = ((n ^ 1) & 1) | ((n + sign) & 2);
  } else {
    *sp = *cp = y - y;
    return;
  }
  const double x2 = x * x;
  *sp = sincos_poly(x, x2, ns);
  *cp = sincos_poly(x, x2, nc);
}

// s_atanf.c (fdlibm)
FS_LIBM_FN float atanf(float x) {
  // atanhi / atanlo: atan(0.5), atan(1), atan(1.5), atan(inf) as hi + lo
  constexpr float kHi0 = 4.6364760399e-01f, kHi1 = 7.8539812565e-01f, kHi2 = 9.8279368877e-01f,
                  kHi3 = 1.5707962513e+00f;
  constexpr float kLo0 = 5.0121582440e-09f, kLo1 = 3.7748947079e-08f, kLo2 = 3.4473217170e-08f,
                  kLo3 = 7.5497894159e-08f;
  constexpr float kAT[11] = {3.3333334327e-01f,  -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                             9.0908870101e-02f,  -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                             4.9768779427e-02f,  -3.6531571299e-02f, 1.6285819933e-02f};
  const int32_t hx = __builtin_bit_cast(int32_t, x);
  const int32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {  // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;
    return hx > 0 ? kHi3 + kLo3 : -kHi3 - kLo3;
  }
  if (ix < 0x3ee00000) {  // |x| < 0.4375
    if (ix < 0x39800000) return x;  // |x| < 2^-12
    id = -1;
  } else {
    x = fabsf(x);
    if (ix < 0x3f980000) {    // |x| < 1.1875
      if (ix < 0x3f300000) {  // 7/16 <= |x| < 11/16
        id = 0;
        x = (2.0f * x - 1.0f) / (2.0f + x);
      } else {  // 11/16 <= |x| < 19/16
        id = 1;
        x = (x - 1.0f) / (x + 1.0f);
      }
    } else if (ix < 0x401c0000) {  // |x| < 2.4375
      id = 2;
      x = (x - 1.5f) / (1.0f + 1.5f * x);
    } else {  // 2.4375 <= |x| < 2^25
      id = 3;
      x = -1.0f / x;
    }
  }
  const float z = x * x;
  const float w = z * z;
  const float s1 = z * (kAT[0] + w * (kAT[2] + w * (kAT[4] + w * (kAT[6] + w * (kAT[8] + w * kAT[10])))));
  const float s2 = w * (kAT[1] + w * (kAT[3] + w * (kAT[5] + w * (kAT[7] + w * kAT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  const float hi = id == 0 ? kHi0 : id == 1 ? kHi1 : id == 2 ? kHi2 : kHi3;
  const float lo = id == 0 ? kLo0 : id == 1 ? kLo1 : id == 2 ? kLo2 : kLo3;
  const float r = hi - ((x * (s1 + s2) - lo) - x);
  return hx < 0 ? -r : r;
}

// e_atan2f.c (fdlibm)
FS_LIBM_FN float atan2f(float y, float x) {
  constexpr float kTiny = 1.0e-30f, kPiO4 = 7.8539818525e-01f, kPiO2 = 1.5707963705e+00f, kPiF = 3.1415927410e+00f,
                  kPiLo = -8.7422776573e-08f;
  const int32_t hx = __builtin_bit_cast(int32_t, x), hy = __builtin_bit_cast(int32_t, y);
  const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;  // NaN
  if (hx == 0x3f800000) return atanf(y);                  // x = 1
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      // 2 * sign(x) + sign(y)
  if (iy == 0) {
    if (m < 2) return y;
    return m == 2 ? kPiF + kTiny : -kPiF - kTiny;
  }
  if (ix == 0) return hy < 0 ? -kPiO2 - kTiny : kPiO2 + kTiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      const float q = m < 2 ? kPiO4 + kTiny : 3.0f * kPiO4 + kTiny;
      return (m & 1) ? -q : q;
    }
    const float q = m < 2 ? 0.0f : kPiF + kTiny;
    return (m & 1) ? -q : q;
  }
  if (iy == 0x7f800000) return hy < 0 ? -kPiO2 - kTiny : kPiO2 + kTiny;
  const int k = (iy - ix) >> 23;
  float z;
  if (k > 26)
    z = kPiO2 + 0.5f * kPiLo;  // |y/x| > 2^26
  else if (hx < 0 && k < -26)
    z = 0.0f;  // |y|/x < -2^26
  else
    z = atanf(fabsf(y / x));
  switch (m) {
    case 0:
      return z;
    case 1:
      return -z;
    case 2:
      return kPiF - (z - kPiLo);
    default:
      return (z - kPiLo) - kPiF;
  }
}

}  // namespace libm
}  // namespace fs
