// libm_check.cpp — csrc/fs_libm.h against the host C library, bit for bit
// (tests/test_exact_rewrites.py builds and runs it; test infrastructure).
//
//   libm_check sincos LO HI STEP   every STEP-th float bit pattern in [LO, HI]:
//                                  fs::libm sinf, cosf and sincosf vs sinf, cosf
//   libm_check atan LO HI STEP     fs::libm atanf vs atanf
//   libm_check atan2 N SEED        N random (y, x) bit patterns, N unit-vector
//                                  components (the sphere map's atan2f(n.x, n.z)),
//                                  and the special values, vs atan2f
// Prints "<checked> <differing>" and the first few differences; 8 threads.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

#define FS_LIBM_FN static inline
#define __constant__
#include "fs_libm.h"

static uint32_t bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
static float flt(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static bool same(float a, float b) { return bits(a) == bits(b) || (a != a && b != b); }

static std::atomic<long> g_checked{0}, g_bad{0};
static void report(const char* what, float y, float x, float want, float got) {
  if (g_bad.fetch_add(1) < 5) printf("%s(%a, %a): libm %a, fs_libm %a\n", what, y, x, want, got);
}

static void sincos_range(uint64_t lo, uint64_t hi, uint64_t step) {
  long n = 0;
  for (uint64_t k = lo; k <= hi; k += step) {
    const float x = flt((uint32_t)k);
    const float s = sinf(x), c = cosf(x);
    float s2, c2;
    fs::libm::sincosf(x, &s2, &c2);
    if (!same(s, fs::libm::sinf(x))) report("sinf", x, 0, s, fs::libm::sinf(x));
    if (!same(c, fs::libm::cosf(x))) report("cosf", x, 0, c, fs::libm::cosf(x));
    if (!same(s, s2) || !same(c, c2)) report("sincosf", x, 0, s, s2);
    n++;
  }
  g_checked += n;
}

static void atan_range(uint64_t lo, uint64_t hi, uint64_t step) {
  long n = 0;
  for (uint64_t k = lo; k <= hi; k += step) {
    const float x = flt((uint32_t)k);
    if (!same(atanf(x), fs::libm::atanf(x))) report("atanf", x, 0, atanf(x), fs::libm::atanf(x));
    n++;
  }
  g_checked += n;
}

static void atan2_pair(float y, float x) {
  const float a = atan2f(y, x), b = fs::libm::atan2f(y, x);
  if (!same(a, b)) report("atan2f", y, x, a, b);
}

static void atan2_random(long n, uint64_t seed) {
  uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
  auto next = [&]() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  };
  for (long i = 0; i < n; i++) {
    const uint64_t r = next();
    atan2_pair(flt((uint32_t)r), flt((uint32_t)(r >> 32)));
    // a unit vector's components, as the sphere map feeds them
    const uint64_t q = next();
    const float a = (float)((q & 0xffffff) / 16777216.0) * 2 - 1, b = (float)(((q >> 24) & 0xffffff) / 16777216.0) * 2 - 1,
                c = (float)(((q >> 48) & 0xffff) / 65536.0) * 2 - 1;
    const float l = sqrtf(a * a + b * b + c * c);
    if (l > 0) atan2_pair(a / l, b / l);
  }
  g_checked += 2 * n;
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int T = 8;
  std::vector<std::thread> th;
  if (!strcmp(argv[1], "atan2")) {
    const long n = atol(argv[2]);
    const uint64_t seed = strtoull(argv[3], 0, 0);
    for (int t = 0; t < T; t++) th.emplace_back(atan2_random, n / T, seed + t);
    const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, INFINITY, -INFINITY, NAN, 1e-45f, -1e-45f, 3e38f, -3e38f, 0.5f, 2.0f};
    for (float y : sp)
      for (float x : sp) atan2_pair(y, x);
  } else {
    const uint64_t lo = strtoull(argv[2], 0, 0), hi = strtoull(argv[3], 0, 0), step = argc > 4 ? strtoull(argv[4], 0, 0) : 1;
    const uint64_t per = ((hi - lo) / step / T + 1) * step;
    for (int t = 0; t < T; t++) {
      const uint64_t a = lo + t * per, b = a + per - step < hi ? a + per - step : hi;
      if (a > hi) break;
      th.emplace_back(!strcmp(argv[1], "atan") ? atan_range : sincos_range, a, b, step);
    }
  }
  for (auto& t : th) t.join();
  printf("%ld %ld\n", g_checked.load(), g_bad.load());
  return g_bad.load() != 0;
}
