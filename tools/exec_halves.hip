// exec_halves.hip — does a wave64 VALU instruction cost less when one
// 32-lane half of its exec mask is empty? (measurement aid, no reference
// counterpart)
//
// gfx950 runs a wave64 VALU instruction on a SIMD-32 in two passes. If a pass
// whose 32 lanes are all inactive were skipped, packing the walking lanes of a
// BVH node loop (about 19 of 64 active per trip on C4) into one half would
// halve its VALU issue time; if not, the lane layout inside a wave does not
// matter to the SIMD and only moving work between waves can help. One and
// four waves per SIMD (one wave alone issues a VALU instruction every ~4
// cycles, so only several waves saturate the pipe) run a loop of independent
// v_fma_f32 under masks of 64, 32 (low half, even lanes), 16 (low quarter,
// spread) and 1 active lane(s) and stamp the shader clock (s_memtime) around
// it; SIMD cycles per instruction = a wave's cycles / (its instructions x the
// waves sharing its SIMD).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/exec_halves.hip -o tools/_bin/exec_halves
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                   \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      return 1;                                                    \
    }                                                              \
  } while (0)

constexpr int kTrips = 20000;

#define F8 \
  "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n" \
  "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n"

// mode: 0 all lanes, 1 lanes 0-31, 2 even lanes, 3 lanes 0-15, 4 every 4th lane, 5 lane 0, 6 lanes 0-31 and 32
__global__ __launch_bounds__(64) void masked_loop(unsigned long long* __restrict__ out, float* __restrict__ sink,
                                                  int mode, int trips) {
  const uint32_t l = threadIdx.x;
  bool on = true;
  if (mode == 1) on = l < 32;
  if (mode == 2) on = (l & 1) == 0;
  if (mode == 3) on = l < 16;
  if (mode == 4) on = (l & 3) == 0;
  if (mode == 5) on = l == 0;
  if (mode == 6) on = l <= 32;
  float a = l, b = a + 1, c = a + 2, d = a + 3, e = a + 4, f = a + 5, g = a + 6, h = a + 7;
  const float m = 0.999f, k = 0.001f;
  unsigned long long t0 = 0, t1 = 0;
  if (on) {
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < trips; i++)
      asm volatile(F8 F8 F8 F8
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h)
                   : "v"(m), "v"(k));
    t1 = __builtin_amdgcn_s_memtime();
  }
  if (l == 0) out[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + l] = a + b + c + d + e + f + g + h;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int rc = 0;
  unsigned long long* d_out;
  float* d_sink;
  CHECK(hipMalloc(&d_out, 8ull * cus * 16));
  CHECK(hipMalloc(&d_sink, 4ull * 64 * cus * 16));
  const char* names[] = {"all 64", "lanes 0-31", "even lanes (32)", "lanes 0-15", "every 4th lane (16)", "lane 0",
                         "lanes 0-32 (33)"};
  std::printf("{\"trips\": %d, \"fma_per_trip\": 32, \"runs\": [\n", kTrips);
  for (int wps : {1, 4})
  for (int mode = 0; mode < 7; mode++) {
    const int grid = cus * 4 * wps;
    hipLaunchKernelGGL(masked_loop, dim3(grid), dim3(64), 0, 0, d_out, d_sink, mode, 100);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(masked_loop, dim3(grid), dim3(64), 0, 0, d_out, d_sink, mode, kTrips);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> c(grid);
    CHECK(hipMemcpy(c.data(), d_out, 8ull * grid, hipMemcpyDeviceToHost));
    double mean = 0;
    for (auto v : c) mean += (double)v;
    mean /= grid;
    std::printf("  {\"waves_per_simd\": %d, \"mask\": \"%s\", \"wave_cycles_per_fma\": %.3f, "
                "\"simd_cycles_per_fma\": %.3f}%s\n",
                wps, names[mode], mean / (32.0 * kTrips), mean / (32.0 * kTrips * wps), wps == 4 && mode == 6 ? "" : ",");
  }
  std::printf("]}\n");
  return rc;
}
