// salu_peak.hip — the scalar unit's issue ceiling on gfx950 (measurement aid,
// no reference counterpart; VERDICT r4 "next" item 1).
//
// The render kernels issue 0.64-0.79 SALU instructions per CU-cycle
// (SQ_INSTS_SALU / (256 CUs x cycles), profiles/pmc_*.json). MI355X_MICROARCH.md
// gives the VALU issue cost but no scalar-unit figure, so the PMC summaries need
// a measured denominator. Each wave runs a loop of independent scalar ALU
// instructions (8 SGPR chains, 32 per trip) and stamps its own shader-clock
// (s_memtime) and 100 MHz (s_memrealtime) counters at the start and the end;
// the host converts them into instructions per CU-cycle for 1, 4, 8, 16, 24
// and 32 waves per CU, plus a VALU-only and a mixed SALU + VALU loop at the
// render kernel's 24 waves per CU, and a dependent scalar chain.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/salu_peak.hip -o tools/_bin/salu_peak
// Run (GPU box): tools/_bin/salu_peak > gpurun_out/<round>/salu_peak.json
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

constexpr int kTrips = 40000;
// shader clock of the first run (one wave per CU, every wave co-resident):
// prices the later runs' kernel time in cycles
double g_clock_ghz = 0.0;

struct Stamp {
  unsigned long long c0, c1, r0, r1;
};

// 32 independent scalar adds per trip (8 chains of 4).
#define S8 \
  "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 3\n s_add_u32 %2, %2, 5\n s_add_u32 %3, %3, 7\n" \
  "s_add_u32 %4, %4, 9\n s_add_u32 %5, %5, 11\n s_add_u32 %6, %6, 13\n s_add_u32 %7, %7, 15\n"
// 32 independent wave64 VALU adds per trip (8 chains of 4).
#define V8 \
  "v_add_u32 %0, %0, 1\n v_add_u32 %1, %1, 3\n v_add_u32 %2, %2, 5\n v_add_u32 %3, %3, 7\n" \
  "v_add_u32 %4, %4, 9\n v_add_u32 %5, %5, 11\n v_add_u32 %6, %6, 13\n v_add_u32 %7, %7, 15\n"
// 16 scalar + 16 vector adds per trip, interleaved.
#define M8 \
  "s_add_u32 %0, %0, 1\n v_add_u32 %8, %8, 1\n s_add_u32 %1, %1, 3\n v_add_u32 %9, %9, 3\n"     \
  "s_add_u32 %2, %2, 5\n v_add_u32 %10, %10, 5\n s_add_u32 %3, %3, 7\n v_add_u32 %11, %11, 7\n" \
  "s_add_u32 %4, %4, 9\n v_add_u32 %12, %12, 9\n s_add_u32 %5, %5, 11\n v_add_u32 %13, %13, 11\n" \
  "s_add_u32 %6, %6, 13\n v_add_u32 %14, %14, 13\n s_add_u32 %7, %7, 15\n v_add_u32 %15, %15, 15\n"
// 32 dependent scalar adds per trip (one chain).
#define D8 \
  "s_add_u32 %0, %0, 1\n s_add_u32 %0, %0, 3\n s_add_u32 %0, %0, 5\n s_add_u32 %0, %0, 7\n" \
  "s_add_u32 %0, %0, 9\n s_add_u32 %0, %0, 11\n s_add_u32 %0, %0, 13\n s_add_u32 %0, %0, 15\n"

__device__ __forceinline__ unsigned long long memtime() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ unsigned long long memrealtime() { return __builtin_amdgcn_s_memrealtime(); }

// mode 0: scalar, 1: vector, 2: mixed, 3: dependent scalar chain
template <int MODE>
__global__ __launch_bounds__(64, 8) void peak_loop(Stamp* __restrict__ out, uint32_t* __restrict__ sink, int trips) {
  uint32_t a = __builtin_amdgcn_readfirstlane(blockIdx.x), b = a + 1, c = a + 2, d = a + 3, e = a + 4, f = a + 5,
           g = a + 6, h = a + 7;
  uint32_t va = threadIdx.x, vb = va + 1, vc = va + 2, vd = va + 3, ve = va + 4, vf = va + 5, vg = va + 6,
           vh = va + 7;
  const unsigned long long c0 = memtime(), r0 = memrealtime();
  for (int i = 0; i < trips; i++) {
    if (MODE == 0) {
      asm volatile(S8 S8 S8 S8 : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h) : : "scc");
    } else if (MODE == 1) {
      asm volatile(V8 V8 V8 V8 : "+v"(va), "+v"(vb), "+v"(vc), "+v"(vd), "+v"(ve), "+v"(vf), "+v"(vg), "+v"(vh));
    } else if (MODE == 2) {
      asm volatile(M8 M8
                   : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h), "+v"(va), "+v"(vb),
                     "+v"(vc), "+v"(vd), "+v"(ve), "+v"(vf), "+v"(vg), "+v"(vh)
                   :
                   : "scc");
    } else {
      asm volatile(D8 D8 D8 D8 : "+s"(a) : : "scc");
    }
  }
  const unsigned long long c1 = memtime(), r1 = memrealtime();
  if (threadIdx.x == 0) out[blockIdx.x] = Stamp{c0, c1, r0, r1};
  // keep every chain live (vector store of the lane values)
  sink[blockIdx.x * 64 + threadIdx.x] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h ^ va ^ vb ^ vc ^ vd ^ ve ^ vf ^ vg ^ vh;
}

int run(const char* name, int mode, int waves_per_cu, int cus, bool last) {
  const int grid = waves_per_cu * cus;
  Stamp* d_out;
  uint32_t* d_sink;
  CHECK(hipMalloc(&d_out, sizeof(Stamp) * grid));
  CHECK(hipMalloc(&d_sink, 4ull * 64 * grid));
  auto launch = [&](int trips) {
    switch (mode) {
      case 0: hipLaunchKernelGGL(peak_loop<0>, dim3(grid), dim3(64), 0, 0, d_out, d_sink, trips); break;
      case 1: hipLaunchKernelGGL(peak_loop<1>, dim3(grid), dim3(64), 0, 0, d_out, d_sink, trips); break;
      case 2: hipLaunchKernelGGL(peak_loop<2>, dim3(grid), dim3(64), 0, 0, d_out, d_sink, trips); break;
      default: hipLaunchKernelGGL(peak_loop<3>, dim3(grid), dim3(64), 0, 0, d_out, d_sink, trips); break;
    }
  };
  launch(100);  // warm-up
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, 0));
  launch(kTrips);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipDeviceSynchronize());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<Stamp> st(grid);
  CHECK(hipMemcpy(st.data(), d_out, sizeof(Stamp) * grid, hipMemcpyDeviceToHost));
  double cyc = 0, rt = 0, cmin = 1e30, cmax = 0;
  unsigned long long rs_max = 0, re_min = ~0ull;
  for (const Stamp& s : st) {
    const double c = (double)(s.c1 - s.c0);
    cyc += c;
    rt += (double)(s.r1 - s.r0);
    cmin = std::min(cmin, c);
    cmax = std::max(cmax, c);
    rs_max = std::max(rs_max, s.r0);
    re_min = std::min(re_min, s.r1);
  }
  cyc /= grid;
  rt /= grid;
  // instructions of one trip: the asm body plus the loop's own counter
  // update and compare (2 scalar instructions; its branch is not counted)
  const double salu = (mode == 1 ? 2.0 : mode == 2 ? 18.0 : 34.0) * kTrips;
  const double valu = (mode == 1 ? 32.0 : mode == 2 ? 16.0 : 0.0) * kTrips;
  const double clock_ghz = cyc / (rt * 10.0);  // s_memrealtime ticks at 100 MHz
  if (g_clock_ghz == 0.0) g_clock_ghz = clock_ghz;
  // Kernel-time rates: every instruction of the launch over the CUs' cycles
  // of the whole kernel (launch and tail included, so a lower bound on the
  // ceiling). The per-wave means above assume every wave co-resident for the
  // whole kernel, which a grid of one-wave workgroups does not guarantee.
  const double cu_cycles = (double)cus * ms * 1e-3 * g_clock_ghz * 1e9;
  std::printf("%s{\"loop\": \"%s\", \"waves_per_cu\": %d, \"grid\": %d, \"kernel_ms\": %.3f, "
              "\"cycles_per_wave_mean\": %.0f, \"cycles_min\": %.0f, \"cycles_max\": %.0f, "
              "\"all_waves_overlap\": %s, \"clock_ghz\": %.3f, \"salu_per_wave_cycle\": %.4f, "
              "\"salu_per_cu_cycle\": %.4f, \"valu_per_cu_cycle\": %.4f, \"valu_per_simd_cycle\": %.4f, "
              "\"salu_per_cu_cycle_kernel\": %.4f, \"valu_per_simd_cycle_kernel\": %.4f}%s\n",
              "  ", name, waves_per_cu, grid, ms, cyc, cmin, cmax, rs_max < re_min ? "true" : "false", clock_ghz,
              salu / cyc, salu * waves_per_cu / cyc, valu * waves_per_cu / cyc,
              valu * waves_per_cu / cyc / 4.0, salu * grid / cu_cycles, valu * grid / cu_cycles / 4.0,
              last ? "" : ",");
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_sink));
  return 0;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::printf("{\"cus\": %d, \"trips\": %d, \"insts_per_trip\": 32, \"runs\": [\n", cus, kTrips);
  int rc = 0;
  for (int w : {1, 4, 8, 16, 24, 32}) rc |= run("salu_independent", 0, w, cus, false);
  rc |= run("salu_dependent", 3, 1, cus, false);
  rc |= run("salu_dependent", 3, 24, cus, false);
  rc |= run("valu_independent", 1, 1, cus, false);
  rc |= run("valu_independent", 1, 24, cus, false);
  rc |= run("mixed_salu_valu", 2, 4, cus, false);
  rc |= run("mixed_salu_valu", 2, 24, cus, true);
  std::printf("]}\n");
  return rc;
}
