// fs_bvh_gpu.hip — binned-SAH BVH2 build of one mesh on the GPU (SURVEY §8f
// rank 1: the reference builds its mesh octree on the CPU at load time,
// mesh.cpp:117-152; the host builder in fs_scene.cpp is the default).
//
// Same tree rules as the host builder (fs_scene.cpp BvhBuilder): 16 SAH bins
// per axis over primitive centroids, cost area(L)·nL + area(R)·nR, leaves of
// at most `leaf` triangles, the depth guard that switches to object-median
// splits so every walk fits the kTraversalStack-entry LDS stack, padded
// child boxes. The node layout and the order of faces with equal keys
// differ; any such tree gives the same frames: the BVH only culls
// (DESIGN.md §3).
//
// Two phases:
//  A. Level-synchronous over tasks of more than kSmall primitives. Per level:
//     centroid bounds, bin histograms (global atomics on order-preserving
//     float bits), one thread per task for the SAH sweep, a partition of
//     the task's range, child boxes, and the parent node record.
//  B. One wave per remaining subtree (<= kSmall primitives), which builds
//     it depth-first out of LDS into a node block reserved in phase A.
// Triangle order: a leaf covers a contiguous range of the final permutation,
// so its word is simply (count, tri_base + first position).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fs_bvh_gpu.h"

namespace fs {
namespace gbvh {

constexpr uint32_t kSmall = 256;  // subtrees at most this large are built by one wave (phase B)
constexpr int kBins = 16;
constexpr uint32_t kGuard = kTraversalStack - 1;  // fs_scene.cpp split_into / partition depth rule

// Order-preserving float <-> uint (so unsigned atomicMin/atomicMax order floats).
__device__ __forceinline__ uint32_t f2o(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

struct Task {
  uint32_t b, e, node, depth;
};

// Per-task scratch of phase A (ordered-uint boxes).
struct TaskData {
  uint32_t cmin[3], cmax[3];                 // centroid bounds
  uint32_t cnt[3][kBins];                    // bin counts
  uint32_t blo[3][kBins][3], bhi[3][kBins][3];  // bin boxes
  uint32_t clo[2][3], chi[2][3];             // child boxes
  int32_t axis;                              // SAH split axis; -1: even split, -2: object median
  uint32_t bin, nl;                          // split bin, left count
  uint32_t maxis, pivot, nless;              // median: axis, pivot key, keys below it
  int32_t child_task[2];                     // next-level task of each side, -1: none
};

struct Box3 {
  float lo[3], hi[3];
};

__device__ __forceinline__ float area(const float* lo, const float* hi) {
  if (lo[0] > hi[0]) return 0.0f;
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return 2.0f * (dx * dy + dy * dz + dz * dx);
}

// fs_scene.cpp BvhBuilder::pad: widen by 4e-5 x max(1, |coord|).
__device__ __forceinline__ void pad(float* lo, float* hi) {
  float s = 1.0f;
  for (int k = 0; k < 3; k++) s = fmaxf(s, fmaxf(fabsf(lo[k]), fabsf(hi[k])));
  const float p = 4e-5f * s;
  for (int k = 0; k < 3; k++) {
    lo[k] -= p;
    hi[k] += p;
  }
}

__device__ __forceinline__ void set_child(BvhNode* nodes, uint32_t node, int slot, const float* lo0, const float* hi0,
                                          uint32_t word) {
  float lo[3] = {lo0[0], lo0[1], lo0[2]}, hi[3] = {hi0[0], hi0[1], hi0[2]};
  pad(lo, hi);
  BvhNode& n = nodes[node];
  n.lo_x[slot] = lo[0];
  n.lo_y[slot] = lo[1];
  n.lo_z[slot] = lo[2];
  n.hi_x[slot] = hi[0];
  n.hi_y[slot] = hi[1];
  n.hi_z[slot] = hi[2];
  n.child[slot] = word;
}

__device__ __forceinline__ uint32_t halvings(uint32_t n, uint32_t leaf) {  // fs_scene.cpp partition(): `need`
  uint32_t need = 0;
  for (uint32_t m = n; m > leaf; m = (m + 1) / 2) need++;
  return need;
}

struct Build {
  const float* lo;  // 3 per primitive
  const float* hi;
  uint32_t n, leaf, tri_base;
  BvhNode* nodes;     // the mesh's node block: local index 0 = root
  uint32_t node_base;  // global index of local node 0 (child words are global)
  uint32_t* perm;    // primitive per position (final order)
  uint32_t* perm2;
  int32_t* task_of;  // phase-A task of each position, -1 when done
  uint32_t* tag;     // (task << 1) | side after a partition
  TaskData* td;
  Task* tasks;
  Task* tasks_next;
  uint32_t* counters;  // [0] nodes reserved, [1] next-level tasks, [2] small subtrees, [3] max depth, [4] overflow,
                       // [5] nodes built
  Task* small;         // phase-B subtrees (node = reserved block base)
  uint32_t max_nodes;
  // Deterministic partition and numbering (the same tree, layout and
  // triangle order on every run): per position, the exclusive prefix of
  // (median ties << 32 | left positions), scanned per block of 256 and then
  // over the blocks; per task, the exclusive prefix of its children's
  // (next-level tasks, phase-B subtrees, nodes).
  uint64_t* pre;        // per position
  uint64_t* bsum;       // per block of 256 positions
  uint4* plan;          // per task: next tasks, small subtrees, nodes, -
};

__device__ __forceinline__ float cen(const Build& B, uint32_t p, int k) {
  return 0.5f * (B.lo[3 * p + k] + B.hi[3 * p + k]);
}

__global__ void k_init(Build B) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= B.n) return;
  B.perm[p] = p;
  B.task_of[p] = 0;
}

__global__ void k_reset(Build B, uint32_t ntasks) {
  const uint32_t t = blockIdx.x;
  if (t >= ntasks) return;
  uint32_t* w = reinterpret_cast<uint32_t*>(B.td + t);
  const uint32_t words = sizeof(TaskData) / 4;
  for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) w[i] = 0;
  __syncthreads();
  if (threadIdx.x < 3) {
    B.td[t].cmin[threadIdx.x] = 0xFFFFFFFFu;
    for (int k = 0; k < 2; k++) B.td[t].clo[k][threadIdx.x] = 0xFFFFFFFFu;
  }
  for (uint32_t i = threadIdx.x; i < 3 * kBins * 3; i += blockDim.x) (&B.td[t].blo[0][0][0])[i] = 0xFFFFFFFFu;
}

// Phase A accumulates per-task reductions with global atomics. Positions of
// one task are contiguous, so nearly every wave (and block) lies inside one
// task: the lanes of the wave's first task ("lead task") are reduced across
// the wave (and, for the bins, the block's LDS) first, and only the rare
// lanes of another task go to global memory one by one. Without this, the
// top levels send ~10^6 atomics to each of a few addresses.
__device__ __forceinline__ float wmin(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wmax(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}
__device__ __forceinline__ int32_t task_at(const Build& B, uint32_t p) { return p < B.n ? B.task_of[p] : -1; }

__global__ __launch_bounds__(256) void k_cbounds(Build B) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t t = task_at(B, p);
  const int32_t lead = __shfl(t, 0, 64);
  float c[3] = {INFINITY, INFINITY, INFINITY};
  if (t >= 0) {
    const uint32_t q = B.perm[p];
    for (int k = 0; k < 3; k++) c[k] = cen(B, q, k);
  }
  if (t >= 0 && t != lead)
    for (int k = 0; k < 3; k++) {
      atomicMin(&B.td[t].cmin[k], f2o(c[k]));
      atomicMax(&B.td[t].cmax[k], f2o(c[k]));
    }
  if (lead < 0) return;
  const bool mine = t == lead;
  for (int k = 0; k < 3; k++) {
    const float mn = wmin(mine ? c[k] : INFINITY), mx = wmax(mine ? c[k] : -INFINITY);
    if ((threadIdx.x & 63u) == 0) {
      atomicMin(&B.td[lead].cmin[k], f2o(mn));
      atomicMax(&B.td[lead].cmax[k], f2o(mx));
    }
  }
}

__device__ __forceinline__ int bin_of(float c, float cmin, float ext) {
  const float scale = kBins / ext;
  return min(kBins - 1, (int)((c - cmin) * scale));
}

// Bins of the block's lead task (that of its first position) accumulate in
// LDS and are flushed once per block.
__global__ __launch_bounds__(256) void k_bins(Build B) {
  __shared__ uint32_t scnt[3 * kBins], slo[3 * kBins * 3], shi[3 * kBins * 3];
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t lead = task_at(B, blockIdx.x * blockDim.x);
  for (uint32_t j = threadIdx.x; j < 3 * kBins * 3; j += blockDim.x) {
    if (j < 3 * kBins) scnt[j] = 0;
    slo[j] = 0xFFFFFFFFu;
    shi[j] = 0u;
  }
  __syncthreads();
  const int32_t t = task_at(B, p);
  if (t >= 0) {
    TaskData& d = B.td[t];
    const uint32_t q = B.perm[p];
    const bool local = t == lead;
    for (int ax = 0; ax < 3; ax++) {
      const float cmin = o2f(d.cmin[ax]), ext = o2f(d.cmax[ax]) - cmin;
      if (!(ext > 0.0f)) continue;
      const int k = bin_of(cen(B, q, ax), cmin, ext);
      if (local) {
        const int j = ax * kBins + k;
        atomicAdd(&scnt[j], 1u);
        for (int c = 0; c < 3; c++) {
          atomicMin(&slo[3 * j + c], f2o(B.lo[3 * q + c]));
          atomicMax(&shi[3 * j + c], f2o(B.hi[3 * q + c]));
        }
      } else {
        atomicAdd(&d.cnt[ax][k], 1u);
        for (int c = 0; c < 3; c++) {
          atomicMin(&d.blo[ax][k][c], f2o(B.lo[3 * q + c]));
          atomicMax(&d.bhi[ax][k][c], f2o(B.hi[3 * q + c]));
        }
      }
    }
  }
  __syncthreads();
  if (lead < 0) return;
  TaskData& d = B.td[lead];
  for (uint32_t j = threadIdx.x; j < 3 * kBins * 3; j += blockDim.x) {
    const uint32_t bin = j / 3;
    if (!scnt[bin]) continue;
    if (j % 3 == 0) atomicAdd(&(&d.cnt[0][0])[bin], scnt[bin]);
    atomicMin(&(&d.blo[0][0][0])[j], slo[j]);
    atomicMax(&(&d.bhi[0][0][0])[j], shi[j]);
  }
}

// One thread per task: the SAH sweep of fs_scene.cpp partition().
__global__ void k_split(Build B, uint32_t ntasks) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntasks) return;
  const Task T = B.tasks[t];
  TaskData& d = B.td[t];
  const uint32_t n = T.e - T.b;
  int axis = 0;
  float ext[3];
  for (int k = 0; k < 3; k++) ext[k] = o2f(d.cmax[k]) - o2f(d.cmin[k]);
  for (int k = 1; k < 3; k++)
    if (ext[k] > ext[axis]) axis = k;
  const bool median = T.depth + halvings(n, B.leaf) + 1 >= kGuard || !(ext[axis] > 0.0f);
  int best_axis = -1, best_bin = -1;
  uint32_t best_nl = 0;
  if (!median) {
    float best = INFINITY;
    for (int ax = 0; ax < 3; ax++) {
      if (!(ext[ax] > 0.0f)) continue;
      float llo[kBins][3], lhi[kBins][3];
      uint32_t lc[kBins];
      float alo[3] = {INFINITY, INFINITY, INFINITY}, ahi[3] = {-INFINITY, -INFINITY, -INFINITY};
      uint32_t acc = 0;
      for (int k = 0; k < kBins; k++) {
        if (d.cnt[ax][k])
          for (int c = 0; c < 3; c++) {
            alo[c] = fminf(alo[c], o2f(d.blo[ax][k][c]));
            ahi[c] = fmaxf(ahi[c], o2f(d.bhi[ax][k][c]));
          }
        acc += d.cnt[ax][k];
        for (int c = 0; c < 3; c++) {
          llo[k][c] = alo[c];
          lhi[k][c] = ahi[c];
        }
        lc[k] = acc;
      }
      float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
      uint32_t rc = 0;
      for (int k = kBins - 1; k > 0; k--) {
        if (d.cnt[ax][k])
          for (int c = 0; c < 3; c++) {
            rlo[c] = fminf(rlo[c], o2f(d.blo[ax][k][c]));
            rhi[c] = fmaxf(rhi[c], o2f(d.bhi[ax][k][c]));
          }
        rc += d.cnt[ax][k];
        if (lc[k - 1] == 0 || rc == 0) continue;
        const float cost = area(llo[k - 1], lhi[k - 1]) * lc[k - 1] + area(rlo, rhi) * rc;
        if (cost < best) {
          best = cost;
          best_axis = ax;
          best_bin = k;
          best_nl = lc[k - 1];
        }
      }
    }
  }
  if (best_axis < 0) {  // object median (k_select) or, all centroids equal, even split of the range
    d.axis = ext[axis] > 0.0f ? -2 : -1;
    d.maxis = (uint32_t)axis;
    d.bin = 0;
    d.nl = n / 2;
  } else {
    d.axis = best_axis;
    d.bin = (uint32_t)best_bin;
    d.nl = best_nl;
  }
}

// Object median of a task near the depth bound (fs_scene.cpp partition's
// nth_element): one block per task radix-selects, over the ordered-uint
// centroid keys on maxis, the key at sorted position n/2 (4 passes of 8 bits
// with an LDS histogram). k_partition sends keys below it left, keys above
// it right, and as many equal keys left as make the left side n/2.
__global__ __launch_bounds__(256) void k_select(Build B) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_prefix, s_rank;
  TaskData& d = B.td[blockIdx.x];
  if (d.axis != -2) return;
  const Task T = B.tasks[blockIdx.x];
  const int ax = (int)d.maxis;
  uint32_t prefix = 0, mask = 0, rank = (T.e - T.b) / 2;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t p = T.b + threadIdx.x; p < T.e; p += blockDim.x) {
      const uint32_t key = f2o(cen(B, B.perm[p], ax));
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t acc = 0, i = 0;
      while (i < 255 && acc + hist[i] <= rank) acc += hist[i++];
      s_prefix = prefix | (i << shift);
      s_rank = rank - acc;
    }
    __syncthreads();
    prefix = s_prefix;
    rank = s_rank;
    mask |= 255u << shift;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    d.pivot = prefix;
    d.nless = (T.e - T.b) / 2 - rank;  // keys below the pivot
  }
}

// The side of position p (task t, primitive q) in its task's split: 0 left,
// 1 right; *tie for a median-split key equal to the pivot (its side is
// decided by its rank among the task's ties, k_partition).
__device__ __forceinline__ uint32_t side_of(const Build& B, uint32_t p, int32_t t, uint32_t q, bool* tie) {
  const Task T = B.tasks[t];
  const TaskData& d = B.td[t];
  *tie = false;
  if (d.axis == -2) {  // the n/2 smallest centroids on maxis go left
    const uint32_t key = f2o(cen(B, q, (int)d.maxis));
    if (key == d.pivot) {
      *tie = true;
      return 0u;
    }
    return key < d.pivot ? 0u : 1u;
  }
  if (d.axis < 0) return (p - T.b) < d.nl ? 0u : 1u;
  const float cmin = o2f(d.cmin[d.axis]), ext = o2f(d.cmax[d.axis]) - cmin;
  return (uint32_t)bin_of(cen(B, q, d.axis), cmin, ext) < d.bin ? 0u : 1u;
}

// Per position: (tie << 32) | (non-tie left), scanned exclusively within
// each block of 256; the block totals go to bsum.
__global__ __launch_bounds__(256) void k_prefix_local(Build B) {
  __shared__ uint64_t wsum[4];
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t t = task_at(B, p);
  uint64_t v = 0;
  if (t >= 0) {
    bool tie;
    const uint32_t side = side_of(B, p, t, B.perm[p], &tie);
    v = tie ? (1ull << 32) : (side == 0 ? 1ull : 0ull);
  }
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint64_t x = v;  // inclusive wave scan (the two 32-bit halves never carry)
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if ((int)lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint64_t off = 0;
  for (uint32_t k = 0; k < w; k++) off += wsum[k];
  if (p < B.n) B.pre[p] = off + x - v;
  if (threadIdx.x == 255) B.bsum[blockIdx.x] = off + x;
}

// Exclusive scan of `count` 64-bit values in place, one block.
__global__ __launch_bounds__(1024) void k_scan_block(uint64_t* v, uint32_t count) {
  __shared__ uint64_t part[1024];
  const uint32_t per = (count + 1023) / 1024, b = threadIdx.x * per, e = min(count, b + per);
  uint64_t s = 0;
  for (uint32_t i = b; i < e; i++) s += v[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // Hillis-Steele over the 1024 partial sums
    const uint64_t y = threadIdx.x >= o ? part[threadIdx.x - o] : 0ull;
    __syncthreads();
    part[threadIdx.x] += y;
    __syncthreads();
  }
  uint64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0ull;
  for (uint32_t i = b; i < e; i++) {
    const uint64_t x = v[i];
    v[i] = run;
    run += x;
  }
}

__device__ __forceinline__ uint64_t prefix_at(const Build& B, uint32_t p) { return B.pre[p] + B.bsum[p >> 8]; }

// Stable scatter of each position to its side of its task's range: a
// position's slot is its rank among the task's positions of that side (the
// scanned prefixes), and the median's ties go left in position order until
// the left side holds n/2. The same input order gives the same output order
// on every run. Lanes of the wave's lead task reduce the child boxes across
// the wave.
__global__ __launch_bounds__(256) void k_partition(Build B) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  const int32_t t = task_at(B, p);
  const int32_t lead = __shfl(t, 0, 64);
  if (p < B.n && t < 0) B.perm2[p] = B.perm[p];
  uint32_t side = 0, q = 0;
  if (t >= 0) {
    const Task T = B.tasks[t];
    const TaskData& d = B.td[t];
    q = B.perm[p];
    bool tie;
    side = side_of(B, p, t, q, &tie);
    const uint64_t a = prefix_at(B, p), a0 = prefix_at(B, T.b);
    const uint32_t ties_before = (uint32_t)(a >> 32) - (uint32_t)(a0 >> 32);
    const uint32_t lefts_before = (uint32_t)a - (uint32_t)a0;
    const uint32_t quota = d.axis == -2 ? d.nl - d.nless : 0u;  // ties that go left
    if (tie) side = ties_before < quota ? 0u : 1u;
    const uint32_t left_rank = lefts_before + min(ties_before, quota);
    const uint32_t np = side ? T.b + d.nl + (p - T.b - left_rank) : T.b + left_rank;
    B.perm2[np] = q;
    B.tag[np] = ((uint32_t)t << 1) | side;
  }
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  if (t >= 0)
    for (int c = 0; c < 3; c++) {
      lo[c] = B.lo[3 * q + c];
      hi[c] = B.hi[3 * q + c];
    }
  if (t >= 0 && t != lead) {
    TaskData& d = B.td[t];
    for (int c = 0; c < 3; c++) {
      atomicMin(&d.clo[side][c], f2o(lo[c]));
      atomicMax(&d.chi[side][c], f2o(hi[c]));
    }
  }
  if (lead < 0) return;
  TaskData& d = B.td[lead];
  const uint32_t lane = threadIdx.x & 63u;
  const bool mine = t == lead;
  for (uint32_t s = 0; s < 2; s++) {
    const bool in = mine && side == s;
    if (!__ballot(in)) continue;
    for (int c = 0; c < 3; c++) {
      const float mn = wmin(in ? lo[c] : INFINITY), mx = wmax(in ? hi[c] : -INFINITY);
      if (lane == 0) {
        atomicMin(&d.clo[s][c], f2o(mn));
        atomicMax(&d.chi[s][c], f2o(mx));
      }
    }
  }
}

// The fate of side s of task T (fs_scene.cpp split_into): 0 leaf, 1 phase-B
// subtree, 2 next-level task.
__device__ __forceinline__ uint32_t fate_of(const Build& B, const Task& T, uint32_t cnt) {
  if (cnt <= B.leaf || T.depth + 1 >= kGuard) return 0u;
  return cnt <= kSmall ? 1u : 2u;
}

// One thread per task: what its two children need (next-level tasks,
// phase-B subtrees, nodes: one per inner child, cnt - 1 per subtree block).
__global__ void k_emit_plan(Build B, uint32_t ntasks) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntasks) return;
  const Task T = B.tasks[t];
  const TaskData& d = B.td[t];
  uint32_t next = 0, small = 0, nodes = 0;
  for (int s = 0; s < 2; s++) {
    const uint32_t cnt = s ? T.e - T.b - d.nl : d.nl;
    const uint32_t f = fate_of(B, T, cnt);
    if (f == 2u) {
      next++;
      nodes++;
    } else if (f == 1u) {
      small++;
      nodes += cnt - 1;
    }
  }
  B.plan[t] = make_uint4(next, small, nodes, 0u);
}

// One block: exclusive scan of the plans in task order, based at the running
// node and subtree totals (counters[0], [2]); the next level's task count
// goes to counters[1]. Numbering follows task order, so it is deterministic.
__global__ __launch_bounds__(1024) void k_emit_scan(Build B, uint32_t ntasks) {
  __shared__ uint32_t part[3][1024];
  const uint32_t per = (ntasks + 1023) / 1024, b = threadIdx.x * per, e = min(ntasks, b + per);
  uint32_t s[3] = {0, 0, 0};
  for (uint32_t i = b; i < e; i++) {
    const uint4 v = B.plan[i];
    s[0] += v.x;
    s[1] += v.y;
    s[2] += v.z;
  }
  for (int k = 0; k < 3; k++) part[k][threadIdx.x] = s[k];
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    uint32_t y[3] = {0, 0, 0};
    if (threadIdx.x >= o)
      for (int k = 0; k < 3; k++) y[k] = part[k][threadIdx.x - o];
    __syncthreads();
    for (int k = 0; k < 3; k++) part[k][threadIdx.x] += y[k];
    __syncthreads();
  }
  const uint32_t node0 = B.counters[0], small0 = B.counters[2];
  uint32_t run[3] = {0, small0, node0};
  if (threadIdx.x)
    for (int k = 0; k < 3; k++) run[k] += part[k][threadIdx.x - 1];
  for (uint32_t i = b; i < e; i++) {
    const uint4 v = B.plan[i];
    B.plan[i] = make_uint4(run[0], run[1], run[2], 0u);
    run[0] += v.x;
    run[1] += v.y;
    run[2] += v.z;
  }
  __syncthreads();
  if (threadIdx.x == 1023) {
    B.counters[1] = part[0][1023];
    B.counters[2] = small0 + part[1][1023];
    B.counters[0] = node0 + part[2][1023];
  }
}

// One thread per task: the parent node record and the children's records at
// the scanned offsets (side 0 first), as fs_scene.cpp split_into.
__global__ void k_emit(Build B, uint32_t ntasks, uint32_t small_max) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntasks) return;
  const Task T = B.tasks[t];
  TaskData& d = B.td[t];
  const uint4 off = B.plan[t];
  uint32_t next = off.x, small = off.y, node = off.z;
  atomicMax(&B.counters[3], T.depth);
  atomicAdd(&B.counters[5], 1u);
  for (int s = 0; s < 2; s++) {
    const uint32_t cb = T.b + (s ? d.nl : 0u), ce = s ? T.e : T.b + d.nl, cnt = ce - cb;
    float lo[3], hi[3];
    for (int c = 0; c < 3; c++) {
      lo[c] = o2f(d.clo[s][c]);
      hi[c] = o2f(d.chi[s][c]);
    }
    uint32_t word;
    d.child_task[s] = -1;
    const uint32_t f = fate_of(B, T, cnt);
    if (f == 0u) {
      if (cnt > kMaxLeafCount) atomicOr(&B.counters[4], 1u);
      word = leaf_word(cnt, B.tri_base + cb);
    } else if (f == 1u) {
      const uint32_t base = node, i = small++;  // a binary tree over cnt: <= cnt-1 inner nodes
      node += cnt - 1;
      if (base + cnt - 1 > B.max_nodes || i >= small_max) {
        atomicOr(&B.counters[4], 2u);
        word = kLeafBit;
      } else {
        B.small[i] = Task{cb, ce, base, T.depth + 1};
        word = B.node_base + base;
      }
    } else {
      const uint32_t nd = node++, i = next++;
      if (nd >= B.max_nodes) {
        atomicOr(&B.counters[4], 2u);
        word = kLeafBit;
      } else {
        B.tasks_next[i] = Task{cb, ce, nd, T.depth + 1};
        d.child_task[s] = (int32_t)i;
        word = B.node_base + nd;
      }
    }
    set_child(B.nodes, T.node, s, lo, hi, word);
  }
}

__global__ void k_retag(Build B) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= B.n) return;
  const int32_t t = B.task_of[p];
  if (t < 0) return;
  const uint32_t g = B.tag[p];
  B.task_of[p] = B.td[g >> 1].child_task[g & 1u];
}

// Phase B: one wave builds one subtree (<= kSmall primitives) depth-first
// into its reserved node block. The subtree's boxes sit in LDS; per node the
// wave reduces the centroid bounds, bins into LDS with LDS atomics, scores
// the 3 x 15 SAH candidates one per lane (the host sweep's order breaks
// cost ties: lower axis, then higher bin), and partitions its slice of the
// local order with ballot prefix counts.

__global__ __launch_bounds__(64) void k_small(Build B, uint32_t nsmall) {
  __shared__ float plo[3 * kSmall], phi[3 * kSmall];
  __shared__ uint32_t pq[kSmall];
  __shared__ uint16_t idx[kSmall], tmp[kSmall];
  __shared__ uint32_t bcnt[3 * kBins], blo[3 * kBins * 3], bhi[3 * kBins * 3];
  __shared__ uint4 stk[kTraversalStack + 2];
  const uint32_t lane = threadIdx.x;
  if (blockIdx.x >= nsmall) return;
  const Task root = B.small[blockIdx.x];
  const uint32_t n0 = root.e - root.b;
  for (uint32_t s = lane; s < n0; s += 64) {
    const uint32_t q = B.perm[root.b + s];
    pq[s] = q;
    idx[s] = (uint16_t)s;
    for (int c = 0; c < 3; c++) {
      plo[3 * s + c] = B.lo[3 * q + c];
      phi[3 * s + c] = B.hi[3 * q + c];
    }
  }
  if (lane == 0) stk[0] = make_uint4(0u, n0, root.node, root.depth);
  __syncthreads();
  uint32_t next = root.node + 1, built = 0, maxd = 0, flags = 0;
  int sp = 1;
  while (sp > 0) {
    sp--;
    const uint4 T = stk[sp];
    __syncthreads();
    const uint32_t b = T.x, e = T.y, node = T.z, depth = T.w, n = e - b;
    built++;
    maxd = max(maxd, depth);
    float cmn[3], cmx[3];
    for (int k = 0; k < 3; k++) {
      cmn[k] = INFINITY;
      cmx[k] = -INFINITY;
    }
    for (uint32_t p = b + lane; p < e; p += 64) {
      const uint32_t s = idx[p];
      for (int k = 0; k < 3; k++) {
        const float c = 0.5f * (plo[3 * s + k] + phi[3 * s + k]);
        cmn[k] = fminf(cmn[k], c);
        cmx[k] = fmaxf(cmx[k], c);
      }
    }
    for (int k = 0; k < 3; k++) {
      cmn[k] = wmin(cmn[k]);
      cmx[k] = wmax(cmx[k]);
    }
    int axis = 0;
    for (int k = 1; k < 3; k++)
      if (cmx[k] - cmn[k] > cmx[axis] - cmn[axis]) axis = k;
    const bool median = depth + halvings(n, B.leaf) + 1 >= kGuard || !(cmx[axis] > cmn[axis]);
    int best_axis = -1, best_bin = -1;
    if (!median) {
      for (uint32_t j = lane; j < 3 * kBins; j += 64) bcnt[j] = 0;
      for (uint32_t j = lane; j < 3 * kBins * 3; j += 64) {
        blo[j] = f2o(INFINITY);
        bhi[j] = f2o(-INFINITY);
      }
      __syncthreads();
      for (uint32_t p = b + lane; p < e; p += 64) {
        const uint32_t s = idx[p];
        for (int ax = 0; ax < 3; ax++) {
          const float ext = cmx[ax] - cmn[ax];
          if (!(ext > 0.0f)) continue;
          const int k = bin_of(0.5f * (plo[3 * s + ax] + phi[3 * s + ax]), cmn[ax], ext);
          const int j = ax * kBins + k;
          atomicAdd(&bcnt[j], 1u);
          for (int c = 0; c < 3; c++) {
            atomicMin(&blo[3 * j + c], f2o(plo[3 * s + c]));
            atomicMax(&bhi[3 * j + c], f2o(phi[3 * s + c]));
          }
        }
      }
      __syncthreads();
      // lane = ax * 16 + k scores the split "bins < k | bins >= k" on axis ax
      float cost = INFINITY;
      const int ax = (int)(lane >> 4), k = (int)(lane & 15u);
      if (ax < 3 && k >= 1 && cmx[ax] - cmn[ax] > 0.0f) {
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t lc = 0, rc = 0;
        for (int j = 0; j < kBins; j++) {
          const int g = ax * kBins + j;
          const bool left = j < k;
          for (int c = 0; c < 3; c++) {
            const float lo = o2f(blo[3 * g + c]), hi = o2f(bhi[3 * g + c]);
            if (left) {
              llo[c] = fminf(llo[c], lo);
              lhi[c] = fmaxf(lhi[c], hi);
            } else {
              rlo[c] = fminf(rlo[c], lo);
              rhi[c] = fmaxf(rhi[c], hi);
            }
          }
          (left ? lc : rc) += bcnt[g];
        }
        if (lc && rc) cost = area(llo, lhi) * lc + area(rlo, rhi) * rc;
        if (!(cost < INFINITY)) cost = INFINITY;
      }
      // argmin over lanes; ties to the host sweep's first candidate
      // (axis ascending, bin descending): order key ax*16 + (15-k)
      uint32_t key = (uint32_t)(ax * kBins + (kBins - 1 - k));
      for (int o = 32; o > 0; o >>= 1) {
        const float oc = __shfl_xor(cost, o, 64);
        const uint32_t ok = (uint32_t)__shfl_xor((int)key, o, 64);
        if (oc < cost || (oc == cost && ok < key)) {
          cost = oc;
          key = ok;
        }
      }
      if (cost < INFINITY) {
        best_axis = (int)(key / kBins);
        best_bin = kBins - 1 - (int)(key % kBins);
      }
    }
    uint32_t m = b + n / 2;  // SAH partition, object median, or (all centroids equal) even split
    if (median && cmx[axis] > cmn[axis]) {
      // object median (fs_scene.cpp partition's nth_element): each element's
      // rank by (centroid key on axis, position) places it; the lower half
      // goes left
      for (uint32_t p = b + lane; p < e; p += 64) {
        const uint32_t s = idx[p];
        const uint32_t key = f2o(0.5f * (plo[3 * s + axis] + phi[3 * s + axis]));
        uint32_t rank = 0;
        for (uint32_t j = b; j < e; j++) {
          const uint32_t sj = idx[j];
          const uint32_t kj = f2o(0.5f * (plo[3 * sj + axis] + phi[3 * sj + axis]));
          rank += (kj < key || (kj == key && j < p)) ? 1u : 0u;
        }
        tmp[b + rank] = (uint16_t)s;
      }
      __syncthreads();
      for (uint32_t p = b + lane; p < e; p += 64) idx[p] = tmp[p];
      __syncthreads();
    } else if (best_axis >= 0) {
      const float cm = cmn[best_axis], ext = cmx[best_axis] - cm;
      uint32_t nl = 0;
      for (int side = 0; side < 2; side++) {
        uint32_t fill = side ? nl : 0u;
        for (uint32_t base = b; base < e; base += 64) {
          const uint32_t p = base + lane;
          const uint32_t s = p < e ? idx[p] : 0u;
          bool want = false;
          if (p < e) {
            const bool left = bin_of(0.5f * (plo[3 * s + best_axis] + phi[3 * s + best_axis]), cm, ext) < best_bin;
            want = side ? !left : left;
          }
          const uint64_t mask = __ballot(want);
          if (want) tmp[b + fill + lanes_below(mask)] = (uint16_t)s;
          fill += (uint32_t)__popcll(mask);
        }
        if (!side) nl = fill;
      }
      __syncthreads();
      for (uint32_t p = b + lane; p < e; p += 64) idx[p] = tmp[p];
      __syncthreads();
      if (nl > 0 && nl < n) m = b + nl;
    }
    const uint32_t rb[2] = {b, m}, re[2] = {m, e};
    for (int s = 0; s < 2; s++) {
      float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (uint32_t p = rb[s] + lane; p < re[s]; p += 64) {
        const uint32_t q = idx[p];
        for (int c = 0; c < 3; c++) {
          lo[c] = fminf(lo[c], plo[3 * q + c]);
          hi[c] = fmaxf(hi[c], phi[3 * q + c]);
        }
      }
      for (int c = 0; c < 3; c++) {
        lo[c] = wmin(lo[c]);
        hi[c] = wmax(hi[c]);
      }
      const uint32_t cnt = re[s] - rb[s];
      uint32_t word;
      if (cnt <= B.leaf || depth + 1 >= kGuard) {
        if (cnt > kMaxLeafCount) flags |= 1u;
        word = leaf_word(cnt, B.tri_base + root.b + rb[s]);
      } else {
        const uint32_t c = next++;
        if (sp >= (int)kTraversalStack + 2 || c >= root.node + (n0 - 1)) {
          flags |= 2u;  // cannot happen for a binary tree; reported, not written
          word = kLeafBit;
        } else {
          if (lane == 0) stk[sp] = make_uint4(rb[s], re[s], c, depth + 1);
          sp++;
          word = B.node_base + c;
        }
      }
      if (lane == 0) set_child(B.nodes, node, s, lo, hi, word);
    }
    __syncthreads();
  }
  for (uint32_t s = lane; s < n0; s += 64) B.perm[root.b + s] = pq[idx[s]];
  if (lane == 0) {
    atomicMax(&B.counters[3], maxd);
    atomicAdd(&B.counters[5], built);
    if (flags) atomicOr(&B.counters[4], flags);
  }
}

template <class T>
__global__ void k_gather(const T* __restrict__ src, T* __restrict__ dst, const uint32_t* __restrict__ perm, uint32_t n,
                         uint32_t per) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)n * per) return;
  const uint32_t p = (uint32_t)(i / per), k = (uint32_t)(i % per);
  dst[i] = src[(uint64_t)perm[p] * per + k];
}

}  // namespace gbvh

#define GB_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      *err = std::string(#call) + ": " + hipGetErrorString(e_);                        \
      return FS_ERR_DEVICE;                                                            \
    }                                                                                  \
  } while (0)

int gpu_build_mesh_bvh(hipStream_t stream, const GpuBvhJob& job, BvhNode* d_nodes, DevTri* d_tris,
                       float* d_tri_normals, float* d_tri_tex, GpuBvhResult* res, std::string* err) {
  using namespace gbvh;
  const uint32_t n = job.num_tris;
  *res = GpuBvhResult{};
  if (n <= job.leaf || n < 2 * kSmall) {
    *err = "mesh too small for the GPU build";
    return FS_ERR_INVALID;
  }
  const uint32_t max_nodes = n;  // <= n-1 inner nodes plus the reserved blocks' slack
  std::vector<void*> allocs;
  auto alloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
    allocs.push_back(p);
    return p;
  };
  struct Free {
    std::vector<void*>* a;
    ~Free() {
      for (void* p : *a) (void)hipFree(p);
    }
  } free_all{&allocs};
  Build B{};
  B.n = n;
  B.leaf = job.leaf;
  B.tri_base = job.tri_base;
  B.max_nodes = max_nodes;
  B.nodes = d_nodes + job.node_base;
  B.node_base = job.node_base;
  float* lo = (float*)alloc(12ull * n);
  float* hi = (float*)alloc(12ull * n);
  B.perm = (uint32_t*)alloc(4ull * n);
  B.perm2 = (uint32_t*)alloc(4ull * n);
  B.task_of = (int32_t*)alloc(4ull * n);
  B.tag = (uint32_t*)alloc(4ull * n);
  const uint32_t max_tasks = n / kSmall + 2;  // phase-A tasks per level have > kSmall primitives
  B.td = (TaskData*)alloc(sizeof(TaskData) * (size_t)max_tasks);
  B.tasks = (Task*)alloc(sizeof(Task) * (size_t)max_tasks);
  B.tasks_next = (Task*)alloc(sizeof(Task) * (size_t)max_tasks);
  const uint32_t small_max = 2 * (n / 3 + 2);
  B.small = (Task*)alloc(sizeof(Task) * (size_t)small_max);
  const uint32_t pblocks = (n + 255) / 256;
  B.pre = (uint64_t*)alloc(8ull * n);
  B.bsum = (uint64_t*)alloc(8ull * pblocks);
  B.plan = (uint4*)alloc(sizeof(uint4) * (size_t)max_tasks);
  B.counters = (uint32_t*)alloc(64);
  for (void* p : allocs)
    if (!p) {
      *err = "GPU BVH build: out of device memory";
      return FS_ERR_NOMEM;
    }
  B.lo = lo;
  B.hi = hi;
  const bool log = job.log;
  auto t0 = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) -> int {  // FS_BUILD_LOG: per-phase wall time
    if (!log) return FS_OK;
    if (hipStreamSynchronize(stream) != hipSuccess) return FS_ERR_DEVICE;
    std::fprintf(stderr, "[fs gpu bvh] %-10s %8.2f ms\n", what,
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    return FS_OK;
  };
  GB_HIP(hipMemcpyAsync(lo, job.lo, 12ull * n, hipMemcpyHostToDevice, stream));
  GB_HIP(hipMemcpyAsync(hi, job.hi, 12ull * n, hipMemcpyHostToDevice, stream));
  GB_HIP(hipMemsetAsync(B.nodes, 0, sizeof(BvhNode) * (size_t)max_nodes, stream));
  GB_HIP(hipMemsetAsync(B.counters, 0, 64, stream));
  const uint32_t one = 1;  // node 0 is the root
  GB_HIP(hipMemcpyAsync(B.counters, &one, 4, hipMemcpyHostToDevice, stream));
  Task root{0, n, 0, 1};
  GB_HIP(hipMemcpyAsync(B.tasks, &root, sizeof(Task), hipMemcpyHostToDevice, stream));
  if (stamp("inputs")) return FS_ERR_DEVICE;
  const uint32_t pg = (n + 255) / 256;
  hipLaunchKernelGGL(k_init, dim3(pg), dim3(256), 0, stream, B);
  uint32_t ntasks = 1, levels = 0;
  while (ntasks) {
    hipLaunchKernelGGL(k_reset, dim3(ntasks), dim3(256), 0, stream, B, ntasks);
    hipLaunchKernelGGL(k_cbounds, dim3(pg), dim3(256), 0, stream, B);
    hipLaunchKernelGGL(k_bins, dim3(pg), dim3(256), 0, stream, B);
    hipLaunchKernelGGL(k_split, dim3((ntasks + 63) / 64), dim3(64), 0, stream, B, ntasks);
    hipLaunchKernelGGL(k_select, dim3(ntasks), dim3(256), 0, stream, B);
    hipLaunchKernelGGL(k_prefix_local, dim3(pg), dim3(256), 0, stream, B);
    hipLaunchKernelGGL(k_scan_block, dim3(1), dim3(1024), 0, stream, B.bsum, pg);
    hipLaunchKernelGGL(k_partition, dim3(pg), dim3(256), 0, stream, B);
    hipLaunchKernelGGL(k_emit_plan, dim3((ntasks + 63) / 64), dim3(64), 0, stream, B, ntasks);
    hipLaunchKernelGGL(k_emit_scan, dim3(1), dim3(1024), 0, stream, B, ntasks);
    hipLaunchKernelGGL(k_emit, dim3((ntasks + 63) / 64), dim3(64), 0, stream, B, ntasks, small_max);
    hipLaunchKernelGGL(k_retag, dim3(pg), dim3(256), 0, stream, B);
    GB_HIP(hipGetLastError());
    std::swap(B.perm, B.perm2);
    std::swap(B.tasks, B.tasks_next);
    GB_HIP(hipMemcpyAsync(&ntasks, B.counters + 1, 4, hipMemcpyDeviceToHost, stream));
    GB_HIP(hipStreamSynchronize(stream));
    if (++levels > kTraversalStack + 2) {
      *err = "GPU BVH build: phase A did not terminate";
      return FS_ERR_DEVICE;
    }
  }
  uint32_t cnt[6];
  GB_HIP(hipMemcpyAsync(cnt, B.counters, sizeof(cnt), hipMemcpyDeviceToHost, stream));
  GB_HIP(hipStreamSynchronize(stream));
  if (stamp("phase A")) return FS_ERR_DEVICE;
  const uint32_t nsmall = cnt[2];
  if (nsmall)
    hipLaunchKernelGGL(k_small, dim3(nsmall), dim3(64), 0, stream, B, nsmall);
  if (stamp("phase B")) return FS_ERR_DEVICE;
  // triangles, vertex normals and texcoords in leaf order
  uint32_t* d_order = B.perm;
  DevTri* src_t = (DevTri*)alloc(sizeof(DevTri) * (size_t)n);
  if (!src_t) {
    *err = "GPU BVH build: out of device memory";
    return FS_ERR_NOMEM;
  }
  GB_HIP(hipMemcpyAsync(src_t, job.tris, sizeof(DevTri) * (size_t)n, hipMemcpyHostToDevice, stream));
  hipLaunchKernelGGL(k_gather<DevTri>, dim3(pg), dim3(256), 0, stream, src_t, d_tris + job.tri_base, d_order, n, 1u);
  if (job.normals && d_tri_normals) {
    float* src = (float*)alloc(48ull * n);
    if (!src) {
      *err = "GPU BVH build: out of device memory";
      return FS_ERR_NOMEM;
    }
    GB_HIP(hipMemcpyAsync(src, job.normals, 48ull * n, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_gather<float>, dim3((12 * n + 255) / 256), dim3(256), 0, stream, src,
                       d_tri_normals + 12ull * job.tri_base, d_order, n, 12u);
  }
  if (job.tex && d_tri_tex) {
    float* src = (float*)alloc(24ull * n);
    if (!src) {
      *err = "GPU BVH build: out of device memory";
      return FS_ERR_NOMEM;
    }
    GB_HIP(hipMemcpyAsync(src, job.tex, 24ull * n, hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_gather<float>, dim3((6 * n + 255) / 256), dim3(256), 0, stream, src,
                       d_tri_tex + 6ull * job.tri_base, d_order, n, 6u);
  }
  GB_HIP(hipGetLastError());
  GB_HIP(hipMemcpyAsync(cnt, B.counters, sizeof(cnt), hipMemcpyDeviceToHost, stream));
  GB_HIP(hipStreamSynchronize(stream));
  if (stamp("gather")) return FS_ERR_DEVICE;
  if (cnt[4]) {
    *err = (cnt[4] & 1u) ? "GPU BVH build: a leaf at the depth bound exceeds 127 triangles"
                         : "GPU BVH build: node storage exhausted";
    return FS_ERR_INVALID;
  }
  res->nodes_used = cnt[5];
  res->max_depth = cnt[3];
  res->levels = levels;
  res->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return FS_OK;
}

}  // namespace fs
