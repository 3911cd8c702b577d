// fs_scene.cpp — host preparation of the device scene.
//
// 1. Restates the reference object constructors (object.cpp, volume.cpp,
//    mesh.cpp:168-275) so the device sees exactly the planes, tangents and
//    baked vertices the reference would hold.
// 2. Replaces the reference's per-mesh 8-ary octree (mesh.cpp:39-152,
//    bvh.h) with a binned-SAH BVH2 per mesh. Only the acceleration structure
//    changes: the leaf test is the reference's ray_intersect_triangle, and the
//    traversal keeps the reference's closest-hit rule (strict '<', the first
//    object in list order wins ties). Boxes are padded so culling is
//    conservative. See DESIGN.md §"Acceleration structure".
#include "fs_scene.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <memory>

namespace fs {
namespace {

// ---- matrix4 (math/matrix4.h, column-major) -------------------------------
struct M4 {
  float m[16];
};
M4 m4_identity() {  // matrix4.h:240-246
  M4 r;
  std::memset(&r, 0, sizeof(r));
  r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1;
  return r;
}
M4 m4_mul(const M4& a, const M4& b) {  // matrix4.h:529-546
  M4 o;
  for (int k = 0; k < 16; k++) {
    int r = k % 4, c = k / 4;
    o.m[k] = 0.0f;
    for (int i = 0; i < 4; i++) o.m[k] += a.m[r + (i * 4)] * b.m[(c * 4) + i];
  }
  return o;
}
M4 m4_rotation(float rad, f3 axis) {  // matrix4.h:270-301
  float c = std::cos(rad), s = std::sin(rad), t = 1.0f - c;
  f3 a = normalize(axis);
  float x = a.x, y = a.y, z = a.z;
  M4 o;
  o.m[0] = t * x * x + c;
  o.m[4] = t * x * y - s * z;
  o.m[8] = t * x * z + s * y;
  o.m[12] = 0.0f;
  o.m[1] = t * x * y + s * z;
  o.m[5] = t * y * y + c;
  o.m[9] = t * y * z - s * x;
  o.m[13] = 0.0f;
  o.m[2] = t * x * z - s * y;
  o.m[6] = t * y * z + s * x;
  o.m[10] = t * z * z + c;
  o.m[14] = 0.0f;
  o.m[3] = 0.0f;
  o.m[7] = 0.0f;
  o.m[11] = 0.0f;
  o.m[15] = 1.0f;
  return o;
}
f3 m4_apply(const M4& M, f3 v) {  // matrix4.h:552-557 with w = 1
  const float* m = M.m;
  const float w = 1.0f;
  return mk3(v.x * m[0] + v.y * m[4] + v.z * m[8] + w * m[12],
             v.x * m[1] + v.y * m[5] + v.z * m[9] + w * m[13],
             v.x * m[2] + v.y * m[6] + v.z * m[10] + w * m[14]);
}

// bounds (volume.cpp:162-191): first point initialises min and max.
struct Bounds {
  f3 mn{0, 0, 0}, mx{0, 0, 0};
  uint32_t count = 0;
  void add(f3 p) {
    if (count == 0) {
      mn = mx = p;
      count = 1;
      return;
    }
    count++;
    if (p.x > mx.x) mx.x = p.x;
    if (p.y > mx.y) mx.y = p.y;
    if (p.z > mx.z) mx.z = p.z;
    if (p.x < mn.x) mn.x = p.x;
    if (p.y < mn.y) mn.y = p.y;
    if (p.z < mn.z) mn.z = p.z;
  }
  f3 center() const { return (mn + mx) * 0.5f; }
};

// ---- BVH builder ------------------------------------------------------------
struct Box {
  float lo[3] = {INFINITY, INFINITY, INFINITY};
  float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const float* p) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  void grow(const Box& b) {
    for (int k = 0; k < 3; k++) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  bool empty() const { return lo[0] > hi[0]; }
  float area() const {
    if (empty()) return 0.0f;
    float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0f * (dx * dy + dy * dz + dz * dx);
  }
};

struct Prim {
  Box box;
  float c[3];
  uint32_t face;
};

// Fills the ray-independent part of the reference triangle test.
void fill_tri(DevTri* t, f3 p0, f3 p1, f3 p2, f4 pl) {
  f3 v0 = p1 - p0, v1 = p2 - p0;
  float ax = std::fabs(pl.x), ay = std::fabs(pl.y), az = std::fabs(pl.z);
  uint32_t axis;
  if (ax >= ay)
    axis = ax >= az ? 0u : 2u;
  else
    axis = ay >= az ? 1u : 2u;
  if (axis == 0) v0.x = v1.x = 0;
  if (axis == 1) v0.y = v1.y = 0;
  if (axis == 2) v0.z = v1.z = 0;
  t->d00 = dot(v0, v0);
  t->d01 = dot(v0, v1);
  t->d11 = dot(v1, v1);
  t->inv = 1 / (t->d00 * t->d11 - t->d01 * t->d01);
  t->plane[0] = pl.x;
  t->plane[1] = pl.y;
  t->plane[2] = pl.z;
  t->plane[3] = pl.w;
  const float P[3] = {p0.x, p0.y, p0.z}, A[3] = {v0.x, v0.y, v0.z}, B[3] = {v1.x, v1.y, v1.z};
  const int ia = axis == 0 ? 1 : 0, ib = axis == 2 ? 1 : 2;
  t->p1[0] = P[ia];
  t->p1[1] = P[ib];
  t->v0[0] = A[ia];
  t->v0[1] = A[ib];
  t->v1[0] = B[ia];
  t->v1[1] = B[ib];
  t->face_axis = (t->face_axis & 0x3FFFFFFFu) | (axis << 30);
}

constexpr int kMaxBins = 64;
// fs_options.node_layout = FS_NODE_LAYOUT_PAIRS: sibling inner nodes share
// one 128-B line (an even/odd slot pair), so the far child of a visited node
// arrives with the near one. Node order never changes a hit (closest hit is
// a total order).
// Rewrites the nodes [begin, end) of one mesh (root at begin, begin even) in
// the pair layout: root, then per node (depth first) its inner children as
// one aligned pair, padding with an unused slot where a pair would straddle.
void relayout_pairs(std::vector<BvhNode>* nodes, uint32_t begin) {
  std::vector<BvhNode> old(nodes->begin() + begin, nodes->end());
  std::vector<BvhNode> out;
  out.reserve(old.size() + old.size() / 8 + 2);
  BvhNode blank;
  std::memset(&blank, 0, sizeof(blank));
  out.push_back(old[0]);
  out.push_back(blank);
  // (new index relative to begin, old index relative to begin)
  std::vector<std::pair<uint32_t, uint32_t>> stack{{0u, 0u}};
  while (!stack.empty()) {
    auto [ni, oi] = stack.back();
    stack.pop_back();
    const BvhNode& o = old[oi];
    uint32_t kids[2], nk = 0;
    for (int c = 0; c < 2; c++)
      if (!(o.child[c] & kLeafBit)) kids[nk++] = (uint32_t)c;
    if (nk == 2 && (out.size() & 1u)) out.push_back(blank);
    uint32_t slot[2];
    for (uint32_t k = 0; k < nk; k++) {
      slot[k] = (uint32_t)out.size();
      out.push_back(old[o.child[kids[k]] - begin]);
    }
    BvhNode& n2 = out[ni];
    for (uint32_t k = 0; k < nk; k++) n2.child[kids[k]] = begin + slot[k];
    // Depth first, child 0's subtree first: push in reverse.
    for (uint32_t k = nk; k-- > 0;) stack.push_back({slot[k], o.child[kids[k]] - begin});
  }
  nodes->resize(begin);
  nodes->insert(nodes->end(), out.begin(), out.end());
}

// Subtrees are built concurrently down to this depth (2^depth threads);
// fs_options.bvh_threads = 1 builds sequentially (same tree, same layout).
uint32_t parallel_depth(uint32_t threads) {
  if (!threads) return 4;
  uint32_t d = 0;
  while (d < 8 && (1u << (d + 1)) <= threads) d++;
  return d;
}

class BvhBuilder {
 public:
  BvhBuilder(std::vector<BvhNode>* nodes, std::vector<DevTri>* tris, std::vector<float>* tri_normals,
             std::vector<float>* tri_tex, const std::vector<DevTri>* mesh_tris,
             const std::vector<float>* mesh_normals, const std::vector<float>* mesh_tex, const BuildOptions& opt)
      : nodes_(nodes),
        tris_(tris),
        tri_normals_(tri_normals),
        tri_tex_(tri_tex),
        mesh_tris_(mesh_tris),
        mesh_normals_(mesh_normals),
        mesh_tex_(mesh_tex),
        leaf_(opt.leaf),
        bins_(opt.bins),
        par_depth_(parallel_depth(opt.threads)) {}

  // Builds the tree over all faces; returns the root node index.
  uint32_t build(std::vector<Prim>& prims, uint32_t* max_depth) {
    prims_ = &prims;
    uint32_t root = alloc_node();
    Box all = range_box(0, (uint32_t)prims.size());
    if (prims.size() <= leaf_) {
      set_child(root, 0, all, make_leaf(0, (uint32_t)prims.size()));
      set_child(root, 1, Box(), kLeafBit);  // empty
    } else {
      split_into(root, 0, (uint32_t)prims.size(), 1);
    }
    *max_depth = std::max(*max_depth, max_depth_);
    return overflow_ ? 0xFFFFFFFFu : root;
  }

 private:
  uint32_t alloc_node() {
    BvhNode n;
    std::memset(&n, 0, sizeof(n));
    nodes_->push_back(n);
    return (uint32_t)nodes_->size() - 1;
  }
  Box range_box(uint32_t b, uint32_t e) const {
    Box r;
    for (uint32_t i = b; i < e; i++) r.grow((*prims_)[i].box);
    return r;
  }
  // Conservative padding: the reference triangle test may accept a hit point
  // a few ulps outside the exact triangle, so boxes are widened.
  static void pad(Box* b) {
    if (b->empty()) return;
    float s = 1.0f;
    for (int k = 0; k < 3; k++) s = std::max(s, std::max(std::fabs(b->lo[k]), std::fabs(b->hi[k])));
    float p = 4e-5f * s;
    for (int k = 0; k < 3; k++) {
      b->lo[k] -= p;
      b->hi[k] += p;
    }
  }
  void set_child(uint32_t node, int slot, Box b, uint32_t word) {
    pad(&b);
    BvhNode& n = (*nodes_)[node];
    if (b.empty()) {  // a far-away point box: never intersected by a segment of the scene
      n.lo_x[slot] = n.lo_y[slot] = n.lo_z[slot] = 3e30f;
      n.hi_x[slot] = n.hi_y[slot] = n.hi_z[slot] = 3e30f;
    } else {
      n.lo_x[slot] = b.lo[0];
      n.lo_y[slot] = b.lo[1];
      n.lo_z[slot] = b.lo[2];
      n.hi_x[slot] = b.hi[0];
      n.hi_y[slot] = b.hi[1];
      n.hi_z[slot] = b.hi[2];
    }
    n.child[slot] = word;
  }
  uint32_t make_leaf(uint32_t b, uint32_t e) {
    if (e - b > kMaxLeafCount) overflow_ = true;  // cannot be encoded: reported by build()
    uint32_t start = (uint32_t)tris_->size();
    for (uint32_t i = b; i < e; i++) {
      uint32_t f = (*prims_)[i].face;
      tris_->push_back((*mesh_tris_)[f]);
      if (!mesh_normals_->empty())
        tri_normals_->insert(tri_normals_->end(), mesh_normals_->begin() + 12 * (size_t)f,
                             mesh_normals_->begin() + 12 * (size_t)f + 12);
      if (!mesh_tex_->empty())
        tri_tex_->insert(tri_tex_->end(), mesh_tex_->begin() + 6 * (size_t)f, mesh_tex_->begin() + 6 * (size_t)f + 6);
    }
    return leaf_word(e - b, start);
  }
  // Partitions [b,e) into two halves; returns the split index.
  uint32_t partition(uint32_t b, uint32_t e, uint32_t depth) {
    std::vector<Prim>& P = *prims_;
    uint32_t n = e - b;
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = b; i < e; i++)
      for (int k = 0; k < 3; k++) {
        cmin[k] = std::min(cmin[k], P[i].c[k]);
        cmax[k] = std::max(cmax[k], P[i].c[k]);
      }
    int axis = 0;
    for (int k = 1; k < 3; k++)
      if (cmax[k] - cmin[k] > cmax[axis] - cmin[axis]) axis = k;
    // Depth guard: fall back to an object median near the stack bound.
    uint32_t need = 0;
    for (uint32_t m = n; m > leaf_; m = (m + 1) / 2) need++;
    bool median = depth + need + 1 >= kTraversalStack - 1 || cmax[axis] <= cmin[axis];
    if (!median) {
      float best_cost = INFINITY;
      int best_axis = -1, best_bin = -1;
      for (int ax = 0; ax < 3; ax++) {
        float ext = cmax[ax] - cmin[ax];
        if (!(ext > 0.0f)) continue;
        Box bb[kMaxBins];
        uint32_t bc[kMaxBins] = {0};
        float scale = bins_ / ext;
        for (uint32_t i = b; i < e; i++) {
          int k = std::min(bins_ - 1, (int)((P[i].c[ax] - cmin[ax]) * scale));
          bb[k].grow(P[i].box);
          bc[k]++;
        }
        Box left[kMaxBins];
        uint32_t lc[kMaxBins];
        Box acc;
        uint32_t cnt = 0;
        for (int k = 0; k < bins_; k++) {
          acc.grow(bb[k]);
          cnt += bc[k];
          left[k] = acc;
          lc[k] = cnt;
        }
        Box racc;
        uint32_t rcnt = 0;
        for (int k = bins_ - 1; k > 0; k--) {
          racc.grow(bb[k]);
          rcnt += bc[k];
          if (lc[k - 1] == 0 || rcnt == 0) continue;
          float cost = left[k - 1].area() * lc[k - 1] + racc.area() * rcnt;
          if (cost < best_cost) {
            best_cost = cost;
            best_axis = ax;
            best_bin = k;
          }
        }
      }
      if (best_axis >= 0) {
        float ext = cmax[best_axis] - cmin[best_axis];
        float scale = bins_ / ext;
        auto mid = std::partition(P.begin() + b, P.begin() + e, [&](const Prim& p) {
          int k = std::min(bins_ - 1, (int)((p.c[best_axis] - cmin[best_axis]) * scale));
          return k < best_bin;
        });
        uint32_t m = (uint32_t)(mid - P.begin());
        if (m > b && m < e) return m;
      }
    }
    uint32_t m = b + n / 2;
    std::nth_element(P.begin() + b, P.begin() + m, P.begin() + e,
                     [&](const Prim& x, const Prim& y) { return x.c[axis] < y.c[axis]; });
    return m;
  }
  // Builds the two children of `node` over [b,e).
  // A subtree built into its own arrays (node and triangle indices local),
  // merged into the parent builder afterwards.
  struct Local {
    std::vector<BvhNode> nodes;
    std::vector<DevTri> tris;
    std::vector<float> normals, tex;
    std::unique_ptr<BvhBuilder> b;
  };
  void init_local(Local* L) const {
    L->b.reset(new BvhBuilder(&L->nodes, &L->tris, &L->normals, &L->tex, mesh_tris_, mesh_normals_, mesh_tex_,
                              BuildOptions{}));
    L->b->prims_ = prims_;
    L->b->leaf_ = leaf_;
    L->b->bins_ = bins_;
    L->b->par_depth_ = par_depth_;
  }
  // Appends a local subtree after everything built so far: the result is the
  // same DFS layout the sequential build produces. Returns the subtree root.
  uint32_t merge(Local& L) {
    const uint32_t node_off = (uint32_t)nodes_->size(), tri_off = (uint32_t)tris_->size();
    for (BvhNode n : L.nodes) {
      for (int c = 0; c < 2; c++) {
        uint32_t w = n.child[c];
        if (!(w & kLeafBit))
          n.child[c] = w + node_off;
        else if (leaf_count(w))
          n.child[c] = (w & ~kLeafFirstMask) | ((w & kLeafFirstMask) + tri_off);
      }
      nodes_->push_back(n);
    }
    tris_->insert(tris_->end(), L.tris.begin(), L.tris.end());
    tri_normals_->insert(tri_normals_->end(), L.normals.begin(), L.normals.end());
    tri_tex_->insert(tri_tex_->end(), L.tex.begin(), L.tex.end());
    max_depth_ = std::max(max_depth_, L.b->max_depth_);
    overflow_ = overflow_ || L.b->overflow_;
    return node_off;
  }

  static constexpr uint32_t kParallelMin = 1u << 14;  // primitives below which a subtree stays on its thread

  void split_into(uint32_t node, uint32_t b, uint32_t e, uint32_t depth) {
    max_depth_ = std::max(max_depth_, depth);
    uint32_t m = partition(b, e, depth);
    uint32_t ranges[2][2] = {{b, m}, {m, e}};
    const bool leaf0 = m - b <= leaf_ || depth + 1 >= kTraversalStack - 1;
    const bool leaf1 = e - m <= leaf_ || depth + 1 >= kTraversalStack - 1;
    if (e - b >= kParallelMin && depth < par_depth_ && !leaf0 && !leaf1) {
      // Both children are subtrees: build them concurrently (disjoint prim
      // ranges), then append them in child order.
      Box boxes[2] = {range_box(b, m), range_box(m, e)};
      Local L0, L1;
      init_local(&L0);
      init_local(&L1);
      auto job = [depth](Local* L, uint32_t cb, uint32_t ce) {
        uint32_t r = L->b->alloc_node();
        L->b->split_into(r, cb, ce, depth + 1);
      };
      std::thread t(job, &L1, m, e);
      job(&L0, b, m);
      t.join();
      set_child(node, 0, boxes[0], merge(L0));
      set_child(node, 1, boxes[1], merge(L1));
      return;
    }
    for (int s = 0; s < 2; s++) {
      uint32_t cb = ranges[s][0], ce = ranges[s][1];
      Box cbox = range_box(cb, ce);
      if (ce - cb <= leaf_ || depth + 1 >= kTraversalStack - 1) {
        set_child(node, s, cbox, make_leaf(cb, ce));
      } else {
        uint32_t c = alloc_node();
        set_child(node, s, cbox, c);
        split_into(c, cb, ce, depth + 1);
      }
    }
  }

  std::vector<BvhNode>* nodes_;
  std::vector<DevTri>* tris_;
  std::vector<float>* tri_normals_;
  std::vector<float>* tri_tex_;
  const std::vector<DevTri>* mesh_tris_;
  const std::vector<float>* mesh_normals_;
  const std::vector<float>* mesh_tex_;
  std::vector<Prim>* prims_ = nullptr;
  uint32_t leaf_;
  int bins_;
  uint32_t par_depth_;
  uint32_t max_depth_ = 0;
  bool overflow_ = false;
};

void cube_planes(const f3* v, float* d) {  // volume.cpp:234-247
  f4 p[6] = {plane_3p(v[0], v[1], v[2]), plane_3p(v[6], v[5], v[4]), plane_3p(v[5], v[6], v[2]),
             plane_3p(v[7], v[4], v[0]), plane_3p(v[4], v[5], v[1]), plane_3p(v[6], v[7], v[3])};
  for (int i = 0; i < 6; i++) {
    d[4 * i + 0] = p[i].x;
    d[4 * i + 1] = p[i].y;
    d[4 * i + 2] = p[i].z;
    d[4 * i + 3] = p[i].w;
  }
}

void put3(float* d, f3 v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}
void put4(float* d, f4 v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
  d[3] = v.w;
}

// Builds one analytic object (object.cpp constructors).
// The corners of a CuboidObject (object.cpp:115-124, volume.cpp:262-283),
// rotated by cube::rotate about the box centre (volume.cpp:434-445).
void cuboid_corners(const fs_object& o, f3 v[8]) {
  const float* a = o.a;
  f3 org = mk3(a[0], a[1], a[2]);
  f3 half = mk3((float)(a[3] * 0.5), (float)(a[4] * 0.5), (float)(a[5] * 0.5));
  Bounds bb;
  bb.add(org - half);
  bb.add(org + half);
  f3 lo = bb.mn, hi = bb.mx;
  const f3 box[8] = {lo,
                     mk3(hi.x, lo.y, lo.z),
                     mk3(hi.x, lo.y, hi.z),
                     mk3(lo.x, lo.y, hi.z),
                     mk3(lo.x, hi.y, lo.z),
                     mk3(hi.x, hi.y, lo.z),
                     mk3(hi.x, hi.y, hi.z),
                     mk3(lo.x, hi.y, hi.z)};
  for (int i = 0; i < 8; i++) v[i] = box[i];
  if (o.rotate) {
    f3 axis = mk3(a[6], a[7], a[8]);
    float c = (float)std::cos(a[9]), s = (float)std::sin(a[9]);
    f3 center = bb.center();
    for (int i = 0; i < 8; i++) v[i] = rotate(v[i] - center, c, s, axis) + center;
  }
}

// Object::GetBounds() as each constructor accumulates it: object.cpp:17-21
// (sphere), 38-57 (plane: +-1000 along the in-plane axes), 75-95 (disc),
// 115-124 + volume.cpp:434-445 (cuboid corners), 167-189 / 191-211 (quads),
// mesh.cpp:218 (the transformed vertices). 2D objects get +-BASE_EPSILON
// along their (raw) normal.
Bounds object_bounds(const fs_object& o, const Bounds& mesh_rb) {
  const float* a = o.a;
  const f3 up = mk3(0, 1, 0);
  const float eps = kEpsilon;
  Bounds b;
  switch (o.kind) {
    case FS_OBJ_SPHERE: {
      f3 org = mk3(a[0], a[1], a[2]), rr = mk3(a[3], a[3], a[3]);
      b.add(org + rr);
      b.add(org - rr);
      break;
    }
    case FS_OBJ_PLANE: {
      f3 n = mk3(a[0], a[1], a[2]);
      float distance = -a[3];
      f3 pop = n * distance;
      f3 right = cross(n, up), forward = cross(n, right);
      b.add(pop + right * 1000.0f);
      b.add(pop - right * 1000.0f);
      b.add(pop + forward * 1000.0f);
      b.add(pop - forward * 1000.0f);
      b.add(pop + n * eps);
      b.add(pop - n * eps);
      break;
    }
    case FS_OBJ_DISC: {
      f3 org = mk3(a[0], a[1], a[2]), n = mk3(a[3], a[4], a[5]);
      f3 right = cross(n, up), forward = cross(n, right);
      b.add(org + right * a[6]);
      b.add(org - right * a[6]);
      b.add(org + forward * a[6]);
      b.add(org - forward * a[6]);
      b.add(org + n * eps);
      b.add(org - n * eps);
      break;
    }
    case FS_OBJ_CUBOID: {
      f3 v[8];
      cuboid_corners(o, v);
      for (int i = 0; i < 8; i++) b.add(v[i]);
      break;
    }
    case FS_OBJ_QUAD_ONWH: {
      f3 n = mk3(a[3], a[4], a[5]), nrm = normalize(n), org = mk3(a[0], a[1], a[2]);
      float hw = (float)(a[6] * 0.5), hh = (float)(a[7] * 0.5);
      f3 bt = cross(nrm, up), tg = cross(nrm, bt);
      b.add(org + bt * hw);
      b.add(org - bt * hw);
      b.add(org + tg * hh);
      b.add(org - tg * hh);
      b.add(org + n * eps);
      b.add(org - n * eps);
      break;
    }
    case FS_OBJ_QUAD_PUV: {
      f3 pos = mk3(a[0], a[1], a[2]), u = mk3(a[3], a[4], a[5]), v = mk3(a[6], a[7], a[8]);
      f3 nrm = normalize(cross(u, v));
      f3 org = pos + u * (float)0.5 + v * (float)0.5;
      float hw = (float)(length(u) * 0.5), hh = (float)(length(v) * 0.5);
      f3 bt = normalize(u), tg = normalize(v);
      b.add(org + nrm * eps);
      b.add(org - nrm * eps);
      b.add(org + bt * hw);
      b.add(org - bt * hw);
      b.add(org + tg * hh);
      b.add(org - tg * hh);
      break;
    }
    default:  // FS_OBJ_MESH
      b = mesh_rb;
      break;
  }
  return b;
}

// bounds::query_volume (volume.cpp:123-126) and bounds_intersect_bounds
// (intersect.cpp:26-43) with BASE_PARAM_CHECK on (base.h:102): a box of zero
// volume intersects nothing.
float bounds_volume(const Bounds& b) { return (b.mx.x - b.mn.x) * (b.mx.y - b.mn.y) * (b.mx.z - b.mn.z); }
bool bounds_overlap(const Bounds& a, const Bounds& b) {
  if (0 == bounds_volume(a) || 0 == bounds_volume(b)) return false;
  f3 ac = a.center(), bc = b.center();
  f3 ae = a.mx - ac, be = b.mx - bc, dd = bc - ac;
  return std::fabs(dd.x) <= (ae.x + be.x) && std::fabs(dd.y) <= (ae.y + be.y) && std::fabs(dd.z) <= (ae.z + be.z);
}

// SceneBvhNode::Subdivide's stop test (scene.cpp:37-46) for a node at `depth`
// holding n objects, under max_tree_depth; min() is the Windows headers'
// two-argument min (uint32 against double, a double result).
bool scene_node_stops(uint32_t depth, uint32_t max_depth, size_t n) {
  if (depth >= max_depth) return true;
  const double a = (double)(uint32_t)(max_depth - depth);
  const double b = (std::log((double)n) / std::log(8.0) + 0.5f) - 2.0f;
  return (double)depth >= (a < b ? a : b);
}

// Scene::Optimize (scene.cpp:216-225) + SceneBvh::BuildBvh (:105-126) +
// SceneBvhNode::Subdivide (:33-74) + ConfigureChildren (bvh.h:108-137).
int build_scene_tree(const fs_scene_desc* d, const std::vector<Bounds>& ob, PreparedScene* S, std::string* err) {
  const size_t n = d->num_objects;
  const int32_t ideal = n ? (int32_t)((std::log((double)n) / std::log(8.0) + 0.5) - 2) : 0;
  S->tree_valid = false;
  if (!(d->flags & FS_SCENE_OPTIMIZED) || ideal <= 0) return FS_OK;
  Bounds root;  // bounds += bounds (volume.cpp:193-224)
  for (const Bounds& b : ob) {
    if (root.count == 0) {
      root.mn = b.mn;
      root.mx = b.mx;
      root.count = 1;
      continue;
    }
    root.count++;
    root.mx = mk3(b.mx.x > root.mx.x ? b.mx.x : root.mx.x, b.mx.y > root.mx.y ? b.mx.y : root.mx.y,
                  b.mx.z > root.mx.z ? b.mx.z : root.mx.z);
    root.mn = mk3(b.mn.x < root.mn.x ? b.mn.x : root.mn.x, b.mn.y < root.mn.y ? b.mn.y : root.mn.y,
                  b.mn.z < root.mn.z ? b.mn.z : root.mn.z);
  }
  // The root node takes SceneBvhNode's default depth limit, 2 (scene.h:47,65).
  constexpr uint32_t kRootMaxDepth = 2;
  if (scene_node_stops(0, kRootMaxDepth, n) || n <= 2) {
    *err = "scene object octree: the root would stay a leaf (unexpected for >= 182 objects)";
    return FS_ERR_INVALID;
  }
  DevSceneTree& T = S->tree;
  std::memset(&T, 0, sizeof(T));
  put3(T.root_mn, root.mn);
  put3(T.root_mx, root.mx);
  const f3 mn = root.mn, center = root.center();
  put3(T.center, center);
  put4(T.split[0], plane_np(mk3(1, 0, 0), center));
  put4(T.split[1], plane_np(mk3(0, 1, 0), center));
  put4(T.split[2], plane_np(mk3(0, 0, 1), center));
  const f3 hx = mk3(center.x, mn.y, mn.z) - mn, hy = mk3(mn.x, center.y, mn.z) - mn, hz = mk3(mn.x, mn.y, center.z) - mn;
  const f3 span = hx + hy + hz;
  Bounds child[8];
  std::vector<std::vector<uint32_t>> lists(8);
  for (int i = 0; i < 8; i++) {
    f3 nmin = mn + hx * (float)(i % 2) + hy * (float)(i >> 2) + hz * (float)((i % 4) >> 1);
    child[i].add(nmin);
    child[i].add(nmin + span);
    put3(T.child_mn[i], child[i].mn);
    put3(T.child_mx[i], child[i].mx);
  }
  for (uint32_t j = 0; j < n; j++)
    for (int i = 0; i < 8; i++)
      if (bounds_overlap(ob[j], child[i])) lists[i].push_back(j);
  S->tree_objs.clear();
  for (int i = 0; i < 8; i++) {
    // A child does not copy max_tree_depth_ (scene.cpp:20-25: undefined). With
    // the parent's 2, or 0 or 1, Subdivide stops at depth 1 for any count.
    if (!scene_node_stops(1, kRootMaxDepth, lists[i].size()) && lists[i].size() > 2) {
      *err = "scene object octree: a leaf would subdivide (unexpected)";
      return FS_ERR_INVALID;
    }
    T.first[i] = (uint32_t)S->tree_objs.size();
    T.count[i] = (uint32_t)lists[i].size();
    S->tree_objs.insert(S->tree_objs.end(), lists[i].begin(), lists[i].end());
  }
  S->tree_valid = true;
  return FS_OK;
}

int build_object(const fs_object& o, DevObject* out, std::string* err) {
  std::memset(out, 0, sizeof(*out));
  out->kind = o.kind;
  out->mat = o.material;
  const float* a = o.a;
  switch (o.kind) {
    case FS_OBJ_SPHERE:  // object.cpp:17-21
      out->d[0] = a[0];
      out->d[1] = a[1];
      out->d[2] = a[2];
      out->d[3] = a[3];
      return FS_OK;
    case FS_OBJ_PLANE:  // object.cpp:38
      for (int i = 0; i < 4; i++) out->d[i] = a[i];
      return FS_OK;
    case FS_OBJ_DISC: {  // object.cpp:75-95 (normal used as given)
      f3 org = mk3(a[0], a[1], a[2]);
      put4(out->d, plane_np(mk3(a[3], a[4], a[5]), org));
      put3(out->d + 4, org);
      out->d[7] = a[6];
      return FS_OK;
    }
    case FS_OBJ_CUBOID: {  // object.cpp:115-124, volume.cpp:262-283, 434-445
      f3 v[8];
      cuboid_corners(o, v);
      cube_planes(v, out->d);
      {  // padded corner box, same padding rule as the BVH node boxes
        f3 mn = v[0], mx = v[0];
        for (int i = 1; i < 8; i++) {
          mn = mk3(std::min(mn.x, v[i].x), std::min(mn.y, v[i].y), std::min(mn.z, v[i].z));
          mx = mk3(std::max(mx.x, v[i].x), std::max(mx.y, v[i].y), std::max(mx.z, v[i].z));
        }
        float sc = 1.0f;
        for (float c : {mn.x, mn.y, mn.z, mx.x, mx.y, mx.z}) sc = std::max(sc, std::fabs(c));
        float pd = 1e-4f * sc;
        put3(out->d + 24, mn - mk3(pd, pd, pd));
        put3(out->d + 27, mx + mk3(pd, pd, pd));
      }
      return FS_OK;
    }
    case FS_OBJ_QUAD_ONWH: {  // object.cpp:167-189
      f3 nrm = normalize(mk3(a[3], a[4], a[5]));
      f3 org = mk3(a[0], a[1], a[2]);
      out->kind = FS_OBJ_QUAD_ONWH;
      put4(out->d, plane_np(nrm, org));
      put3(out->d + 4, org);
      out->d[7] = (float)(a[6] * 0.5);
      out->d[8] = (float)(a[7] * 0.5);
      f3 bt = cross(nrm, mk3(0, 1, 0));
      put3(out->d + 9, bt);
      put3(out->d + 12, cross(nrm, bt));
      return FS_OK;
    }
    case FS_OBJ_QUAD_PUV: {  // object.cpp:191-211
      f3 pos = mk3(a[0], a[1], a[2]), u = mk3(a[3], a[4], a[5]), v = mk3(a[6], a[7], a[8]);
      f3 nrm = normalize(cross(u, v));
      out->kind = FS_OBJ_QUAD_ONWH;
      put4(out->d, plane_np(nrm, pos));
      put3(out->d + 4, pos + u * (float)0.5 + v * (float)0.5);
      out->d[7] = (float)(length(u) * 0.5);
      out->d[8] = (float)(length(v) * 0.5);
      put3(out->d + 9, normalize(u));
      put3(out->d + 12, normalize(v));
      return FS_OK;
    }
    default:
      *err = "unknown object kind " + std::to_string(o.kind);
      return FS_ERR_INVALID;
  }
}

}  // namespace

// Per-face preparation of large meshes runs on up to kPrepThreads threads
// (each face's record depends only on that face).
constexpr uint32_t kPrepThreads = 16;
constexpr uint32_t kPrepParallelMin = 1u << 16;
template <class F>
void parallel_chunks(uint32_t n, F&& fn) {
  uint32_t t = std::min<uint32_t>(kPrepThreads, std::max(1u, std::thread::hardware_concurrency()));
  if (n < kPrepParallelMin) t = 1;
  const uint32_t per = (n + t - 1) / t;
  std::vector<std::thread> pool;
  for (uint32_t c = 1; c < t; c++) {
    const uint32_t b = std::min(n, c * per), e = std::min(n, b + per);
    if (b < e) pool.emplace_back(fn, c, b, e);
  }
  fn(0u, 0u, std::min(n, per));
  for (std::thread& th : pool) th.join();
}

BuildOptions BuildOptions::from(const fs_options* o) {
  fs_options def;
  fs_options_default(&def);
  if (!o) o = &def;
  BuildOptions b;
  b.leaf = (o->bvh_leaf && o->bvh_leaf <= kMaxLeafCount) ? o->bvh_leaf : def.bvh_leaf;
  b.bins = (o->bvh_bins >= 2 && o->bvh_bins <= (uint32_t)kMaxBins) ? (int)o->bvh_bins : (int)def.bvh_bins;
  b.threads = o->bvh_threads;
  b.pair_layout = o->node_layout == FS_NODE_LAYOUT_PAIRS;
  b.park_min_tris = o->park_min_tris;
  b.small_mesh_tris = o->small_mesh_tris <= kMaxSmallMeshTris ? o->small_mesh_tris : def.small_mesh_tris;
  b.log = o->build_log != 0;
  return b;
}

int prepare_scene(const fs_scene_desc* d, PreparedScene* out, std::string* err, const BuildOptions& opt,
                  uint32_t gpu_bvh_min_tris) {
  auto t0 = std::chrono::steady_clock::now();
  if (!d || !out) {
    *err = "null scene";
    return FS_ERR_INVALID;
  }
  if (!d->materials || d->num_materials == 0 || !d->normal_table) {
    *err = "scene needs materials and a normal table (InitializeMaterials)";
    return FS_ERR_INVALID;
  }
  if (d->sky_material < 0 || (uint32_t)d->sky_material >= d->num_materials) {
    *err = "sky_material out of range";
    return FS_ERR_INVALID;
  }
  if (d->num_objects && !d->objects) {
    *err = "objects pointer is null";
    return FS_ERR_INVALID;
  }
  PreparedScene& S = *out;
  S = PreparedScene();
  S.sky = d->sky_material;
  S.materials.assign(d->materials, d->materials + d->num_materials);
  for (const fs_material& m : S.materials) {
    if (m.kind < FS_MAT_DIFFUSE || m.kind > FS_MAT_FOG) {
      *err = "unknown material kind " + std::to_string(m.kind);
      return FS_ERR_INVALID;
    }
    if (m.texture >= 0 && (uint32_t)m.texture >= d->num_textures) {
      *err = "material texture index out of range";
      return FS_ERR_INVALID;
    }
  }
  // Textures (material.h:42-52): one packed texel array. A map with no texels
  // is no map (material.cpp:47, 111: buffer.size() && width && height).
  std::vector<int32_t> tex_slot(d->num_textures, -1);
  for (uint32_t i = 0; i < d->num_textures; i++) {
    const fs_texture& t = d->textures[i];
    size_t n = (size_t)t.width * t.height * 3;
    if (!n) continue;
    if (!t.rgb) {
      *err = "texture " + std::to_string(i) + " has no texels";
      return FS_ERR_INVALID;
    }
    if ((size_t)t.width * t.height * 3 > 0xFFFFFFFFull || S.tex_rgb.size() + n > 0xFFFFFFFFull) {
      *err = "textures exceed 2^32 floats";
      return FS_ERR_INVALID;
    }
    tex_slot[i] = (int32_t)(S.tex_info.size() / 4);
    S.tex_info.push_back((uint32_t)S.tex_rgb.size());
    S.tex_info.push_back(t.width);
    S.tex_info.push_back(t.height);
    S.tex_info.push_back(0);
    S.tex_rgb.insert(S.tex_rgb.end(), t.rgb, t.rgb + n);
  }
  for (fs_material& m : S.materials) m.texture = m.texture >= 0 ? tex_slot[m.texture] : -1;
  S.table.resize(4 * (size_t)FS_NORMAL_TABLE_SIZE);
  for (uint32_t i = 0; i < FS_NORMAL_TABLE_SIZE; i++) {
    S.table[4 * i + 0] = d->normal_table[3 * i + 0];
    S.table[4 * i + 1] = d->normal_table[3 * i + 1];
    S.table[4 * i + 2] = d->normal_table[3 * i + 2];
    S.table[4 * i + 3] = 0.0f;
  }

  // Meshes: MeshObject::MeshObject + BuildBvh face planes.
  struct MeshOut {
    uint32_t root = 0;
    uint32_t first_tri = 0, small = 0;  // a small mesh's triangle slots (host build)
    bool tree = false;
    bool normals = false;
    bool texcoords = false;
    Bounds rb;
  };
  std::vector<MeshOut> mesh_out(d->num_meshes);
  bool any_normals = false, any_tex = false;
  size_t all_tris = 0;
  for (uint32_t mi = 0; mi < d->num_meshes; mi++) {
    if (d->meshes[mi].normals && d->meshes[mi].num_normals) any_normals = true;
    if (d->meshes[mi].texcoords && d->meshes[mi].num_texcoords) any_tex = true;
    all_tris += d->meshes[mi].num_triangles;
  }
  // A BVH2 over n faces has at most n-1 inner nodes: size the arrays once
  // (regrowing a 1 M-face scene's arrays costs tens of ms of copies).
  if (all_tris <= kMaxTriangles) {
    S.nodes.reserve(all_tris + d->num_meshes);
    S.tris.reserve(all_tris);
    if (any_normals) S.tri_normals.reserve(12 * all_tris);
    if (any_tex) S.tri_tex.reserve(6 * all_tris);
  }
  for (uint32_t mi = 0; mi < d->num_meshes; mi++) {
    const fs_mesh& m = d->meshes[mi];
    if (m.num_triangles && (!m.corners || !m.positions)) {
      *err = "mesh " + std::to_string(mi) + " has triangles but no positions/corners";
      return FS_ERR_INVALID;
    }
    bool need = false;
    M4 T = m4_identity(), Sc = m4_identity(), R = m4_identity();
    if (m.translation[0] || m.translation[1] || m.translation[2]) {
      need = true;
      T.m[12] = m.translation[0];
      T.m[13] = m.translation[1];
      T.m[14] = m.translation[2];
    }
    if (m.scale[0] || m.scale[1] || m.scale[2]) {
      need = true;
      Sc.m[0] = m.scale[0];
      Sc.m[5] = m.scale[1];
      Sc.m[10] = m.scale[2];
    }
    if (m.rotation[0] || m.rotation[1] || m.rotation[2]) {
      need = true;
      R = m4_rotation(m.rotation[3], mk3(m.rotation[0], m.rotation[1], m.rotation[2]));
    }
    std::vector<f3> verts;
    if (need) {  // vertices_ is only filled when a transform is needed (mesh.cpp:211-221)
      M4 M = m4_mul(m4_mul(T, R), Sc);
      verts.resize(m.num_positions);
      for (uint32_t i = 0; i < m.num_positions; i++) {
        f3 v = m4_apply(M, mk3(m.positions[3 * i], m.positions[3 * i + 1], m.positions[3 * i + 2]));
        verts[i] = v;
        mesh_out[mi].rb.add(v);
      }
    }
    uint32_t nn = (m.normals ? m.num_normals : 0);
    std::vector<f3> normals(nn);
    for (uint32_t i = 0; i < nn; i++) {  // mesh.cpp:223-234
      f3 n = normalize(mk3(m.normals[3 * i], m.normals[3 * i + 1], m.normals[3 * i + 2]));
      if (m.invert_normals) n = n * (float)-1.0;
      normals[i] = n;
    }
    mesh_out[mi].normals = nn > 0;
    uint32_t nt = m.texcoords ? m.num_texcoords : 0;
    std::vector<DevTri> mtris(m.num_triangles);
    std::vector<float> corner_pos(need ? 9 * (size_t)m.num_triangles : 0);
    std::vector<float> mnormals, mtex;
    if (any_normals) mnormals.assign(12 * (size_t)m.num_triangles, 0.0f);
    if (any_tex) mtex.assign(6 * (size_t)m.num_triangles, 0.0f);
    // Faces are independent: large meshes fill their records on several
    // threads. The first bad face (lowest index) is reported, as the
    // sequential loop would.
    std::vector<uint64_t> bad(kPrepThreads, ~0ull);  // per chunk: (face << 2) | kind of the first bad face
    auto fill_faces = [&](uint32_t chunk, uint32_t f0, uint32_t f1) {
    for (uint32_t f = f0; f < f1; f++) {
      const int32_t* c = m.corners + 9 * (size_t)f;
      uint32_t vi[3], ni[3], ti[3];
      uint32_t kind = 0;
      for (int k = 0; k < 3; k++) {  // winding reversed (mesh.cpp:250-260)
        vi[k] = (uint32_t)c[3 * (2 - k) + 0];
        ni[k] = (uint32_t)c[3 * (2 - k) + 1];
        ti[k] = (uint32_t)c[3 * (2 - k) + 2];
        if (!kind && vi[k] >= m.num_positions) kind = 1;
        if (!kind && nn && ni[k] >= nn) kind = 2;  // normals_.at() would throw (mesh.cpp:292)
        if (!kind && nt && ti[k] >= nt) kind = 3;
      }
      if (kind) {
        bad[chunk] = ((uint64_t)f << 2) | kind;
        return;
      }
      DevTri& t = mtris[f];
      std::memset(&t, 0, sizeof(t));
      t.face_axis = f;
      if (need) {
        f3 p0 = verts[vi[0]], p1 = verts[vi[1]], p2 = verts[vi[2]];
        fill_tri(&t, p0, p1, p2, plane_np(calc_normal(p0, p1, p2), p0));  // mesh.cpp:136-146
        for (int k = 0; k < 3; k++) corner_pos[9 * (size_t)f + 3 * k + 0] = verts[vi[k]].x;
        for (int k = 0; k < 3; k++) corner_pos[9 * (size_t)f + 3 * k + 1] = verts[vi[k]].y;
        for (int k = 0; k < 3; k++) corner_pos[9 * (size_t)f + 3 * k + 2] = verts[vi[k]].z;
      }
      if (nn)
        for (int k = 0; k < 3; k++) put3(&mnormals[12 * (size_t)f + 4 * k], normals[ni[k]]);
      if (nt)  // mesh.cpp:236-239, texcoords_ in face (reversed) corner order
        for (int k = 0; k < 3; k++) {
          mtex[6 * (size_t)f + 2 * k] = m.texcoords[2 * (size_t)ti[k]];
          mtex[6 * (size_t)f + 2 * k + 1] = m.texcoords[2 * (size_t)ti[k] + 1];
        }
    }
    };
    parallel_chunks(m.num_triangles, fill_faces);
    const uint64_t first_bad = *std::min_element(bad.begin(), bad.end());
    if (first_bad != ~0ull) {
      static const char* what[4] = {"", "vertex", "normal", "texcoord"};
      *err = "mesh " + std::to_string(mi) + " face " + std::to_string(first_bad >> 2) + ": " + what[first_bad & 3u] +
             " index out of range";
      return FS_ERR_INVALID;
    }
    mesh_out[mi].texcoords = nt > 0;
    mesh_out[mi].tree = need && !verts.empty() && m.num_triangles > 0;  // mesh.cpp:119-121
    if (!mesh_out[mi].tree) continue;
    if (S.tris.size() + S.deferred_tris + m.num_triangles > kMaxTriangles) {
      *err = "scene has more than 2^27 triangles (the leaf encoding's 27-bit first-triangle slot)";
      return FS_ERR_INVALID;
    }
    for (DevTri& t : mtris) t.mesh_obj = mi;
    if (gpu_bvh_min_tris && m.num_triangles >= gpu_bvh_min_tris) {
      // Deferred to the device build: reserve the node block (a binary tree
      // over n faces has at most n-1 inner nodes) and the triangle slots.
      DeferredMesh D;
      D.mesh = mi;
      D.num_tris = m.num_triangles;
      S.deferred_nodes += m.num_triangles;  // bases are assigned after the host-built meshes
      S.deferred_tris += m.num_triangles;
      D.lo.resize(3 * (size_t)m.num_triangles);
      D.hi.resize(3 * (size_t)m.num_triangles);
      parallel_chunks(m.num_triangles, [&](uint32_t, uint32_t f0, uint32_t f1) {
        for (uint32_t f = f0; f < f1; f++) {
          Box b;
          for (int k = 0; k < 3; k++) b.grow(&corner_pos[9 * (size_t)f + 3 * k]);
          for (int k = 0; k < 3; k++) {
            D.lo[3 * (size_t)f + k] = b.lo[k];
            D.hi[3 * (size_t)f + k] = b.hi[k];
          }
        }
      });
      D.tris = std::move(mtris);
      if (any_normals) D.normals = std::move(mnormals);
      if (any_tex) D.tex = std::move(mtex);
      S.deferred.push_back(std::move(D));
      continue;
    }
    auto tp = std::chrono::steady_clock::now();
    std::vector<Prim> prims(m.num_triangles);
    for (uint32_t f = 0; f < m.num_triangles; f++) {
      Prim& p = prims[f];
      p.box.grow(&corner_pos[9 * (size_t)f]);
      p.box.grow(&corner_pos[9 * (size_t)f + 3]);
      p.box.grow(&corner_pos[9 * (size_t)f + 6]);
      for (int k = 0; k < 3; k++) p.c[k] = 0.5f * (p.box.lo[k] + p.box.hi[k]);
      p.face = f;
    }
    const bool pairs = opt.pair_layout;
    if (pairs && (S.nodes.size() & 1u)) {
      BvhNode blank;
      std::memset(&blank, 0, sizeof(blank));
      S.nodes.push_back(blank);
    }
    const uint32_t node_begin = (uint32_t)S.nodes.size();
    mesh_out[mi].first_tri = (uint32_t)S.tris.size();  // the builder appends the mesh's faces in leaf order
    if (m.num_triangles <= opt.small_mesh_tris) mesh_out[mi].small = m.num_triangles;
    BvhBuilder builder(&S.nodes, &S.tris, &S.tri_normals, &S.tri_tex, &mtris, &mnormals, &mtex, opt);
    auto tb = std::chrono::steady_clock::now();
    mesh_out[mi].root = builder.build(prims, &S.max_depth);
    if (pairs && mesh_out[mi].root == node_begin) relayout_pairs(&S.nodes, node_begin);
    if (mesh_out[mi].small) {  // faces whose plane has the previous slot's bits share its plane test
      const uint32_t f0 = mesh_out[mi].first_tri;
      for (uint32_t f = f0 + 1; f < f0 + m.num_triangles; f++)
        if (!std::memcmp(S.tris[f].plane, S.tris[f - 1].plane, sizeof(S.tris[f].plane)))
          S.tris[f].mesh_obj |= kSamePlaneBit;
    }
    if (opt.log)
      std::fprintf(stderr, "[fs build] mesh %u: %u tris, prepare %.1f ms, prims %.1f ms, bvh %.1f ms\n", mi,
                   m.num_triangles, std::chrono::duration<double, std::milli>(tp - t0).count(),
                   std::chrono::duration<double, std::milli>(tb - tp).count(),
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count());
    if (mesh_out[mi].root == 0xFFFFFFFFu) {
      *err = "mesh " + std::to_string(mi) + ": BVH leaf exceeds 15 triangles at the depth bound";
      return FS_ERR_INVALID;
    }
  }

  // Device-built meshes take the node and triangle slots after the host arrays.
  S.any_normals = any_normals;
  S.any_tex = any_tex;
  {
    uint32_t nb = (uint32_t)S.nodes.size(), tb = (uint32_t)S.tris.size();
    for (DeferredMesh& D : S.deferred) {
      D.node_base = nb;
      D.tri_base = tb;
      mesh_out[D.mesh].root = nb;
      mesh_out[D.mesh].first_tri = tb;
      nb += D.num_tris;
      tb += D.num_tris;
    }
  }

  // fs_options.park_min_tris (tests exercise the parked-walk schedule on
  // small meshes by lowering it).
  const uint32_t park_min = opt.park_min_tris;
  S.objects.resize(d->num_objects);
  std::vector<Bounds> obj_bounds(d->num_objects);
  for (uint32_t i = 0; i < d->num_objects; i++) {
    const fs_object& o = d->objects[i];
    if (o.material < 0 || (uint32_t)o.material >= d->num_materials) {
      *err = "object " + std::to_string(i) + " has no valid material";
      return FS_ERR_INVALID;
    }
    if (o.kind == FS_OBJ_MESH) {
      if (o.mesh < 0 || (uint32_t)o.mesh >= d->num_meshes) {
        *err = "object " + std::to_string(i) + " references a missing mesh";
        return FS_ERR_INVALID;
      }
      DevObject& D = S.objects[i];
      std::memset(&D, 0, sizeof(D));
      const MeshOut& mo = mesh_out[o.mesh];
      D.kind = FS_OBJ_MESH;
      D.mat = o.material;
      D.i0 = (int32_t)mo.root;
      D.i1 = mo.normals ? 1 : 0;
      D.i2 = mo.tree ? 1 : 0;
      D.i3 = (int32_t)mo.small;
      std::memcpy(&D.d[6], &mo.first_tri, 4);  // small meshes: their faces from here
      D.i4 = mo.texcoords ? 1 : 0;
      const uint32_t nt = d->meshes[o.mesh].num_triangles;
      D.i5 = nt >= park_min ? (nt >= kParkLargeTris ? 2 : 1) : 0;
      put3(D.d, mo.rb.mn);
      put3(D.d + 3, mo.rb.mx);
      obj_bounds[i] = mo.rb;
    } else {
      int rc = build_object(o, &S.objects[i], err);
      if (rc) return rc;
      obj_bounds[i] = object_bounds(o, Bounds());
    }
  }
  if (int rc = build_scene_tree(d, obj_bounds, &S, err)) return rc;
  S.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return FS_OK;
}

}  // namespace fs
