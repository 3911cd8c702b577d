// fs_host.cpp — the reference render API (namespace base) on top of the
// MI355X path-trace layer. See fs_host.h for the mapping.
#include "fs_host.h"
#include "fs_image.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <mutex>
#include <sstream>

namespace base {

// ============================================================================
// RNG — math/random.cpp:6-49
// ============================================================================
static thread_local uint64 g_random_seed = 521288629;

void set_seed(uint64 seed) { g_random_seed = seed; }
uint64 random_integer() {
  uint64 x = g_random_seed;
  x ^= x << 12;
  x ^= x >> 25;
  x ^= x << 27;
  g_random_seed = x;
  return x * 0x2545F4914F6CDD1Dull;
}
float32 random_float() { return ((float32)(random_integer() % 0x7FFFFFFFull)) / (float32)0x7FFFFFFF; }
int64_t random_integer_range(int32 imin, int32 imax) {
  if (imax < imin) return 0;
  if (imin == imax) return imin;
  uint32 span = (uint32)(imax - imin) + 1;
  return ((int32)imin + (int64_t)(random_integer() % span));
}
float32 random_float_range(float32 imin, float32 imax) {
  if (imax < imin) return 0.0f;
  return imin + random_float() * (imax - imin);
}

// ============================================================================
// Materials — material.cpp
// ============================================================================
Material::Material() { material_id_ = (uint32)random_integer(); }  // material.cpp:26

static bool file_exists(const std::string& f) {
  FILE* fp = std::fopen(f.c_str(), "rb");
  if (!fp) return false;
  std::fclose(fp);
  return true;
}
static bool ends_with(const std::string& s, const std::string& e) {
  return s.size() >= e.size() && s.compare(s.size() - e.size(), e.size(), e) == 0;
}

DiffuseMaterial::DiffuseMaterial(const vector3& diffuse) : texture_scale_(0) { diffuse_ = diffuse; }
DiffuseMaterial::DiffuseMaterial(const std::string& filename, float32 tex_scale) : texture_scale_(0) {
  diffuse_map_.filename = filename;
  LoadDiffuseTexture(filename, tex_scale);
}
void DiffuseMaterial::LoadDiffuseTexture(const std::string& filename, float32 tex_scale) {  // material.cpp:63-95
  diffuse_map_.filename = filename;
  texture_scale_ = tex_scale;
  if (ends_with(filename, ".bmp")) {
    LoadBitmap(filename, &diffuse_map_.buffer, &diffuse_map_.width, &diffuse_map_.height);
  } else if (ends_with(filename, ".exr")) {
    float* rgba = nullptr;
    const char* errors = nullptr;
    int width, height;
    if (LoadEXR(&rgba, &width, &height, filename.c_str(), &errors) < 0) {
      std::printf("Failed to load %s. Errors: %s.\n", filename.c_str(), errors ? errors : "");
      return;
    }
    std::printf("Loaded %s with dims: <%i, %i>.\n", filename.c_str(), width, height);
    diffuse_map_.width = (uint32)width;
    diffuse_map_.height = (uint32)height;
    diffuse_map_.buffer.resize((size_t)width * height * 3);
    for (size_t i = 0; i < (size_t)width * height; i++) {
      diffuse_map_.buffer[i * 3 + 0] = rgba[i * 4 + 0];
      diffuse_map_.buffer[i * 3 + 1] = rgba[i * 4 + 1];
      diffuse_map_.buffer[i * 3 + 2] = rgba[i * 4 + 2];
    }
    std::free(rgba);
  }
}
fs_material DiffuseMaterial::Base(int kind) const {
  fs_material m;
  std::memset(&m, 0, sizeof(m));
  m.kind = kind;
  m.id = material_id_;
  m.diffuse[0] = diffuse_.x;
  m.diffuse[1] = diffuse_.y;
  m.diffuse[2] = diffuse_.z;
  m.texture = -1;  // assigned by Scene::Describe
  m.texture_scale = texture_scale_;
  return m;
}
fs_material DiffuseMaterial::Describe() const { return Base(FS_MAT_DIFFUSE); }

LightMaterial::LightMaterial(const vector3& emissive) {  // material.cpp:28-31
  emissive_ = emissive;
  diffuse_ = vector3(1, 1, 1);
}
fs_material LightMaterial::Describe() const {
  fs_material m = Base(FS_MAT_LIGHT);
  m.emissive[0] = emissive_.x;
  m.emissive[1] = emissive_.y;
  m.emissive[2] = emissive_.z;
  return m;
}
MetalMaterial::MetalMaterial(const vector3& diffuse, float32 roughness) : roughness_(roughness) { diffuse_ = diffuse; }
fs_material MetalMaterial::Describe() const {
  fs_material m = Base(FS_MAT_METAL);
  m.roughness = roughness_;
  return m;
}
MirrorMaterial::MirrorMaterial(const vector3& diffuse) { diffuse_ = diffuse; }
fs_material MirrorMaterial::Describe() const { return Base(FS_MAT_MIRROR); }
GlassMaterial::GlassMaterial(const vector3 diffuse, float32 index, float32 reflectivity, float32 frost)
    : index_(index), frost_(frost), reflectivity_(reflectivity) {
  diffuse_ = diffuse;
}
fs_material GlassMaterial::Describe() const {
  fs_material m = Base(FS_MAT_GLASS);
  m.index = index_;
  m.frost = frost_;
  m.reflectivity = reflectivity_;
  return m;
}
LiquidMaterial::LiquidMaterial(const vector3 diffuse, float32 index, float32 reflectivity)
    : index_(index), reflectivity_(reflectivity) {
  diffuse_ = diffuse;
}
fs_material LiquidMaterial::Describe() const {
  fs_material m = Base(FS_MAT_LIQUID);
  m.index = index_;
  m.reflectivity = reflectivity_;
  return m;
}
CeramicMaterial::CeramicMaterial(const vector3& diffuse, float32 shininess) : shininess_(shininess) {
  diffuse_ = diffuse;
}
fs_material CeramicMaterial::Describe() const {
  fs_material m = Base(FS_MAT_CERAMIC);
  m.shininess = shininess_;
  return m;
}
GlowMaterial::GlowMaterial(const vector3& diffuse, const vector3& glow, float32 shininess) : glow_(glow) {
  diffuse_ = diffuse;
  shininess_ = shininess;
}
fs_material GlowMaterial::Describe() const {
  fs_material m = Base(FS_MAT_GLOW);
  m.shininess = shininess_;
  m.glow[0] = glow_.x;
  m.glow[1] = glow_.y;
  m.glow[2] = glow_.z;
  return m;
}
FogMaterial::FogMaterial(const vector3 diffuse, float32 density) : density_(density * 1000.0f) {  // material.cpp:303-307
  diffuse_ = diffuse;
}
fs_material FogMaterial::Describe() const {
  fs_material m = Base(FS_MAT_FOG);
  m.density = density_;
  return m;
}

// normal_sphere::initialize (normal.cpp:9-27). The three draws of
// vector3(rfr(), rfr(), rfr()) are evaluated right to left by g++, so z is
// drawn first.
static std::vector<float32> g_normal_table;
static uint64 g_table_version = 0;
static inline float32 fast_len(float32 x, float32 y, float32 z) {
  float32 d = x * x + y * y + z * z;
  float32 half = 0.5f * d;
  int32_t i;
  std::memcpy(&i, &d, 4);
  i = 0x5f3759df - (i >> 1);
  float32 f;
  std::memcpy(&f, &i, 4);
  f = f * (1.5f - half * f * f);
  return 1.0f / f;
}
void InitializeMaterials() {
  const uint32 count = FS_NORMAL_TABLE_SIZE;
  g_normal_table.assign(3 * (size_t)count, 0.0f);
  for (uint32 i = 0; i < count; i++) {
    float32 x = 10, y = 10, z = 10;
    while (fast_len(x, y, z) > 1.0) {
      z = random_float_range(-1.0f, 1.0f);
      y = random_float_range(-1.0f, 1.0f);
      x = random_float_range(-1.0f, 1.0f);
    }
    float32 l = fast_len(x, y, z);
    if (l == 0.0) l = 1.0f;
    g_normal_table[3 * i + 0] = x / l;
    g_normal_table[3 * i + 1] = y / l;
    g_normal_table[3 * i + 2] = z / l;
  }
  g_table_version++;
}
const std::vector<float32>& NormalTable() { return g_normal_table; }

// ============================================================================
// Camera — camera.cpp:6-24
// ============================================================================
Camera::Camera()
    : z_near(1.0f),
      z_far(10000.0f),
      origin(0, 0, -200),
      target(0, 0, 0),
      fov_y(45),
      aperture_size(1.5),
      focal_depth(80),
      fast_render_enabled(false) {}
Camera::Camera(const vector3& new_origin, const vector3& new_target)
    : z_near(1.0f),
      z_far(10000.0f),
      origin(new_origin),
      target(new_target),
      fov_y(45),
      aperture_size(1.5),
      focal_depth(80),
      fast_render_enabled(false) {}
fs_camera Camera::Describe() const {
  fs_camera c;
  c.origin[0] = origin.x;
  c.origin[1] = origin.y;
  c.origin[2] = origin.z;
  c.target[0] = target.x;
  c.target[1] = target.y;
  c.target[2] = target.z;
  c.fov_y = fov_y;
  c.aperture_size = aperture_size;
  c.focal_depth = focal_depth;
  c.z_near = z_near;
  c.z_far = z_far;
  c.fast_render = fast_render_enabled ? 1 : 0;
  return c;
}

// ============================================================================
// Objects
// ============================================================================
static fs_object obj_base(int kind) {
  fs_object o;
  std::memset(&o, 0, sizeof(o));
  o.kind = kind;
  o.material = -1;
  o.mesh = -1;
  return o;
}
fs_object SphericalObject::Describe() const {
  fs_object o = obj_base(FS_OBJ_SPHERE);
  o.a[0] = origin_.x;
  o.a[1] = origin_.y;
  o.a[2] = origin_.z;
  o.a[3] = radius_;
  return o;
}
fs_object PlanarObject::Describe() const {
  fs_object o = obj_base(FS_OBJ_PLANE);
  o.a[0] = plane_.x;
  o.a[1] = plane_.y;
  o.a[2] = plane_.z;
  o.a[3] = plane_.w;
  return o;
}
fs_object DiscObject::Describe() const {
  fs_object o = obj_base(FS_OBJ_DISC);
  o.a[0] = origin_.x;
  o.a[1] = origin_.y;
  o.a[2] = origin_.z;
  o.a[3] = normal_.x;
  o.a[4] = normal_.y;
  o.a[5] = normal_.z;
  o.a[6] = radius_;
  return o;
}
void CuboidObject::Rotate(const vector3& axis, float32 angle) {
  rotated_ = true;
  axis_ = axis;
  angle_ = angle;
}
fs_object CuboidObject::Describe() const {
  fs_object o = obj_base(FS_OBJ_CUBOID);
  o.a[0] = origin_.x;
  o.a[1] = origin_.y;
  o.a[2] = origin_.z;
  o.a[3] = width_;
  o.a[4] = height_;
  o.a[5] = depth_;
  o.rotate = rotated_ ? 1 : 0;
  o.a[6] = axis_.x;
  o.a[7] = axis_.y;
  o.a[8] = axis_.z;
  o.a[9] = angle_;
  return o;
}
QuadObject::QuadObject(const vector3& origin, const vector3& normal, float32 width, float32 height)
    : puv_(false), a_(origin), b_(normal), w_(width), h_(height) {}
QuadObject::QuadObject(const vector3& position, const vector3& u, const vector3& v)
    : puv_(true), a_(position), b_(u), c_(v) {}
fs_object QuadObject::Describe() const {
  fs_object o = obj_base(puv_ ? FS_OBJ_QUAD_PUV : FS_OBJ_QUAD_ONWH);
  o.a[0] = a_.x;
  o.a[1] = a_.y;
  o.a[2] = a_.z;
  o.a[3] = b_.x;
  o.a[4] = b_.y;
  o.a[5] = b_.z;
  if (puv_) {
    o.a[6] = c_.x;
    o.a[7] = c_.y;
    o.a[8] = c_.z;
  } else {
    o.a[6] = w_;
    o.a[7] = h_;
  }
  return o;
}

// ---- Wavefront OBJ ----------------------------------------------------------
// Restates the parts of the vendored tinyobj loader (tiny_obj_loader.h) that
// decide the triangles MeshObject sees: its number parser, index fixing and
// the ear-clipping triangulation of polygons.
//
// try_parse_double, pnpoly and triangulate_face below are derived from
// tinyobjloader v1.2.2 (the copy vendored by the reference), which carries
// this notice:
//
//   The MIT License (MIT)
//   Copyright (c) 2012-2018 Syoyo Fujita and many contributors.
//   Permission is hereby granted, free of charge, to any person obtaining a
//   copy of this software and associated documentation files (the
//   "Software"), to deal in the Software without restriction, including
//   without limitation the rights to use, copy, modify, merge, publish,
//   distribute, sublicense, and/or sell copies of the Software, and to permit
//   persons to whom the Software is furnished to do so, subject to the
//   following conditions:
//   The above copyright notice and this permission notice shall be included
//   in all copies or substantial portions of the Software.
//   THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY KIND, EXPRESS
//   OR IMPLIED, INCLUDING BUT NOT LIMITED TO THE WARRANTIES OF
//   MERCHANTABILITY, FITNESS FOR A PARTICULAR PURPOSE AND NONINFRINGEMENT. IN
//   NO EVENT SHALL THE AUTHORS OR COPYRIGHT HOLDERS BE LIABLE FOR ANY CLAIM,
//   DAMAGES OR OTHER LIABILITY, WHETHER IN AN ACTION OF CONTRACT, TORT OR
//   OTHERWISE, ARISING FROM, OUT OF OR IN CONNECTION WITH THE SOFTWARE OR THE
//   USE OR OTHER DEALINGS IN THE SOFTWARE.
namespace {

// tryParseDouble (tiny_obj_loader.h:537-650): digits accumulated in double,
// fraction digits as digit * 10^-k, exponent applied as ldexp(m * 5^e, e).
bool try_parse_double(const char* s, const char* s_end, double* result) {
  if (s >= s_end) return false;
  double mantissa = 0.0;
  int exponent = 0;
  char sign = '+', exp_sign = '+';
  const char* curr = s;
  int read = 0;
  bool end_not_reached = false;
  auto is_digit = [](char c) { return c >= '0' && c <= '9'; };
  if (*curr == '+' || *curr == '-') {
    sign = *curr;
    curr++;
  } else if (!is_digit(*curr)) {
    return false;
  }
  end_not_reached = curr != s_end;
  while (end_not_reached && is_digit(*curr)) {
    mantissa *= 10;
    mantissa += (int)(*curr - 0x30);
    curr++;
    read++;
    end_not_reached = curr != s_end;
  }
  if (read == 0) return false;
  if (end_not_reached) {
    bool parse_exp = false;
    if (*curr == '.') {
      curr++;
      read = 1;
      end_not_reached = curr != s_end;
      static const double pow_lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
      while (end_not_reached && is_digit(*curr)) {
        mantissa += (int)(*curr - 0x30) * (read < 8 ? pow_lut[read] : std::pow(10.0, -read));
        read++;
        curr++;
        end_not_reached = curr != s_end;
      }
      parse_exp = end_not_reached;
    } else if (*curr == 'e' || *curr == 'E') {
      parse_exp = true;
    }
    if (parse_exp && (*curr == 'e' || *curr == 'E')) {
      curr++;
      end_not_reached = curr != s_end;
      if (end_not_reached && (*curr == '+' || *curr == '-')) {
        exp_sign = *curr;
        curr++;
      } else if (!is_digit(*curr)) {
        return false;
      }
      read = 0;
      end_not_reached = curr != s_end;
      while (end_not_reached && is_digit(*curr)) {
        exponent *= 10;
        exponent += (int)(*curr - 0x30);
        curr++;
        read++;
        end_not_reached = curr != s_end;
      }
      exponent *= (exp_sign == '+' ? 1 : -1);
      if (read == 0) return false;
    }
  }
  *result = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
  return true;
}

// parseReal (tiny_obj_loader.h:652-660): the token ends at space, tab or CR.
float32 parse_real(const char** token, double default_value = 0.0) {
  (*token) += std::strspn(*token, " \t");
  const char* end = (*token) + std::strcspn(*token, " \t\r\n");
  double val = default_value;
  try_parse_double(*token, end, &val);
  *token = end;
  return (float32)val;
}

// fixIndex (tiny_obj_loader.h:471-492): 1-based, negative = relative.
bool fix_index(int idx, int n, int* ret) {
  if (idx > 0) {
    *ret = idx - 1;
    return true;
  }
  if (idx == 0) return false;
  *ret = n + idx;
  return true;
}

struct Corner {
  int v = -1, t = -1, n = -1;
};

// parseTriple (v, v/vt, v//vn, v/vt/vn).
bool parse_corner(const char** token, int nv, int nn, int nt, Corner* c) {
  const char* p = *token;
  if (!fix_index(std::atoi(p), nv, &c->v)) return false;
  p += std::strcspn(p, "/ \t\r\n");
  if (*p == '/') {
    p++;
    if (*p == '/') {  // v//vn
      p++;
      if (!fix_index(std::atoi(p), nn, &c->n)) return false;
      p += std::strcspn(p, "/ \t\r\n");
    } else {  // v/vt or v/vt/vn
      if (!fix_index(std::atoi(p), nt, &c->t)) return false;
      p += std::strcspn(p, "/ \t\r\n");
      if (*p == '/') {
        p++;
        if (!fix_index(std::atoi(p), nn, &c->n)) return false;
        p += std::strcspn(p, "/ \t\r\n");
      }
    }
  }
  *token = p;
  return true;
}

// pnpoly (tiny_obj_loader.h:1019-1029)
int pnpoly(int nvert, const float32* vertx, const float32* verty, float32 testx, float32 testy) {
  int c = 0;
  for (int i = 0, j = nvert - 1; i < nvert; j = i++) {
    if (((verty[i] > testy) != (verty[j] > testy)) &&
        (testx < (vertx[j] - vertx[i]) * (testy - verty[i]) / (verty[j] - verty[i]) + vertx[i]))
      c = !c;
  }
  return c;
}

// exportGroupsToShape with triangulate = true (tiny_obj_loader.h:1042-1236):
// ear clipping in the dominant plane of the first non-degenerate corner.
void triangulate_face(const std::vector<float32>& v, const std::vector<Corner>& face, std::vector<Corner>* out) {
  size_t npolys = face.size();
  if (npolys < 3) return;
  size_t axes[2] = {1, 2};
  const float32 epsilon = std::numeric_limits<float32>::epsilon();
  for (size_t k = 0; k < npolys; ++k) {
    size_t vi0 = (size_t)face[(k + 0) % npolys].v, vi1 = (size_t)face[(k + 1) % npolys].v,
           vi2 = (size_t)face[(k + 2) % npolys].v;
    if (3 * vi0 + 2 >= v.size() || 3 * vi1 + 2 >= v.size() || 3 * vi2 + 2 >= v.size()) continue;
    float32 e0x = v[vi1 * 3 + 0] - v[vi0 * 3 + 0], e0y = v[vi1 * 3 + 1] - v[vi0 * 3 + 1],
            e0z = v[vi1 * 3 + 2] - v[vi0 * 3 + 2];
    float32 e1x = v[vi2 * 3 + 0] - v[vi1 * 3 + 0], e1y = v[vi2 * 3 + 1] - v[vi1 * 3 + 1],
            e1z = v[vi2 * 3 + 2] - v[vi1 * 3 + 2];
    float32 cx = std::fabs(e0y * e1z - e0z * e1y);
    float32 cy = std::fabs(e0z * e1x - e0x * e1z);
    float32 cz = std::fabs(e0x * e1y - e0y * e1x);
    if (cx > epsilon || cy > epsilon || cz > epsilon) {
      if (!(cx > cy && cx > cz)) {
        axes[0] = 0;
        if (cz > cx && cz > cy) axes[1] = 1;
      }
      break;
    }
  }
  float32 area = 0;
  for (size_t k = 0; k < npolys; ++k) {
    size_t vi0 = (size_t)face[(k + 0) % npolys].v, vi1 = (size_t)face[(k + 1) % npolys].v;
    if (vi0 * 3 + axes[0] >= v.size() || vi0 * 3 + axes[1] >= v.size() || vi1 * 3 + axes[0] >= v.size() ||
        vi1 * 3 + axes[1] >= v.size())
      continue;
    float32 v0x = v[vi0 * 3 + axes[0]], v0y = v[vi0 * 3 + axes[1]];
    float32 v1x = v[vi1 * 3 + axes[0]], v1y = v[vi1 * 3 + axes[1]];
    area += (v0x * v1y - v0y * v1x) * (float32)0.5;
  }
  int max_rounds = 10;
  std::vector<Corner> rem = face;
  size_t guess_vert = 0;
  Corner ind[3];
  float32 vx[3], vy[3];
  while (rem.size() > 3 && max_rounds > 0) {
    npolys = rem.size();
    if (guess_vert >= npolys) {
      max_rounds -= 1;
      guess_vert -= npolys;
    }
    for (size_t k = 0; k < 3; k++) {
      ind[k] = rem[(guess_vert + k) % npolys];
      size_t vi = (size_t)ind[k].v;
      if (vi * 3 + axes[0] >= v.size() || vi * 3 + axes[1] >= v.size()) {
        vx[k] = 0.0f;
        vy[k] = 0.0f;
      } else {
        vx[k] = v[vi * 3 + axes[0]];
        vy[k] = v[vi * 3 + axes[1]];
      }
    }
    float32 e0x = vx[1] - vx[0], e0y = vy[1] - vy[0], e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
    float32 cross = e0x * e1y - e0y * e1x;
    if (cross * area < (float32)0.0) {  // an internal (reflex) angle
      guess_vert += 1;
      continue;
    }
    bool overlap = false;
    for (size_t other = 3; other < npolys; ++other) {
      size_t idx = (guess_vert + other) % npolys;
      size_t ovi = (size_t)rem[idx].v;
      if (ovi * 3 + axes[0] >= v.size() || ovi * 3 + axes[1] >= v.size()) continue;
      if (pnpoly(3, vx, vy, v[ovi * 3 + axes[0]], v[ovi * 3 + axes[1]])) {
        overlap = true;
        break;
      }
    }
    if (overlap) {
      guess_vert += 1;
      continue;
    }
    out->push_back(ind[0]);  // an ear
    out->push_back(ind[1]);
    out->push_back(ind[2]);
    size_t removed = (guess_vert + 1) % npolys;
    while (removed + 1 < npolys) {
      rem[removed] = rem[removed + 1];
      removed += 1;
    }
    rem.pop_back();
  }
  if (rem.size() == 3) {
    out->push_back(rem[0]);
    out->push_back(rem[1]);
    out->push_back(rem[2]);
  }
}

}  // namespace

bool LoadObjFile(const std::string& filename, MeshData* out, std::string* err) {
  std::ifstream in(filename, std::ios::in | std::ios::binary);
  if (!in) {
    *err = "cannot open " + filename;
    return false;
  }
  MeshData d;
  std::string line;
  std::vector<Corner> face, tris;
  while (std::getline(in, line)) {
    const char* token = line.c_str();
    token += std::strspn(token, " \t");
    if (token[0] == '\0' || token[0] == '#') continue;
    auto is_space = [](char c) { return c == ' ' || c == '\t'; };
    if (token[0] == 'v' && is_space(token[1])) {  // v x y z
      token += 2;
      float32 x = parse_real(&token), y = parse_real(&token), z = parse_real(&token);
      d.positions.insert(d.positions.end(), {x, y, z});
    } else if (token[0] == 'v' && token[1] == 'n' && is_space(token[2])) {
      token += 3;
      float32 x = parse_real(&token), y = parse_real(&token), z = parse_real(&token);
      d.normals.insert(d.normals.end(), {x, y, z});
    } else if (token[0] == 'v' && token[1] == 't' && is_space(token[2])) {
      token += 3;
      float32 u = parse_real(&token), v = parse_real(&token);
      d.texcoords.insert(d.texcoords.end(), {u, v});
    } else if (token[0] == 'f' && is_space(token[1])) {
      token += 2;
      token += std::strspn(token, " \t");
      face.clear();
      int nv = (int)(d.positions.size() / 3), nn = (int)(d.normals.size() / 3), nt = (int)(d.texcoords.size() / 2);
      while (*token && *token != '\r' && *token != '\n') {
        Corner c;
        if (!parse_corner(&token, nv, nn, nt, &c)) {
          *err = filename + ": failed to parse a face";
          return false;
        }
        face.push_back(c);
        token += std::strspn(token, " \t\r");
      }
      tris.clear();
      triangulate_face(d.positions, face, &tris);
      for (const Corner& c : tris) d.corners.insert(d.corners.end(), {c.v, c.n, c.t});
    }
  }
  *out = std::move(d);
  return true;
}

MeshObject::MeshObject(const std::string& filename, bool invert_normals, const vector3& translation,
                       const vector3& scale, const vector4& rotation)
    : invert_(invert_normals), t_(translation), s_(scale), r_(rotation) {
  std::string err;
  ok_ = LoadObjFile(filename, &data_, &err);
  if (!ok_) std::printf("Error loading obj file %s: %s.\n", filename.c_str(), err.c_str());  // mesh.cpp:179
}
MeshObject::MeshObject(MeshData data, bool invert_normals, const vector3& translation, const vector3& scale,
                       const vector4& rotation)
    : data_(std::move(data)), ok_(true), invert_(invert_normals), t_(translation), s_(scale), r_(rotation) {}
fs_object MeshObject::Describe() const { return obj_base(FS_OBJ_MESH); }
fs_mesh MeshObject::DescribeMesh() const {
  fs_mesh m;
  std::memset(&m, 0, sizeof(m));
  m.positions = data_.positions.empty() ? nullptr : data_.positions.data();
  m.num_positions = (uint32_t)(data_.positions.size() / 3);
  m.normals = data_.normals.empty() ? nullptr : data_.normals.data();
  m.num_normals = (uint32_t)(data_.normals.size() / 3);
  m.texcoords = data_.texcoords.empty() ? nullptr : data_.texcoords.data();
  m.num_texcoords = (uint32_t)(data_.texcoords.size() / 2);
  m.corners = data_.corners.empty() ? nullptr : data_.corners.data();
  m.num_triangles = (uint32_t)(data_.corners.size() / 9);
  m.invert_normals = invert_ ? 1 : 0;
  m.translation[0] = t_.x;
  m.translation[1] = t_.y;
  m.translation[2] = t_.z;
  m.scale[0] = s_.x;
  m.scale[1] = s_.y;
  m.scale[2] = s_.z;
  m.rotation[0] = r_.x;
  m.rotation[1] = r_.y;
  m.rotation[2] = r_.z;
  m.rotation[3] = r_.w;
  return m;
}

// ============================================================================
// Scene — scene.cpp
// ============================================================================
Scene::Scene() { sky_material_.reset(new LightMaterial(vector3(0, 0, 0))); }  // scene.cpp:142-144

Camera* Scene::GetCamera(uint32 index) {
  if (index >= camera_list_.size()) return nullptr;
  return &camera_list_[index];
}
void Scene::SetSkyMaterial(std::shared_ptr<LightMaterial> material) {
  sky_material_ = material;
  Touch();
}
void Scene::SetSkyMaterial(std::shared_ptr<Material> material) {
  sky_material_ = material;
  Touch();
}
MeshObject* Scene::AddMeshObject(const std::string& filename, bool invert_normals, const vector3& translation,
                                 const vector3& scale, const vector4& rotation) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new MeshObject(filename, invert_normals, translation, scale, rotation));
  return static_cast<MeshObject*>(object_list_.back().get());
}
MeshObject* Scene::AddMeshObject(MeshData data, bool invert_normals, const vector3& translation,
                                 const vector3& scale, const vector4& rotation) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new MeshObject(std::move(data), invert_normals, translation, scale, rotation));
  return static_cast<MeshObject*>(object_list_.back().get());
}
SphericalObject* Scene::AddSphericalObject(const vector3& origin, float32 radius) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new SphericalObject(origin, radius));
  return static_cast<SphericalObject*>(object_list_.back().get());
}
DiscObject* Scene::AddDiscObject(const vector3& origin, const vector3& normal, float32 radius) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new DiscObject(origin, normal, radius));
  return static_cast<DiscObject*>(object_list_.back().get());
}
PlanarObject* Scene::AddPlanarObject(const plane& data) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new PlanarObject(data));
  return static_cast<PlanarObject*>(object_list_.back().get());
}
CuboidObject* Scene::AddCuboidObject(const vector3& origin, float32 width, float32 height, float32 depth) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new CuboidObject(origin, width, height, depth));
  return static_cast<CuboidObject*>(object_list_.back().get());
}
QuadObject* Scene::AddQuadObject(const vector3& origin, const vector3& normal, float32 width, float32 height) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new QuadObject(origin, normal, width, height));
  return static_cast<QuadObject*>(object_list_.back().get());
}
QuadObject* Scene::AddQuadObject(const vector3& position, const vector3& u, const vector3& v) {
  Touch();
  optimized_ = false;  // is_tree_valid_ = false (scene.cpp:165-214)
  object_list_.emplace_back(new QuadObject(position, u, v));
  return static_cast<QuadObject*>(object_list_.back().get());
}

namespace {
typedef std::map<std::string, std::shared_ptr<Material>> MaterialMap;

// Reads block lines up to (and including) the first line containing '}'
// (scene.cpp:267-268).
template <class F>
void read_block(std::ifstream* in, F&& per_line) {
  std::string line;
  while (std::getline(*in, line)) {
    if (std::strchr(line.c_str(), '}')) break;
    per_line(line.c_str());
  }
}
std::string resolve(const std::string& file, const std::string& scene_dir) {
  if (file_exists(file) || scene_dir.empty() || (!file.empty() && file[0] == '/')) return file;
  std::string alt = scene_dir + "/" + file;
  return file_exists(alt) ? alt : file;
}
}  // namespace

bool Scene::LoadScene(const std::string& filename) {  // scene.cpp:493-535
  MaterialMap materials;
  std::ifstream in(filename, std::ios::in);
  if (!in.is_open()) {
    std::printf("Failed to read scene file %s.\n", filename.c_str());
    last_error_ = "cannot open scene file " + filename;
    return false;
  }
  std::string scene_dir;
  size_t slash = filename.find_last_of('/');
  if (slash != std::string::npos) scene_dir = filename.substr(0, slash);
  std::string line;
  while (std::getline(in, line)) {
    if (line[0] == '#') continue;
    char name[260] = {0};
    const char* s = line.c_str();
    if (std::sscanf(s, " material %259s", name) == 1) {  // ParseMaterial, scene.cpp:251-310
      vector3 color, emission;
      float32 metallic = 0, roughness = 0, refraction_index = 1, texture_scale = 1.0;
      int32 brdf = 0;
      float32 frostiness = 0.0, reflectivity = 0.1f;
      char texture_name[260] = {0};
      read_block(&in, [&](const char* l) {
        std::sscanf(l, " color %f %f %f", &color.x, &color.y, &color.z);
        std::sscanf(l, " emission %f %f %f", &emission.x, &emission.y, &emission.z);
        std::sscanf(l, " metallic %f", &metallic);
        std::sscanf(l, " roughness %f", &roughness);
        std::sscanf(l, " index %f", &refraction_index);
        std::sscanf(l, " texture %259s", texture_name);
        std::sscanf(l, " texture_scale %f", &texture_scale);
        std::sscanf(l, " brdf %i", &brdf);
        std::sscanf(l, " frostiness %f", &frostiness);
        std::sscanf(l, " reflectivity %f", &reflectivity);
      });
      std::shared_ptr<DiffuseMaterial> m;
      if (emission.x || emission.y || emission.z)
        m = std::make_shared<LightMaterial>(emission);
      else if (roughness)
        m = std::make_shared<CeramicMaterial>(color, roughness);
      else if (metallic) {
        if (metallic == 1.0)
          m = std::make_shared<MirrorMaterial>(color);
        else
          m = std::make_shared<MetalMaterial>(color, metallic);
      } else if (brdf == 1)
        m = std::make_shared<LiquidMaterial>(color, refraction_index, reflectivity);
      else if (brdf == 2)
        m = std::make_shared<GlassMaterial>(color, refraction_index, reflectivity, frostiness);
      else
        m = std::make_shared<DiffuseMaterial>(color);
      if (std::strlen(texture_name) && std::strcmp(texture_name, "None") != 0)
        m->LoadDiffuseTexture(resolve(texture_name, scene_dir), texture_scale);
      materials[std::string(name)] = m;
    } else if (std::strstr(s, "sphere")) {  // ParseSphere, scene.cpp:312-337
      float32 radius = 0;
      vector3 position;
      char mat[260] = {0};
      read_block(&in, [&](const char* l) {
        std::sscanf(l, " material %259s", mat);
        std::sscanf(l, " position %f %f %f", &position.x, &position.y, &position.z);
        std::sscanf(l, " radius %f", &radius);
      });
      Object* o = AddSphericalObject(position, radius);
      if (std::strlen(mat) && materials.count(mat)) o->SetMaterial(materials[mat]);
    } else if (std::strstr(s, "camera")) {  // ParseCamera, scene.cpp:339-366
      Camera cam;
      vector3 position = cam.origin, target = cam.target;
      float32 fov = cam.fov_y, aperture = cam.aperture_size, focal_depth = cam.focal_depth;
      read_block(&in, [&](const char* l) {
        std::sscanf(l, " position %f %f %f", &position.x, &position.y, &position.z);
        std::sscanf(l, " target %f %f %f", &target.x, &target.y, &target.z);
        std::sscanf(l, " fov %f", &fov);
        std::sscanf(l, " aperture %f", &aperture);
        std::sscanf(l, " focal_depth %f", &focal_depth);
      });
      cam.origin = position;
      cam.target = target;
      cam.fov_y = fov;
      cam.aperture_size = aperture;
      cam.focal_depth = focal_depth;
      camera_list_.push_back(cam);
      Touch();
    } else if (std::strstr(s, "sky")) {  // ParseSky, scene.cpp:368-386
      char mat[260] = {0};
      read_block(&in, [&](const char* l) { std::sscanf(l, " material %259s", mat); });
      if (std::strlen(mat) && materials.count(mat)) SetSkyMaterial(materials[mat]);
    } else if (std::strstr(s, "quad")) {  // ParseQuad, scene.cpp:388-418
      vector3 position, normal;
      float32 width = 0, height = 0;
      char mat[260] = {0};
      read_block(&in, [&](const char* l) {
        std::sscanf(l, " material %259s", mat);
        std::sscanf(l, " position %f %f %f", &position.x, &position.y, &position.z);
        std::sscanf(l, " normal %f %f %f", &normal.x, &normal.y, &normal.z);
        std::sscanf(l, " width %f", &width);
        std::sscanf(l, " height %f", &height);
      });
      Object* o = AddQuadObject(position, normal, width, height);
      if (std::strlen(mat) && materials.count(mat)) o->SetMaterial(materials[mat]);
    } else if (std::strstr(s, "cuboid")) {  // ParseCuboid, scene.cpp:420-454
      vector3 position;
      float32 width = 0, height = 0, depth = 0;
      vector4 rot;
      char mat[260] = {0};
      read_block(&in, [&](const char* l) {
        std::sscanf(l, " material %259s", mat);
        std::sscanf(l, " position %f %f %f", &position.x, &position.y, &position.z);
        std::sscanf(l, " width %f", &width);
        std::sscanf(l, " height %f", &height);
        std::sscanf(l, " depth %f", &depth);
        std::sscanf(l, " rotation %f %f %f %f", &rot.x, &rot.y, &rot.z, &rot.w);
      });
      CuboidObject* o = AddCuboidObject(position, width, height, depth);
      if (std::strlen(mat) && materials.count(mat)) o->SetMaterial(materials[mat]);
      o->Rotate(vector3(rot.x, rot.y, rot.z), rot.w);
    } else if (std::strstr(s, "mesh")) {  // ParseMesh, scene.cpp:456-491
      char file[260] = {0}, mat[260] = {0};
      vector3 t, sc(1, 1, 1);
      vector4 rot;
      read_block(&in, [&](const char* l) {
        std::sscanf(l, " file %259s", file);
        std::sscanf(l, " material %259s", mat);
        std::sscanf(l, " translation %f %f %f", &t.x, &t.y, &t.z);
        std::sscanf(l, " scale %f %f %f", &sc.x, &sc.y, &sc.z);
        std::sscanf(l, " rotation %f %f %f %f", &rot.x, &rot.y, &rot.z, &rot.w);
      });
      if (std::strlen(file)) {
        Object* o = AddMeshObject(resolve(file, scene_dir), false, t, sc, rot);
        if (std::strlen(mat) && materials.count(mat)) o->SetMaterial(materials[mat]);
      }
    }
  }
  Optimize();
  return true;
}

const fs_scene_desc* Scene::Describe(std::string* err) {
  desc_mat_ptrs_.clear();
  desc_mats_.clear();
  desc_objs_.clear();
  desc_meshes_.clear();
  desc_tex_.clear();
  std::map<Material*, int32> index;
  auto mat_index = [&](const std::shared_ptr<Material>& m) -> int32 {
    if (!m) return -1;
    auto it = index.find(m.get());
    if (it != index.end()) return it->second;
    int32 i = (int32)desc_mats_.size();
    index[m.get()] = i;
    desc_mat_ptrs_.push_back(m);
    fs_material d = m->Describe();
    auto* dm = dynamic_cast<const DiffuseMaterial*>(m.get());
    if (dm && dm->HasDiffuseMap()) {
      const Texture& t = dm->diffuse_map();
      d.texture = (int32)desc_tex_.size();
      desc_tex_.push_back(fs_texture{t.buffer.data(), t.width, t.height});
    }
    desc_mats_.push_back(d);
    return i;
  };
  int32 sky = mat_index(sky_material_);
  for (size_t i = 0; i < object_list_.size(); i++) {
    Object* o = object_list_[i].get();
    fs_object d = o->Describe();
    d.material = mat_index(o->material_ptr());
    if (d.material < 0) {
      *err = "object " + std::to_string(i) + " has no material (the reference dereferences a null Material* on hit)";
      return nullptr;
    }
    if (d.kind == FS_OBJ_MESH) {
      d.mesh = (int32)desc_meshes_.size();
      desc_meshes_.push_back(static_cast<MeshObject*>(o)->DescribeMesh());
    }
    desc_objs_.push_back(d);
  }
  if (g_normal_table.empty()) InitializeMaterials();  // normal.cpp:29-32 lazy initialisation
  std::memset(&desc_, 0, sizeof(desc_));
  desc_.materials = desc_mats_.data();
  desc_.num_materials = (uint32_t)desc_mats_.size();
  desc_.sky_material = sky;
  desc_.objects = desc_objs_.empty() ? nullptr : desc_objs_.data();
  desc_.num_objects = (uint32_t)desc_objs_.size();
  desc_.meshes = desc_meshes_.empty() ? nullptr : desc_meshes_.data();
  desc_.num_meshes = (uint32_t)desc_meshes_.size();
  desc_.textures = desc_tex_.empty() ? nullptr : desc_tex_.data();
  desc_.num_textures = (uint32_t)desc_tex_.size();
  desc_.normal_table = g_normal_table.data();
  desc_.flags = optimized_ ? FS_SCENE_OPTIMIZED : 0u;
  return &desc_;
}

// ============================================================================
// Engine state: one process-wide device context (engine.cpp has none)
// ============================================================================
namespace {
struct Engine {
  std::mutex mu;
  int device = 0;
  fs_context* ctx = nullptr;
  const Scene* scene = nullptr;
  uint64 scene_version = 0, table_version = 0;
  int status = FS_OK;
  std::string error;
  uint32 frame_counter = 0;
  TraceSettings settings;
  bool settings_init = false;
};
Engine& engine() {
  static Engine e;
  return e;
}
int engine_fail(Engine& e, int rc, const std::string& where) {
  e.status = rc;
  e.error = where + ": " + fs_last_error();
  std::fprintf(stderr, "[fs] %s\n", e.error.c_str());
  return rc;
}
void init_settings(Engine& e) {
  if (e.settings_init) return;
  fs_options_default(&e.settings.options);
  e.settings_init = true;
}
int ensure_context(Engine& e) {
  if (e.ctx) return FS_OK;
  init_settings(e);
  int rc = fs_create(e.device, &e.ctx);
  if (rc) return engine_fail(e, rc, "fs_create");
  rc = fs_set_options(e.ctx, &e.settings.options);
  if (rc) return engine_fail(e, rc, "fs_set_options");
  return FS_OK;
}
}  // namespace

bool SetTraceDevice(int device) {
  Engine& e = engine();
  std::lock_guard<std::mutex> g(e.mu);
  if (e.ctx) return false;
  e.device = device;
  return true;
}
TraceSettings GetTraceSettings() {
  Engine& e = engine();
  std::lock_guard<std::mutex> g(e.mu);
  init_settings(e);
  return e.settings;
}
bool SetTraceSettings(const TraceSettings& s) {
  Engine& e = engine();
  std::lock_guard<std::mutex> g(e.mu);
  init_settings(e);
  if (e.ctx) {
    int rc = fs_set_options(e.ctx, &s.options);
    if (rc) {
      engine_fail(e, rc, "fs_set_options");
      return false;
    }
  }
  const bool rebuild = std::memcmp(&s.options, &e.settings.options, sizeof(fs_options)) != 0 ||
                       s.device_bvh != e.settings.device_bvh;
  e.settings = s;
  if (rebuild) e.scene = nullptr;  // re-upload with the new build settings
  return true;
}
int LastTraceStatus() { return engine().status; }
const char* LastTraceError() { return engine().error.c_str(); }

// ============================================================================
// DisplayFrame — frame.cpp, device resident
// ============================================================================
DisplayFrame::DisplayFrame(uint32 width, uint32 height) : width_(width), height_(height) {
  Engine& e = engine();
  std::lock_guard<std::mutex> g(e.mu);
  if (ensure_context(e) == FS_OK) {
    int rc = fs_frame_create(e.ctx, width, height, &frame_);
    if (rc) engine_fail(e, rc, "fs_frame_create");
  }
}
DisplayFrame::~DisplayFrame() { fs_frame_destroy(frame_); }
void DisplayFrame::Reset() {
  samples_ = 0;
  if (frame_) fs_frame_reset(frame_);
}
// The planes are read into page-locked buffers the device frame owns
// (fs_frame_map): the window loop's per-frame display read runs at pinned
// PCIe speed and no copy into pageable memory follows (ABI 9). Without a
// device frame (creation failed, LastTraceStatus says why) they are zeros.
uint8* DisplayFrame::GetDisplayBuffer() {
  const void* p = nullptr;
  if (frame_ && fs_frame_map(frame_, FS_PLANE_DISPLAY, &p) == FS_OK) return (uint8*)p;
  display_.assign(3 * (size_t)width_ * height_, 0);
  return display_.data();
}
const float32* DisplayFrame::GetRenderTarget() {
  const void* p = nullptr;
  if (frame_ && fs_frame_map(frame_, FS_PLANE_COLOR, &p) == FS_OK) return (const float32*)p;
  color_.assign(3 * (size_t)width_ * height_, 0.0f);
  return color_.data();
}
const uint32* DisplayFrame::GetCountBuffer() {
  const void* p = nullptr;
  if (frame_ && fs_frame_map(frame_, FS_PLANE_COUNT, &p) == FS_OK) return (const uint32*)p;
  count_.assign((size_t)width_ * height_, 0u);
  return count_.data();
}

// ============================================================================
// TraceScene — engine.cpp:253-296
// ============================================================================
namespace {
// Uploads `scene` when it (or the normal table) changed since the last trace.
bool ensure_scene(Engine& e, Scene* scene) {
  if (ensure_context(e)) return false;
  if (e.scene != scene || e.scene_version != scene->version() || e.table_version != g_table_version) {
    std::string err;
    const fs_scene_desc* d = scene->Describe(&err);
    if (!d) {
      e.status = FS_ERR_INVALID;
      e.error = err;
      std::fprintf(stderr, "[fs] %s\n", err.c_str());
      return false;
    }
    // Large meshes get their BVH built on the device (same frames, about a
    // tenth of the host build time) unless TraceSettings::device_bvh is off.
    const uint32_t flags = e.settings.device_bvh ? FS_UPLOAD_GPU_BVH : 0u;
    int rc = fs_upload_scene_ex(e.ctx, d, flags);
    if (rc) {
      engine_fail(e, rc, "fs_upload_scene_ex");
      return false;
    }
    e.scene = scene;
    e.scene_version = scene->version();
    e.table_version = g_table_version;
  }
  return true;
}
}  // namespace

void TraceSceneBatch(const Camera& view, Scene* scene, DisplayFrame* output, uint32 spp) {
  Engine& e = engine();
  std::lock_guard<std::mutex> g(e.mu);
  e.status = FS_OK;
  e.error.clear();
  if (!scene || !output || !output->device_frame()) {
    e.status = FS_ERR_INVALID;
    e.error = "TraceScene: null scene or frame";
    return;
  }
  if (!ensure_scene(e, scene)) return;
  fs_camera cam = view.Describe();
  fs_render_params p;
  std::memset(&p, 0, sizeof(p));
  p.width = output->GetWidth();
  p.height = output->GetHeight();
  auto t0 = std::chrono::steady_clock::now();
  // The C ABI seeds sample k of a pixel from (pixel << 20) ^ k ^ seed with
  // k < 2^20; a frame that keeps accumulating past 2^20 samples (the
  // reference has no limit) moves on to epoch e = samples >> 20 with seed
  // e << 48, above every pixel bit of frames up to 2^28 pixels.
  uint64 have = output->samples();
  for (uint32 left = spp; left;) {
    const uint64 epoch = have >> 20, k = have & ((1u << 20) - 1);
    const uint32 n = (uint32)std::min<uint64>(left, (1u << 20) - k);
    p.spp = n;
    p.sample_base = (uint32)k;
    p.seed = epoch << 48;
    int rc = fs_render(e.ctx, &cam, &p, output->device_frame());
    if (rc) {
      engine_fail(e, rc, "fs_render");
      return;
    }
    have += n;
    left -= n;
  }
  // The frame's accessors (GetDisplayBuffer & co.) read it on the same
  // stream, so the call returns once its work is enqueued; it waits for the
  // device only to time the frame for the reference's log line (the window
  // loop then overlaps this frame's fold with the host's previous display).
  const bool timed = !view.fast_render_enabled && e.settings.timing_log;
  if (timed) {
    int rc = fs_synchronize(e.ctx);
    if (rc) {
      engine_fail(e, rc, "fs_synchronize");
      return;
    }
  }
  output->add_samples(spp);
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (timed)  // engine.cpp:284-293
    std::printf("Frame %u render time: %.2f sec. Msamples/sec: %.2f\n", e.frame_counter, sec,
                (double)p.width * p.height * spp / (1e6 * sec));
  e.frame_counter++;
  output->SetFrameCount(e.frame_counter);
}

void TraceScene(const Camera& view, Scene* scene, DisplayFrame* output, ImagePlaneCache*) {
  TraceSceneBatch(view, scene, output, 1);
}

float32 TraceRange(const Camera& view, Scene* scene, DisplayFrame* frame, float32 x, float32 y) {
  Engine& e = engine();
  std::lock_guard<std::mutex> g(e.mu);
  e.status = FS_OK;
  e.error.clear();
  if (!scene || !frame) {
    e.status = FS_ERR_INVALID;
    e.error = "TraceRange: null scene or frame";
    return view.z_far;
  }
  if (!ensure_scene(e, scene)) return view.z_far;
  fs_camera cam = view.Describe();
  float xy[2] = {x, y}, d = view.z_far;
  int rc = fs_trace_range(e.ctx, &cam, frame->GetWidth(), frame->GetHeight(), xy, 1, &d);
  if (rc) engine_fail(e, rc, "fs_trace_range");
  return d;
}

}  // namespace base

// ============================================================================
// C entry points (used by the Python tooling and tests)
// ============================================================================
namespace {
thread_local std::string g_host_error;
}

extern "C" {

const char* fsh_last_error(void) { return g_host_error.c_str(); }

void* fsh_scene_new(void) { return new base::Scene(); }

void* fsh_scene_load(const char* path) {
  base::Scene* s = new base::Scene();
  if (!s->LoadScene(path ? path : "")) {
    g_host_error = s->last_error();
    delete s;
    return nullptr;
  }
  return s;
}

void fsh_scene_free(void* scene) { delete static_cast<base::Scene*>(scene); }

const fs_scene_desc* fsh_scene_describe(void* scene) {
  if (!scene) {
    g_host_error = "null scene";
    return nullptr;
  }
  std::string err;
  const fs_scene_desc* d = static_cast<base::Scene*>(scene)->Describe(&err);
  if (!d) g_host_error = err;
  return d;
}

int fsh_scene_camera_count(void* scene) { return scene ? (int)static_cast<base::Scene*>(scene)->GetCameraCount() : 0; }

int fsh_scene_camera(void* scene, uint32_t index, fs_camera* out) {
  if (!scene || !out) return FS_ERR_INVALID;
  base::Camera* c = static_cast<base::Scene*>(scene)->GetCamera(index);
  if (!c) return FS_ERR_INVALID;
  *out = c->Describe();
  return FS_OK;
}

void fsh_set_seed(uint64_t seed) { base::set_seed(seed); }
uint64_t fsh_random_integer(void) { return base::random_integer(); }
float fsh_random_float(void) { return base::random_float(); }
void fsh_initialize_materials(void) { base::InitializeMaterials(); }

int fsh_normal_table(float* out) {
  const std::vector<float>& t = base::NormalTable();
  if (!out || t.empty()) return FS_ERR_STATE;
  std::memcpy(out, t.data(), t.size() * sizeof(float));
  return FS_OK;
}

// Loads an OBJ into flat arrays owned by the returned handle.
void* fsh_obj_load(const char* path) {
  base::MeshData* m = new base::MeshData();
  std::string err;
  if (!base::LoadObjFile(path ? path : "", m, &err)) {
    g_host_error = err;
    delete m;
    return nullptr;
  }
  return m;
}
int fsh_obj_info(void* h, uint32_t* positions, uint32_t* normals, uint32_t* texcoords, uint32_t* triangles) {
  if (!h) return FS_ERR_INVALID;
  base::MeshData* m = static_cast<base::MeshData*>(h);
  if (positions) *positions = (uint32_t)(m->positions.size() / 3);
  if (normals) *normals = (uint32_t)(m->normals.size() / 3);
  if (texcoords) *texcoords = (uint32_t)(m->texcoords.size() / 2);
  if (triangles) *triangles = (uint32_t)(m->corners.size() / 9);
  return FS_OK;
}
int fsh_obj_copy(void* h, float* positions, int32_t* corners) {
  if (!h) return FS_ERR_INVALID;
  base::MeshData* m = static_cast<base::MeshData*>(h);
  if (positions) std::memcpy(positions, m->positions.data(), m->positions.size() * 4);
  if (corners) std::memcpy(corners, m->corners.data(), m->corners.size() * 4);
  return FS_OK;
}
void fsh_obj_free(void* h) { delete static_cast<base::MeshData*>(h); }

// Texture loaders (host/fs_image.h), for tests. fsh_load_bitmap returns
// LoadBitmap's result and hands back whatever it left in the buffer (n floats).
int fsh_load_bitmap(const char* path, float** out, uint32_t* w, uint32_t* h, size_t* n) {
  std::vector<float> buf;
  uint32_t ww = 0, hh = 0;
  bool ok = base::LoadBitmap(path ? path : "", &buf, &ww, &hh);
  *out = static_cast<float*>(std::malloc(sizeof(float) * (buf.size() ? buf.size() : 1)));
  if (buf.size()) std::memcpy(*out, buf.data(), sizeof(float) * buf.size());
  *w = ww;
  *h = hh;
  *n = buf.size();
  return ok ? 1 : 0;
}
int fsh_load_exr(const char* path, float** rgba, int* w, int* h) {
  const char* err = nullptr;
  int rc = base::LoadEXR(rgba, w, h, path, &err);
  if (rc) g_host_error = err ? err : "LoadEXR failed";
  return rc;
}
void fsh_free(void* p) { std::free(p); }

}  // extern "C"
