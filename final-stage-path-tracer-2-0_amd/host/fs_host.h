// fs_host.h — C++ mirror of the reference's render API, backed by the
// MI355X path-trace layer (include/fs_trace.h).
//
// Same names, arguments and call order as the reference (namespace base):
//   Scene::LoadScene / Add*Object / SetSkyMaterial / GetCamera   scene.h:94-140
//   Camera                                                      camera.h:43-63
//   DiffuseMaterial ... FogMaterial, InitializeMaterials()      material.h:54-330
//   DisplayFrame                                                frame.h:49-92
//   TraceScene(camera, scene, frame)                            engine.h:74-75
// Material ids and the normal table draw from the main-thread xorshift64*
// stream exactly as the reference does (material.cpp:26, normal.cpp:9-27),
// so a scene built here renders with the reference's table.
#pragma once

#include <stdint.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "fs_trace.h"

namespace base {

typedef int32_t int32;
typedef uint32_t uint32;
typedef uint64_t uint64;
typedef uint8_t uint8;
typedef float float32;

// ---- minimal value types (math/vector3.h, vector4.h) ----------------------
struct vector2 {
  float32 x = 0, y = 0;
  vector2() {}
  vector2(float32 a, float32 b) : x(a), y(b) {}
};
struct vector3 {
  float32 x = 0, y = 0, z = 0;
  vector3() {}
  vector3(float32 a, float32 b, float32 c) : x(a), y(b), z(c) {}
};
struct vector4 {
  float32 x = 0, y = 0, z = 0, w = 0;
  vector4() {}
  vector4(float32 a, float32 b, float32 c, float32 d) : x(a), y(b), z(c), w(d) {}
  explicit vector4(const vector3& v) : x(v.x), y(v.y), z(v.z), w(1.0f) {}  // vector4.cpp:40-47
};
typedef vector4 plane;

// ---- RNG (math/random.h): thread_local xorshift64*, seed 521288629 -------
void set_seed(uint64 seed);
uint64 random_integer();
float32 random_float();
int64_t random_integer_range(int32 imin, int32 imax);
float32 random_float_range(float32 imin, float32 imax);

// ---- materials (material.h) ----------------------------------------------
class Material {
 public:
  virtual ~Material() {}
  uint32 GetID() { return material_id_; }
  virtual bool IsLight() { return false; }
  // Flattened record for the device (fs_material).
  virtual fs_material Describe() const = 0;

 protected:
  Material();
  uint32 material_id_;
};

// Texture (material.h:42-52): RGB floats, rows in file order.
struct Texture {
  std::string filename;
  std::vector<float32> buffer;
  uint32 width = 0;
  uint32 height = 0;
};

class DiffuseMaterial : public Material {
 public:
  DiffuseMaterial() : texture_scale_(0) {}
  explicit DiffuseMaterial(const vector3& diffuse);
  DiffuseMaterial(const std::string& filename, float32 tex_scale = 1.0f);
  // material.cpp:63-95: .bmp through LoadBitmap, .exr through LoadEXR
  // (host/fs_image.h); any other extension leaves the map empty.
  void LoadDiffuseTexture(const std::string& filename, float32 tex_scale = 1.0f);
  fs_material Describe() const override;
  // material.cpp:111: a map is used only when it holds texels.
  bool HasDiffuseMap() const { return diffuse_map_.buffer.size() && diffuse_map_.width && diffuse_map_.height; }
  const Texture& diffuse_map() const { return diffuse_map_; }

 protected:
  fs_material Base(int kind) const;
  vector3 diffuse_;
  Texture diffuse_map_;
  float32 texture_scale_;
};

class LightMaterial : public DiffuseMaterial {
 public:
  LightMaterial() : emissive_(1, 1, 1) { diffuse_ = vector3(1, 1, 1); }
  explicit LightMaterial(const vector3& emissive);
  bool IsLight() override { return true; }
  fs_material Describe() const override;

 protected:
  vector3 emissive_;
};

class MetalMaterial : public DiffuseMaterial {
 public:
  MetalMaterial() : roughness_(0.5f) {}
  MetalMaterial(const vector3& diffuse, float32 roughness);
  fs_material Describe() const override;

 protected:
  float32 roughness_;
};

class MirrorMaterial : public DiffuseMaterial {
 public:
  MirrorMaterial() {}
  explicit MirrorMaterial(const vector3& diffuse);
  fs_material Describe() const override;
};

class GlassMaterial : public DiffuseMaterial {
 public:
  GlassMaterial() : index_(0.75f), frost_(0.0f), reflectivity_(0.1f) {}
  GlassMaterial(const vector3 diffuse, float32 index = 0.75f, float32 reflectivity = 0.1, float32 frost = 0.0f);
  fs_material Describe() const override;

 protected:
  float32 index_, frost_, reflectivity_;
};

class LiquidMaterial : public DiffuseMaterial {
 public:
  LiquidMaterial() : index_(0.75f), reflectivity_(0.4f) {}
  LiquidMaterial(const vector3 diffuse, float32 index = 0.75f, float32 reflectivity = 0.4f);
  fs_material Describe() const override;

 protected:
  float32 index_, reflectivity_;
};

class CeramicMaterial : public DiffuseMaterial {
 public:
  CeramicMaterial() : shininess_(0.0f) {}
  CeramicMaterial(const vector3& diffuse, float32 shininess);
  fs_material Describe() const override;

 protected:
  float32 shininess_;
};

class GlowMaterial : public CeramicMaterial {
 public:
  GlowMaterial(const vector3& diffuse, const vector3& glow, float32 shininess);
  fs_material Describe() const override;

 protected:
  vector3 glow_;
};

class FogMaterial : public DiffuseMaterial {
 public:
  FogMaterial() : density_(0) {}
  FogMaterial(const vector3 diffuse, float32 density);
  fs_material Describe() const override;

 protected:
  float32 density_;
};

// Builds the 32768-entry normal table from the main-thread stream
// (material.cpp:15-17, normal.cpp:9-27). Call after the scene is loaded.
void InitializeMaterials();
// The table built by the last InitializeMaterials() (3 floats per entry).
const std::vector<float32>& NormalTable();

// ---- camera (camera.h:43-63) ----------------------------------------------
struct Camera {
  float32 z_near;
  float32 z_far;
  vector3 origin;
  vector3 target;
  float32 fov_y;
  float32 aperture_size;
  float32 focal_depth;
  bool fast_render_enabled;
  Camera();
  Camera(const vector3& new_origin, const vector3& new_target);
  fs_camera Describe() const;
};

// ---- objects (object.h, mesh.h) -------------------------------------------
class Object {
 public:
  virtual ~Object() {}
  void SetMaterial(std::shared_ptr<Material> material) { material_ = material; }
  Material* GetMaterial() { return material_.get(); }
  virtual fs_object Describe() const = 0;
  std::shared_ptr<Material> material_ptr() const { return material_; }

 protected:
  std::shared_ptr<Material> material_;
};

class SphericalObject : public Object {
 public:
  SphericalObject(const vector3& origin, float32 radius) : origin_(origin), radius_(radius) {}
  fs_object Describe() const override;

 private:
  vector3 origin_;
  float32 radius_;
};

class PlanarObject : public Object {
 public:
  explicit PlanarObject(const plane& data) : plane_(data) {}
  fs_object Describe() const override;

 private:
  plane plane_;
};

class DiscObject : public Object {
 public:
  DiscObject(const vector3& origin, const vector3& normal, float32 radius)
      : origin_(origin), normal_(normal), radius_(radius) {}
  fs_object Describe() const override;

 private:
  vector3 origin_, normal_;
  float32 radius_;
};

class CuboidObject : public Object {
 public:
  CuboidObject(const vector3& origin, float32 width, float32 height, float32 depth)
      : origin_(origin), width_(width), height_(height), depth_(depth) {}
  // cube::rotate (volume.cpp:434-445). Only one rotation is recorded; the
  // reference parser applies exactly one (scene.cpp:452).
  void Rotate(const vector3& axis, float32 angle);
  fs_object Describe() const override;

 private:
  vector3 origin_;
  float32 width_, height_, depth_;
  bool rotated_ = false;
  vector3 axis_;
  float32 angle_ = 0;
};

class QuadObject : public Object {
 public:
  QuadObject(const vector3& origin, const vector3& normal, float32 width, float32 height);
  QuadObject(const vector3& position, const vector3& u, const vector3& v);
  fs_object Describe() const override;

 private:
  bool puv_;
  vector3 a_, b_, c_;
  float32 w_ = 0, h_ = 0;
};

// Triangle-mesh data as tinyobj would hand it to MeshObject (mesh.cpp:177).
struct MeshData {
  std::vector<float32> positions, normals, texcoords;
  std::vector<int32> corners;  // 9 per triangle: v,n,t x 3 (OBJ order)
};
// Parses a Wavefront OBJ (v/vn/vt/f; polygons fan-triangulated).
bool LoadObjFile(const std::string& filename, MeshData* out, std::string* err);

class MeshObject : public Object {
 public:
  MeshObject(const std::string& filename, bool invert_normals = false, const vector3& translation = vector3(0, 0, 0),
             const vector3& scale = vector3(1, 1, 1), const vector4& rotation = vector4(0, 0, 0, 0));
  MeshObject(MeshData data, bool invert_normals, const vector3& translation, const vector3& scale,
             const vector4& rotation);
  fs_object Describe() const override;
  fs_mesh DescribeMesh() const;
  bool ok() const { return ok_; }
  const MeshData& data() const { return data_; }

 private:
  MeshData data_;
  bool ok_ = false;
  bool invert_;
  vector3 t_, s_;
  vector4 r_;
};

// ---- scene (scene.h) ------------------------------------------------------
class Scene {
 public:
  Scene();
  bool LoadScene(const std::string& filename);
  MeshObject* AddMeshObject(const std::string& filename, bool invert_normals = false,
                            const vector3& translation = vector3(0, 0, 0), const vector3& scale = vector3(1, 1, 1),
                            const vector4& rotation = vector4(0, 0, 0, 0));
  MeshObject* AddMeshObject(MeshData data, bool invert_normals = false, const vector3& translation = vector3(0, 0, 0),
                            const vector3& scale = vector3(1, 1, 1), const vector4& rotation = vector4(0, 0, 0, 0));
  SphericalObject* AddSphericalObject(const vector3& origin, float32 radius);
  DiscObject* AddDiscObject(const vector3& origin, const vector3& normal, float32 radius);
  PlanarObject* AddPlanarObject(const plane& data);
  CuboidObject* AddCuboidObject(const vector3& origin, float32 width, float32 height, float32 depth);
  QuadObject* AddQuadObject(const vector3& origin, const vector3& normal, float32 width, float32 height);
  QuadObject* AddQuadObject(const vector3& position, const vector3& u, const vector3& v);
  void SetSkyMaterial(std::shared_ptr<LightMaterial> material);
  void SetSkyMaterial(std::shared_ptr<Material> material);  // scene.cpp:383 cast
  Material* GetSkyMaterial() { return sky_material_.get(); }
  // scene.cpp:216-225: marks the object list as optimised; the consumers
  // (device layer, oracle) then trace a scene of >= 182 objects through the
  // reference's object octree (fs_scene_desc.flags FS_SCENE_OPTIMIZED).
  // Adding an object clears it, as in the reference.
  void Optimize() {
    optimized_ = true;
    Touch();
  }
  bool optimized() const { return optimized_; }
  uint32 GetCameraCount() { return (uint32)camera_list_.size(); }
  Camera* GetCamera(uint32 index);

  // Flattens the scene for fs_upload_scene; pointers stay valid until the
  // scene is modified or destroyed. The normal table is the global one.
  const fs_scene_desc* Describe(std::string* err);
  uint64 version() const { return version_; }
  const std::string& last_error() const { return last_error_; }

 private:
  void Touch() { version_++; }
  std::shared_ptr<Material> sky_material_;
  std::vector<Camera> camera_list_;
  std::vector<std::unique_ptr<Object>> object_list_;
  uint64 version_ = 1;
  bool optimized_ = false;  // Scene::is_tree_valid_ once Optimize() ran
  std::string last_error_;
  // Describe() storage
  std::vector<std::shared_ptr<Material>> desc_mat_ptrs_;
  std::vector<fs_material> desc_mats_;
  std::vector<fs_object> desc_objs_;
  std::vector<fs_mesh> desc_meshes_;
  std::vector<fs_texture> desc_tex_;
  fs_scene_desc desc_{};
};

// ---- frame (frame.h) --------------------------------------------------------
class DisplayFrame {
 public:
  DisplayFrame(uint32 width, uint32 height);
  ~DisplayFrame();
  void Reset();
  // Host copies (page-locked, owned by the frame) are refreshed from the
  // device on access; a pointer stays valid until the next access of that plane.
  uint8* GetDisplayBuffer();
  const float32* GetRenderTarget();
  const uint32* GetCountBuffer();
  uint32 GetWidth() { return width_; }
  uint32 GetHeight() { return height_; }
  float32 GetAspectRatio() { return (float32)width_ / height_; }
  void SetFrameCount(uint32 count) { frame_count_ = count; }
  uint32 GetFrameCount() const { return frame_count_; }
  fs_frame* device_frame() { return frame_; }
  uint64 samples() const { return samples_; }
  void add_samples(uint32 n) { samples_ += n; }

 private:
  uint32 frame_count_ = 0, width_, height_;
  uint64 samples_ = 0;
  fs_frame* frame_ = nullptr;
  std::vector<uint8> display_;
  std::vector<float32> color_;
  std::vector<uint32> count_;
};

// ---- engine (engine.h) ------------------------------------------------------
class ImagePlaneCache;  // accepted and ignored, as main.cpp:157 never passes one
// Adds one sample per pixel (engine.cpp:253-296).
void TraceScene(const Camera& view, Scene* scene, DisplayFrame* output, ImagePlaneCache* cache = nullptr);
// Adds `spp` samples per pixel in one device submission (== spp TraceScene calls).
void TraceSceneBatch(const Camera& view, Scene* scene, DisplayFrame* output, uint32 spp);
// engine.cpp:298-329: distance from view.origin to the first hit of the
// jitter-free ray through frame point (x, y), or view.z_far (focus picking).
float32 TraceRange(const Camera& view, Scene* scene, DisplayFrame* frame, float32 x, float32 y);
// Device used by TraceScene (default 0); must be called before the first trace.
bool SetTraceDevice(int device);
// Mirror-only settings (no reference counterpart): the device context's
// fs_options, whether large meshes build their BVH on the device (default
// true; frames are identical either way), and whether each TraceScene call
// prints the reference's per-frame timing line (engine.cpp:284-293; default
// off). Scene-build fields apply from the next upload.
struct TraceSettings {
  fs_options options;
  bool device_bvh = true;
  bool timing_log = false;
};
TraceSettings GetTraceSettings();
bool SetTraceSettings(const TraceSettings& s);
// fs_status of the last engine call and its message.
int LastTraceStatus();
const char* LastTraceError();

}  // namespace base
