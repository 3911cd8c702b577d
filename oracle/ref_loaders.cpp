// ref_loaders.cpp — TEST INFRASTRUCTURE, container only (never shipped, never
// on the GPU box): a harness around the reference's OWN vendored loaders,
// compiled unmodified from /root/reference/source/third_party by
// oracle/Makefile into oracle/_ref/ref_loaders. It writes what the loaders
// return, so tests/golden/make_loader_fixtures.py can pin the C++ mirror's
// OBJ and EXR readers (host/fs_host.cpp, host/fs_image.cpp) against them.
//
//   ref_loaders obj IN.obj OUT.bin   LoadObj(triangulate = true), the call of
//                                    mesh.cpp:177-178
//   ref_loaders exr IN.exr OUT.bin   LoadEXR, the call of material.cpp:75
//
// OUT.bin (little endian): int32 status (LoadObj's bool / LoadEXR's return)
// then, for obj: uint32 counts (vertices, normals, texcoords floats; shapes),
// the three float arrays, and per shape uint32 (indices, faces), the index
// triples (vertex, normal, texcoord) and num_face_vertices as uint32;
// for exr: int32 width, height, then width*height*4 floats (RGBA).
#define TINYOBJLOADER_IMPLEMENTATION
#include "tiny_obj_loader.h"
#define TINYEXR_IMPLEMENTATION
#include "tiny_exr_loader.h"

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {
struct Out {
  FILE* f;
  template <class T>
  void put(const T& v) { std::fwrite(&v, sizeof(T), 1, f); }
  template <class T>
  void arr(const std::vector<T>& v) { if (!v.empty()) std::fwrite(v.data(), sizeof(T), v.size(), f); }
};

int obj(const char* in, Out& o) {
  tinyobj::attrib_t attrib;
  std::vector<tinyobj::shape_t> shapes;
  std::vector<tinyobj::material_t> materials;
  std::string err;
  bool ok = tinyobj::LoadObj(&attrib, &shapes, &materials, &err, in, nullptr, true);
  o.put<int32_t>(ok ? 1 : 0);
  o.put<uint32_t>((uint32_t)attrib.vertices.size());
  o.put<uint32_t>((uint32_t)attrib.normals.size());
  o.put<uint32_t>((uint32_t)attrib.texcoords.size());
  o.put<uint32_t>((uint32_t)shapes.size());
  o.arr(attrib.vertices);
  o.arr(attrib.normals);
  o.arr(attrib.texcoords);
  for (const tinyobj::shape_t& s : shapes) {
    o.put<uint32_t>((uint32_t)s.mesh.indices.size());
    o.put<uint32_t>((uint32_t)s.mesh.num_face_vertices.size());
    for (const tinyobj::index_t& ix : s.mesh.indices) {
      o.put<int32_t>(ix.vertex_index);
      o.put<int32_t>(ix.normal_index);
      o.put<int32_t>(ix.texcoord_index);
    }
    for (unsigned char n : s.mesh.num_face_vertices) o.put<uint32_t>(n);
  }
  return 0;
}

int exr(const char* in, Out& o) {
  float* rgba = nullptr;
  int w = 0, h = 0;
  const char* err = nullptr;
  int rc = LoadEXR(&rgba, &w, &h, in, &err);
  o.put<int32_t>(rc);
  if (rc < 0) return 0;
  o.put<int32_t>(w);
  o.put<int32_t>(h);
  std::fwrite(rgba, sizeof(float), (size_t)w * h * 4, o.f);
  std::free(rgba);
  return 0;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc != 4) {
    std::fprintf(stderr, "usage: ref_loaders obj|exr IN OUT\n");
    return 2;
  }
  Out o{std::fopen(argv[3], "wb")};
  if (!o.f) return 2;
  int rc = std::strcmp(argv[1], "obj") == 0 ? obj(argv[2], o) : std::strcmp(argv[1], "exr") == 0 ? exr(argv[2], o) : 2;
  std::fclose(o.f);
  return rc;
}
