// trace_scene.cpp — the reference's main.cpp render loop (main.cpp:47-165)
// without the window: LoadScene -> InitializeMaterials -> TraceScene per
// frame -> GetDisplayBuffer, written as a PPM (top row first).
//
//   trace_scene <file.scene> <width> <height> <frames> <out.ppm> [out.f32]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fs_host.h"

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s scene width height frames out.ppm [color.f32]\n", argv[0]);
    return 2;
  }
  base::Scene scene;                              // main.cpp:88
  if (!scene.LoadScene(argv[1])) return 1;        // main.cpp:90
  base::InitializeMaterials();                    // main.cpp:102
  base::Camera camera;                            // main.cpp:104-112
  if (scene.GetCameraCount()) camera = *scene.GetCamera(0);
  base::DisplayFrame frame(std::atoi(argv[2]), std::atoi(argv[3]));
  int frames = std::atoi(argv[4]);
  for (int i = 0; i < frames; i++) {
    base::TraceScene(camera, &scene, &frame);     // main.cpp:157
    if (base::LastTraceStatus() != 0) {
      std::fprintf(stderr, "TraceScene failed: %s\n", base::LastTraceError());
      return 1;
    }
  }
  const base::uint8* rgb = frame.GetDisplayBuffer();  // main.cpp:162
  unsigned W = frame.GetWidth(), H = frame.GetHeight();
  FILE* f = std::fopen(argv[5], "wb");
  std::fprintf(f, "P6\n%u %u\n255\n", W, H);
  for (unsigned y = 0; y < H; y++) std::fwrite(rgb + 3 * (size_t)(H - 1 - y) * W, 1, 3 * W, f);  // row 0 = bottom
  std::fclose(f);
  if (argc > 6) {
    FILE* g = std::fopen(argv[6], "wb");
    std::fwrite(frame.GetRenderTarget(), 4, 3 * (size_t)W * H, g);
    std::fclose(g);
  }
  return 0;
}
