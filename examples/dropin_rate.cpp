// dropin_rate.cpp — samples/s of the drop-in API as an application drives it
// (measurement aid for DESIGN.md §6): the reference's window loop calls
// TraceScene once per displayed frame and reads the display bytes back
// (main.cpp:157-162), so every frame of 1 spp pays a launch, a fold and a
// PCIe read of W x H x 3 bytes; TraceSceneBatch submits many samples at once.
// Scene load and BVH build are excluded (one warm-up frame first).
//
//   dropin_rate <file.scene> <width> <height> <frames> [lookahead depth, default the library's]
#include <algorithm>
#include <chrono>
#include <vector>
#include <cstdio>
#include <cstdlib>

#include "fs_host.h"

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s scene width height frames\n", argv[0]);
    return 2;
  }
  base::Scene scene;
  if (!scene.LoadScene(argv[1])) return 1;
  base::InitializeMaterials();
  base::Camera camera;
  if (scene.GetCameraCount()) camera = *scene.GetCamera(0);
  const unsigned W = std::atoi(argv[2]), H = std::atoi(argv[3]), frames = std::atoi(argv[4]);
  if (W < 2 || H < 2 || frames == 0) {
    std::fprintf(stderr, "width and height must be >= 2 and frames > 0\n");
    return 2;
  }
  if (argc > 5) {  // fs_options.lookahead: how many TraceScene calls ahead the device traces
    base::TraceSettings ts = base::GetTraceSettings();
    ts.options.lookahead = (uint32_t)std::atoi(argv[5]);
    if (!base::SetTraceSettings(ts)) {
      std::fprintf(stderr, "SetTraceSettings: %s\n", base::LastTraceError());
      return 2;
    }
  }
  base::DisplayFrame frame(W, H);
  // not timed: the upload and BVH build (first call) and the lookahead's
  // buffers (allocated by the second, the first that continues a sequence)
  for (int i = 0; i < 2; i++) {
    base::TraceScene(camera, &scene, &frame);
    frame.GetDisplayBuffer();
  }
  if (base::LastTraceStatus() != 0) {
    std::fprintf(stderr, "TraceScene failed: %s\n", base::LastTraceError());
    return 1;
  }
  // the window loop: one TraceScene (1 spp) and one display read per frame
  std::vector<double> per(frames);
  double t0 = now_s();
  for (unsigned i = 0; i < frames; i++) {
    const double tf = now_s();
    base::TraceScene(camera, &scene, &frame);
    frame.GetDisplayBuffer();
    per[i] = now_s() - tf;
    if (base::LastTraceStatus() != 0) {  // a failed frame must not count as rendered
      std::fprintf(stderr, "frame %u failed: %s\n", i, base::LastTraceError());
      return 1;
    }
  }
  const double loop_s = now_s() - t0;
  // the same samples in one submission, one display read
  frame.Reset();
  t0 = now_s();
  base::TraceSceneBatch(camera, &scene, &frame, frames);
  frame.GetDisplayBuffer();
  const double batch_s = now_s() - t0;
  if (base::LastTraceStatus() != 0) {
    std::fprintf(stderr, "trace failed: %s\n", base::LastTraceError());
    return 1;
  }
  const double samples = (double)W * H * frames;
  std::sort(per.begin(), per.end());
  auto pct = [&](double q) { return per[std::min<size_t>(per.size() - 1, (size_t)(q * per.size()))] * 1e3; };
  std::printf("{\"width\": %u, \"height\": %u, \"frames\": %u, \"lookahead\": %u, \"loop_msamples_per_s\": %.2f, "
              "\"loop_ms_per_frame\": %.3f, \"frame_ms_p10_p50_p90_max\": [%.3f, %.3f, %.3f, %.3f], "
              "\"batch_msamples_per_s\": %.2f}\n",
              W, H, frames, base::GetTraceSettings().options.lookahead, samples / loop_s / 1e6, loop_s * 1e3 / frames,
              pct(0.1), pct(0.5), pct(0.9), per.back() * 1e3, samples / batch_s / 1e6);
  return 0;
}
