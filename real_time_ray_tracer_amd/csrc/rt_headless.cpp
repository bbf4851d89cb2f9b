// rt_headless.cpp — headless frame driver over the C ABI: the render()/compute() loop of
// src/main.cpp:763-781 and 553-578 without GLFW/GL.  Per frame it updates the light
// (moving_light, main.cpp:541-551) or the rand buffer (fill_rand_buffer, main.cpp:535-539),
// uploads the header, dispatches the mode's programs, advances the 8-slot ring
// (main.cpp:619) and finally writes the last image as a PPM in place of the GL blit
// (main.cpp:783-797, shader_fragment.glsl).
//
//   rt_headless [--width W] [--height H] [--objects N] [--spp A] [--mode 1..4] [--frames K]
//               [--scene synthetic|1|5|6] [--seed S] [--device D] [--ppm out.ppm] [--pipeline 0|1]
//               [--strips G] [--devices d0,d1,...] [--balance ROUNDS]
// --strips G > 1 renders the frame as G row strips through the rt_group_* entry points: strip i
// on device devices[i % #devices] (default, without --devices: every visible device in turn,
// starting at --device), cost-balanced with --balance ROUNDS timed plans (0: equal strips),
// assembled on the first device.  A --devices list naming a device that does not exist, or
// more devices than are visible, is refused with a message.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt/abi.h"

static int check(int rc, const char* what) {
  if (rc < 0) {
    std::fprintf(stderr, "rt_headless: %s failed: %s (%d)\n", what, rt_strerror(rc), rc);
    std::exit(1);
  }
  return rc;
}

static void write_ppm(const char* path, const std::vector<float>& img, int W, int H) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return;
  std::fprintf(f, "P6\n%d %d\n255\n", W, H);
  std::vector<unsigned char> row(3 * (size_t)W);
  for (int r = H - 1; r >= 0; --r) {  // GL texture origin is bottom-left
    for (int x = 0; x < W; ++x)
      for (int c = 0; c < 3; ++c) {
        float v = img[((size_t)r * W + x) * 4 + c];
        v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
        row[3 * x + c] = (unsigned char)(v * 255.0f + 0.5f);
      }
    std::fwrite(row.data(), 1, row.size(), f);
  }
  std::fclose(f);
}

// The frame as `strips` row strips over the devices in `devlist` (rt_group_*).
static int run_strips(const rt_config& cfg, std::vector<float>& header, int mode, int frames, int pipeline,
                      int strips, const std::string& devlist, int device, int balance, const std::string& ppm) {
  std::vector<int> devs;
  for (size_t p = 0; p < devlist.size();) {
    size_t q = devlist.find(',', p);
    if (q == std::string::npos) q = devlist.size();
    devs.push_back(std::atoi(devlist.substr(p, q - p).c_str()));
    p = q + 1;
  }
  const int ndev = rt_device_count();
  if (ndev <= 0) {
    std::fprintf(stderr, "rt_headless: no HIP device is visible\n");
    return 1;
  }
  if (devs.empty()) {
    for (int k = 0; k < ndev; ++k) devs.push_back((device + k) % ndev);
  } else {
    // (every entry < ndev also bounds the distinct devices by the visible ones)
    for (int d : devs)
      if (d < 0 || d >= ndev) {
        std::fprintf(stderr, "rt_headless: --devices names device %d, but only %d device(s) are visible (0..%d)\n",
                     d, ndev, ndev - 1);
        return 1;
      }
  }
  std::vector<int> sd(strips);
  for (int i = 0; i < strips; ++i) sd[i] = devs[i % devs.size()];
  rt_group* g = nullptr;
  check(rt_group_create(strips, sd.data(), &cfg, nullptr, &g), "rt_group_create (peer access to the first device?)");
  if (pipeline) check(rt_group_enable_pipelining(g, 1), "rt_group_enable_pipelining");
  std::vector<double> strip_ms(strips, 0.0);
  if (balance > 0) check(rt_group_balance(g, header.data(), mode, balance, strip_ms.data()), "rt_group_balance");
  std::vector<int> b(strips + 1);
  check(rt_group_bounds(g, b.data()), "rt_group_bounds");
  std::printf("strips:");
  for (int i = 0; i < strips; ++i)
    std::printf(" [%d,%d)@%d%s", b[i], b[i + 1], sd[i], rt_group_strip_copies(g, i) > 0 ? "+copy" : "");
  std::printf("\n");
  auto t0 = std::chrono::steady_clock::now();
  check(rt_group_compute_frames(g, header.data(), mode, 0, frames, 7000, 0), "rt_group_compute_frames");
  check(rt_group_synchronize(g), "rt_group_synchronize");
  double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const int W = cfg.width, H = cfg.height, A = cfg.spp;
  std::printf("%dx%d spp=%d mode=%d %d strips%s: %.3f ms/frame (wall), %.1f Mrays/s\n", W, H, A, mode, strips,
              pipeline ? " pipelined" : "", wall / frames, (double)W * H * (mode <= 2 ? A : 1) * frames / (wall * 1e3));
  if (!ppm.empty()) {
    std::vector<float> img((size_t)W * H * 4);
    check(rt_group_download_image(g, img.data()), "rt_group_download_image");
    write_ppm(ppm.c_str(), img, W, H);
  }
  rt_group_destroy(g);
  return 0;
}

int main(int argc, char** argv) {
  int W = 440, H = 330, N = 5, A = 4, mode = 1, frames = 8, device = 0, pipeline = 0, strips = 1, balance = 0;
  std::string scene = "1", ppm, devlist;
  unsigned long long seed = 1234;
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string k = argv[i], v = argv[i + 1];
    if (k == "--width") W = std::atoi(v.c_str());
    else if (k == "--height") H = std::atoi(v.c_str());
    else if (k == "--objects") N = std::atoi(v.c_str());
    else if (k == "--spp") A = std::atoi(v.c_str());
    else if (k == "--mode") mode = std::atoi(v.c_str());
    else if (k == "--frames") frames = std::atoi(v.c_str());
    else if (k == "--scene") scene = v;
    else if (k == "--seed") seed = std::strtoull(v.c_str(), nullptr, 10);
    else if (k == "--device") device = std::atoi(v.c_str());
    else if (k == "--ppm") ppm = v;
    else if (k == "--pipeline") pipeline = std::atoi(v.c_str());
    else if (k == "--strips") strips = std::atoi(v.c_str());
    else if (k == "--devices") devlist = v;
    else if (k == "--balance") balance = std::atoi(v.c_str());
    else { std::fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
  }
  const float aspect = (W * 3 == H * 4) ? 1.333333f : 1.777777f;  // main.cpp:39-40
  int S = scene == "synthetic" ? N : 10;
  std::vector<float> header(rt_header_bytes(S, A) / 4, 0.0f);
  if (scene == "synthetic") check(rt_scenegen(header.data(), S, N, A, seed, aspect), "rt_scenegen");
  else check(rt_init_scene(header.data(), S, A, std::atoi(scene.c_str()), aspect), "rt_init_scene");

  rt_config cfg{W, H, S, A, RT_NUM_FRAMES, RT_RECURSION_DEPTH, 0, 0};
  if (strips > 1) return run_strips(cfg, header, mode, frames, pipeline, strips, devlist, device, balance, ppm);
  rt_ctx* ctx = nullptr;
  check(rt_create(device, &cfg, &ctx), "rt_create");
  check(rt_enable_timing(ctx, 1), "rt_enable_timing");
  if (pipeline) check(rt_enable_pipelining(ctx, 1, nullptr), "rt_enable_pipelining");
  int frame = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < frames; ++k) {
    if (mode <= 2) check(rt_fill_rand_buffer(header.data(), S, A, 7000 + (uint64_t)k), "fill_rand_buffer");
    else check(rt_moving_light(header.data(), 0), "moving_light");
    check(rt_set_mode(header.data(), frame, (int)header[4 * RT_HDR_MODE + 2]), "set_mode");
    check(rt_upload_header(ctx, header.data(), header.size() * 4), "rt_upload_header");
    frame = check(rt_dispatch(ctx, mode, frame), "rt_dispatch");
  }
  check(rt_synchronize(ctx), "rt_synchronize");
  double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  double total = 0.0;
  for (int p = 1; p < RT_PROG_COUNT; ++p) {
    int n = 0;
    double ms = 0;
    check(rt_kernel_stats(ctx, p, &n, &ms), "rt_kernel_stats");
    if (n) std::printf("program %d: %d launches, %.3f ms avg\n", p, n, ms / n);
    total += ms;
  }
  // pipelined: kernel spans overlap, so the frame rate comes from the wall clock
  double ms_frame = pipeline ? wall / frames : total / frames;
  std::printf("%dx%d spp=%d objects=%d mode=%d%s: %.3f ms/frame (%s), %.1f Mrays/s, wall %.1f ms\n", W, H, A, N,
              mode, pipeline ? " pipelined" : "", ms_frame, pipeline ? "wall" : "kernels",
              (double)W * H * (mode <= 2 ? A : 1) / (ms_frame * 1e3), wall);
  if (!ppm.empty()) {
    std::vector<float> img((size_t)W * H * 4);
    check(rt_download(ctx, nullptr, nullptr, nullptr, img.data()), "rt_download");
    write_ppm(ppm.c_str(), img, W, H);
  }
  rt_destroy(ctx);
  return 0;
}
