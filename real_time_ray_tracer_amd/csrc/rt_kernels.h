// rt_kernels.h — launch interface between the C-ABI shim and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace rt {

constexpr int kMaxFrames = 16;
constexpr int kCounters = 8;
constexpr int kCounterSlots = 256;  // per counter, summed by the host

// Everything one program launch needs.  Passed by value as the kernel argument (lives in the
// kernarg segment -> SGPRs).  Row ranges are in frame coordinates (row 0 = bottom row).
struct FrameParams {
  int W, H;                  // full frame (WIDTH, HEIGHT)
  int trace_row0, trace_rows;  // rows this launch computes
  int band_row0, band_rows;  // rows held by the g-buffer ring (strip + halo)
  int img_row0, img_rows;    // rows of the image (the strip, no halo)
  int nobj;                  // int(mode.z)
  int S;                     // stride of the compact shape table (capacity)
  int spp, D, F, frame;
  int b1_min;                // AO: least live lanes of a prepared batch for its batched first bounce (set at launch)
  float inv_spp, fW, fH;     // 1.0f / spp, (float)W, (float)H: host-computed wave-uniform constants
  float inv_W, inv_H;        // 1.0f / fW, 1.0f / fH (correctly rounded; div_rn_by)
  float hx, hy, hz;          // horizontal
  float vx, vy, vz;          // vertical
  float lx, ly, lz;          // llc_minus_campos
  float cx, cy, cz;          // camera_location
  float Lx, Ly, Lz;          // light_pos
  float4 bg;                 // background
  const float4* shapes;      // compact table [4][S]: geo, geo2, col, aux (rt_device.h)
  const float4* rb;          // rand_buffer[2*spp]
  float4* out_pix;           // colour destination [band_rows][W]
  float4* nrm;               // normals_buffer slot `frame` [band_rows][W]
  float4* dep;               // depth_buffer slot `frame`
  const float4* nrm_prev;    // the slot's previous normals / depth (stale reads); == nrm / dep
  const float4* dep_prev;    // unless the frame is pipelined (written to a fresh buffer)
  float4* image;             // [img_rows][W] or nullptr
  const float4* raw;         // post-process input (pre-filter snapshot of slot `frame`)
  const float4* hist_pix[kMaxFrames];  // per slot
  const float4* hist_nrm[kMaxFrames];
  const float4* hist_dep[kMaxFrames];
  // optional work counters (nullptr in timed runs): [0] primary samples, [1] closest-hit
  // segments, [2] shadow rays, [3] ray-shape tests = (segments + shadow rays) * nobj,
  // [4] executed lane-tests = sum over waves of 64 x (shapes tested by the wave's scene loops);
  // post-process: [5] filtered pixels, [6] history slots read, [7] history slots accepted;
  // each counter has kCounterSlots copies (index k * kCounterSlots + slot)
  unsigned long long* counters;
  // optional per-row closest-hit segment counts, indexed by (y - band_row0) (nullptr = off)
  unsigned long long* row_counters;
};

enum KernelId { K_AOP = 1, K_POST = 2, K_AO = 3, K_PHONG = 4, K_HYBRID = 5 };

// Launch `program` (RT_PROG_* numbering) on `stream`.  all_spheres selects the specialised
// intersection loop.  Returns hipSuccess or the launch error.
hipError_t launch_program(int program, const FrameParams& p, bool all_spheres, hipStream_t stream);

// Device math self-test (rt_selftest_math).
hipError_t launch_selftest(int fn, const float* d_in, float* d_out, size_t n, hipStream_t stream);

}  // namespace rt
