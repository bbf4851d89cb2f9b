// rt_kernels.h — launch interface between the C-ABI shim and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

// Normals slot layout, shared by the kernels and the shim (rt_download_rect reads the slots
// directly): 1 = an xyz plane then a w plane (production), 0 = interleaved float4 (the round-2
// layout, A/B builds only; set it for both translation units or neither).
#ifndef RT_NRM_PLANES
#define RT_NRM_PLANES 1
#endif

namespace rt {

constexpr int kMaxFrames = 16;
constexpr int kMaxBatch = 32;  // frames per multi-frame Phong/hybrid launch
// Hybrid (mode 4) workgroups of kHyBW x kHyBW waves, each wave an 8x8 pixel tile; the tile
// schedule's units are these workgroups (rt_shim launch_sched).  2x2 (16x16 pixels, 4 waves).
// Round 5 A/Bs at (b), tables read through the caches: in row order 1x1 33.1, 2x1 33.6, 2x2 34.2,
// 4x1 33.7, 4x2 35.0 us per launch (profiles/r05o_*), but with the longest-first schedule 1x1
// (its order at 8x8 granularity) 28.3 vs 2x2 26.5 us (r05p_*).  Set for both translation units.
#ifndef RT_HY_BW
#define RT_HY_BW 2
#endif
constexpr int kHyBW = RT_HY_BW, kHyTile = 8 * RT_HY_BW;
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
  int pool_rot;              // AO: pools per rotation group (one row's; 0 = pools in row order; set at launch)
  int tile_run;              // post-process: tiles per XCD run (xcd_tile; set at launch)
  int post_sx, post_sy;      // post-process: super-tiles of post_sx x post_sy blocks per XCD visit (xcd_tile)
  float inv_spp, fW, fH;     // 1.0f / spp, (float)W, (float)H: host-computed wave-uniform constants
  float inv_W, inv_H;        // 1.0f / fW, 1.0f / fH (correctly rounded; div_rn_by)
  float hx, hy, hz;          // horizontal
  float vx, vy, vz;          // vertical
  float lx, ly, lz;          // llc_minus_campos
  float cx, cy, cz;          // camera_location
  float Lx, Ly, Lz;          // light_pos
  float4 bg;                 // background
  const float4* shapes;      // compact table [4][S]: geo, geo2, col, aux (rt_device.h)
  // derived from `shapes` by launch_program (sphere_table / plane_table below):
  const float4* sph;         // [S] sphere-only geometry: geo for spheres, NaN for every other shape
  const float4* planes;      // [nplanes][2]: (normal, bits(index)), (p0, 0) of the planes among [0, nobj)
  int nplanes;               // set by the host (rt_shim) from the header's shape ids
  // AO bounce-ray cluster culling (set by the host, rt_shim build_clusters; ncl = 0: off):
  const float4* clus;        // [ncl] (centre, R): every member sphere lies within R of the centre
  const unsigned long long* clmask;  // [1 + kMaxClusters][kClusterWords]: always-tested spheres, then members
  const float4* camrel;              // [S] (camera - centre, |camera - centre|^2 as the kernels' dot) per sphere
  int ncl;
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
  // multi-frame Phong/hybrid launch (mf_n > 0, gridDim.z = mf_n): frame j of the batch renders
  // into slot (mf_slot0 + j) % F (hist_pix) with light mf_light[j]; only frame mf_n - 1 writes
  // the image.  The shape table is the same for every frame of the batch.
  int mf_n, mf_slot0;
  float4 mf_light[kMaxBatch];
  // multi-frame AO launch (mode 2, gridDim.y = mf_n): frame j reads rand_buffer mf_rb[j * 2 spp ..]
  // and writes slot (mf_slot0 + j) % F (hist_pix / hist_nrm / hist_dep); the image by frame mf_n - 1
  const float4* mf_rb;
  // hybrid (mode 4) tile schedule (rt_shim hy_schedule): block (x, y) renders the 16x16 tile
  // tile_order[x + y * gridDim.x] (packed x | y << 16) when non-null, else tile (x, y); each wave
  // stores its bounce-round count at tile_cost[tile * 4 + wave] when non-null
  const unsigned* tile_order;
  unsigned* tile_cost;
};

// Bounce-ray cluster culling (AO later bounce rounds): at most kMaxClusters clusters (a wave-uniform
// u64 of kept clusters), member masks over the first kClusterWords * 64 spheres.
constexpr int kMaxClusters = 64;
constexpr int kClusterWords = 4;

// Device shape table of one header copy, in float4 units from its base (rt_shim fills it):
//   [0, 4S)          geo, geo2, col, aux        (rt_device.h "scene tables")
//   [4S, 5S)         sph: geo of spheres, NaN of other shapes (never accepted by sphere_candidate)
//   [5S, 7S)         planes: 2 float4 per plane, compacted, ascending index
//   [7S, 7S + 64)    clusters: (centre, R) per cluster
//   then (1 + 64) * 4 u64 cluster masks (the always-tested spheres, then each cluster's members)
//   then [S) camrel: per sphere (camera - centre, dot of it with itself), NaN for other shapes:
//        the camera rays' sphere tests without the per-lane subtraction and self dot (phong /
//        hybrid primary rays; the same float operations, done once per frame on the host)
//   then rand_buffer[2 spp]
__host__ __device__ constexpr size_t sphere_table(int S) { return (size_t)4 * S; }
__host__ __device__ constexpr size_t plane_table(int S) { return (size_t)5 * S; }
__host__ __device__ constexpr size_t cluster_table(int S) { return (size_t)7 * S; }
__host__ __device__ constexpr size_t cluster_mask_table(int S) { return cluster_table(S) + kMaxClusters; }
__host__ __device__ constexpr size_t camrel_table(int S) {
  return cluster_mask_table(S) + (size_t)(1 + kMaxClusters) * kClusterWords / 2;
}
__host__ __device__ constexpr size_t rand_table(int S) { return camrel_table(S) + (size_t)S; }
__host__ __device__ constexpr size_t table_vec4(int S, int spp) { return rand_table(S) + (size_t)2 * spp; }

enum KernelId { K_AOP = 1, K_POST = 2, K_AO = 3, K_PHONG = 4, K_HYBRID = 5 };

// Launch `program` (RT_PROG_* numbering) on `stream`.  Scenes with planes (p.nplanes > 0)
// take the plane-testing instantiations; every other shape but spheres and planes is never
// hit (eval_ray returns -1 for it, p_compute.glsl:121-138) and is skipped through the NaN
// entries of the sphere table.  Returns hipSuccess or the launch error.
hipError_t launch_program(int program, const FrameParams& p, hipStream_t stream);

// g-buffer layout conversion between the reference's [F][W][R] vec4 (x-major, y fastest:
// src/main.cpp:49-85 over a context's R rows) and the device slots of one array kind (0 pixels:
// [band_rows][W] float4; 1 normals: xyz plane + w plane; 2 depth: (x, y) plane + (z, w) plane),
// rows r0 .. r0 + R - 1 of the band; n = band_rows * W.  to_ref: slots -> ref, else ref -> slots.
struct GbufXfer {
  int W, R, r0, F, kind, to_ref;
  size_t n;
  float4* ref;
  float4* slot[kMaxFrames];
};
hipError_t launch_gbuf_convert(const GbufXfer& x, hipStream_t stream);

// Device math self-test (rt_selftest_math).
hipError_t launch_selftest(int fn, const float* d_in, float* d_out, size_t n, hipStream_t stream);

}  // namespace rt
