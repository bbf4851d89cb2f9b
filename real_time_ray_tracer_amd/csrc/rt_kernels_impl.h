// rt_kernels_impl.h — the gfx950 kernels of the per-pixel ray-scene hot path (device code and
// kernel templates), included by the production launcher (rt_kernels.hip) and by the A/B tools
// library (tools/ab/rt_kernels_ab.hip, make ablib).
//
//   phong_kernel     <- resources/p_compute.glsl   (mode 3)
//   hybrid_kernel    <- resources/h_compute.glsl   (mode 4)
//   ao_batch_kernel  <- resources/ao_compute.glsl  (mode 2) / aop_compute.glsl (mode 1 pass 1)
//   post_kernel      <- resources/aop_postprocessing.glsl (mode 1 pass 2)
//
// The reference dispatches W x H single-lane workgroups (local_size 1x1, p_compute.glsl:26).
// Here a 256-lane workgroup (4 wave64) owns a 16x16 pixel tile (modes 3/4, one lane per
// pixel), and a one-wave workgroup owns a pool of 256 pixel-samples (modes 1/2).  The sphere
// table is read on the scalar path with wave-uniform loads; camera rays are cone-culled per
// wave / pool.  Planes are tested after the spheres of each segment.  Per-sample AO results are
// combined in sample order, so the sum order matches the reference's sequential
// `result_color += ambient_occlusion(dir, aa)` (ao_compute.glsl:303-330).
//
// The kernel templates carry diagnostic parameters (ABL: timing ablations, section clocks and
// event counts; !ALLSPH: the unculled LDS-table Phong/hybrid kernels) that only the A/B tools
// library instantiates; the production launcher (launch_production below) never does.
#pragma once
#include <hip/hip_runtime.h>

#include "rt_device.h"
#include "rt_kernels.h"

namespace rt {

namespace {

constexpr int kBlock = 256;
constexpr float kGamma = 1.0f / 2.2f;  // p_compute.glsl:240

// Stage the first nobj entries of the four [S] tables into LDS as [4][nobj].
__device__ __forceinline__ void stage_shapes(const FrameParams& P, float4* lds) {
  const int n = P.nobj;
  for (int k = threadIdx.x; k < 4 * n; k += blockDim.x) {
    int tab = k / n, i = k - tab * n;
    lds[k] = P.shapes[(size_t)tab * P.S + i];
  }
}

__device__ __forceinline__ f3 primary_dir(const FrameParams& P, float hp, float vp) {
  // normalize(llc_minus_campos + hp*horizontal + vp*vertical), p_compute.glsl:235
  f3 a = mk(P.lx + hp * P.hx, P.ly + hp * P.hy, P.lz + hp * P.hz);
  return normalize(mk(a.x + vp * P.vx, a.y + vp * P.vy, a.z + vp * P.vz));
}

__device__ __forceinline__ float4 gamma_out(float r, float g, float b) {
  // pow(c, 1/2.2) as exp2(log2(c) / 2.2) on the hardware v_log_f32 / v_exp_f32: relative
  // error ~5e-6 at worst (|log2 c| <= 126), inside the 1e-4 output tolerance; outputs only,
  // never feeds control flow (0 -> 0, inf -> inf, NaN -> NaN as powf)
  auto gm = [](float c) { return __builtin_amdgcn_exp2f(kGamma * __builtin_amdgcn_logf(c)); };
  return make_float4(gm(r), gm(g), gm(b), 0.0f);
}

// pow(x, 500) of the specular term (p_compute.glsl:230, h_compute.glsl:266) for x = clamp(.., 0,
// 1), by squaring: x^500 = x^256 x^128 x^64 x^32 x^16 x^4, 13 multiplies instead of powf's
// extended-precision log/exp.  Each squaring at most doubles the relative error and adds half an
// ulp, so the result is within ~500 ulp (3e-5 relative) of x^500 while it is normal, and below
// 1e-38 (the tolerance's 1e-6 absolute slack) where intermediate powers go subnormal.  The term
// only feeds the colour (never control flow); 0 -> 0, 1 -> 1, NaN -> NaN as powf.
__device__ __forceinline__ float pow500(float x) {
  const float x2 = x * x, x4 = x2 * x2, x8 = x4 * x4, x16 = x8 * x8, x32 = x16 * x16, x64 = x32 * x32,
              x128 = x64 * x64, x256 = x128 * x128;
  return ((((x256 * x128) * x64) * x32) * x16) * x4;
}

// 8x8 pixels per wave (ray coherence inside a wave), BWX x BWY waves per block (16x16 pixels
// per 256-lane block by default); block tile (bx, by) of the trace rows.
template <int BWX = 2, int BWY = 2>
__device__ __forceinline__ void tile_xy(int& x, int& y, int row0, int bx, int by) {
  int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  x = bx * 8 * BWX + (wave % BWX) * 8 + (lane & 7);
  y = row0 + by * 8 * BWY + (wave / BWX) * 8 + (lane >> 3);
}
__device__ __forceinline__ void tile_xy(int& x, int& y, int row0) { tile_xy<2, 2>(x, y, row0, blockIdx.x, blockIdx.y); }

// Work counters for the algorithmic-FLOP roofline (only when P.counters is set).  Called by
// every lane of a wave with the wave converged; one atomic per counter per wave.
__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ unsigned wave_max(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor(v, o));
  return v;
}
// Float wave reductions over all 64 lanes on the DPP path (quad perms, row mirrors, row
// broadcasts), result read from lane 63 (wave-uniform).  The whole wave must be active.
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWMASK, 0xf, false));
}
template <typename Op>
__device__ __forceinline__ float wave_reduce_f(float v, Op op) {
  v = op(v, dpp_f<0xB1>(v));        // quad_perm [1,0,3,2]
  v = op(v, dpp_f<0x4E>(v));        // quad_perm [2,3,0,1]
  v = op(v, dpp_f<0x141>(v));       // row_half_mirror: 8 lanes
  v = op(v, dpp_f<0x140>(v));       // row_mirror: 16 lanes
  v = op(v, dpp_f<0x142, 0xA>(v));  // row_bcast:15 into rows 1, 3
  v = op(v, dpp_f<0x143, 0xC>(v));  // row_bcast:31 into rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_min_f(float v) { return wave_reduce_f(v, [](float a, float b) { return fminf(a, b); }); }
__device__ __forceinline__ float wave_max_f(float v) { return wave_reduce_f(v, [](float a, float b) { return fmaxf(a, b); }); }
__device__ __forceinline__ float wave_sum_f(float v) { return wave_reduce_f(v, [](float a, float b) { return a + b; }); }

__device__ __forceinline__ void count_work(const FrameParams& P, bool active, int y, unsigned segs, unsigned shadows) {
  if (P.row_counters && active) atomicAdd(&P.row_counters[y - P.band_row0], (unsigned long long)(segs + shadows));
  if (!P.counters) return;
  if (!active) segs = shadows = 0;
  unsigned n = wave_sum(active ? 1u : 0u), sg = wave_sum(segs), sh = wave_sum(shadows);
  unsigned slots = wave_max(segs + shadows) * 64u;  // lane slots spent in scene loops (divergence)
  if ((threadIdx.x & 63) == 0) {
    // kCounterSlots copies per counter, spread by wave id, so waves do not serialise on one
    // address; the host sums the slots
    unsigned long long* c = P.counters + ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kCounterSlots - 1));
    atomicAdd(&c[0 * kCounterSlots], (unsigned long long)n);
    atomicAdd(&c[1 * kCounterSlots], (unsigned long long)sg);
    atomicAdd(&c[2 * kCounterSlots], (unsigned long long)sh);
    atomicAdd(&c[3 * kCounterSlots], (unsigned long long)(sg + sh) * (unsigned long long)P.nobj);
    atomicAdd(&c[4 * kCounterSlots], (unsigned long long)slots * (unsigned long long)P.nobj);
  }
}

// Colour stores (g-buffer slot + image) non-temporal: written once, read by a later launch at
// the earliest.  Hybrid (b) 26.25 -> 25.78 us, post_kernel (d) 0.311 -> 0.293 ms, AO and Phong
// unchanged (profiles/r05u_*).  RT_NT_GBUF: the AO pass's normal and depth stores as well.
#ifndef RT_NT_STORE
#define RT_NT_STORE 1
#endif
#ifndef RT_NT_GBUF
#define RT_NT_GBUF 0
#endif
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_nt(float4* p, float4 c) {
  __builtin_nontemporal_store(f4v{c.x, c.y, c.z, c.w}, (f4v*)p);
}
__device__ __forceinline__ void store_color(const FrameParams& P, float4* out_pix, float4* image, int x, int y,
                                            float4 c) {
  float4* const po = out_pix + (size_t)(y - P.band_row0) * P.W + x;
  if (RT_NT_STORE) st_nt(po, c);
  else *po = c;
  if (image) {
    int r = y - P.img_row0;
    if (r >= 0 && r < P.img_rows) {
      float4* const pi = image + (size_t)r * P.W + x;
      if (RT_NT_STORE) st_nt(pi, c);
      else *pi = c;
    }
  }
}
__device__ __forceinline__ void store_color(const FrameParams& P, int x, int y, float4 c) {
  store_color(P, P.out_pix, P.image, x, y, c);
}

// The frame a Phong/hybrid block renders: its light, colour slot and image (multi-frame
// launches: frame blockIdx.z of the batch, see FrameParams::mf_n).
// Depth g-buffer slot layout: two planes of [band_rows][W] float2, (x, y) then (z, w).  The
// post-process reads only depth.x and depth.y (aop_postprocessing.glsl: the neighbour weights and
// the history test), so it reads 8 B per depth instead of 16; the AO pass writes both planes and
// reads both for its stale-depth pixels.  rt_download / rt_upload_gbuffer convert to the
// reference's vec4 layout.
__device__ __forceinline__ size_t dep_plane(const FrameParams& P) { return (size_t)P.band_rows * P.W; }
__device__ __forceinline__ void dep_store(float4* base, size_t n, size_t off, float4 d) {
  float2* p = (float2*)base;
  if (RT_NT_GBUF) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(f2v{d.x, d.y}, (f2v*)(p + off));
    __builtin_nontemporal_store(f2v{d.z, d.w}, (f2v*)(p + n + off));
    return;
  }
  p[off] = make_float2(d.x, d.y);
  p[n + off] = make_float2(d.z, d.w);
}
__device__ __forceinline__ float4 dep_load(const float4* base, size_t n, size_t off) {
  const float2* p = (const float2*)base;
  const float2 a = p[off], b = p[n + off];
  return make_float4(a.x, a.y, b.x, b.y);
}
__device__ __forceinline__ float2 dep_load_xy(const float4* base, size_t off) { return ((const float2*)base)[off]; }
// Normals g-buffer slot layout: a [band_rows][W] plane of xyz (12 B per pixel) then a
// [band_rows][W] plane of w (the hit flag, 4 B).  The post-process's temporal test reads only
// the history normals' xyz (aop_postprocessing.glsl:180), 12 B per history slot instead of 16;
// the pixel itself and its neighbours read both planes.  rt_download / rt_upload_gbuffer convert
// to the reference's vec4 layout.
// (RT_NRM_PLANES=0: interleaved float4, the round-2 layout, for A/B builds)
__device__ __forceinline__ void nrm_store(float4* base, size_t n, size_t off, float4 v) {
  if (!RT_NRM_PLANES) {
    base[off] = v;
    return;
  }
  float* p = (float*)base;
  if (RT_NT_GBUF) {
    __builtin_nontemporal_store(v.x, p + 3 * off);
    __builtin_nontemporal_store(v.y, p + 3 * off + 1);
    __builtin_nontemporal_store(v.z, p + 3 * off + 2);
    __builtin_nontemporal_store(v.w, p + 3 * n + off);
    return;
  }
  p[3 * off] = v.x;
  p[3 * off + 1] = v.y;
  p[3 * off + 2] = v.z;
  p[3 * n + off] = v.w;
}
__device__ __forceinline__ f3 nrm_load_xyz(const float4* base, size_t off) {
  if (!RT_NRM_PLANES) return xyz(base[off]);
  const float* p = (const float*)base;
  return mk(p[3 * off], p[3 * off + 1], p[3 * off + 2]);
}
__device__ __forceinline__ float nrm_load_w(const float4* base, size_t n, size_t off) {
  if (!RT_NRM_PLANES) return base[off].w;
  return ((const float*)base)[3 * n + off];
}
__device__ __forceinline__ float4 nrm_load(const float4* base, size_t n, size_t off) {
  const f3 v = nrm_load_xyz(base, off);
  return make_float4(v.x, v.y, v.z, nrm_load_w(base, n, off));
}

struct FrameDst {
  f3 light;
  float4* out_pix;
  float4* image;
};
// MF = false: a single-frame launch (mf_n = 0, the host's choice): the frame's light and
// destinations come straight from the kernel arguments, with no branch on mf_n, so a wave's
// first scalar loads issue together instead of one dependent round trip after another
template <bool MF = true>
__device__ __forceinline__ FrameDst frame_dst(const FrameParams& P, int j) {
  if (!MF || P.mf_n <= 0) return FrameDst{mk(P.Lx, P.Ly, P.Lz), P.out_pix, P.image};
  const float4 L = P.mf_light[j];
  return FrameDst{mk(L.x, L.y, L.z), (float4*)P.hist_pix[(P.mf_slot0 + j) % P.F], j == P.mf_n - 1 ? P.image : nullptr};
}
// Multi-frame launches of modes 3/4 (FrameParams::mf_n frames): each block renders its tile in
// frames blockIdx.z * FPB ... (up to FPB of them, one after another), so a launch dispatches FPB x
// fewer workgroups and stages its LDS tables once per tile, not once per frame.  Every frame's
// tile is traced and shaded in full.  Phong (config (a), short waves bound by the workgroup
// dispatch rate): FPB 4, +5% over 1 (2: +3%, 8: +0%); hybrid (config (b)): 1 (2: -1.3%,
// 4: -2.7%, 8: -17%; its waves are longer and the mirror bounces of a few tiles set the tail)
// (tools/explore/r02m.sh).
constexpr int kPhongFramesPerBlock = 4, kHybridFramesPerBlock = 1;
#ifndef RT_HY_TPB
#define RT_HY_TPB 1
#endif
constexpr int kHybridTilesPerBlock = RT_HY_TPB;  // tiles per hybrid block, one after another (A/B)

template <int FPB>
__device__ __forceinline__ int block_frames(const FrameParams& P, int& j0) {
  if (P.mf_n <= 0) {
    j0 = 0;
    return 1;
  }
  j0 = (int)blockIdx.z * FPB;
  return P.mf_n - j0 < FPB ? P.mf_n - j0 : FPB;
}

// ---------------------------------------------------------------------------------------
// Primary-ray cone culling (used by ao_batch_kernel, phong_kernel, hybrid_kernel).  Every primary ray starts at the camera
// and passes through the pool's pixel rectangle (jitter < 0.0834 px), so one cone bounds
// them.  A sphere whose line distance from every ray of the cone exceeds its radius by a
// float-error margin has a computed discriminant < 0 for every lane (-1 in the reference,
// never accepted) and is skipped.
// ---------------------------------------------------------------------------------------
constexpr float kInv6 = 1.0f / 6.0f;  // correctly rounded (div_rn_by)
constexpr int kPool = 256;
constexpr int kSetupCost = 24;
constexpr int kTailMaxObj = 128;  // split tail rounds stage the sphere table in LDS up to this size  // per-sample setup (hashes, directions, shading) in sphere-test units

// Float form of the same cull (no trig): cone axis a, cos/sin of the half-angle; a sphere
// with inflated radius r_eff (r_eff^2 = r^2 + 1e-5 (d^2 + r^2)) lies outside the forward and
// the backward cone iff |cos phi| < cos(theta + alpha), sin alpha = r_eff / d.  Float error
// (~1e-6) is covered by the 2e-5 slack on the cosine and the 1e-5 inflation.
// threadIdx.x & 63 recomputed at the point of use (volatile: not hoisted or shared)
__device__ __forceinline__ int lane_id_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

struct ConeF {
  float ax, ay, az, ct, st;
};

// The cone only has to be conservative, not bit-exact: it is built with the raw
// v_rcp/v_sqrt/v_rsq instructions (<= 1 ulp, ~1e-7 relative), far inside the 2e-5 cosine
// slack and the 1e-5 radius inflation.
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float fast_rsq(float x) { return __builtin_amdgcn_rsqf(x); }

__device__ inline ConeF pool_cone_f(const FrameParams& P, int xmin, int xmax, int ymin, int ymax) {
  const float iw = fast_rcp(P.fW), ih = fast_rcp(P.fH);
  const float hps[2] = {((float)xmin - 0.1f) * iw, ((float)xmax + 0.1f) * iw};
  const float vps[2] = {((float)ymin - 0.1f) * ih, ((float)ymax + 0.1f) * ih};
  f3 d[4];
  f3 sum = mk(0.0f, 0.0f, 0.0f);
  for (int k = 0; k < 4; ++k) {
    float hp = hps[k & 1], vp = vps[k >> 1];
    f3 v = mk(P.lx + hp * P.hx + vp * P.vx, P.ly + hp * P.hy + vp * P.vy, P.lz + hp * P.hz + vp * P.vz);
    d[k] = fast_rsq(dot(v, v)) * v;
    sum = sum + d[k];
  }
  const float il = fast_rsq(dot(sum, sum));
  ConeF c;
  c.ax = sum.x * il; c.ay = sum.y * il; c.az = sum.z * il;
  float ct = 1.0f;
  for (int k = 0; k < 4; ++k) ct = fminf(ct, c.ax * d[k].x + c.ay * d[k].y + c.az * d[k].z);
  ct = fminf(fmaxf(ct - 2e-5f, -1.0f), 1.0f);  // widen the cone a little (direction rounding)
  c.ct = ct;
  c.st = fast_sqrt(fmaxf(0.0f, 1.0f - ct * ct));
  return c;
}

__device__ inline bool cone_misses_f(const ConeF& c, float4 g, float cx, float cy, float cz) {
  float Lx = g.x - cx, Ly = g.y - cy, Lz = g.z - cz;
  float d2 = Lx * Lx + Ly * Ly + Lz * Lz, r2 = g.w * g.w;
  float reff2 = r2 + 1e-5f * (d2 + r2);
  if (!(d2 > reff2 * 1.01f + 1e-6f)) return false;  // camera inside / near the sphere: keep
  float id = fast_rsq(d2);
  float sa2 = reff2 * (id * id);
  float sa = fast_sqrt(sa2), ca = fast_sqrt(fmaxf(0.0f, 1.0f - sa2));
  float K = c.ct * ca - c.st * sa - 2e-5f;  // cos(theta + alpha), made smaller (conservative)
  if (!(K > 0.0f)) return false;
  float cphi = (c.ax * Lx + c.ay * Ly + c.az * Lz) * id;
  return fabsf(cphi) < K;
}

// First-bounce cone of a prepared batch (ao_batch_kernel).  The live lanes' bounce rays start
// at primary hit points of the batch's few pixels and go into a hemisphere about the hit
// normal (or around the mirror direction), so their origins lie in a small ball (centre o,
// radius rho) and their directions in a cone (axis a, half-angle theta).  A sphere is skipped
// for the whole batch when, for every such ray, the reference's test provably rejects it:
//  (1) every origin is clearly outside the sphere: |c - o| - rho - r > 1e-2 (|c - o| + rho);
//  (2) the forward cone from o misses the sphere inflated to r_eff + rho, r_eff^2 = r^2 +
//      1e-5 (Lmax^2 + r^2): beta > theta + alpha with sin alpha = (r_eff + rho) / |c - o|.
// A ray from p (|p - o| <= rho) that met B(c, r_eff) would give the ray from o with the same
// direction a point within rho of it, so by (2) every ray's forward half-line misses
// B(c, r_eff).  If its closest approach to c lies ahead, the line passes at distance >= r_eff
// and the exact discriminant is <= -1e-5 (Lmax^2 + r^2), > 10x the computed-discriminant
// error (~7e-7 Lmax^2): the computed del is < 0 (-1, never accepted).  If it lies behind, both
// real roots are negative and, by (1), the larger one is below -(|p - c| - r) <= -1e-2 Lmax,
// > 10x the computed-root error (sqrt of the del error, ~8.4e-4 Lmax): the computed roots are
// negative, never above the 1e-4 threshold.  NaN anywhere fails a comparison and keeps the
// sphere.  Must be called by every lane of the wave.
struct ConeB {
  float ox, oy, oz, rho, ax, ay, az, ct, st;
};

__device__ __forceinline__ ConeB bounce_cone(bool live, f3 p, f3 d, unsigned long long lm) {
  ConeB c;
  const int first = __builtin_ctzll(lm);
  c.ox = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.x), first));
  c.oy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.y), first));
  c.oz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p.z), first));
  const float ex = p.x - c.ox, ey = p.y - c.oy, ez = p.z - c.oz;
  const float e2 = wave_max_f(live ? ex * ex + ey * ey + ez * ez : 0.0f);
  const float sx = wave_sum_f(live ? d.x : 0.0f), sy = wave_sum_f(live ? d.y : 0.0f), sz = wave_sum_f(live ? d.z : 0.0f);
  c.rho = fast_sqrt(e2) * 1.0001f + 1e-6f * (fabsf(c.ox) + fabsf(c.oy) + fabsf(c.oz));
  const float s2 = sx * sx + sy * sy + sz * sz;
  const float il = fast_rsq(s2);
  c.ax = sx * il; c.ay = sy * il; c.az = sz * il;
  float ct = wave_min_f(live ? c.ax * d.x + c.ay * d.y + c.az * d.z : 1.0f) - 2e-5f;
  if (!(s2 > 1e-6f)) ct = -1.0f;  // directions cancel: no usable axis
  ct = fminf(fmaxf(ct, -1.0f), 1.0f);
  c.ct = ct;
  c.st = fast_sqrt(fmaxf(0.0f, 1.0f - ct * ct));
  return c;
}

__device__ __forceinline__ bool bounce_cone_misses(const ConeB& c, float4 g) {
  const float vx = g.x - c.ox, vy = g.y - c.oy, vz = g.z - c.oz;
  const float L = fast_sqrt(vx * vx + vy * vy + vz * vz);
  const float r = fabsf(g.w), Lmax = L + c.rho;
  if (!((L - c.rho - r) > 1e-2f * Lmax)) return false;  // (1)
  const float R = fast_sqrt(r * r + 1e-5f * (Lmax * Lmax + r * r)) * 1.00001f + c.rho;
  const float sa = R * fast_rcp(L), ca = fast_sqrt(fmaxf(0.0f, 1.0f - sa * sa));
  if (!(c.st * ca + c.ct * sa > 1e-5f)) return false;  // theta + alpha >= pi: the cone covers the sphere
  const float K = c.ct * ca - c.st * sa - 2e-5f;         // cos(theta + alpha), made smaller
  const float cphi = (c.ax * vx + c.ay * vy + c.az * vz) * fast_rcp(L);
  return cphi < K;  // (2)
}

// bounce_cone_misses plus the sphere's per-ray pre-test for the batch: with theta = 0 (the
// cone of ONE ray, around its own direction d) the same argument shows that a live lane
// whose direction has dot(d, (c - o) / |c - o|) < cos(alpha) - 2e-5 cannot accept the sphere
// (|d| = 1 within 3e-7 and u's fast-math error is ~1e-7, both far inside the 2e-5 slack).
// pt = (u, K) with K = cos(alpha) - 2e-5, or K = -2 (every lane tests) when (1) fails.
__device__ __forceinline__ bool bounce_cone_keep_pt(const ConeB& c, float4 g, float4& pt) {
  const float vx = g.x - c.ox, vy = g.y - c.oy, vz = g.z - c.oz;
  const float L = fast_sqrt(vx * vx + vy * vy + vz * vz);
  const float r = fabsf(g.w), Lmax = L + c.rho;
  pt = make_float4(0.0f, 0.0f, 0.0f, -2.0f);
  if (!((L - c.rho - r) > 1e-2f * Lmax)) return true;  // (1)
  const float R = fast_sqrt(r * r + 1e-5f * (Lmax * Lmax + r * r)) * 1.00001f + c.rho;
  const float il = fast_rcp(L);
  const float sa = R * il, ca = fast_sqrt(fmaxf(0.0f, 1.0f - sa * sa));
  const float ux = vx * il, uy = vy * il, uz = vz * il;
  if (sa < 1.0f) pt = make_float4(ux, uy, uz, ca - 2e-5f);
  if (!(c.st * ca + c.ct * sa > 1e-5f)) return true;
  const float K = c.ct * ca - c.st * sa - 2e-5f;
  const float cphi = c.ax * ux + c.ay * uy + c.az * uz;
  return !(cphi < K);  // (2)
}

// Bounce-ray cluster cull (ao_batch_kernel's later bounce rounds).  A cluster cb = (centre, R)
// holds spheres with |c_i - centre| + |r_i| <= R (rt_shim build_clusters).  The ray (p, d), |d|
// = 1 within 3e-7, provably accepts none of them when
//  (A) its line passes the centre at distance h > R' = R + 0.0032 (Lmax + R), Lmax = |p - centre|
//      + R >= |p - c_i|: then every member's line distance is h_i > r_i + sqrt(1e-5 (d_i^2 +
//      r_i^2)) >= r_eff (the cone culls' inflated radius, d_i = |p - c_i|), so the exact
//      discriminant is <= -1e-5 (d_i^2 + r_i^2), > 5x the computed one's float error:
//      the computed del is < 0 (-1 in the reference, never accepted).  The computed h^2 =
//      fmaf(-b, b, L2) is within ~1.3e-6 L2 of the exact one, covered by the 4e-6 L2 slack;
//  (B) or the ball lies behind the origin (d . (centre - p) < -R' - 1e-3 (u + R')) while the
//      origin is outside it (u - R' > 1e-2 (u + R'), u = |p - centre|): for every member the
//      closest approach is behind (b_i > 0 with margin) and the origin is outside it by more than
//      1e-2 (|p - c_i| + r_i), so both roots are negative by more than 10x the computed-root error
//      (bounce_cone_misses (1)): never above the 1e-4 threshold.
// NaN anywhere fails both tests and keeps the cluster.
#ifndef RT_TL_CLUSTERS
#define RT_TL_CLUSTERS 1
#endif
#ifndef RT_CL_MASKS
#define RT_CL_MASKS 1
#endif
#ifndef RT_GLOBAL_TAIL
#define RT_GLOBAL_TAIL 1  // config (e), 256 spheres: 140.6 -> 128.3 ms per frame (r03i)
#endif
#ifndef RT_CLUSTER_TAIL_MAX_G
#define RT_CLUSTER_TAIL_MAX_G 8
#endif
constexpr int kClusterTailMaxG = RT_CLUSTER_TAIL_MAX_G;  // split tail rounds with G <= this use the cluster cull
__device__ __forceinline__ bool cluster_may_hit(f3 p, f3 d, float4 cb) {
  const float vx = cb.x - p.x, vy = cb.y - p.y, vz = cb.z - p.z;
  const float L2 = fmaf(vz, vz, fmaf(vy, vy, vx * vx));
  const float b = fmaf(d.z, vz, fmaf(d.y, vy, d.x * vx));  // > 0: the centre lies ahead
  const float u = fast_sqrt(L2);
  const float Rp = fmaf(0.0032f, u + 2.0f * cb.w, cb.w);
  const bool line_miss = fmaf(-b, b, L2) > fmaf(Rp, Rp, 4e-6f * L2);
  const bool behind = (b + Rp) < -1e-3f * (u + Rp) && (u - Rp) > 1e-2f * (u + Rp);
  return !(line_miss || behind);
}
// The wave mask of the lanes (full exec mask) whose ray may hit the cluster: cluster_may_hit as
// three ballots of single compares, !line_miss & (!c1 | !c2), each a negated compare that is true
// on NaN (so NaN keeps the cluster, as above).  The compiler's ballot of the combined bool went
// through a v_cndmask + v_cmp pair per cluster.
__device__ __forceinline__ unsigned long long cluster_may_hit_mask(f3 p, f3 d, float4 cb) {
  const float vx = cb.x - p.x, vy = cb.y - p.y, vz = cb.z - p.z;
  const float L2 = fmaf(vz, vz, fmaf(vy, vy, vx * vx));
  const float b = fmaf(d.z, vz, fmaf(d.y, vy, d.x * vx));
  const float u = fast_sqrt(L2);
  const float Rp = fmaf(0.0032f, u + 2.0f * cb.w, cb.w);
  const unsigned long long nlm = __builtin_amdgcn_ballot_w64(!(fmaf(-b, b, L2) > fmaf(Rp, Rp, 4e-6f * L2)));
  const unsigned long long nc1 = __builtin_amdgcn_ballot_w64(!((b + Rp) < -1e-3f * (u + Rp)));
  const unsigned long long nc2 = __builtin_amdgcn_ballot_w64(!((u - Rp) > 1e-2f * (u + Rp)));
  return nlm & (nc1 | nc2);
}

// ---------------------------------------------------------------------------------------
// Planes (plane_eval_ray, p_compute.glsl:111-119) in the cone-culled kernels.  The spheres
// keep their culled, ascending scan over the sphere table (P.sph: planes and every other
// shape are NaN there, never accepted); the planes are tested after it from the compact plane
// table and merged by plane_candidate's lexicographic (t, index) rule, which is the result of
// the reference's ascending scan whatever the visiting order.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long uniform_mask(unsigned long long m) {
  return ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(m >> 32)) << 32) |
         (unsigned)__builtin_amdgcn_readfirstlane((unsigned)m);
}

// every plane of the scene
__device__ __forceinline__ void plane_pass(const FrameParams& P, f3 pos, f3 dir, float thr, float& t, int& ind) {
  for (int k = 0; k < P.nplanes; ++k) plane_candidate(pos, dir, P.planes[2 * k], P.planes[2 * k + 1], thr, t, ind);
}

// the planes k < 64 whose bit is set in the wave-uniform mask m, and every plane k >= 64
__device__ __forceinline__ void plane_pass_masked(const FrameParams& P, unsigned long long m, f3 pos, f3 dir, float thr,
                                                  float& t, int& ind) {
  while (m) {
    const int k = __builtin_ctzll(m);
    m &= m - 1;
    plane_candidate(pos, dir, P.planes[2 * k], P.planes[2 * k + 1], thr, t, ind);
  }
  for (int k = 64; k < P.nplanes; ++k) plane_candidate(pos, dir, P.planes[2 * k], P.planes[2 * k + 1], thr, t, ind);
}

// A plane that no camera ray of the cone can accept.  Every such ray starts at the camera, so
// its numerator dot(n, p0 - cam) is the same float on every lane (computed here by the same
// operations).  The ray's t = num / denom is accepted only if denom has num's sign and is
// outside (-0.001, 0.001); the denominators dot(n, d) of the cone's directions lie within
// |n| [cos(min(phi + theta, pi)), cos(max(phi - theta, 0))], phi = angle(n, axis).  With a
// 1e-4 |n| slack (the cone's float error is ~1e-6; the lanes' dot error ~3e-7 |n|) a plane
// outside that window for its sign is missed by every lane (-1 or a value <= 0, never accepted).
// NaN fails every comparison and keeps the plane.
__device__ __forceinline__ bool plane_cone_misses(const ConeF& c, float4 a, float4 b, f3 cam) {
  const f3 n = xyz(a);
  const float num = dot(n, xyz(b) - cam);
  if (num == 0.0f) return true;  // res = +-0 (or NaN): never above a threshold >= 0
  const float n2 = n.x * n.x + n.y * n.y + n.z * n.z;
  if (n2 == 0.0f) return true;  // denom = 0: the parallel case, -1
  const float nl = fast_sqrt(n2);
  const float cphi = (c.ax * n.x + c.ay * n.y + c.az * n.z) * fast_rcp(nl);
  const float sphi = fast_sqrt(fmaxf(0.0f, 1.0f - cphi * cphi));
  if (num > 0.0f) {  // accepted only with denom >= 0.001
    const float cmax = cphi > c.ct ? 1.0f : cphi * c.ct + sphi * c.st;
    return nl * (cmax + 1e-4f) < 0.001f;
  }
  if (num < 0.0f) {  // accepted only with denom <= -0.001
    const float cmin = cphi < -c.ct ? -1.0f : cphi * c.ct - sphi * c.st;
    return nl * (cmin - 1e-4f) > -0.001f;
  }
  return false;  // NaN
}

// wave-uniform mask of the planes k < 64 that the cone does not exclude
__device__ __forceinline__ unsigned long long plane_cone_mask(const FrameParams& P, const ConeF& cone, f3 cam) {
  const int k = lane_id_here();
  const bool keep = k < P.nplanes && !plane_cone_misses(cone, P.planes[2 * k], P.planes[2 * k + 1], cam);
  return uniform_mask(__ballot(keep));
}

// Closest hit of the camera rays of a pixel rectangle whose cone is `cone`: per 64-sphere
// word the wave culls the spheres lane-parallel, then tests the survivors in ascending index
// order, reading them on the scalar path (wave-uniform index).  PL: then the planes the cone
// does not exclude.  Same result as closest_hit.  Must be called by every lane of the wave.
// SKIP (timing ablation): cull only, no tests.
template <bool PL, bool SKIP = false>
__device__ __forceinline__ int closest_hit_cone(const FrameParams& P, const float4* __restrict__ geo, int nobj,
                                                const ConeF& cone, f3 cam, f3 dir, float thr, float& t_out,
                                                const float4* pre0 = nullptr) {
  float t = -1.0f;
  int ind = -1;
  const int lane = threadIdx.x & 63;
  // cam is the header's camera (P.cx, P.cy, P.cz): the survivors are tested from the per-frame
  // camera-relative rows (P.camrel: cam - centre and its self dot, computed on the host with the
  // same float operations), so each test skips the three subtractions and the self dot
  const float4* const cr = P.camrel;
  auto word = [&](int w, bool keep) {
    unsigned long long m = uniform_mask(__ballot(keep));
    const float4* const gw = geo + w;  // (unsigned row offset: one scalar shift per survivor)
    const float4* const cw = cr + w;
    while (m && !SKIP) {
      const unsigned j = (unsigned)pop_lowest(m);
      sphere_candidate_rel(dir, cw[j], gw[j].w, w + (int)j, thr, t, ind);
    }
  };
  int w = 0;
  if (pre0 && nobj > 0) {  // the first word's rows, already requested by the caller
    word(0, lane < nobj && !cone_misses_f(cone, *pre0, cam.x, cam.y, cam.z));
    w = 64;
  }
  for (; w < nobj; w += 64) {
    const int i = w + lane;
    word(w, i < nobj && !cone_misses_f(cone, geo[i], cam.x, cam.y, cam.z));
  }
  if (PL) plane_pass_masked(P, plane_cone_mask(P, cone, cam), cam, dir, thr, t, ind);
  t_out = t;
  return ind;
}

// The cone of the camera rays through this wave's 8x8 pixel tile (tile_xy of tile (bx, by)).
template <int BWX = 2, int BWY = 2>
__device__ __forceinline__ ConeF wave_tile_cone(const FrameParams& P, int bx, int by) {
  const int wave = threadIdx.x >> 6;
  const int x0 = bx * 8 * BWX + (wave % BWX) * 8, y0 = P.trace_row0 + by * 8 * BWY + (wave / BWX) * 8;
  return pool_cone_f(P, x0, x0 + 7, y0, y0 + 7);
}

// shadow_ray (p_compute.glsl:145-166) for the whole wave at once, all-sphere scenes: every
// shadow line passes (within ~3e-5) through the light, so the lines of the lanes that need
// one lie in a cone with its apex at the light.  Spheres outside that cone (radius inflated
// by 1e-4 plus cone_misses_f's margins) are missed by every line (-1, never an occluder); the
// rest are tested as shadow_lit does.  "Some occluder exists" does not depend on the order.
// Must be called by every lane of the wave (ballots and shuffles).
#ifndef RT_SHADOW_CONE_MIN
#define RT_SHADOW_CONE_MIN 8
#endif
constexpr int kShadowConeMinObj = RT_SHADOW_CONE_MIN;
// the binary64 occluder test of shadow_ray (p_compute.glsl:155-163) for one object's float t:
// t > 0.0001 and length(dvec3(t * l)) < len.  With |l| within 2^-18.8 of 1 (checked per ray, see
// shadow_bounds) the binary64 length is t |l| (1 +- 2^-51), so t < len (1 - 2^-12) and
// t > len (1 + 2^-12) (float products, each within 2^-24) decide the test exactly; only t within
// 2^-12 of len (an occluder at the light's distance) runs the binary64 sequence.
// (RT_SHADOW_FAST=0: the binary64 sequence for every t, A/B builds)
#ifndef RT_SHADOW_FAST
#define RT_SHADOW_FAST 0
#endif
struct ShadowBounds {
  float lo, hi;  // t < lo: occludes; t > hi: does not (finite bounds only when |l|^2 is within 2^-19 of 1)
};
__device__ __forceinline__ ShadowBounds shadow_bounds(f3 l, float len) {
  const float l2 = dot(l, l);  // within 3 ulps of |l|^2
  const bool ok = RT_SHADOW_FAST && fabsf(l2 - 1.0f) < 0x1p-19f;
  return ok ? ShadowBounds{len * (1.0f - 0x1p-12f), len * (1.0f + 0x1p-12f)} : ShadowBounds{0.0f, INFINITY};
}
__device__ __forceinline__ bool shadow_occludes(float tf, f3 l, double dlen, ShadowBounds sb) {
  if (!(tf > 0.0001f)) return false;  // (double)tf > (double)0.0001f, exactly
  if (tf < sb.lo) return true;
  if (tf > sb.hi) return false;
  const double t = (double)tf;
  const double dx = t * (double)l.x, dy = t * (double)l.y, dz = t * (double)l.z;
  return sqrt(fma(dz, dz, fma(dy, dy, dx * dx))) < dlen;
}
// PL: planes occlude too (any shape type does, p_compute.glsl:153); they are tested after the
// spheres ("some occluder exists" does not depend on the order).
template <bool PL>
__device__ __forceinline__ bool shadow_lit_cone(const FrameParams& P, const float4* __restrict__ geo, int n, f3 light,
                                                f3 pos, bool need, const float4* pre0 = nullptr) {
  const f3 lv = light - pos;
  const f3 l = normalize(lv);
  const float len = sqrtf(dot(lv, lv));
  const f3 np = pos + 0.01f * l;
  const double dlen = (double)len;
  const ShadowBounds sb = shadow_bounds(l, len);
  if (__ballot(need) == 0) return true;
  bool lit = true;
  if (PL)
    for (int k = 0; k < P.nplanes; ++k)
      if (need && lit && shadow_occludes(plane_eval(np, l, P.planes[2 * k], P.planes[2 * k + 1]), l, dlen, sb)) lit = false;
  if (n <= kShadowConeMinObj) {  // small scenes: the cone costs more than it saves
    for (int k = 0; k < n; ++k) {
      if (need && lit && shadow_occludes(sphere_eval_shadow(np, l, geo[k]), l, dlen, sb)) lit = false;
    }
    return lit;
  }
  // cone at the light over the directions -l of the lanes that need a shadow ray (DPP
  // reductions; the cone only has to contain every lane's direction, whatever the sum order)
  const float sx = wave_sum_f(need ? -l.x : 0.0f), sy = wave_sum_f(need ? -l.y : 0.0f),
              sz = wave_sum_f(need ? -l.z : 0.0f);
  const float il = __builtin_amdgcn_rsqf(sx * sx + sy * sy + sz * sz);
  ConeF cone;
  cone.ax = sx * il; cone.ay = sy * il; cone.az = sz * il;
  float cd = wave_min_f(need ? -(cone.ax * l.x + cone.ay * l.y + cone.az * l.z) : 1.0f);
  cd = fminf(fmaxf(cd - 2e-5f, -1.0f), 1.0f);
  cone.ct = cd;
  cone.st = __builtin_amdgcn_sqrtf(fmaxf(0.0f, 1.0f - cd * cd));
  const bool wide = !(cd > 0.05f);  // nearly a half-space: test everything
  const int lane = threadIdx.x & 63;
  auto word = [&](int w, bool keep) {
    unsigned long long m = uniform_mask(__ballot(keep));
    const float4* const gw = geo + w;
    while (m) {
      const unsigned j = (unsigned)pop_lowest(m);
      if (need && lit && shadow_occludes(sphere_eval_shadow(np, l, gw[j]), l, dlen, sb)) lit = false;
    }
  };
  auto keep_row = [&](float4 g) {
    return wide || !cone_misses_f(cone, make_float4(g.x, g.y, g.z, g.w + 1e-4f), light.x, light.y, light.z);
  };
  int w = 0;
  if (pre0) {  // the first word's rows, already requested by the caller (n > kShadowConeMinObj here)
    word(0, lane < n && keep_row(*pre0));
    w = 64;
  }
  for (; w < n; w += 64) {
    const int i = w + lane;
    word(w, i < n && keep_row(geo[i]));
  }
  return lit;
}

// ---------------------------------------------------------------------------------------
// mode 3 — p_compute.glsl:168-245
// ---------------------------------------------------------------------------------------
// shadow_ray over the sphere table (every lane on its own; the hybrid kernel's bounces), with
// the planes first when the scene has some (any order: "some occluder exists")
template <bool PL>
__device__ __forceinline__ bool shadow_lit_sph(const FrameParams& P, const float4* __restrict__ geo, int n, f3 light,
                                               f3 pos) {
  const f3 lv = light - pos;
  const f3 l = normalize(lv);
  const float len = sqrtf(dot(lv, lv));
  const f3 np = pos + 0.01f * l;
  const double dlen = (double)len;
  const ShadowBounds sb = shadow_bounds(l, len);
  if (PL)
    for (int k = 0; k < P.nplanes; ++k)
      if (shadow_occludes(plane_eval(np, l, P.planes[2 * k], P.planes[2 * k + 1]), l, dlen, sb)) return false;
  for (int i = 0; i < n; ++i)
    if (shadow_occludes(sphere_eval_shadow(np, l, geo[i]), l, dlen, sb)) return false;
  return true;
}

// The kernels below come in two families.  ALLSPH (production): the sphere table P.sph is
// read on the scalar path from global memory, the camera rays of each wave's 8x8 tile and
// their shadow rays are cone-culled, and PL adds the scene's planes (plane table, tested after
// the spheres).  !ALLSPH (A/B builds only): the whole shape table staged in LDS, every shape
// tested through eval_ray's id dispatch, no culling.
template <bool ALLSPH, bool PL, bool LT, int BWX = 2, int BWY = 2>
__device__ __forceinline__ void phong_tile(const FrameParams& P, const float4* lds, int bx, int by, const FrameDst& fd,
                                           const float4* __restrict__ gsph, const float4* __restrict__ gshp,
                                           const float4* pre0 = nullptr) {
  const int n = P.nobj;
  const float4* tab = (ALLSPH && !LT) ? gshp : lds;                       // geo | geo2 | col
  const float4* geo = (ALLSPH && !LT) ? gsph : (ALLSPH ? lds + 4 * n : lds);  // what the sphere tests read
  const int stride = (ALLSPH && !LT) ? P.S : n;
  const float4 *geo2 = tab + stride, *col = tab + 2 * stride;
  int x, y;
  tile_xy<BWX, BWY>(x, y, P.trace_row0, bx, by);
  const bool active = x < P.W && y < P.trace_row0 + P.trace_rows;
  const f3 cam = mk(P.cx, P.cy, P.cz), light = fd.light;
  const f3 dir = primary_dir(P, div_rn_by((float)x, P.fW, P.inv_W), div_rn_by((float)y, P.fH, P.inv_H));
  float t;
  int ind;
  if (ALLSPH) {
    const ConeF cone = wave_tile_cone<BWX, BWY>(P, bx, by);
    ind = closest_hit_cone<PL>(P, geo, n, cone, cam, dir, 0.0f, t, pre0);
  } else {
    ind = closest_hit<ALLSPH>(geo, geo2, n, cam, dir, 0.0f, t);
  }
  count_work(P, active, y, 1u, active && ind != -1 ? 1u : 0u);
  const bool need = active && ind != -1;
  bool lit_w = true;
  if (ALLSPH) lit_w = shadow_lit_cone<PL>(P, geo, n, light, cam + t * dir, need, pre0);  // every lane takes part
  if (!active) return;
  float r, g, b;
  if (ind == -1) {
    r = P.bg.x; g = P.bg.y; b = P.bg.z;
  } else {
    f3 curr = cam + t * dir;
    bool lit = ALLSPH ? lit_w : shadow_lit<ALLSPH>(geo, geo2, n, light, curr);
    int id = (ALLSPH && !PL) ? SHAPE_SPHERE : __float_as_int(geo2[ind].w);
    f3 nn = shape_normal(tab[ind], id, curr);
    float4 c = col[ind];
    if (lit) {
      f3 l = normalize(light - curr);
      float spec = pow500(gclamp(dot(normalize(l - dir), nn), 0.0f, 1.0f));
      float k = gclamp(dot(nn, l), 0.06f, 1.0f);
      r = c.x * k + spec; g = c.y * k + spec; b = c.z * k + spec;
    } else {
      r = c.x * 0.06f; g = c.y * 0.06f; b = c.z * 0.06f;
    }
  }
  // result_color = vec4(0) + phong(dir); gamma; w = 0
  store_color(P, fd.out_pix, fd.image, x, y, gamma_out(0.0f + r, 0.0f + g, 0.0f + b));
}

// LT (ALLSPH, scenes of at most kTabLdsMax objects): the block stages the shape tables and the
// sphere table in LDS once ([4][n] + [n] float4), so the culls, the survivors' tests, the shadow
// rays and the shading read LDS instead of making dependent global round trips, whose latency
// the few resident waves of these short kernels do not hide.
#ifndef RT_TAB_LDS_MAX
#define RT_TAB_LDS_MAX 128
#endif
constexpr int kTabLdsMax = RT_TAB_LDS_MAX;
__device__ __forceinline__ void stage_tables(const FrameParams& P, float4* lds) {
  const int n = P.nobj;
  stage_shapes(P, lds);
  for (int k = threadIdx.x; k < n; k += blockDim.x) lds[4 * n + k] = P.sph[k];
}

// (the sphere and shape tables lead the arguments: preloaded into SGPRs, as for hybrid_kernel)
template <bool ALLSPH, bool PL = false, bool LT = false, bool MF = true>
__global__ __launch_bounds__(kBlock) void phong_kernel(const float4* __restrict__ gsph, const float4* __restrict__ gshp,
                                                       FrameParams P) {
  extern __shared__ float4 lds[];
  if (!ALLSPH || LT) {
    if (LT) stage_tables(P, lds);
    else stage_shapes(P, lds);
    __syncthreads();
  }
  if constexpr (!MF) {  // single-frame launch (frame_dst<false>)
    // the lane's row of the first 64-sphere word, requested before anything else (in bounds for
    // any scene: the sphere table is followed by >= 64 rows of other tables, rt_kernels.h)
    const float4 g0 = gsph[threadIdx.x & 63];
    phong_tile<ALLSPH, PL, LT>(P, lds, blockIdx.x, blockIdx.y, frame_dst<false>(P, 0), gsph, gshp,
                               (ALLSPH && !LT) ? &g0 : nullptr);
    return;
  }
  int j0;
  const int nj = block_frames<kPhongFramesPerBlock>(P, j0);
#pragma unroll 1
  for (int j = 0; j < nj; ++j)
    phong_tile<ALLSPH, PL, LT>(P, lds, blockIdx.x, blockIdx.y, frame_dst(P, j0 + j), gsph, gshp);
}

// ---------------------------------------------------------------------------------------
// mode 4 — h_compute.glsl:186-321
// ---------------------------------------------------------------------------------------
// Mirror bounces (segments >= 1) of the live paths of a wave, one segment per round.  Few
// paths bounce (~3% of the pixels at config (b)), so a round usually has a handful of live
// lanes; then each live path gets a group of G = 64 / 2^ceil(log2 L) lanes: lane p of the group
// tests spheres p, p+G, ... and the group merges the partial closest hits (minimum t, lowest
// index on ties: exactly the ascending scan of h_compute.glsl:121-139), and likewise splits the
// segment's shadow ray ("some occluder exists" is order-free, p_compute.glsl:145-166).  With
// more than 32 live paths every lane traces its own.  Returns (for the owner lanes) t, ind, lit.
// Must be called by every lane of the wave; perm: this wave's 64-int LDS slice.
template <bool PL>
__device__ __forceinline__ void bounce_round(const FrameParams& P, const float4* __restrict__ geo, int n, f3 light,
                                             bool live, f3 pos, f3 dir, int* perm, float& t_out, int& ind_out,
                                             bool& lit_out) {
  const unsigned long long lm = __ballot(live);
  const int L = __popcll(lm);
  const int lane = threadIdx.x & 63;
  if (L > 32) {
    float t = -1.0f;
    int ind = -1;
    bool lit = true;
    if (live) {
      ind = closest_hit_pf(geo, n, pos, dir, 0.001f, t);
      if (PL) plane_pass(P, pos, dir, 0.001f, t, ind);
      if (ind != -1) lit = shadow_lit_sph<PL>(P, geo, n, light, pos + t * dir);
    }
    t_out = t;
    ind_out = ind;
    lit_out = lit;
    return;
  }
  int c = 0;
  while ((1 << c) < L) ++c;
  const int G = 64 >> c;  // the largest power of 2 with G * L <= 64
  const int rk = __builtin_amdgcn_mbcnt_hi((unsigned)(lm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)lm, 0u));
  if (live) perm[rk] = lane;
  __builtin_amdgcn_wave_barrier();
  const int g = lane / G, pl = lane - g * G;
  const bool act = g < L;
  const int owner = act ? perm[g] : lane;
  __builtin_amdgcn_wave_barrier();
  const f3 o = mk(__shfl(pos.x, owner), __shfl(pos.y, owner), __shfl(pos.z, owner));
  const f3 d = mk(__shfl(dir.x, owner), __shfl(dir.y, owner), __shfl(dir.z, owner));
  float t = -1.0f;
  int ind = -1;
  if (act)
    for (int i = pl; i < n; i += G) sphere_candidate(o, d, geo[i], i, 0.001f, t, ind);
  for (int m = 1; m < G; m <<= 1) {  // every lane of the group ends with the group's result
    const float tb = __shfl_xor(t, m);
    const int ib = __shfl_xor(ind, m);
    const bool take = ib >= 0 && (ind < 0 || tb < t || (tb == t && ib < ind));
    t = take ? tb : t;
    ind = take ? ib : ind;
  }
  if (PL && act) plane_pass(P, o, d, 0.001f, t, ind);  // same planes, same result on every group lane
  // the segment's shadow ray, split the same way (the owner's hit point, same float ops)
  bool occ = false;
  if (act && ind != -1) {
    const f3 curr = o + t * d;
    const f3 lv = light - curr;
    const f3 l = normalize(lv);
    const float len = sqrtf(dot(lv, lv));
    const f3 np = curr + 0.01f * l;
    const double dlen = (double)len;
    const ShadowBounds sb = shadow_bounds(l, len);
    if (PL)
      for (int k = pl; k < P.nplanes && !occ; k += G)
        occ = shadow_occludes(plane_eval(np, l, P.planes[2 * k], P.planes[2 * k + 1]), l, dlen, sb);
    for (int i = pl; i < n && !occ; i += G) occ = shadow_occludes(sphere_eval_shadow(np, l, geo[i]), l, dlen, sb);
  }
  unsigned oc = occ ? 1u : 0u;
  for (int m = 1; m < G; m <<= 1) oc |= (unsigned)__shfl_xor((int)oc, m);
  const int src = live ? rk * G : lane;
  t_out = __shfl(t, src);
  ind_out = __shfl(ind, src);
  lit_out = __shfl((int)oc, src) == 0;
}

// ABL (A/B builds only, timing ablations): 1 = no shadow rays, 2 = no scene tests at all,
// 3 = primary cull only, 5 = no bounce segments, 6 = bounces without the split rounds
template <bool ALLSPH, bool PL, bool LT, int ABL = 0, int BWX = 2, int BWY = 2>
__device__ __forceinline__ void hybrid_tile(const FrameParams& P, const float4* lds, int* perm, int bx, int by,
                                            const FrameDst& fd, const float4* __restrict__ gsph,
                                            const float4* __restrict__ gshp, const float4* pre0 = nullptr) {
  const int n = P.nobj;  // !ALLSPH or LT: LDS tables (see phong_kernel)
  const float4* tab = (ALLSPH && !LT) ? gshp : lds;
  const float4* geo = (ALLSPH && !LT) ? gsph : (ALLSPH ? lds + 4 * n : lds);
  const int stride = (ALLSPH && !LT) ? P.S : n;
  const float4 *geo2 = tab + stride, *col = tab + 2 * stride, *aux = tab + 3 * stride;
  int x, y;
  tile_xy<BWX, BWY>(x, y, P.trace_row0, bx, by);
  const bool active = x < P.W && y < P.trace_row0 + P.trace_rows;
  const f3 light = fd.light;
  const unsigned long long tstart = ABL == 7 ? __builtin_amdgcn_s_memrealtime() : 0;
  f3 pos = mk(P.cx, P.cy, P.cz);
  f3 dir = primary_dir(P, div_rn_by((float)x, P.fW, P.inv_W), div_rn_by((float)y, P.fH, P.inv_H));
  float arefl = 0.0f;          // array[2].w
  float rr = 0, rg = 0, rb = 0;  // result_color.rgb
  float c = 0.0f;
  unsigned nseg = 0, nshadow = 0;
  // hybrid_helper's shading of one segment's hit (or miss) plus hybrid's accumulation
  // (h_compute.glsl:241-295); returns true when the path stops
  auto segment = [&](int seg, float t, int ind, bool lit) -> bool {
    ++nseg;
    nshadow += ind == -1 ? 0u : 1u;
    float ar, ag, ab;
    bool stop;
    if (ind == -1) {
      ar = P.bg.x; ag = P.bg.y; ab = P.bg.z;
      stop = true;
    } else {
      // (ABL 9, timing ablation with ABL 5's single segment: the shading without its table loads)
      float4 att = ABL == 9 ? make_float4(0.5f, 0.5f, 0.5f, 0.0f) : col[ind];
      f3 curr = pos + t * dir;
      int id = (ALLSPH && !PL) ? SHAPE_SPHERE : __float_as_int(geo2[ind].w);
      f3 nn = ABL == 9 ? normalize(curr) : shape_normal(tab[ind], id, curr);
      if (lit) {
        f3 l = normalize(light - curr);
        float spec = pow500(gclamp(dot(normalize(l - dir), nn), 0.0f, 1.0f));
        float k = gclamp(dot(nn, l), 0.06f, 1.0f);
        ar = att.x * k + spec; ag = att.y * k + spec; ab = att.z * k + spec;
      } else {
        ar = att.x * 0.06f; ag = att.y * 0.06f; ab = att.z * 0.06f;
      }
      float refl = ABL == 9 ? 0.0f : 1.0f - aux[ind].y;
      if (refl < 0.001f) {
        stop = true;
      } else {
        stop = false;
        float dn = dot(dir, nn);
        dir = normalize(mk(dir.x - 2.0f * (dn * nn.x), dir.y - 2.0f * (dn * nn.y),
                           dir.z - 2.0f * (dn * nn.z)));
        pos = curr;
        arefl = refl;
      }
    }
    if (seg == 0) {
      c = arefl;
      rr = ar; rg = ag; rb = ab;
    } else {
      float den = 1.0f + c;
      rr = (rr + c * ar) / den;
      rg = (rg + c * ag) / den;
      rb = (rb + c * ab) / den;
      c = c * arefl;
    }
    return stop;
  };
  if (ALLSPH) {
    // segment 0: the camera rays of the wave's 8x8 tile and their shadow rays, cone-culled
    float t0 = -1.0f;
    int ind0 = -1;
    bool lit0 = true;
    const ConeF cone = wave_tile_cone<BWX, BWY>(P, bx, by);
    if (ABL != 2) ind0 = closest_hit_cone<PL, ABL == 3>(P, geo, n, cone, pos, dir, 0.001f, t0, pre0);
    if (ABL == 0 || ABL >= 4) lit0 = shadow_lit_cone<PL>(P, geo, n, light, pos + t0 * dir, active && ind0 != -1, pre0);  // every lane takes part
    bool live = active && !segment(0, t0, ind0, lit0);
    // segments 1 .. D-1: bounce rounds with the whole wave
    int rounds = 0;  // wave-uniform: the wave's cost beyond its camera rays (tile schedule)
    for (int seg = 1; seg < ((ABL == 5 || ABL == 9) ? 1 : P.D); ++seg) {
      if (__ballot(live) == 0) break;
      ++rounds;
      float t;
      int ind;
      bool lit = true;
      if (ABL == 6) {
        if (live) {
          ind = closest_hit_pf(geo, n, pos, dir, 0.001f, t);
          if (PL) plane_pass(P, pos, dir, 0.001f, t, ind);
          if (ind != -1) lit = shadow_lit_sph<PL>(P, geo, n, light, pos + t * dir);
        }
      } else {
        bounce_round<PL>(P, geo, n, light, live, pos, dir, perm, t, ind, lit);
      }
      if (live) live = !segment(seg, t, ind, lit);
    }
    if (P.tile_cost && (threadIdx.x & 63) == 0)  // (a vector store from lane 0)
      P.tile_cost[((unsigned)by * gridDim.x + (unsigned)bx) * (BWX * BWY) + (threadIdx.x >> 6)] = (unsigned)rounds;
  } else {
    for (int seg = 0; active && seg < P.D; ++seg) {  // helper depth D, D-1, ..., 1
      float t;
      const int ind = closest_hit<ALLSPH>(geo, geo2, n, pos, dir, 0.001f, t);
      const bool lit = ind == -1 || shadow_lit<ALLSPH>(geo, geo2, n, light, pos + t * dir);
      if (segment(seg, t, ind, lit)) break;
    }
  }
  count_work(P, active, y, nseg, nshadow);
  if (active) store_color(P, fd.out_pix, fd.image, x, y, gamma_out(0.0f + rr, 0.0f + rg, 0.0f + rb));
  if (ABL == 7) {  // per-wave timeline (tools/explore/wave_timeline.py): lane 0's pixel slot holds
    // (start, end) of the wave's s_memtime and its longest path in segments
    const unsigned mx = wave_max(active ? nseg : 0u);
    const unsigned long long tend = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0 && active)
      P.out_pix[(size_t)(y - P.band_row0) * P.W + x] =
          make_float4(__uint_as_float((unsigned)tstart), __uint_as_float((unsigned)tend), __uint_as_float(mx),
                      __uint_as_float((unsigned)(tstart >> 32)));
  }
}

// The schedule's order table and the sphere / shape tables lead the argument list: the build
// preloads the first kernel arguments into SGPRs (-mllvm -amdgpu-kernarg-preload-count, Makefile),
// so a wave's first loads (its tile, then the culls' sphere rows) need not wait for a kernarg load.
// (FrameParams, an aggregate, is never preloaded.)
template <bool ALLSPH, bool PL = false, bool LT = false, int ABL = 0, int BWX = 2, int BWY = 2, bool MF = true>
__global__ __launch_bounds__(64 * BWX * BWY) void hybrid_kernel(const unsigned* __restrict__ tord,
                                                                const float4* __restrict__ gsph,
                                                                const float4* __restrict__ gshp, unsigned gx,
                                                                FrameParams P) {
  extern __shared__ float4 lds[];
  __shared__ int hperm[64 * BWX * BWY];  // bounce_round's live-rank -> lane map, a slice per wave
  if (!ALLSPH || LT) {
    if (LT) stage_tables(P, lds);
    else stage_shapes(P, lds);
    __syncthreads();
  }
  if constexpr (kHybridTilesPerBlock == 2) {
    // A/B builds: two tiles per block, half the waves.  Block b takes the tiles at positions b and
    // n - 1 - b of the schedule's order (row order without one): one of the longest with one of
    // the shortest, so block durations stay even.  The grid is gx x ceil(gy / 2).
    const unsigned gx = gridDim.x, gy = (unsigned)(P.trace_rows + 8 * BWY - 1) / (8 * BWY), n = gx * gy;
    const unsigned b = blockIdx.x + blockIdx.y * gx;
#pragma unroll 1
    for (int t = 0; t < 2; ++t) {
      const unsigned u = t == 0 ? b : n - 1 - b;
      if (b > n - 1 - b || (t == 1 && u == b)) break;  // (block-uniform; blocks past n / 2 have no tiles)
      unsigned bx = u % gx, by = u / gx;
      if (tord) {
        const unsigned v = tord[u];
        bx = v & 0xffffu;
        by = v >> 16;
      }
      hybrid_tile<ALLSPH, PL, LT, ABL, BWX, BWY>(P, lds, hperm + 64 * (threadIdx.x >> 6), bx, by, frame_dst(P, blockIdx.z), gsph, gshp);
    }
  } else if constexpr (kHybridTilesPerBlock > 1) {  // A/B builds: TPB vertically adjacent tiles per block
#pragma unroll 1
    for (int t = 0; t < kHybridTilesPerBlock; ++t)
      hybrid_tile<ALLSPH, PL, LT, ABL, BWX, BWY>(P, lds, hperm + 64 * (threadIdx.x >> 6), blockIdx.x,
                                                 blockIdx.y * kHybridTilesPerBlock + t, frame_dst(P, blockIdx.z), gsph, gshp);
  } else if constexpr (kHybridFramesPerBlock == 1) {  // no frame loop (the loop form costs 3-4% at (b))
    // the host's tile schedule (longest first, from the previous frames' bounce rounds): the
    // few tiles whose mirror paths bounce for many rounds start early instead of setting the
    // launch's tail (config (b): 32.0 -> 25.4 us per frame with the reverse of row order, which
    // happens to put that scene's bouncing tiles first)
    // MF = false: the lane's row of the first 64-sphere word requested before the tile order (in
    // bounds for any scene: the sphere table is followed by >= 64 rows of other tables)
    const bool pre = !MF && ALLSPH && !LT;
    float4 g0;
    if (pre) g0 = gsph[threadIdx.x & 63];
    unsigned bx = blockIdx.x, by = blockIdx.y;
    if (tord) {
      const unsigned t = tord[blockIdx.x + blockIdx.y * gx];  // (gx = gridDim.x, a preloaded argument)
      bx = t & 0xffffu;
      by = t >> 16;
    }
    hybrid_tile<ALLSPH, PL, LT, ABL, BWX, BWY>(P, lds, hperm + 64 * (threadIdx.x >> 6), bx, by,
                                               frame_dst<MF>(P, blockIdx.z), gsph, gshp, pre ? &g0 : nullptr);
  } else {
    int j0;
    const int nj = block_frames<kHybridFramesPerBlock>(P, j0);
#pragma unroll 1
    for (int j = 0; j < nj; ++j)
      hybrid_tile<ALLSPH, PL, LT, ABL, BWX, BWY>(P, lds, hperm + 64 * (threadIdx.x >> 6), blockIdx.x, blockIdx.y,
                                                 frame_dst(P, j0 + j), gsph, gshp);
  }
}

// ---------------------------------------------------------------------------------------
// modes 1/2 pass 1 — ao_compute.glsl:143-339 (aop_compute.glsl:141-336)
// lane = (pixel, sample); ppb = blockDim / spp pixels per block, consecutive in a row.
// ---------------------------------------------------------------------------------------
enum { PRIM_HIT = 0, PRIM_MISS = 1, PRIM_EMISSIVE = 2 };

// ---------------------------------------------------------------------------------------
// Pooled AO (production, all scenes).  One wave per workgroup owns a pool of kPool pixel-samples
// (TP = kPool/spp consecutive pixels x spp samples).  New samples are prepared 64 at a time
// with the whole wave active: primary direction + hemisphere vector + primary hit
// over the culled set + first-hit shading.  Samples whose path ended at the primary hit are
// final at once; the live post-primary states are kept in the lanes that prepared them and
// handed to idle lanes by ds_bpermute whenever lanes run out of work.  Bounce rounds then
// run with (nearly) all lanes live, and no per-sample setup runs at partial utilisation.
// ---------------------------------------------------------------------------------------
// LDS layout of ao_batch_kernel, in bytes.  Every offset is a compile-time constant when spp
// is (SPPC), so the kernel then holds no LDS addresses in scalar registers.
struct BatchLds {
  int prec, sres, pstop, pkind, perm, cmask, rls, geol, total;
};
__host__ __device__ constexpr BatchLds batch_lds(int spp, int pool, int ntail, bool rls_lds = true) {
  const int TP = pool / spp > 0 ? pool / spp : 1, NS = TP * spp;
  BatchLds L{};
  L.prec = 0;                                   // [TP] float4: first-segment (normal, t) of sample 0
  L.sres = 16 * TP;                             // [3][NS] float: per-sample r, g, b (channel-major)
  L.pstop = L.sres + 12 * NS;                   // [TP] int: max (aa << 16 | stop) of the stop writes
  L.pkind = L.pstop + 4 * TP;                   // [TP] int
  L.perm = L.pkind + 4 * ((TP + 1) & ~1);       // [64] int: live rank -> lane of the prepared batch
  L.cmask = (L.perm + 256 + 7) & ~7;            // [32] u64: primary cull mask (nobj <= 2048)
  L.rls = (L.cmask + 8 * 32 + 15) & ~15;        // [2 spp] float4: rand_buffer
  L.geol = L.rls + (rls_lds ? 32 * spp : 0);   // [ntail] float4: sphere table (split tail rounds)
  L.total = L.geol + 16 * ntail;
  return L;
}

// geo: the sphere table (P.sph).  PL: the scene has planes, tested after the spheres of every
// segment (plane_candidate) and, for the primary rays, culled against the pool cone.
// MF: frame blockIdx.y of a multi-frame mode-2 launch (FrameParams::mf_rb): its own rand_buffer
// and slot buffers, the image by the launch's last frame only.
// CL: the bounce-ray cluster cull of the later bounce rounds (P.ncl > 0); without it the rounds
// test every sphere.
// PTW (with PT, above kTailMaxObj spheres): the first bounce's pre-test rows one 64-sphere word at a
// time, the split tail rounds on the global table, rand_buffer read from global memory (RT_PT_WIDE).
// waves per SIMD the production AO kernel is compiled for (its register budget: 7 -> 72 VGPRs)
#ifndef RT_AO_MINW
#define RT_AO_MINW 7
#endif
// Scenes above kTailMaxObj spheres (config (e)): the first bounce's per-ray pre-test with its rows
// one 64-sphere word at a time in LDS, rand_buffer read from global memory to make room for them.
// Before, every cone survivor (95 of 256 per batch at (e)) ran the exact test; the pre-test leaves
// ~15 that some lane passes (tools/explore/b1_pairs_sim.py).  Config (e) 121.5 -> 97.3 ms per
// launch, bit-identical (profiles/r06t_*).  0 = the exact tests on every survivor (A/B builds).
#ifndef RT_PT_WIDE
#define RT_PT_WIDE 1
#endif
// the batched first bounce's exact tests deferred and merged over survivors with disjoint
// pre-test masks (see the survivor loop): (d) 2.439 -> 2.414 ms, (c) 0.738 -> 0.730 ms
// (profiles/r05z3_*); 0 = one exact pass per survivor that some lane passes (A/B builds)
#ifndef RT_B1_DEFER
#define RT_B1_DEFER 1
#endif
// The batched first bounce at wave issue priority 1 (s_setprio), every other phase at 0: among
// the ready waves of a SIMD, those in the first bounce's latency-bound survivor loop issue first.
// Per launch (d) 2.382 -> 2.349 ms, (c) 0.707 -> 0.698, (e) 93.0 -> 91.4; pipelined (d) frames
// 2.172 -> 2.141 ms over three alternating rounds; images identical.  The later bounce rounds at
// priority 1 too: level or worse; all of prepare(): worse pipelined (profiles/r06pm_*).
#ifndef RT_B1_PRIO
#define RT_B1_PRIO 1
#endif
// The pool's start (its LDS set-up, the rand_buffer copy and the primary cone cull: two dependent
// global-load round trips) at priority 1 as well, so a new wave's loads issue ahead of the
// resident waves' arithmetic: per launch (d) 2.441 -> 2.407 ms, (c) 0.714 -> 0.703, pipelined (d)
// frames 2.144-2.154 -> 2.139-2.148 ms on top of RT_B1_PRIO; the split tail rounds at priority 1
// instead: per launch -1.8% but pipelined frames +0.3% (profiles/r06px_*).
#ifndef RT_START_PRIO
#define RT_START_PRIO 1
#endif
#ifndef RT_B1_CREAD
#define RT_B1_CREAD 1
#endif
constexpr int kAoMinWaves = RT_AO_MINW;
template <int MINW, bool LAZY = true, int POOL = kPool, int ABL = 0, bool TAIL = false, bool B1 = false,
          int SPPC = 0, bool PT = false, bool CNT = true, bool PL = false, bool MF = false, bool CL = true, int DC = 0,
          bool CLON = false, bool PTW = false>
__global__ __launch_bounds__(64, MINW) void ao_batch_kernel(FrameParams P, const float4* __restrict__ geo) {
  if (RT_START_PRIO) __builtin_amdgcn_s_setprio(1);
  // CNT = false: the work counters compiled out (timed launches pass none): fewer live scalars
  unsigned long long* const cnts = CNT ? P.counters : nullptr;
  unsigned long long* const rowc = CNT ? P.row_counters : nullptr;
  extern __shared__ float4 lds[];
  const int spp = SPPC ? SPPC : P.spp, W = P.W, D = DC ? DC : P.D, nobj = P.nobj;
  // CLON: launched only with clusters (P.ncl > 0), so the rounds' plain full-scan path is not compiled
  const bool use_cl = CL && (CLON || P.ncl > 0);
  // this frame's buffers (the launch's frame unless MF)
  const int fj = MF ? (int)blockIdx.y : 0;
  const int fslot = MF ? (P.mf_slot0 + fj) % P.F : 0;
  float4* const f_nrm = MF ? (float4*)P.hist_nrm[fslot] : P.nrm;
  float4* const f_dep = MF ? (float4*)P.hist_dep[fslot] : P.dep;
  const float4* const f_nrm_prev = MF ? f_nrm : P.nrm_prev;  // sequential frames: the slot itself
  const float4* const f_dep_prev = MF ? f_dep : P.dep_prev;
  float4* const f_out = MF ? (float4*)P.hist_pix[fslot] : P.out_pix;
  float4* const f_img = MF ? (fj == P.mf_n - 1 ? P.image : nullptr) : P.image;
  const float4* const f_rb = MF ? P.mf_rb + (size_t)fj * 2 * spp : P.rb;
  const int TP = POOL / spp > 0 ? POOL / spp : 1;
  const int lane = threadIdx.x;
  const int NS = TP * spp;
  // PTW (scenes above kTailMaxObj spheres): the first bounce's pre-test rows one 64-sphere word at a
  // time in LDS, the split tail rounds on the global table, and rand_buffer read from global memory
  // (its LDS copy would not leave room for the rows at 7 waves per SIMD with spp 64)
  const BatchLds LO = batch_lds(spp, POOL, 0, !PTW);
  char* lbase = (char*)lds;
  float4* prec = (float4*)(lbase + LO.prec);
  float* sres = (float*)(lbase + LO.sres);
  int* pstop = (int*)(lbase + LO.pstop);
  int* pkind = (int*)(lbase + LO.pkind);
  int* perm = (int*)(lbase + LO.perm);
  unsigned long long* cmask = (unsigned long long*)(lbase + LO.cmask);
  float4* rls = (float4*)(lbase + LO.rls);
  if (!PTW)
    for (int k = lane; k < 2 * spp; k += 64) rls[k] = f_rb[k];
  for (int k = lane; k < TP; k += 64) pstop[k] = -1;
  // TAIL: the sphere table in LDS (per-lane sphere indices in the split tail rounds)
  float4* geol = (float4*)(lbase + LO.geol);  // [nobj] when TAIL && nobj <= kTailMaxObj
  // split tail rounds: the sphere table in LDS up to kTailMaxObj spheres; above (TAIL instantiations
  // launched without the LDS table), per-lane reads of the global table (L1/L2-resident)
  constexpr bool tail_lds = TAIL && PT && !PTW;  // launch_batch: the LDS-table instantiations (<= kTailMaxObj) have PT
  const bool tail_ok = TAIL;
  const float4* const tgeo = tail_lds ? geol : geo;
  // PT: the batched first bounce keeps its per-ray pre-test table in the same LDS rows, so the
  // sphere table is (re)staged only when a split tail round needs it
  const bool pt_ok = PT && B1 && (tail_lds || PTW);
  bool geol_valid = false;  // wave-uniform
  if (tail_lds && !pt_ok) {
    for (int k = lane; k < nobj; k += 64) geol[k] = geo[k];
    geol_valid = true;
  }
  // the cluster table and masks (rt_kernels.h layout: shapes + 7S, i.e. geo + 3S) read through the
  // read-only, non-aliased sphere-table pointer: their wave-uniform loads in the bounce rounds are
  // then scalar loads (through FrameParams they were vector loads, one memory round trip each)
  const float4* const clus = geo + (size_t)3 * P.S;
  const unsigned long long* const clm = (const unsigned long long*)(geo + (size_t)3 * P.S + kMaxClusters);
  // col[ind] / aux[ind] (rt_device.h scene tables) addressed from the sphere table (geo = shapes + 4S, launch_program) with a
  // per-lane offset the compiler cannot fold into a hoisted pointer: the two extra 64-bit base
  // pointers were the most reloaded of the kernel's scalar spills (a v_readlane pair each, per shade)
  auto col_at = [&](int ind) -> float4 {
    int o = ind - P.S;
    asm("" : "+v"(o));
    return geo[o - P.S];
  };
  auto aux_at = [&](int ind) -> float4 {
    int o = ind - P.S;
    asm("" : "+v"(o));
    return geo[o];
  };

  const long long npix = (long long)P.trace_rows * W;
  // pool of this workgroup
  unsigned pb = blockIdx.x;
  // XCD balance: workgroups are dealt round-robin to the 8 XCDs (b mod 8), so in row order an XCD
  // would take the same pool columns in every row (the same 16-px column stripes of the image);
  // rotating row r's pools by r (groups of pool_rot = pools per row) moves each XCD's columns by
  // one pool per row, so over 8 rows every XCD samples every column residue (a bijection on the
  // full groups; the last, partial group keeps its order).  Config (d) AO launch: -3%.
  if (P.pool_rot > 0) {
    const unsigned Q = (unsigned)P.pool_rot, r = pb / Q;
    if ((r + 1) * Q <= gridDim.x) {
      unsigned c = pb - r * Q + r % Q;
      c = c >= Q ? c - Q : c;
      pb = r * Q + c;
    }
  }
  const long long p0 = (long long)pb * TP;
  const int np = (int)(npix - p0 < TP ? npix - p0 : TP);
  const int total = np * spp;

  // ABL == 3: per-section wave clock (s_memtime) into the counters, timing ablation only
  unsigned long long tsec[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // 5..7: bounce rounds, sum ncull, prepares
  // ABL == 6: the same, with slots 5..7 timing the batched first bounce's cone + cull, survivor
  // loop and shading; ABL == 7: event counts of the first bounce and the bounce rounds instead
  // ABL == 8: the ABL == 3 sections with the later bounce rounds split: split tail rounds in slot
  // 5, full rounds in slot 3; slots 6 / 7 count full / tail rounds
  constexpr bool kLaps = ABL == 3 || ABL == 6 || ABL == 8;
  unsigned long long tmark = kLaps ? __builtin_amdgcn_s_memtime() : 0;
  auto lap = [&](int k) {
    if (kLaps) {
      unsigned long long now = __builtin_amdgcn_s_memtime();
      tsec[k] += now - tmark;
      tmark = now;
    }
  };
  // ---- frustum cull of the primary rays -------------------------------------------------
  const int yf = P.trace_row0 + (int)(p0 / W), xf = (int)(p0 % W);  // once per pool (scalar)
  // pixel lp of the pool: (xf + lp, yf), wrapped into the next row(s) when it passes W
  auto pool_xy = [&](int lp, int& x, int& y) {
    int xi = xf + lp;
    y = yf;
    if (xi >= W) {  // only pools that straddle a row end (none when TP divides W)
      int q = (int)((unsigned)xi / (unsigned)W);
      y += q;
      xi -= q * W;
    }
    x = xi;
  };
  const int yl = P.trace_row0 + (int)((p0 + np - 1) / W), xl = (int)((p0 + np - 1) % W);
  int ncull = 0;
  const int nwords = (nobj + 63) >> 6;
  unsigned long long pmask = 0;  // PL: planes k < 64 the pool's camera rays may hit (wave-uniform)
  {
    const ConeF cone = pool_cone_f(P, yf == yl ? xf : 0, yf == yl ? xl : W - 1, yf, yl);
    for (int w = 0; w < nwords; ++w) {
      int i = (w << 6) + lane;
      bool keep = i < nobj && !cone_misses_f(cone, geo[i], P.cx, P.cy, P.cz);
      if (PL) keep = keep && geo[i].x == geo[i].x;  // not a plane / other shape (NaN in the sphere table)
      unsigned long long m = __ballot(keep);
      ncull += __popcll(m);
      if (lane == 0) cmask[w] = m;
    }
    if (PL) {
      pmask = plane_cone_mask(P, cone, mk(P.cx, P.cy, P.cz));
      ncull += __popcll(pmask) + (P.nplanes > 64 ? P.nplanes - 64 : 0);
    }
  }
  __syncthreads();
  lap(0);
  if (RT_START_PRIO) __builtin_amdgcn_s_setprio(0);

  if (LAZY && ncull == 0) {
    // Empty frustum: every primary ray of the pool provably misses every sphere, so each
    // sample is "miss at the first segment": colour 1*background, depth.y = 0, zero g-buffer.
    // Same float sequence as the general path (sum of spp background values, then / spp).
    const float fa = (float)spp;
    float sr = 0.0f, sg = 0.0f, sb = 0.0f;
    for (int k = 0; k < spp; ++k) {
      sr = sr + 1.0f * P.bg.x; sg = sg + 1.0f * P.bg.y; sb = sb + 1.0f * P.bg.z;
    }
    const float4 col = gamma_out(sr / fa, sg / fa, sb / fa);
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int lp = lane; lp < np; lp += 64) {
      int x, y;
      pool_xy(lp, x, y);
      const size_t off = (size_t)(y - P.band_row0) * W + x;
      nrm_store(f_nrm, dep_plane(P), off, z);
      dep_store(f_dep, dep_plane(P), off, z);  // (0, 0, 0, 0) / AA
      store_color(P, f_out, f_img, x, y, col);
      if (rowc) atomicAdd(&rowc[y - P.band_row0], (unsigned long long)spp);  // ~free
    }
    if (cnts && lane == 0 && ABL < 3) {  // (ABL >= 3: the counters hold section clocks / events)
      unsigned long long* c = cnts + (blockIdx.x & (kCounterSlots - 1));
      atomicAdd(&c[0 * kCounterSlots], (unsigned long long)total);
      atomicAdd(&c[1 * kCounterSlots], (unsigned long long)total);
      atomicAdd(&c[3 * kCounterSlots], (unsigned long long)total * (unsigned long long)nobj);
    }
    return;
  }

  const f3 cam = mk(P.cx, P.cy, P.cz);
  const float4* rbuf = PTW ? f_rb : rls;
  // live path of this lane
  bool has = false;
  int item = 0, depth = 0;
  f3 pos = cam, dir = cam, hemi = cam;
  float rr = 1.0f, rg = 1.0f, rb = 1.0f;
  // prepared batch slot of this lane
  int bitem = 0;
  f3 bpos = cam, bdir = cam, bhemi = cam;
  float br = 1.0f, bg = 1.0f, bb = 1.0f;
  int next = 0, cursor = 0, nlive = 0, bdepth = D - 1;  // wave-uniform
  int b1cost = nobj;  // spheres the latest batched first bounce tested (row cost profile)
  unsigned nseg = 0;
  unsigned long long exec_tests = 0;

  const float inv_spp = P.inv_spp;
  // it / spp for pool items (< 2^16): exact via the float reciprocal (error << 0.5/spp)
  auto div_spp = [&](int it) { return SPPC ? (int)((unsigned)it / (unsigned)SPPC) : (int)(((float)it + 0.5f) * inv_spp); };
  // row cost profile (strip balancing), in sphere-test units: setup + culled primary + bounces
  auto finish = [&](int it, float r, float g, float b, float stopv, int segs) {
    sres[it] = r;
    sres[NS + it] = g;
    sres[2 * NS + it] = b;
    if (stopv >= 0.0f) {  // depth_buffer.y: the last writer in sample order wins
      const int lq = div_spp(it);
      atomicMax(&pstop[lq], ((it - lq * spp) << 16) | (int)stopv);
    }
    if (rowc) {
      int x, y;
      pool_xy(div_spp(it), x, y);
      atomicAdd(&rowc[y - P.band_row0],
                (unsigned long long)(kSetupCost + ncull + (segs >= 2 ? b1cost + (segs - 2) * nobj : 0)));
    }
  };

  // hit shading shared by primary and bounce segments; returns true when the path goes on
  // (written with one exit: the attenuation product, the kind store and finish() each appear
  // once, and the diffuse and mirror directions share their final normalize, so lanes that
  // take different cases do not run duplicated code)
  auto shade = [&](int ind, float t, f3& ps, f3& dr, f3 hm, float& r, float& g, float& b, int dpt, int it,
                   bool first) -> bool {
    const int lp = div_spp(it), aa = it - lp * spp;
    // a miss (ind == -1) reads the background: the host stores it as the colour table's row -1
    float4 att = col_at(ind);
    int kind = PRIM_MISS;
    bool go = false;
    if (ind != -1) {
      const float4 ax = aux_at(ind);
      // all-sphere scenes: the hit sphere's centre requested with its colour and flags, one memory
      // round trip (pinned here: the compiler would sink the load behind the emissive test)
      float4 gc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (!PL) {
        gc = geo[ind];
        asm volatile("" ::"v"(gc.x), "v"(gc.y), "v"(gc.z));
      }
      if (ax.x > 0.9f) {
        kind = PRIM_EMISSIVE;
      } else {
        kind = PRIM_HIT;
        f3 curr = cam + t * dr;  // sic: camera origin (ao_compute.glsl:210)
        f3 nn;
        if (PL) {  // ao_compute.glsl:211-218: the stored normal of a plane
          const float4 gi = P.shapes[ind];
          nn = __float_as_int(P.shapes[P.S + ind].w) == SHAPE_PLANE ? xyz(gi) : normalize(curr - xyz(gi));
        } else {
          nn = normalize(curr - xyz(gc));
        }
        if (aa == 0 && first) prec[lp] = make_float4(nn.x, nn.y, nn.z, t);
        if (ABL == 9) {  // instruction-budget ablation: the hit shading's arithmetic twice
          float z;
          asm volatile("v_mov_b32 %0, 0" : "=v"(z));
          const f3 c2 = cam + (t + z) * dr;
          const f3 n2 = normalize(c2 - (PL ? xyz(P.shapes[ind]) : xyz(gc)));
          const float d2 = dot(dr, n2);
          const f3 R2 = normalize(mk(dr.x - 2.0f * (d2 * n2.x), dr.y - 2.0f * (d2 * n2.y), dr.z - 2.0f * (d2 * n2.z)));
          const f3 X2 = normalize(ax.y > 0.999f ? hm + n2 : R2 + ax.y * hm);
          if (__float_as_uint(X2.x + X2.y + X2.z) == 0x7fc00001u) t = X2.x;
        }
        ps = curr;
        const float reflect = ax.y;
        f3 X;
        if (reflect > 0.999f) {
          X = hm + nn;
        } else {
          float dn = dot(dr, nn);
          f3 R = normalize(mk(dr.x - 2.0f * (dn * nn.x), dr.y - 2.0f * (dn * nn.y), dr.z - 2.0f * (dn * nn.z)));
          X = R + reflect * hm;
        }
        dr = normalize(X);
        go = dpt - 1 != 0;  // RECURSION_DEPTH non-emissive hits end without a stop write
      }
    }
    r = r * att.x; g = g * att.y; b = b * att.z;
    if (aa == 0 && first) pkind[lp] = kind;
    if (!go) finish(it, r, g, b, kind == PRIM_HIT ? -1.0f : (float)(D - dpt), kind == PRIM_HIT ? D : D - dpt + 1);
    return go;
  };

  // Prepare the next 64 samples with the whole wave.
  auto prepare = [&]() {
    bitem = next + lane;
    bool live = false;
    if (ABL == 3) { tsec[6] += (unsigned long long)ncull; tsec[7] += 1; }
    exec_tests += (unsigned long long)ncull;
    if (bitem < total) {
      const int lp = div_spp(bitem), aa = bitem - lp * spp;
      int x, y;
      pool_xy(lp, x, y);
      const float px = (float)x, py = (float)y;
      float hp, vp;
      {  // ao_compute.glsl:310-323; sample 0 is unjittered: px + 0 == px, so one path for
        // every lane (no divergent branch in the batch)
        float4 f = rbuf[2 * aa], s = rbuf[2 * aa + 1];
        float uw[2];
        grandom_n<2>({((s.x + px * f.z) - px) + f.x, s.z * px - (f.x * px) * f.z},
                     {((f.y + py * s.w) - py) + s.y, f.w * py - (s.y * py) * s.w}, uw);
        if (ABL == 4) {  // instruction-budget ablation: the jitter hashes twice
          float z, uw2[2];
          asm volatile("v_mov_b32 %0, 0" : "=v"(z));
          grandom_n<2>({((s.x + px * f.z) - px) + f.x + z, s.z * px - (f.x * px) * f.z + z},
                       {((f.y + py * s.w) - py) + s.y, f.w * py - (s.y * py) * s.w}, uw2);
          if (__float_as_uint(uw2[0]) == 0x7fc00001u && __float_as_uint(uw2[1]) == 0x7fc00001u) uw[0] = uw2[0];
        }
        float u = uw[0], w = uw[1];
        normalize2(u, w);
        const float jx = aa == 0 ? 0.0f : div_rn_by(u, 6.0f, kInv6) - 0.08333f;
        const float jy = aa == 0 ? 0.0f : div_rn_by(w, 6.0f, kInv6) - 0.08333f;
        hp = div_rn_by(px + jx, P.fW, P.inv_W);
        vp = div_rn_by(py + jy, P.fH, P.inv_H);
      }
      bdir = primary_dir(P, hp, vp);
      if (ABL == 10) {  // instruction-budget ablation: the primary setup after the hashes twice
        float z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        float u2 = hp + z, w2 = vp + z;
        normalize2(u2, w2);
        const float jx2 = aa == 0 ? 0.0f : div_rn_by(u2, 6.0f, kInv6) - 0.08333f;
        const float jy2 = aa == 0 ? 0.0f : div_rn_by(w2, 6.0f, kInv6) - 0.08333f;
        const f3 d2 = primary_dir(P, div_rn_by(px + jx2, P.fW, P.inv_W), div_rn_by(py + jy2, P.fH, P.inv_H));
        if (__float_as_uint(d2.x + d2.y + d2.z) == 0x7fc00001u) bdir.x = d2.y;
      }
      // get_pt_within_unit_sphere(aa), hoisted: it depends on aa and the pixel only, so it is
      // computed once per sample — after the primary hit when LAZY, for hits only (a non-emissive
      // hit uses it)
      auto hemisphere = [&]() {
        float4 f = rbuf[2 * aa], s = rbuf[2 * aa + 1];
        float abe[3];
        grandom_n<3>({f.x + px * s.z, f.z - px * s.z, s.x * px + s.z}, {f.y + py * s.w, f.w - py * s.w, s.y * py + s.w},
                     abe);
        if (ABL == 4) {  // instruction-budget ablation: the hemisphere hashes twice
          float z, abe2[3];
          asm volatile("v_mov_b32 %0, 0" : "=v"(z));
          grandom_n<3>({f.x + px * s.z + z, f.z - px * s.z + z, s.x * px + s.z + z},
                       {f.y + py * s.w, f.w - py * s.w, s.y * py + s.w}, abe2);
          if (__float_as_uint(abe2[0]) == 0x7fc00001u && __float_as_uint(abe2[2]) == 0x7fc00001u) abe[1] = abe2[1];
        }
        return normalize(mk(abe[0] * 2.0f - 1.0f, abe[1] * 2.0f - 1.0f, abe[2] * 2.0f - 1.0f));
      };
      if (!LAZY) bhemi = hemisphere();
      // the camera in VGPRs for the primary tests: with the uniform camera and the sphere both in
      // SGPRs, each of the three subtractions would need a copy first (one scalar operand per
      // vector instruction)
      f3 cv = cam;
      asm("" : "+v"(cv.x), "+v"(cv.y), "+v"(cv.z));
      bpos = cv;
      br = bg = bb = 1.0f;
      float t = -1.0f;
      int ind = -1;
      for (int w = 0; w < nwords; ++w) {
        unsigned long long m = cmask[w];
        m = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(m >> 32)) << 32) |
            (unsigned)__builtin_amdgcn_readfirstlane((unsigned)m);
        const float4* const gw = geo + (w << 6);  // (unsigned row offset: see the bounce rounds)
        while (m) {
          const unsigned j = (unsigned)pop_lowest(m);
          const int i = (w << 6) + (int)j;
          sphere_candidate(bpos, bdir, gw[j], i, 0.0001f, t, ind);
          if (ABL == 2) {  // timing ablation: the culled primary tests twice
            float z;
            asm volatile("v_mov_b32 %0, 0" : "=v"(z));
            float t2 = -1.0f;
            int i2 = -1;
            sphere_candidate(mk(bpos.x + z, bpos.y, bpos.z), bdir, geo[i], i, 0.0001f, t2, i2);
            if (i2 == 0x7fffffff) t = t2;
          }
        }
      }
      if (PL) plane_pass_masked(P, pmask, bpos, bdir, 0.0001f, t, ind);
      ++nseg;
      // (every hit, emissive or not: only non-emissive hits use it, but waiting for the hit's flags
      // first cost a memory round trip, and a wave with any non-emissive hit computes it anyway)
      if (LAZY && ind != -1) bhemi = hemisphere();
      live = shade(ind, t, bpos, bdir, bhemi, br, bg, bb, D, bitem, true);
    }
    bdepth = D - 1;
    b1cost = nobj;
    if (B1) {
      // The batch's live paths take their first bounce together, against the spheres their
      // bounce cone does not exclude (bounce_cone), in ascending index order as closest_hit.
      const unsigned long long lm1 = __ballot(live);
      if (lm1 != 0 && __popcll(lm1) >= P.b1_min) {
        lap(1);
        if (RT_B1_PRIO) __builtin_amdgcn_s_setprio(1);
        const ConeB cb = bounce_cone(live, bpos, bdir, lm1);
        float t = -1.0f;
        int ind = -1;
        b1cost = 0;
        if (ABL == 12) {  // instruction-budget ablation: the first bounce's cone and cull twice
          float z;
          asm volatile("v_mov_b32 %0, 0" : "=v"(z));
          const ConeB c2 = bounce_cone(live, mk(bpos.x + z, bpos.y, bpos.z), bdir, lm1);
          unsigned long long acc = 0;
          for (int w = 0; w < nwords; ++w) {
            const int i = (w << 6) + lane_id_here();
            float4 pt;
            const bool k2 = i < nobj && bounce_cone_keep_pt(c2, geo[i], pt);
            acc ^= __ballot(k2 && pt.w != 7.0f);
          }
          if (acc == 0x123456789abcdefull) b1cost = 1;
        }
        // RT_B1_DEFER: the exact tests of the survivors whose pre-test passes somewhere are
        // deferred and merged: survivors whose pass masks are disjoint share one exact-test
        // pass, each lane testing the one sphere it passed (ksel, read per lane); a survivor
        // whose mask meets the pending ones first runs them.  Every lane still meets its spheres
        // in ascending index order, so (t, ind) is the sequential scan's.
        // (Two pending spheres per lane, flushed when a lane would need a third: no better,
        // profiles/r05z4_*.)
        unsigned long long ru = 0;  // lanes with a pending sphere (wave-uniform)
        int ksel = 0;               // the pending sphere of each lane in ru
        // the pre-test's direction, NaN on the lanes that are not live (their pre-test then
        // fails, NaN >= K being false), so the ballot needs no live mask (RT_B1_DEFER)
        f3 tdir = bdir;
        if (RT_B1_DEFER && !live) tdir = mk(__int_as_float(0x7fc00000), __int_as_float(0x7fc00000), __int_as_float(0x7fc00000));
        auto flush = [&]() {
          const float4 gs = geo[ksel];
          sphere_candidate_if(bpos, bdir, gs, ksel, 0.0001f, t, ind, ru);
          ru = 0;
        };
        for (int w = 0; w < nwords; ++w) {
          // the lane index re-read here (not the kernel-wide one): otherwise the compiler keeps
          // this loop's per-lane addresses live across the whole pool and spills them to scratch
          const int i = (w << 6) + lane_id_here();
          bool keep;
          if (pt_ok) {
            float4 pt;
            keep = i < nobj && bounce_cone_keep_pt(cb, geo[i], pt);
            if (i < nobj) geol[PTW ? i - (w << 6) : i] = pt;  // (PTW: this word's rows only)
          } else {
            keep = i < nobj && !bounce_cone_misses(cb, geo[i]);
          }
          if (PL) keep = keep && geo[i].x == geo[i].x;  // planes are tested after the spheres
          unsigned long long m = __ballot(keep);
          m = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(m >> 32)) << 32) |
              (unsigned)__builtin_amdgcn_readfirstlane((unsigned)m);
          exec_tests += (unsigned long long)__popcll(m);
          b1cost += __popcll(m);
          if (ABL == 3) tsec[6] += (unsigned long long)__popcll(m) << 24;  // sections: first-bounce survivors
          if (pt_ok) {
            geol_valid = false;
            __syncthreads();  // the pre-test rows are written
            if (ABL == 6) lap(5);
            const float4* const qw = geol + (PTW ? 0 : (w << 6));  // this word's rows and spheres (fewer
            const float4* const gw = geo + (w << 6);   // scalar address operations per survivor)
            // the row's LDS address is formed by one vector instruction from the row base held in
            // a VGPR (the compiler builds the uniform address with two scalar instructions and
            // copies it to a VGPR), and the broadcast read waits at once, as the loop would
            int qbase;
            asm("v_mov_b32 %0, %1" : "=v"(qbase) : "s"((int)(size_t)((const char*)qw - lbase)));
            // (RT_B1_DEFER: the loop on every lane, the live lanes picked by lm1 in the ballots, so
            // the pending mask stays a scalar value across the loop)
            if (RT_B1_DEFER || live)
              while (m) {
                const int j = pop_lowest(m), k = (w << 6) + j;
#if RT_B1_CREAD
                // the row read in C from the VGPR row base: one v_lshl_add_u32 for the address, the
                // compiler's own wait (no inline-asm boundary, whose hazard padding cost an s_nop)
                const float4 q = *(const float4*)(lbase + (qbase + (j << 4)));
#else
                typedef float v4f __attribute__((ext_vector_type(4)));
                v4f qv;
                int j_addr_scratch;
                asm volatile("v_lshl_add_u32 %1, %2, 4, %3\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(qv), "=&v"(j_addr_scratch)
                             : "s"(j), "v"(qbase));
                const float4 q = make_float4(qv.x, qv.y, qv.z, qv.w);  // wave-uniform address: LDS broadcast
#endif
                const float4 g = gw[j];
                if (ABL == 7) {  // survivor iterations; with any pre-test pass; with any del >= 0 there
                  const bool pass = fmaf(bdir.z, q.z, fmaf(bdir.y, q.y, bdir.x * q.x)) >= q.w;
                  const f3 pmc = bpos - xyz(g);
                  const float bb = dot(bdir, pmc);
                  const float del = fmaf(g.w, g.w, fmaf(bb, bb, -dot(pmc, pmc)));
                  const unsigned long long pm = __ballot(pass), dm = __ballot(pass && del >= 0.0f);
                  tsec[0] += 1; tsec[1] += pm != 0; tsec[2] += dm != 0;
                  tsec[3] += (unsigned long long)__popcll(pm);
                }
                // the skip as a branch on the ballot (VCC), not an exec-mask save / restore per survivor
                const bool pass = fmaf(tdir.z, q.z, fmaf(tdir.y, q.y, tdir.x * q.x)) >= q.w;
                if (ABL == 5) {  // instruction-budget ablation: each survivor iteration twice
                  float z, t2 = t;
                  int i2 = ind;
                  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
                  const bool pass2 = fmaf(bdir.z + z, q.z, fmaf(bdir.y, q.y, bdir.x * q.x)) >= q.w;
                  const unsigned long long pm2 = __builtin_amdgcn_ballot_w64(pass2);
                  if (pm2 != 0) sphere_candidate_if(mk(bpos.x + z, bpos.y, bpos.z), bdir, g, k, 0.0001f, t2, i2, pm2);
                  if (i2 == 0x7fffffff) t = t2;
                }
                const unsigned long long pm = __builtin_amdgcn_ballot_w64(pass);
                if (RT_B1_DEFER) {
                  if (pm != 0) {
                    if (pm & ru) flush();
                    ru |= pm;
                    int kv = k;
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(ksel) : "v"(ksel), "v"(kv), "s"(pm));
                  }
                } else if (pm != 0) {
                  sphere_candidate_if(bpos, bdir, g, k, 0.0001f, t, ind, pm);
                }
              }
            if (ABL == 6) lap(6);
          } else if (live) {
            while (m) {
              const int k = (w << 6) + __builtin_ctzll(m);
              m &= m - 1;
              sphere_candidate(bpos, bdir, geo[k], k, 0.0001f, t, ind);
            }
          }
        }
        if (RT_B1_DEFER && ru != 0) flush();
        if (RT_B1_PRIO) __builtin_amdgcn_s_setprio(0);
        if (ABL == 7) { tsec[4] += 1; tsec[5] += (unsigned long long)__popcll(lm1); }
        if (live) {
          if (PL) plane_pass(P, bpos, bdir, 0.0001f, t, ind);
          ++nseg;
          live = shade(ind, t, bpos, bdir, bhemi, br, bg, bb, D - 1, bitem, false);
        }
        if (ABL == 6) lap(7);
        bdepth = D - 2;
        lap(4);  // sections: the batched first bounce (shares slot 4 with combine + stores)
      }
    }
    unsigned long long lm = __ballot(live);
    if (live) perm[__builtin_amdgcn_mbcnt_hi((unsigned)(lm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)lm, 0u))] = lane;
    nlive = __popcll(lm);
    cursor = 0;
    next = next + 64 < total ? next + 64 : total;
    __syncthreads();  // perm[] visible to the whole wave
  };

  for (;;) {
    // ---- hand prepared live states to idle lanes; prepare more when the batch is used up --
    for (;;) {
      unsigned long long need = __ballot(!has);
      if (need == 0) break;
      if (cursor >= nlive) {
        if (next >= total) break;
        lap(2);
        prepare();
        lap(1);
        continue;
      }
      int r = __builtin_amdgcn_mbcnt_hi((unsigned)(need >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)need, 0u));
      int take = __popcll(need) < nlive - cursor ? __popcll(need) : nlive - cursor;
      bool get = !has && r < take;
      int src = get ? perm[cursor + r] : lane;
      // every lane executes the shuffles (ds_bpermute reads the source lane's register)
      float sx = __shfl(bpos.x, src), sy = __shfl(bpos.y, src), sz = __shfl(bpos.z, src);
      float dx = __shfl(bdir.x, src), dy = __shfl(bdir.y, src), dz = __shfl(bdir.z, src);
      float hx = __shfl(bhemi.x, src), hy = __shfl(bhemi.y, src), hz = __shfl(bhemi.z, src);
      float cr = __shfl(br, src), cg = __shfl(bg, src), cb = __shfl(bb, src);
      int ci = __shfl(bitem, src);
      if (ABL == 11) {  // instruction-budget ablation: the hand-out's 13 shuffles twice
        int zi;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zi));
        const int s2 = src + zi;
        float q = __shfl(bpos.x, s2) + __shfl(bpos.y, s2) + __shfl(bpos.z, s2) + __shfl(bdir.x, s2) + __shfl(bdir.y, s2) +
                  __shfl(bdir.z, s2) + __shfl(bhemi.x, s2) + __shfl(bhemi.y, s2) + __shfl(bhemi.z, s2) + __shfl(br, s2) +
                  __shfl(bg, s2) + __shfl(bb, s2) + (float)__shfl(bitem, s2);
        if (__float_as_uint(q) == 0x7fc00001u) cr = q;
      }
      if (get) {
        pos = mk(sx, sy, sz);
        dir = mk(dx, dy, dz);
        hemi = mk(hx, hy, hz);
        rr = cr; rg = cg; rb = cb;
        item = ci;
        depth = bdepth;
        has = true;
      }
      cursor += take;
    }
    const unsigned long long hm = __ballot(has);
    if (hm == 0) break;
    lap(2);
    if (ABL == 3) tsec[5] += 1;
    // ---- split tail round: the pool has no fresh samples left and at most 32 paths are live.
    // Each live path gets a group of G = 64/2^ceil(log2 L) lanes; lane p of the group tests
    // spheres p, p+G, ... (ascending), and the group merges the partial results: minimum t,
    // lowest index on ties = exactly the sequential scan's result (ao_compute.glsl:183-194).
    const int L = __popcll(hm);
    if (tail_ok && next >= total && cursor >= nlive && L <= 32) {
      if (tail_lds && !geol_valid) {
        __syncthreads();
        for (int k = lane_id_here(); k < nobj; k += 64) geol[k] = geo[k];
        geol_valid = true;
      }
      int c = 0;
      while ((1 << c) < L) ++c;
      const int G = 64 >> c;  // the largest power of 2 with G * L <= 64
      const int rk = __builtin_amdgcn_mbcnt_hi((unsigned)(hm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)hm, 0u));
      if (has) perm[rk] = lane;
      __syncthreads();
      const int g = lane / G, pl = lane - g * G;
      const bool act = g < L;
      const int owner = act ? perm[g] : lane;
      const f3 o = mk(__shfl(pos.x, owner), __shfl(pos.y, owner), __shfl(pos.z, owner));
      const f3 d = mk(__shfl(dir.x, owner), __shfl(dir.y, owner), __shfl(dir.z, owner));
      float t = -1.0f;
      int ind = -1;
      if (use_cl && G <= kClusterTailMaxG) {
        // cluster cull over the round's L paths (cluster_may_hit): lane pl of group g tests
        // clusters pl, pl + G, ... for path g; the ballot folded over the groups gives the clusters
        // some path may hit.  Their spheres plus the always-tested ones, compacted in ascending
        // order into a byte list (LDS: the primary cull mask's words, dead once the pool's samples
        // are all prepared), are split over the group's lanes as before: the group merge below
        // returns the lexicographic minimum (t, index) over them = the full scan's result.
        unsigned long long kc = 0;
        for (int c0 = 0; c0 < P.ncl; c0 += G) {
          const int c = c0 + pl;
          const bool may = act && c < P.ncl && cluster_may_hit(o, d, clus[c]);
          unsigned long long b = __builtin_amdgcn_ballot_w64(may);
          for (int sh = 32; sh >= G; sh >>= 1) b |= b >> sh;
          kc |= (G == 64 ? b : (b & ((1ull << G) - 1))) << c0;
        }
        unsigned char* list = (unsigned char*)cmask;
        int cnt = 0;
        for (int w = 0; w < nwords; ++w) {
          unsigned long long m = clm[w];
          for (unsigned long long k2 = kc; k2;) m |= clm[(size_t)(1 + pop_lowest(k2)) * kClusterWords + w];
          const int ln = lane_id_here();
          if ((m >> ln) & 1ull)
            list[cnt + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                (unsigned char)((w << 6) + ln);
          cnt += __popcll(m);
        }
        __syncthreads();  // the list is written (one wave per workgroup)
        exec_tests += (unsigned long long)((P.ncl + G - 1) / G + (cnt + G - 1) / G);
        if (act) {
          // the next list entry is requested before this one's test: one LDS round trip per
          // sphere (entry, then the sphere row) instead of two dependent ones
          int i = list[pl < cnt ? pl : 0];
          for (int k = pl; k < cnt; k += G) {
            const float4 g = tgeo[i];
            const int inext = list[k + G < cnt ? k + G : cnt - 1];  // (no exec-mask branch around it)
            sphere_candidate(o, d, g, i, 0.0001f, t, ind);
            i = inext;
          }
        }
      } else if (act) {
        for (int i = pl; i < nobj; i += G) sphere_candidate(o, d, tgeo[i], i, 0.0001f, t, ind);
      }
      for (int m = 1; m < G; m <<= 1) {
        const float tb = __shfl_xor(t, m);
        const int ib = __shfl_xor(ind, m);
        const bool take = ib >= 0 && (ind < 0 || tb < t || (tb == t && ib < ind));
        t = take ? tb : t;
        ind = take ? ib : ind;
      }
      float tt = __shfl(t, rk * G);
      int ii = __shfl(ind, rk * G);
      if (!(use_cl && G <= kClusterTailMaxG)) exec_tests += (unsigned long long)((nobj + G - 1) / G);
      if (has) {
        if (PL) plane_pass(P, pos, dir, 0.0001f, tt, ii);
        ++nseg;
        has = shade(ii, tt, pos, dir, hemi, rr, rg, rb, depth, item, false);
        depth -= 1;
      }
      if (ABL == 8) tsec[7] += 1;
      lap(ABL == 8 ? 5 : 3);
      continue;
    }
    // ---- one bounce segment for every live path, against every sphere ------------------
    exec_tests += (unsigned long long)(use_cl ? P.ncl : nobj);
    if (ABL == 7) {  // later bounce rounds: sphere iterations, and those with any live lane's del >= 0
      tsec[6] += (unsigned long long)nobj;
      for (int i = 0; i < nobj; ++i) {
        const float4 g = geo[i];
        const f3 pmc = pos - xyz(g);
        const float bb = dot(dir, pmc);
        const float del = fmaf(g.w, g.w, fmaf(bb, bb, -dot(pmc, pmc)));
        tsec[7] += __ballot(has && del >= 0.0f) != 0;
      }
    }
    if (use_cl) {
      // cluster cull: a cluster is skipped when no live lane's ray may hit it (cluster_may_hit);
      // the spheres of the kept clusters plus the always-tested ones are visited in ascending
      // index order, so (t, ind) is the full scan's (ao_compute.glsl:183-194)
      // Four clusters per step, their records requested together (one scalar-load round trip per
      // four; slots past ncl are still inside the table, the cluster masks follow the 64 slots,
      // and their bits are dropped below).  Every lane tests (a lane without a path only sets a
      // bit that the live mask drops), so the loop runs with the full exec mask.
      unsigned long long kc = 0;
      for (int c = 0; c < P.ncl; c += 4) {
        const float4 c0 = clus[c], c1 = clus[c + 1], c2 = clus[c + 2], c3 = clus[c + 3];
#if RT_CL_MASKS
        // (the kept bits by scalar selects: the compiler's (b != 0) | ... << k went through VGPRs)
        const unsigned long long b0 = cluster_may_hit_mask(pos, dir, c0) & hm;
        const unsigned long long b1 = cluster_may_hit_mask(pos, dir, c1) & hm;
        const unsigned long long b2 = cluster_may_hit_mask(pos, dir, c2) & hm;
        const unsigned long long b3 = cluster_may_hit_mask(pos, dir, c3) & hm;
        // (bits 4..7 first and an opaque move before the shift: with bit 0 selected directly the
        // compiler builds it as a zero-extended bool through v_cndmask + v_readfirstlane)
        unsigned nib = (b0 ? 16u : 0u) | (b1 ? 32u : 0u) | (b2 ? 64u : 0u) | (b3 ? 128u : 0u);
        asm("" : "+s"(nib));
        kc |= (unsigned long long)(nib >> 4) << c;
#else
        const unsigned long long b0 = __builtin_amdgcn_ballot_w64(cluster_may_hit(pos, dir, c0)) & hm;
        const unsigned long long b1 = __builtin_amdgcn_ballot_w64(cluster_may_hit(pos, dir, c1)) & hm;
        const unsigned long long b2 = __builtin_amdgcn_ballot_w64(cluster_may_hit(pos, dir, c2)) & hm;
        const unsigned long long b3 = __builtin_amdgcn_ballot_w64(cluster_may_hit(pos, dir, c3)) & hm;
        kc |= (unsigned long long)((b0 != 0) | (b1 != 0) << 1 | (b2 != 0) << 2 | (b3 != 0) << 3) << c;
#endif
      }
      // (bits of the slots past ncl need no mask: their member words are zero, rt_shim build_clusters)
      float t = -1.0f;
      int ind = -1;
      if (ABL == 13) {  // instruction-budget ablation: the cluster cull twice
        float z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        const f3 p2 = mk(pos.x + z, pos.y, pos.z);
        unsigned long long k2 = 0;
        for (int c = 0; c < P.ncl; c += 4) {
          const unsigned long long b0 = cluster_may_hit_mask(p2, dir, clus[c]) & hm;
          const unsigned long long b1 = cluster_may_hit_mask(p2, dir, clus[c + 1]) & hm;
          const unsigned long long b2 = cluster_may_hit_mask(p2, dir, clus[c + 2]) & hm;
          const unsigned long long b3 = cluster_may_hit_mask(p2, dir, clus[c + 3]) & hm;
          unsigned nib = (b0 ? 16u : 0u) | (b1 ? 32u : 0u) | (b2 ? 64u : 0u) | (b3 ? 128u : 0u);
          asm("" : "+s"(nib));
          k2 |= (unsigned long long)(nib >> 4) << c;
        }
        if (k2 == 0x123456789abcdefull) t = 1.0f;
      }
      for (int w = 0; w < nwords; ++w) {
        unsigned long long m = clm[w];
        // the kept clusters' member words, up to four requested per round trip (a repeated index
        // when fewer are left: the same word OR-ed twice)
        for (unsigned long long k2 = kc; k2;) {
          const int a = pop_lowest(k2);
          const int b = k2 ? pop_lowest(k2) : a;
          const int e = k2 ? pop_lowest(k2) : a;
          const int f = k2 ? pop_lowest(k2) : a;
          m |= clm[(size_t)(1 + a) * kClusterWords + w] | clm[(size_t)(1 + b) * kClusterWords + w] |
               clm[(size_t)(1 + e) * kClusterWords + w] | clm[(size_t)(1 + f) * kClusterWords + w];
        }
        exec_tests += (unsigned long long)__popcll(m);
        if (has) {
          // (streaming the word's 4-sphere groups with a per-nibble skip, or loading 4 survivors
          // per wait, were slower: configs d / e +1.2% / +0% and +0% / +5%, r03f / r03i)
          if (ABL == 1) {  // instruction-budget ablation: the cluster rounds' tests twice
            float z, t2 = -1.0f;
            int i2 = -1;
            asm volatile("v_mov_b32 %0, 0" : "=v"(z));
            for (unsigned long long m2 = m; m2;) {
              const int i = (w << 6) + pop_lowest(m2);
              sphere_candidate(mk(pos.x + z, pos.y, pos.z), dir, geo[i], i, 0.0001f, t2, i2);
            }
            if (i2 == 0x7fffffff) t = t2;
          }
          // (the word's sphere pointer hoisted and the row index unsigned: the row's scalar load takes
          // it as a 32-bit byte offset instead of a sign-extended 64-bit address, 3 scalar
          // instructions fewer per survivor)
          const float4* const gw = geo + (w << 6);
          while (m) {
            const unsigned j = (unsigned)pop_lowest(m);
            sphere_candidate(pos, dir, gw[j], (w << 6) + (int)j, 0.0001f, t, ind);
          }
        }
      }
      if (has) {
        if (PL) plane_pass(P, pos, dir, 0.0001f, t, ind);
        ++nseg;
        has = shade(ind, t, pos, dir, hemi, rr, rg, rb, depth, item, false);
        depth -= 1;
      }
    } else if (has) {
      float t;
      int ind = closest_hit_pf(geo, nobj, pos, dir, 0.0001f, t);  // 4-sphere scalar groups (pf2: +0.9%)
      if (PL) plane_pass(P, pos, dir, 0.0001f, t, ind);
      if (ABL == 1) {  // timing ablation: the bounce tests twice
        float z, t2;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        int i2 = closest_hit_pf(geo, nobj, mk(pos.x + z, pos.y, pos.z), dir, 0.0001f, t2);
        if (i2 == 0x7fffffff) t = t2;
      }
      ++nseg;
      has = shade(ind, t, pos, dir, hemi, rr, rg, rb, depth, item, false);
      depth -= 1;
    }
    if (ABL == 8) tsec[6] += 1;
    lap(3);
  }
  lap(2);

  if (cnts && !kLaps && ABL != 7) {
    unsigned sg = wave_sum(nseg);
    if (lane == 0) {
      unsigned long long* c = cnts + (blockIdx.x & (kCounterSlots - 1));
      atomicAdd(&c[0 * kCounterSlots], (unsigned long long)total);
      atomicAdd(&c[1 * kCounterSlots], (unsigned long long)sg);
      atomicAdd(&c[3 * kCounterSlots], (unsigned long long)sg * (unsigned long long)nobj);
      atomicAdd(&c[4 * kCounterSlots], 64ull * exec_tests);
    }
  }
  __syncthreads();

  // ---- sample combine in aa order (ao_compute.glsl:303-339) ----------------------------
  for (int lp = lane; lp < np; lp += 64) {
    int x, y;
    pool_xy(lp, x, y);
    float sr = 0.0f, sg = 0.0f, sb = 0.0f;
    const float* ps = sres + lp * spp;
    if (SPPC % 4 == 0 && SPPC > 0) {
      // spp a multiple of 4 (constant): the pixel's samples read 4 at a time (ds_read_b128;
      // 16-byte aligned: lp * spp and NS are multiples of 4), summed in the same aa order
#pragma unroll 1
      for (int k = 0; k < SPPC; k += 4) {
        const float4 a = *(const float4*)(ps + k), g = *(const float4*)(ps + NS + k),
                     c = *(const float4*)(ps + 2 * NS + k);
        sr = sr + a.x; sr = sr + a.y; sr = sr + a.z; sr = sr + a.w;
        sg = sg + g.x; sg = sg + g.y; sg = sg + g.z; sg = sg + g.w;
        sb = sb + c.x; sb = sb + c.y; sb = sb + c.z; sb = sb + c.w;
      }
    } else {
#pragma unroll 1
      for (int k = 0; k < spp; ++k) {
        sr = sr + ps[k]; sg = sg + ps[NS + k]; sb = sb + ps[2 * NS + k];
      }
    }
    const int st = pstop[lp];
    const float ystop = st < 0 ? -1.0f : (float)(st & 0xffff);
    const float fa = (float)spp;
    const size_t off = (size_t)(y - P.band_row0) * W + x;
    const int kind = pkind[lp];
    float4 d;
    if (kind == PRIM_HIT) {
      float4 r0 = prec[lp];
      d = make_float4(r0.w, 0.0f, 0.0f, 1.0f);
      nrm_store(f_nrm, dep_plane(P), off, make_float4(r0.x, r0.y, r0.z, 1.0f));
    } else if (kind == PRIM_MISS) {
      d = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      nrm_store(f_nrm, dep_plane(P), off, d);
    } else {  // stale: the slot's previous normal / depth (an emissive first hit writes neither)
      d = dep_load(f_dep_prev, dep_plane(P), off);
      if (f_nrm_prev != f_nrm) nrm_store(f_nrm, dep_plane(P), off, nrm_load(f_nrm_prev, dep_plane(P), off));
    }
    if (ystop >= 0.0f) d.y = ystop;
    d.x = d.x / fa; d.y = d.y / fa; d.z = d.z / fa; d.w = d.w / fa;
    dep_store(f_dep, dep_plane(P), off, d);
    store_color(P, f_out, f_img, x, y, gamma_out(sr / fa, sg / fa, sb / fa));
  }
  if ((kLaps || ABL == 7) && cnts && lane == 0) {
    lap(4);
    unsigned long long* c = cnts + (blockIdx.x & (kCounterSlots - 1));
    for (int k = 0; k < 8; ++k) atomicAdd(&c[k * kCounterSlots], tsec[k]);
  }
}

// (the streaming AO kernel of rounds 1-2, rejected in DESIGN.md §5, was removed in round 2)

// ---------------------------------------------------------------------------------------
// mode 1 pass 2 — aop_postprocessing.glsl:57-208, with the documented snapshot semantics:
// neighbours read `raw` (slot f before filtering); right iff x+1<W, left iff x>0,
// up iff y+1<H, down iff y>=2.  Output goes to out_pix (the shim swaps it into slot f).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void post_pixel(const FrameParams& P, int x, int y, unsigned& filtered, unsigned& visited,
                                           unsigned& accepted);

// XCD-local tile order: workgroups are dealt round-robin to the 8 XCDs (linear block id L on
// XCD L mod 8), each with its own L2, so in plain row-major order horizontally adjacent tiles
// sit on different XCDs and every tile's left / right neighbour columns (whole 128-B lines of
// raw, normals and depth) are fetched into a second L2.  Here the tiles are cut into runs of R
// consecutive tiles in row-major order and the runs are dealt round-robin to the XCDs, so most
// left / right neighbour lines were just brought into the tile's own L2 by the tile before it.
// The host picks R (launch_params: a divisor of gx / 8 when gx is a multiple of 8, so the tile
// below a tile is on its XCD too; >= 4).  Runs must stay short: every XCD has to take an equal
// share of every part of the frame, since sky costs far less than ground (one contiguous band
// per XCD cut the bytes by 19% but made the launch 43% slower; runs of 1/8 row, 11% slower).
// L -> run (L / 8 / R) * 8 + L mod 8, offset (L / 8) mod R: a bijection on the first multiple
// of 8R tiles; the rest keep their order.
//
// Round 4: when the host finds super-tiles of SX x SY blocks that tile the grid (launch_params:
// SX, SY in {4, 2} dividing gx, gy), each XCD takes whole super-tiles, dealt round-robin (row-major
// blocks inside), so a block's upper and lower neighbour rows are mostly in its own L2 too:
// config (d) post-process PMC 1.085 -> 1.044x the byte model, per-launch and pipelined-frame
// times unchanged (profiles/r04o_ab_post_super_tiles.txt; 4 x 12: 1.035x, 2 x 6: 1.052x).
// L -> super-tile (L / 8 / SS) * 8 + L mod 8, block (L / 8) mod SS for the first multiple of 8
// super-tiles; the rest in order: a bijection.
__device__ __forceinline__ void xcd_tile(unsigned R, unsigned SX, unsigned SY, unsigned& bx, unsigned& by) {
  if (SX * SY > 1) {
    const unsigned gx = gridDim.x, L = blockIdx.x + blockIdx.y * gx, SS = SX * SY;
    const unsigned gsx = gx / SX, Q = gsx * (gridDim.y / SY), M = Q / 8 * 8;
    unsigned q, o;
    if (L < M * SS) {
      const unsigned j = L >> 3;
      q = (j / SS) * 8 + (L & 7u);
      o = j % SS;
    } else {
      const unsigned L2 = L - M * SS;
      q = M + L2 / SS;
      o = L2 % SS;
    }
    bx = (q % gsx) * SX + o % SX;
    by = (q / gsx) * SY + o / SX;
    return;
  }
  const unsigned gx = gridDim.x, n = gx * gridDim.y, L = blockIdx.x + blockIdx.y * gx;
  const unsigned M = R ? n / (8 * R) * (8 * R) : 0;
  unsigned t = L;
  if (L < M) {
    const unsigned j = L >> 3;
    t = ((j / R) * 8 + (L & 7u)) * R + j % R;
  }
  by = t / gx;
  bx = t - by * gx;
}

// Post-process tile shape: a wave covers kPostWX x (64 / kPostWX) pixels, a block kPostBWX x
// kPostBWY waves (RT_POST_* overrides: A/B builds).  Round 4: a wave is one 64-pixel row segment
// and a block 64 x 4 pixels (was 8 x 8 waves in 16 x 16 blocks): a wave's loads of an array are
// then whole contiguous lines (1 KiB of colour, 768 B of normals, 512 B of depth), its left /
// right neighbours are its own lanes' lines but for the two edge pixels, and the up / down rows
// are the block's other waves'.  Config (d): 0.350 -> 0.300 ms per launch, same process
// (128 x 2 blocks 0.317, row-major tile order 0.321; profiles/r04d_ab_post.txt)
#ifndef RT_POST_WX
#define RT_POST_WX 64
#endif
#ifndef RT_POST_BWX
#define RT_POST_BWX 1
#endif
#ifndef RT_POST_BWY
#define RT_POST_BWY 4
#endif
constexpr int kPostWX = RT_POST_WX, kPostWY = 64 / RT_POST_WX, kPostBWX = RT_POST_BWX, kPostBWY = RT_POST_BWY;
constexpr int kPostTileW = kPostWX * kPostBWX, kPostTileH = kPostWY * kPostBWY;
static_assert(kPostWX * kPostWY == 64 && kPostBWX * kPostBWY * 64 == kBlock, "post tile shape");

__global__ __launch_bounds__(kBlock) void post_kernel(FrameParams P) {
  int x, y;
  unsigned bx, by;
  xcd_tile((unsigned)P.tile_run, (unsigned)P.post_sx, (unsigned)P.post_sy, bx, by);
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    x = (int)bx * kPostTileW + (wave % kPostBWX) * kPostWX + lane % kPostWX;
    y = P.trace_row0 + (int)by * kPostTileH + (wave / kPostBWX) * kPostWY + lane / kPostWX;
  }
  const bool active = x < P.W && y < P.trace_row0 + P.trace_rows;
  unsigned filtered = 0, visited = 0, accepted = 0;
  if (active) post_pixel(P, x, y, filtered, visited, accepted);
  if (P.counters) {
    unsigned n = wave_sum(filtered), v = wave_sum(visited), a = wave_sum(accepted);
    if ((threadIdx.x & 63) == 0) {
      unsigned long long* c = P.counters + ((blockIdx.x * 4 + blockIdx.y * 4 * gridDim.x + (threadIdx.x >> 6)) &
                                            (kCounterSlots - 1));
      atomicAdd(&c[5 * kCounterSlots], (unsigned long long)n);
      atomicAdd(&c[6 * kCounterSlots], (unsigned long long)v);
      atomicAdd(&c[7 * kCounterSlots], (unsigned long long)a);
    }
  }
}

// History slots read ahead of the acceptance test (see post_pixel).  1: the next slot's keys and
// colour are in flight while a slot is tested.  2 needs 76 VGPRs, more than the 72 an AO wave
// holds, so a post-process wave no longer fits in the registers one retiring AO wave frees and
// pipelined frames got 8% slower (profiles/r03s_ab_post_prefetch.txt).
constexpr int kPostAhead = 1;
struct HistSlot {
  f3 n;
  float2 d;
  float4 p;
};
__device__ __forceinline__ HistSlot hist_load(const FrameParams& P, int cf, size_t off) {
  HistSlot h;
  h.n = nrm_load_xyz(P.hist_nrm[cf], off);
  h.d = dep_load_xy(P.hist_dep[cf], off);
  h.p = P.hist_pix[cf][off];
  return h;
}

__device__ __forceinline__ void post_pixel(const FrameParams& P, int x, int y, unsigned& filtered, unsigned& visited,
                                           unsigned& accepted) {
  const int W = P.W, f = P.frame, F = P.F;
  const size_t off = (size_t)(y - P.band_row0) * W + x;
  float4 color = P.raw[off];
  const size_t np = dep_plane(P);  // normals: xyz plane + w plane (nrm_store)
  if (nrm_load_w(P.nrm, np, off) > 0.99f) {
    filtered = 1;
    // Memory round trips, not bytes, are what this kernel costs in the pipelined frame: there it
    // runs beside the next frame's AO pass, and each resident post-process wave holds registers
    // an AO wave could use for as long as it waits on memory.  So the neighbours are requested in
    // one round trip, and history slots f-1, f-2, ... kPostAhead ahead of the acceptance test with
    // keys and colour together (the colour of the slot that fails is read and dropped): ~F + 2
    // round trips per filtered pixel instead of ~2F + 9 (pipelined frames 2.368 -> 2.305 ms,
    // profiles/r03u_ab_post_round_trips.txt).  The arithmetic is the reference's, in its order.
    const float2 cd = dep_load_xy(P.dep, off);
    const f3 nv = nrm_load_xyz(P.nrm, off);
    const float nd = cd.x, nb = cd.y;
    float4 acc = color;
    float den = 1.0f;
    const int band_end = P.band_row0 + P.band_rows;
    // GLSL order: up, down, left, right (line 173).  Every neighbour's flag, keys and colour are
    // requested together (an absent neighbour reads the pixel itself and is dropped).
    {
      size_t o[4];
      bool pr[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int xx = x + (k == 2 ? -1 : (k == 3 ? 1 : 0));
        int yy = y + (k == 0 ? 1 : (k == 1 ? -1 : 0));
        bool present = (k == 0) ? (y + 1 < P.H) : (k == 1) ? (y >= 2) : (k == 2) ? (x > 0) : (x + 1 < W);
        pr[k] = present && yy >= P.band_row0 && yy < band_end;
        const int xc = pr[k] ? xx : x, yc = pr[k] ? yy : y;  // (a select, not a branch on a shared load)
        o[k] = (size_t)(unsigned)((yc - P.band_row0) * W + xc);
      }
      float wn[4];
      f3 nn[4];
      float2 dd[4];
      float4 rv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        wn[k] = nrm_load_w(P.nrm, np, o[k]);
        nn[k] = nrm_load_xyz(P.nrm, o[k]);
        dd[k] = dep_load_xy(P.dep, o[k]);
        rv[k] = P.raw[o[k]];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // the neighbour weight (aop_postprocessing.glsl:82-171: 1 for a sky neighbour), branch-free
        // so the compiler keeps the loads above together
        const float normal_dot = dot(nv, nn[k]);
        const float depth_diff = 1.0f - gclamp(fabsf(nd - dd[k].x), 0.0f, 1.0f);
        const float bounces_diff = 1.0f - gclamp(fabsf(nb - dd[k].y) / 1.7f, 0.0f, 1.0f);
        const float wf = normal_dot * depth_diff * bounces_diff + 0.2f;
        const float wk = pr[k] ? (wn[k] < 0.001f ? 1.0f : wf) : 0.0f;
        const float4 v = pr[k] ? rv[k] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        acc.x = acc.x + wk * v.x; acc.y = acc.y + wk * v.y;
        acc.z = acc.z + wk * v.z; acc.w = acc.w + wk * v.w;
        den = den + wk;
      }
    }
    color = make_float4(acc.x / den, acc.y / den, acc.z / den, acc.w / den);
    // temporal, lines 177-201
    HistSlot ring[kPostAhead];
    int cf = f;
    int issued = 0;
#pragma unroll
    for (int k = 0; k < kPostAhead; ++k)
      if (k < F - 1) {
        cf = cf == 0 ? F - 1 : cf - 1;
        ring[k] = hist_load(P, cf, off);
        ++issued;
      }
    float4 cs = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float denominator = 0.9f;
    for (int i = 1; i < F; ++i) {
      const HistSlot h = ring[0];
#pragma unroll
      for (int k = 0; k + 1 < kPostAhead; ++k) ring[k] = ring[k + 1];
      if (issued < F - 1) {  // slot f-i-kPostAhead, in flight while slot f-i is tested
        cf = cf == 0 ? F - 1 : cf - 1;
        ring[kPostAhead - 1] = hist_load(P, cf, off);
        ++issued;
      }
      float normal_dot = dot(nv, h.n);
      float depth_diff = 1.0f - gclamp(fabsf(nd - h.d.x), 0.0f, 1.0f);
      float bounces_diff = 1.0f - gclamp(fabsf(nb - h.d.y) / 1.7f, 0.0f, 1.0f);
      float coeff = normal_dot * depth_diff * bounces_diff;
      ++visited;
      if (!(coeff > 0.85f)) break;
      ++accepted;
      cs.x = cs.x + coeff * h.p.x; cs.y = cs.y + coeff * h.p.y;
      cs.z = cs.z + coeff * h.p.z; cs.w = cs.w + coeff * h.p.w;
      denominator = denominator + coeff;
    }
    color = make_float4((color.x * 0.9f + cs.x) / denominator, (color.y * 0.9f + cs.y) / denominator,
                        (color.z * 0.9f + cs.z) / denominator, (color.w * 0.9f + cs.w) / denominator);
  }
  store_color(P, x, y, color);
}

// ---------------------------------------------------------------------------------------
// math self-test
// ---------------------------------------------------------------------------------------
__global__ void selftest_kernel(int fn, const float* __restrict__ in, float* __restrict__ out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (fn) {
    case 0: out[i] = det_sin(in[i]); break;
    case 9: out[i] = det_sin(__uint_as_float(__float_as_uint(in[0]) + (unsigned)i)); break;  // bit patterns in[0].., wrapping
    case 1: out[i] = grandom(in[2 * i], in[2 * i + 1]); break;
    case 2: out[i] = sqrt_rn(in[i]); break;
    case 6: {  // exhaustive sqrt_rn == sqrtf over bit patterns [i*per, (i+1)*per) of [0, 0x7f800000]
      const unsigned per = (unsigned)in[0];
      unsigned bad = 0;
      for (unsigned k = 0; k < per; ++k) {
        unsigned long long u = (unsigned long long)i * per + k;
        if (u > 0x7f800000ull) break;
        float x = __uint_as_float((unsigned)u);
        bad += __float_as_uint(sqrt_rn(x)) != __float_as_uint(sqrtf(x));
      }
      out[i] = (float)bad;
      break;
    }
    case 7: {  // exhaustive inv_len_rn == 1/sqrtf over [0, 0x7f800000]; rcp_rn_normal == 1/x on [2^-126, 2^126]
      const unsigned per = (unsigned)in[0];
      unsigned bad = 0;
      for (unsigned k = 0; k < per; ++k) {
        unsigned long long u = (unsigned long long)i * per + k;
        if (u > 0x7f800000ull) break;
        float x = __uint_as_float((unsigned)u);
        bad += __float_as_uint(inv_len_rn(x)) != __float_as_uint(1.0f / sqrtf(x));
        if (u >= 0x00800000ull && u <= 0x7e800000ull) bad += __float_as_uint(rcp_rn_normal(x)) != __float_as_uint(1.0f / x);
      }
      out[i] = (float)bad;
      break;
    }
    case 8: {  // exhaustive sqrt_rn_tail contract over [0, 0x7f7fffff]: == sqrtf on [2^-96, FLT_MAX], in [0, 2^-47] below
      const unsigned per = (unsigned)in[0];
      unsigned bad = 0;
      for (unsigned k = 0; k < per; ++k) {
        unsigned long long u = (unsigned long long)i * per + k;
        if (u > 0x7f7fffffull) break;
        float x = __uint_as_float((unsigned)u);
        const float s = sqrt_rn_tail(x);
        if (u >= 0x0f800000ull) bad += __float_as_uint(s) != __float_as_uint(sqrtf(x));
        else bad += !(s >= 0.0f && s <= 0x1p-47f);
      }
      out[i] = (float)bad;
      break;
    }
    case 3: out[i] = in[2 * i] / in[2 * i + 1]; break;
    case 11: {  // the exception table against this build's device code: entry i is an input whose
      // binary64 sin (det_sin_rare's sin_binary64) is ambiguous to round, so its table value is used
      if (i < (size_t)kSinTableN) {
        const float x = __uint_as_float(kSinTableX[i]);
        out[2 * i] = sin_ambiguous(sin_binary64(x)) ? 1.0f : 0.0f;
        out[2 * i + 1] = __uint_as_float(kSinTableX[i]);
      } else {
        out[2 * i] = -1.0f;
        out[2 * i + 1] = 0.0f;
      }
      break;
    }
    case 10: {  // shadow_lit_cone's per-ray set-up and occluder test for one (light - pos, t)
      const f3 lv = mk(in[4 * i], in[4 * i + 1], in[4 * i + 2]);
      const f3 l = normalize(lv);
      const float len = sqrtf(dot(lv, lv));
      const bool occ = shadow_occludes(in[4 * i + 3], l, (double)len, shadow_bounds(l, len));
      out[5 * i] = l.x; out[5 * i + 1] = l.y; out[5 * i + 2] = l.z; out[5 * i + 3] = len;
      out[5 * i + 4] = occ ? 1.0f : 0.0f;
      break;
    }
    case 4: {
      f3 v = normalize(mk(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
      out[3 * i] = v.x; out[3 * i + 1] = v.y; out[3 * i + 2] = v.z;
      break;
    }
    case 5: {
      const float* a = in + 10 * i;
      out[i] = sphere_eval(mk(a[0], a[1], a[2]), mk(a[3], a[4], a[5]), make_float4(a[6], a[7], a[8], a[9]));
      break;
    }
    default: break;
  }
}

size_t shapes_lds_bytes(const FrameParams& p) { return (size_t)4 * p.nobj * sizeof(float4); }
size_t tab_lds_bytes(const FrameParams& p) { return (size_t)5 * (p.nobj > 0 ? p.nobj : 1) * sizeof(float4); }

}  // namespace

// The production pooled AO kernel: split tail rounds and the per-ray first-bounce pre-test when
// the sphere table fits in LDS (tl), with or without the work counters (cnt), with or without
// planes (PL).
constexpr int kRefDepth = 20;  // RECURSION_DEPTH, ao_compute.glsl:9

template <int SPPC, bool PL, int DC = 0, bool CLON = false>
inline void launch_batch(bool tl, bool cnt, dim3 g, dim3 b, size_t lds, hipStream_t stream, const FrameParams& q) {
  constexpr bool GT = RT_GLOBAL_TAIL;  // split tail rounds above kTailMaxObj spheres (global table)
  constexpr bool TLC = RT_TL_CLUSTERS;  // the cluster cull in the LDS-table (<= kTailMaxObj) instantiations
  constexpr bool PTWV = RT_PT_WIDE;     // above kTailMaxObj spheres: the pre-test rows word by word
  if (q.mf_n > 0) {  // multi-frame mode-2 launch (never with counters: rt_compute_frames checks)
    g.y = (unsigned)q.mf_n;
    if (tl)
      hipLaunchKernelGGL((ao_batch_kernel<kAoMinWaves, true, kPool, 0, true, true, SPPC, true, false, PL, true, TLC, DC, CLON>), g, b, lds, stream, q, q.sph);
    else
      hipLaunchKernelGGL((ao_batch_kernel<kAoMinWaves, true, kPool, 0, GT, true, SPPC, PTWV, false, PL, true, true, DC, CLON, PTWV>), g, b, lds, stream, q, q.sph);
    return;
  }
  if (tl && cnt)
    hipLaunchKernelGGL((ao_batch_kernel<kAoMinWaves, true, kPool, 0, true, true, SPPC, true, true, PL, false, TLC, DC, CLON>), g, b, lds, stream, q, q.sph);
  else if (tl)
    hipLaunchKernelGGL((ao_batch_kernel<kAoMinWaves, true, kPool, 0, true, true, SPPC, true, false, PL, false, TLC, DC, CLON>), g, b, lds, stream, q, q.sph);
  else if (cnt)
    hipLaunchKernelGGL((ao_batch_kernel<kAoMinWaves, true, kPool, 0, GT, true, SPPC, PTWV, true, PL, false, true, DC, CLON, PTWV>), g, b, lds, stream, q, q.sph);
  else
    hipLaunchKernelGGL((ao_batch_kernel<kAoMinWaves, true, kPool, 0, GT, true, SPPC, PTWV, false, PL, false, true, DC, CLON, PTWV>), g, b, lds, stream, q, q.sph);
}

// g-buffer layout conversion (rt_download / rt_upload_gbuffer, the host-buffer path of
// compute_one_shader / compute_two_shaders): one thread per reference vec4, reference side
// coalesced.
__global__ __launch_bounds__(256) void gbuf_convert_kernel(GbufXfer x) {
  const size_t total = (size_t)x.F * x.W * x.R;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const size_t wr = (size_t)x.W * x.R;
  const int f = (int)(idx / wr);
  const size_t rem = idx - (size_t)f * wr;
  const int xx = (int)(rem / x.R), r = (int)(rem - (size_t)xx * x.R);
  const size_t o = (size_t)(x.r0 + r) * x.W + xx;
  float4* base = x.slot[f];
  if (x.to_ref) {
    x.ref[idx] = x.kind == 0 ? base[o] : x.kind == 1 ? nrm_load(base, x.n, o) : dep_load(base, x.n, o);
  } else {
    const float4 v = x.ref[idx];
    if (x.kind == 0) base[o] = v;
    else if (x.kind == 1) nrm_store(base, x.n, o, v);
    else dep_store(base, x.n, o, v);
  }
}

inline hipError_t launch_gbuf_convert_impl(const GbufXfer& x, hipStream_t stream) {
  const size_t total = (size_t)x.F * x.W * x.R;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(gbuf_convert_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, x);
  return hipGetLastError();
}

// The production launch of `program` (rt_kernels.hip's launch_program; the A/B tools library
// falls back to it): q = p with the derived table pointers and launch constants.
inline FrameParams launch_params(const FrameParams& p) {
  FrameParams q = p;
  q.sph = p.shapes + sphere_table(p.S);
  q.planes = p.shapes + plane_table(p.S);
  q.clus = p.shapes + cluster_table(p.S);
  q.clmask = (const unsigned long long*)(p.shapes + cluster_mask_table(p.S));
  q.camrel = p.shapes + camrel_table(p.S);
  q.b1_min = 1;
  {  // rotation group: the pools of one image row (at least 8)
    const int TP = kPool / p.spp > 0 ? kPool / p.spp : 1;
    const int ppr = p.W / TP;
    q.pool_rot = ppr >= 8 ? ppr : 8;
  }
  {  // post-process XCD runs (xcd_tile): the least R in [4, gx / 16] dividing gx / 8 (a tile row
    // is a whole number of 8-run rounds, at least two per XCD), else 4; narrow frames: none
    const int gx = (p.W + kPostTileW - 1) / kPostTileW;
    int R = 0;
    if (gx % 8 == 0)
      for (int r = 4; r <= gx / 16 && !R; ++r)
        if ((gx / 8) % r == 0) R = r;
    q.tile_run = R ? R : (gx >= 32 ? 4 : 0);
#ifdef RT_POST_RUN
    q.tile_run = RT_POST_RUN;  // A/B builds: a fixed run length (0 = row-major order)
#endif
    // super-tiles (xcd_tile): 4 or 2 blocks each way where that divides the grid
    const int gy = (p.trace_rows + kPostTileH - 1) / kPostTileH;
    q.post_sx = gx % 4 == 0 ? 4 : (gx % 2 == 0 ? 2 : 1);
    q.post_sy = gy % 4 == 0 ? 4 : (gy % 2 == 0 ? 2 : 1);
    if (gx < 8 * q.post_sx) q.post_sx = q.post_sy = 1;  // narrow frames: the runs (or none)
  }
  return q;
}

inline hipError_t launch_production(int program, const FrameParams& p, const FrameParams& q, hipStream_t stream) {
  const bool pl = p.nplanes > 0;
  if (program == K_AOP || program == K_AO) {
    const long long npix = (long long)p.trace_rows * p.W;
    const int TP = kPool / p.spp > 0 ? kPool / p.spp : 1;
    const long long pools = (npix + TP - 1) / TP;
    const bool tl = p.nobj <= kTailMaxObj;
    const size_t psh = (size_t)batch_lds(p.spp, kPool, tl ? p.nobj : (RT_PT_WIDE ? 64 : 0), tl || !RT_PT_WIDE).total;
    const dim3 g((unsigned)pools), b(64);
    // timed launches pass no counters: the counter code is compiled out (fewer live scalars)
    const bool cnt = p.counters || p.row_counters;
    // spp 4 (the reference's AA), 16 (configs c/d) and 64 (config e) have their own
    // instantiations: constant LDS offsets and it / spp, fewer scalar registers
    // The reference's RECURSION_DEPTH (20, ao_compute.glsl:9) with bounce-ray clusters (every
    // scene of 16..256 spheres) also has its own instantiations for spp 16 and 64: with the depth
    // a constant and the rounds' plain full-scan fallback compiled out, fewer scalar registers are
    // spilled to vector lanes (each reload is a v_readlane on the bounce rounds' path)
    if (!pl) {
      const bool ref_d = p.D == kRefDepth && p.ncl > 0;
      if (p.spp == 16 && ref_d) launch_batch<16, false, kRefDepth, true>(tl, cnt, g, b, psh, stream, q);
      else if (p.spp == 64 && ref_d) launch_batch<64, false, kRefDepth, true>(tl, cnt, g, b, psh, stream, q);
      else if (p.spp == 16) launch_batch<16, false>(tl, cnt, g, b, psh, stream, q);
      else if (p.spp == 64) launch_batch<64, false>(tl, cnt, g, b, psh, stream, q);
      else if (p.spp == 4) launch_batch<4, false>(tl, cnt, g, b, psh, stream, q);
      else launch_batch<0, false>(tl, cnt, g, b, psh, stream, q);
    } else {
      if (p.spp == 16) launch_batch<16, true>(tl, cnt, g, b, psh, stream, q);
      else if (p.spp == 4) launch_batch<4, true>(tl, cnt, g, b, psh, stream, q);
      else launch_batch<0, true>(tl, cnt, g, b, psh, stream, q);
    }
    return hipGetLastError();
  }
  // modes 3/4 multi-frame launches: FPB frames per block (block_frames)
  const int fpb = program == K_PHONG ? kPhongFramesPerBlock : kHybridFramesPerBlock;
  const int tpb = program == K_HYBRID ? kHybridTilesPerBlock : 1;
  // hybrid blocks: kHyBW x kHyBW waves of 8x8 pixels (kHyTile = 8 kHyBW px); phong: 2x2 waves
  const int tw = program == K_HYBRID ? kHyTile : 16;
  dim3 grid((p.W + tw - 1) / tw, ((p.trace_rows + tw - 1) / tw + tpb - 1) / tpb, p.mf_n > 0 ? (p.mf_n + fpb - 1) / fpb : 1);
  const dim3 hyb(64 * kHyBW * kHyBW);
  // scenes of at most kTabLdsMax objects: the tables staged in LDS per wave (LT)
// Modes 3/4 read the shape tables through the caches (scalar loads for the wave-uniform culls
// and survivor tests, vector loads for the hit's material) instead of staging them in LDS per
// block: no staging round trip and no block barrier before a wave's first test.  Round 5,
// burst A/Bs: hybrid (b) 28.15 -> 26.78 us per launch (-4.9%), phong (a) 6.87 -> 6.75 us
// (-1.7%), bit-identical (profiles/r05n_*).  Round 2 had measured the LDS tables faster
// (40.4 -> 37.9 us) on the kernels of that time.  0 restores the LDS tables (A/B builds).
#ifndef RT_HY_NOLT
#define RT_HY_NOLT 1
#endif
#ifndef RT_PH_NOLT
#define RT_PH_NOLT 1
#endif
  const bool lt = p.nobj <= kTabLdsMax && !(RT_HY_NOLT && program == K_HYBRID) && !(RT_PH_NOLT && program == K_PHONG);
  const size_t ltb = lt ? tab_lds_bytes(p) : 0;
  const bool mf = p.mf_n > 0;  // multi-frame launch; single-frame ones take the MF = false kernels
  switch (program) {
    case K_PHONG:
      if (pl && lt) hipLaunchKernelGGL((phong_kernel<true, true, true>), grid, dim3(kBlock), ltb, stream, q.sph, q.shapes, q);
      else if (pl && mf) hipLaunchKernelGGL((phong_kernel<true, true, false>), grid, dim3(kBlock), 0, stream, q.sph, q.shapes, q);
      else if (pl) hipLaunchKernelGGL((phong_kernel<true, true, false, false>), grid, dim3(kBlock), 0, stream, q.sph, q.shapes, q);
      else if (lt) hipLaunchKernelGGL((phong_kernel<true, false, true>), grid, dim3(kBlock), ltb, stream, q.sph, q.shapes, q);
      else if (mf) hipLaunchKernelGGL((phong_kernel<true, false, false>), grid, dim3(kBlock), 0, stream, q.sph, q.shapes, q);
      else hipLaunchKernelGGL((phong_kernel<true, false, false, false>), grid, dim3(kBlock), 0, stream, q.sph, q.shapes, q);
      break;
    case K_HYBRID:
      if (pl && lt) hipLaunchKernelGGL((hybrid_kernel<true, true, true, 0, kHyBW, kHyBW>), grid, hyb, ltb, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
      else if (pl && mf) hipLaunchKernelGGL((hybrid_kernel<true, true, false, 0, kHyBW, kHyBW>), grid, hyb, 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
      else if (pl) hipLaunchKernelGGL((hybrid_kernel<true, true, false, 0, kHyBW, kHyBW, false>), grid, hyb, 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
      else if (lt) hipLaunchKernelGGL((hybrid_kernel<true, false, true, 0, kHyBW, kHyBW>), grid, hyb, ltb, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
      else if (mf) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, kHyBW, kHyBW>), grid, hyb, 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
      else hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, kHyBW, kHyBW, false>), grid, hyb, 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
      break;
    case K_POST:
      hipLaunchKernelGGL(post_kernel,
                         dim3((p.W + kPostTileW - 1) / kPostTileW, (p.trace_rows + kPostTileH - 1) / kPostTileH),
                         dim3(kBlock), 0, stream, q);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

inline hipError_t launch_selftest_impl(int fn, const float* d_in, float* d_out, size_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(selftest_kernel, dim3(grid), dim3(256), 0, stream, fn, d_in, d_out, n);
  return hipGetLastError();
}

}  // namespace rt
