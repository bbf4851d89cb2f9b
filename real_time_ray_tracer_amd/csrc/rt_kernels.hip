// rt_kernels.hip — gfx950 kernels for the per-pixel ray-scene hot path.
//
//   phong_kernel   <- resources/p_compute.glsl   (mode 3)
//   hybrid_kernel  <- resources/h_compute.glsl   (mode 4)
//   ao_kernel      <- resources/ao_compute.glsl  (mode 2) / aop_compute.glsl (mode 1 pass 1)
//   post_kernel    <- resources/aop_postprocessing.glsl (mode 1 pass 2)
//
// The reference dispatches W x H single-lane workgroups (local_size 1x1, p_compute.glsl:26).
// Here a 256-lane workgroup (4 wave64) owns a tile: one lane per pixel (modes 3/4) or one
// lane per pixel-sample (modes 1/2).  The scene table (<= a few KB) is staged into LDS once
// per workgroup and read by wave-uniform broadcast.  AO samples of a pixel are combined in
// sample order by the pixel's sample-0 lane, so the sum order matches the reference's
// sequential `result_color += ambient_occlusion(dir, aa)` (ao_compute.glsl:303-330).
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
  return make_float4(powf(r, kGamma), powf(g, kGamma), powf(b, kGamma), 0.0f);
}

// 16x16 pixel tile per 256-lane block, 8x8 per wave (ray coherence inside a wave).
__device__ __forceinline__ void tile_xy(int& x, int& y, int row0) {
  int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
  y = row0 + blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
}

// Work counters for the algorithmic-FLOP roofline (only when P.counters is set; the atomic
// optimizer turns the uniform-address adds into one add per wave).
__device__ __forceinline__ void count_work(const FrameParams& P, int y, unsigned samples, unsigned segs,
                                           unsigned shadows) {
  if (P.row_counters) atomicAdd(&P.row_counters[y - P.band_row0], (unsigned long long)(segs + shadows));
  if (!P.counters) return;
  atomicAdd(&P.counters[0], (unsigned long long)samples);
  atomicAdd(&P.counters[1], (unsigned long long)segs);
  atomicAdd(&P.counters[2], (unsigned long long)shadows);
  atomicAdd(&P.counters[3], (unsigned long long)(segs + shadows) * (unsigned long long)P.nobj);
}

__device__ __forceinline__ void store_color(const FrameParams& P, int x, int y, float4 c) {
  P.out_pix[(size_t)(y - P.band_row0) * P.W + x] = c;
  if (P.image) {
    int r = y - P.img_row0;
    if (r >= 0 && r < P.img_rows) P.image[(size_t)r * P.W + x] = c;
  }
}

// ---------------------------------------------------------------------------------------
// mode 3 — p_compute.glsl:168-245
// ---------------------------------------------------------------------------------------
template <bool ALLSPH>
__global__ __launch_bounds__(kBlock) void phong_kernel(FrameParams P) {
  extern __shared__ float4 lds[];
  stage_shapes(P, lds);
  __syncthreads();
  const int n = P.nobj;
  const float4 *geo = lds, *geo2 = lds + n, *col = lds + 2 * n;
  int x, y;
  tile_xy(x, y, P.trace_row0);
  if (x >= P.W || y >= P.trace_row0 + P.trace_rows) return;

  const f3 cam = mk(P.cx, P.cy, P.cz), light = mk(P.Lx, P.Ly, P.Lz);
  f3 dir = primary_dir(P, (float)x / (float)P.W, (float)y / (float)P.H);
  float t;
  int ind = closest_hit<ALLSPH>(geo, geo2, n, cam, dir, 0.0f, t);
  count_work(P, y, 1u, 1u, ind == -1 ? 0u : 1u);
  float r, g, b;
  if (ind == -1) {
    r = P.bg.x; g = P.bg.y; b = P.bg.z;
  } else {
    f3 curr = cam + t * dir;
    bool lit = shadow_lit<ALLSPH>(geo, geo2, n, light, curr);
    int id = ALLSPH ? SHAPE_SPHERE : __float_as_int(geo2[ind].w);
    f3 nn = shape_normal(geo[ind], id, curr);
    float4 c = col[ind];
    if (lit) {
      f3 l = normalize(light - curr);
      float spec = powf(gclamp(dot(normalize(l - dir), nn), 0.0f, 1.0f), 500.0f);
      float k = gclamp(dot(nn, l), 0.06f, 1.0f);
      r = c.x * k + spec; g = c.y * k + spec; b = c.z * k + spec;
    } else {
      r = c.x * 0.06f; g = c.y * 0.06f; b = c.z * 0.06f;
    }
  }
  // result_color = vec4(0) + phong(dir); gamma; w = 0
  store_color(P, x, y, gamma_out(0.0f + r, 0.0f + g, 0.0f + b));
}

// ---------------------------------------------------------------------------------------
// mode 4 — h_compute.glsl:186-321
// ---------------------------------------------------------------------------------------
template <bool ALLSPH>
__global__ __launch_bounds__(kBlock) void hybrid_kernel(FrameParams P) {
  extern __shared__ float4 lds[];
  stage_shapes(P, lds);
  __syncthreads();
  const int n = P.nobj;
  const float4 *geo = lds, *geo2 = lds + n, *col = lds + 2 * n, *aux = lds + 3 * n;
  int x, y;
  tile_xy(x, y, P.trace_row0);
  if (x >= P.W || y >= P.trace_row0 + P.trace_rows) return;

  const f3 light = mk(P.Lx, P.Ly, P.Lz);
  f3 pos = mk(P.cx, P.cy, P.cz);
  f3 dir = primary_dir(P, (float)x / (float)P.W, (float)y / (float)P.H);
  float arefl = 0.0f;          // array[2].w
  float rr = 0, rg = 0, rb = 0;  // result_color.rgb
  float c = 0.0f;
  unsigned nseg = 0, nshadow = 0;
  for (int seg = 0; seg < P.D; ++seg) {  // helper depth D, D-1, ..., 1
    // ---- hybrid_helper ----
    float t;
    int ind = closest_hit<ALLSPH>(geo, geo2, n, pos, dir, 0.001f, t);
    ++nseg;
    nshadow += ind == -1 ? 0u : 1u;
    float ar, ag, ab;
    bool stop;
    if (ind == -1) {
      ar = P.bg.x; ag = P.bg.y; ab = P.bg.z;
      stop = true;
    } else {
      float4 att = col[ind];
      f3 curr = pos + t * dir;
      bool lit = shadow_lit<ALLSPH>(geo, geo2, n, light, curr);
      int id = ALLSPH ? SHAPE_SPHERE : __float_as_int(geo2[ind].w);
      f3 nn = shape_normal(geo[ind], id, curr);
      if (lit) {
        f3 l = normalize(light - curr);
        float spec = powf(gclamp(dot(normalize(l - dir), nn), 0.0f, 1.0f), 500.0f);
        float k = gclamp(dot(nn, l), 0.06f, 1.0f);
        ar = att.x * k + spec; ag = att.y * k + spec; ab = att.z * k + spec;
      } else {
        ar = att.x * 0.06f; ag = att.y * 0.06f; ab = att.z * 0.06f;
      }
      float refl = 1.0f - aux[ind].y;
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
    // ---- hybrid (h_compute.glsl:279-295) ----
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
    if (stop) break;
  }
  count_work(P, y, 1u, nseg, nshadow);
  store_color(P, x, y, gamma_out(0.0f + rr, 0.0f + rg, 0.0f + rb));
}

// ---------------------------------------------------------------------------------------
// modes 1/2 pass 1 — ao_compute.glsl:143-339 (aop_compute.glsl:141-336)
// lane = (pixel, sample); ppb = blockDim / spp pixels per block, consecutive in a row.
// ---------------------------------------------------------------------------------------
enum { PRIM_HIT = 0, PRIM_MISS = 1, PRIM_EMISSIVE = 2 };

template <bool ALLSPH>
__global__ __launch_bounds__(kBlock) void ao_kernel(FrameParams P) {
  extern __shared__ float4 lds[];
  stage_shapes(P, lds);
  const int n = P.nobj;
  const float4 *geo = lds, *geo2 = lds + n, *col = lds + 2 * n, *aux = lds + 3 * n;
  float4* samp = lds + 4 * n;  // [blockDim] per-sample (r, g, b, stop value or -1)
  __syncthreads();

  const int spp = P.spp;
  const int ppb = blockDim.x / spp;
  const int lp = threadIdx.x / spp, aa = threadIdx.x - lp * spp;
  const long long pix = (long long)blockIdx.x * ppb + lp;
  const bool valid = lp < ppb && pix < (long long)P.trace_rows * P.W;
  const int x = valid ? (int)(pix % P.W) : 0;
  const int y = valid ? P.trace_row0 + (int)(pix / P.W) : 0;

  int kind = PRIM_HIT;
  float t0 = 0.0f;
  f3 n0 = mk(0.0f, 0.0f, 0.0f);
  float rr = 1.0f, rg = 1.0f, rb = 1.0f;
  float stopv = -1.0f;
  if (valid) {
    const float px = (float)x, py = (float)y;
    const float4* rbuf = P.rb;
    float hp, vp;
    if (aa == 0) {
      hp = px / (float)P.W;
      vp = py / (float)P.H;
    } else {  // jitter, ao_compute.glsl:310-323
      float4 f = rbuf[2 * aa], s = rbuf[2 * aa + 1];
      float u = grandom(((s.x + px * f.z) - px) + f.x, ((f.y + py * s.w) - py) + s.y);
      float w = grandom(s.z * px - (f.x * px) * f.z, f.w * py - (s.y * py) * s.w);
      float l = sqrtf(fmaf(w, w, u * u));
      float jx = (u / l) / 6.0f - 0.08333f;
      float jy = (w / l) / 6.0f - 0.08333f;
      hp = (px + jx) / (float)P.W;
      vp = (py + jy) / (float)P.H;
    }
    f3 dir = primary_dir(P, hp, vp);
    // get_pt_within_unit_sphere(aa): depends on (aa, pixel) only -> hoisted out of the bounce loop
    f3 hemi;
    {
      float4 f = rbuf[2 * aa], s = rbuf[2 * aa + 1];
      float a = grandom(f.x + px * s.z, f.y + py * s.w);
      float b = grandom(f.z - px * s.z, f.w - py * s.w);
      float e = grandom(s.x * px + s.z, s.y * py + s.w);
      hemi = normalize(mk(a * 2.0f - 1.0f, b * 2.0f - 1.0f, e * 2.0f - 1.0f));
    }
    const f3 cam = mk(P.cx, P.cy, P.cz);
    f3 pos = cam;
    unsigned nseg = 0;
    for (int depth = P.D; depth > 0; --depth) {
      float t;
      int ind = closest_hit<ALLSPH>(geo, geo2, n, pos, dir, 0.0001f, t);
      ++nseg;
      if (ind != -1) {
        float4 att = col[ind];
        float4 ax = aux[ind];
        if (ax.x > 0.9f) {  // emissive: stop
          rr = rr * att.x; rg = rg * att.y; rb = rb * att.z;
          stopv = (float)(P.D - depth);
          if (aa == 0 && depth == P.D) kind = PRIM_EMISSIVE;
          break;
        }
        f3 curr = cam + t * dir;  // sic: camera origin (ao_compute.glsl:210)
        int id = ALLSPH ? SHAPE_SPHERE : __float_as_int(geo2[ind].w);
        f3 nn = shape_normal(geo[ind], id, curr);
        if (aa == 0 && depth == P.D) {
          kind = PRIM_HIT;
          t0 = t;
          n0 = nn;
        }
        rr = rr * att.x; rg = rg * att.y; rb = rb * att.z;
        pos = curr;
        float reflect = ax.y;
        if (reflect > 0.999f) {
          dir = normalize(hemi + nn);
        } else {
          float dn = dot(dir, nn);
          f3 R = normalize(mk(dir.x - 2.0f * (dn * nn.x), dir.y - 2.0f * (dn * nn.y),
                              dir.z - 2.0f * (dn * nn.z)));
          dir = normalize(R + reflect * hemi);
        }
      } else {
        if (aa == 0 && depth == P.D) kind = PRIM_MISS;
        rr = rr * P.bg.x; rg = rg * P.bg.y; rb = rb * P.bg.z;
        stopv = (float)(P.D - depth);
        break;
      }
    }
    count_work(P, y, 1u, nseg, 0u);
  }
  samp[threadIdx.x] = make_float4(rr, rg, rb, stopv);
  __syncthreads();
  if (!valid || aa != 0) return;

  // ---- sample combine in aa order (ao_compute.glsl:303-339) ----
  float sr = 0.0f, sg = 0.0f, sb = 0.0f, ystop = -1.0f;
  const float4* ps = samp + lp * spp;
  for (int k = 0; k < spp; ++k) {
    float4 s = ps[k];
    sr = sr + s.x; sg = sg + s.y; sb = sb + s.z;
    if (s.w >= 0.0f) ystop = s.w;  // depth_buffer.y: last writer wins
  }
  const float fa = (float)spp;
  const size_t off = (size_t)(y - P.band_row0) * P.W + x;
  float4 d;
  if (kind == PRIM_HIT) {
    d = make_float4(t0, 0.0f, 0.0f, 1.0f);
    P.nrm[off] = make_float4(n0.x, n0.y, n0.z, 1.0f);
  } else if (kind == PRIM_MISS) {
    d = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    P.nrm[off] = d;
  } else {
    d = P.dep[off];  // stale: sample 0 hit an emissive shape first (no g-buffer write)
  }
  if (ystop >= 0.0f) d.y = ystop;
  d.x = d.x / fa; d.y = d.y / fa; d.z = d.z / fa; d.w = d.w / fa;
  P.dep[off] = d;
  store_color(P, x, y, gamma_out(sr / fa, sg / fa, sb / fa));
}

// ---------------------------------------------------------------------------------------
// mode 1 pass 2 — aop_postprocessing.glsl:57-208, with the documented snapshot semantics:
// neighbours read `raw` (slot f before filtering); right iff x+1<W, left iff x>0,
// up iff y+1<H, down iff y>=2.  Output goes to out_pix (the shim swaps it into slot f).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float nbr_weight(f3 n, float nd, float nb, float4 kn, float4 kd) {
  if (kn.w < 0.001f) return 1.0f;
  float normal_dot = dot(n, xyz(kn));
  float depth_diff = 1.0f - gclamp(fabsf(nd - kd.x), 0.0f, 1.0f);
  float bounces_diff = 1.0f - gclamp(fabsf(nb - kd.y) / 1.7f, 0.0f, 1.0f);
  return normal_dot * depth_diff * bounces_diff + 0.2f;
}

__global__ __launch_bounds__(kBlock) void post_kernel(FrameParams P) {
  int x, y;
  tile_xy(x, y, P.trace_row0);
  if (x >= P.W || y >= P.trace_row0 + P.trace_rows) return;
  const int W = P.W, f = P.frame;
  const size_t off = (size_t)(y - P.band_row0) * W + x;
  float4 color = P.raw[off];
  const float4 cn = P.nrm[off];
  if (cn.w > 0.99f) {
    const float4 cd = P.dep[off];
    const f3 nv = xyz(cn);
    const float nd = cd.x, nb = cd.y;
    float4 acc = color;
    float den = 1.0f;
    const int band_end = P.band_row0 + P.band_rows;
    // GLSL order: up, down, left, right (line 173)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int xx = x + (k == 2 ? -1 : (k == 3 ? 1 : 0));
      int yy = y + (k == 0 ? 1 : (k == 1 ? -1 : 0));
      bool present = (k == 0) ? (y + 1 < P.H) : (k == 1) ? (y >= 2) : (k == 2) ? (x > 0) : (x + 1 < W);
      present = present && yy >= P.band_row0 && yy < band_end;
      float wk = 0.0f;
      float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (present) {
        size_t o = (size_t)(yy - P.band_row0) * W + xx;
        wk = nbr_weight(nv, nd, nb, P.nrm[o], P.dep[o]);
        v = P.raw[o];
      }
      acc.x = acc.x + wk * v.x; acc.y = acc.y + wk * v.y;
      acc.z = acc.z + wk * v.z; acc.w = acc.w + wk * v.w;
      den = den + wk;
    }
    color = make_float4(acc.x / den, acc.y / den, acc.z / den, acc.w / den);
    // temporal, lines 177-201
    float4 cs = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float denominator = 0.9f;
    for (int i = 1; i < P.F; ++i) {
      int cf = (f + P.F - i) % P.F;
      float4 hn = P.hist_nrm[cf][off];
      float4 hd = P.hist_dep[cf][off];
      float normal_dot = dot(nv, xyz(hn));
      float depth_diff = 1.0f - gclamp(fabsf(nd - hd.x), 0.0f, 1.0f);
      float bounces_diff = 1.0f - gclamp(fabsf(nb - hd.y) / 1.7f, 0.0f, 1.0f);
      float coeff = normal_dot * depth_diff * bounces_diff;
      if (!(coeff > 0.85f)) break;
      float4 hp = P.hist_pix[cf][off];
      cs.x = cs.x + coeff * hp.x; cs.y = cs.y + coeff * hp.y;
      cs.z = cs.z + coeff * hp.z; cs.w = cs.w + coeff * hp.w;
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
    case 1: out[i] = grandom(in[2 * i], in[2 * i + 1]); break;
    case 2: out[i] = sqrtf(in[i]); break;
    case 3: out[i] = in[2 * i] / in[2 * i + 1]; break;
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

}  // namespace

hipError_t launch_program(int program, const FrameParams& p, bool all_spheres, hipStream_t stream) {
  if (p.trace_rows <= 0) return hipSuccess;
  const size_t lds = shapes_lds_bytes(p);
  if (program == K_AOP || program == K_AO) {
    const int ppb = kBlock / p.spp >= 1 ? kBlock / p.spp : 1;
    const int block = ppb * p.spp;
    const long long npix = (long long)p.trace_rows * p.W;
    const long long grid = (npix + ppb - 1) / ppb;
    const size_t sh = lds + (size_t)block * sizeof(float4);
    if (all_spheres)
      hipLaunchKernelGGL(ao_kernel<true>, dim3((unsigned)grid), dim3(block), sh, stream, p);
    else
      hipLaunchKernelGGL(ao_kernel<false>, dim3((unsigned)grid), dim3(block), sh, stream, p);
    return hipGetLastError();
  }
  dim3 grid((p.W + 15) / 16, (p.trace_rows + 15) / 16);
  switch (program) {
    case K_PHONG:
      if (all_spheres) hipLaunchKernelGGL(phong_kernel<true>, grid, dim3(kBlock), lds, stream, p);
      else hipLaunchKernelGGL(phong_kernel<false>, grid, dim3(kBlock), lds, stream, p);
      break;
    case K_HYBRID:
      if (all_spheres) hipLaunchKernelGGL(hybrid_kernel<true>, grid, dim3(kBlock), lds, stream, p);
      else hipLaunchKernelGGL(hybrid_kernel<false>, grid, dim3(kBlock), lds, stream, p);
      break;
    case K_POST:
      hipLaunchKernelGGL(post_kernel, grid, dim3(kBlock), 0, stream, p);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_selftest(int fn, const float* d_in, float* d_out, size_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(selftest_kernel, dim3(grid), dim3(256), 0, stream, fn, d_in, d_out, n);
  return hipGetLastError();
}

}  // namespace rt
