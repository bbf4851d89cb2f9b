// rt_kernels_ab.hip — the A/B tools library's launcher (make ablib -> build/librtrt_ab.so; never
// part of librtrt.so).  Same kernels (../../real_time_ray_tracer_amd/csrc/rt_kernels_impl.h) plus
// the experimental / superseded ones, selected per launch by environment switches read by
// tools/ab.py, tools/sections.py and tools/variant_counters.py:
//   RTRT_AO_VARIANT  AO kernel variant (see ab_launch_ao), RTRT_B1_MIN, RTRT_POOL_ROT=0,
//   RTRT_NO_CLUSTERS=1  the AO bounce rounds without the cluster cull,
//   RTRT_GENERAL=1   every program on the unculled LDS-table kernels,
//   RTRT_HY_ABL      hybrid timing ablations, RTRT_HY_BLK hybrid block shapes.
// Anything not selected runs the production launch (launch_production).
#include <cstdlib>

#include "rt_kernels_impl.h"

namespace rt {

namespace {

// the lane-per-sample AO kernel (the round-1 baseline; the pooled kernel is production)
template <bool ALLSPH, int V>
__global__ __launch_bounds__(kBlock) void ao_kernel(FrameParams P, const float4* __restrict__ gtab) {
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
  unsigned nseg = 0;
  if (valid) {
    const float px = (float)x, py = (float)y;
    const float4* rbuf = P.rb;
    float hp, vp;
    if (aa == 0) {
      hp = div_rn_by(px, P.fW, P.inv_W);
      vp = div_rn_by(py, P.fH, P.inv_H);
    } else {  // jitter, ao_compute.glsl:310-323
      float4 f = rbuf[2 * aa], s = rbuf[2 * aa + 1];
      float u = grandom(((s.x + px * f.z) - px) + f.x, ((f.y + py * s.w) - py) + s.y);
      float w = grandom(s.z * px - (f.x * px) * f.z, f.w * py - (s.y * py) * s.w);
      normalize2(u, w);
      float jx = div_rn_by(u, 6.0f, kInv6) - 0.08333f;
      float jy = div_rn_by(w, 6.0f, kInv6) - 0.08333f;
      hp = div_rn_by(px + jx, P.fW, P.inv_W);
      vp = div_rn_by(py + jy, P.fH, P.inv_H);
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
    for (int depth = P.D; depth > 0; --depth) {
      float t;
      int ind = V == 2 ? closest_hit_v<ALLSPH, 2>(gtab, gtab + P.S, n, pos, dir, 0.0001f, t)
                       : closest_hit_v<ALLSPH, V>(geo, geo2, n, pos, dir, 0.0001f, t);
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
  }
  count_work(P, valid, y, nseg, 0u);
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
    nrm_store(P.nrm, dep_plane(P), off, make_float4(n0.x, n0.y, n0.z, 1.0f));
  } else if (kind == PRIM_MISS) {
    d = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    nrm_store(P.nrm, dep_plane(P), off, d);
  } else {
    // stale: sample 0 hit an emissive shape first (no g-buffer write): the slot keeps its
    // previous normal and depth (read from the slot's previous buffers when pipelined)
    d = dep_load(P.dep_prev, dep_plane(P), off);
    if (P.nrm_prev != P.nrm) nrm_store(P.nrm, dep_plane(P), off, nrm_load(P.nrm_prev, dep_plane(P), off));
  }
  if (ystop >= 0.0f) d.y = ystop;
  d.x = d.x / fa; d.y = d.y / fa; d.z = d.z / fa; d.w = d.w / fa;
  dep_store(P.dep, dep_plane(P), off, d);
  store_color(P, x, y, gamma_out(sr / fa, sg / fa, sb / fa));
}

}  // namespace

// ---- A/B build only (make ablib -> build/librtrt_ab.so; tools/ab.py, tools/sections.py) -----
// RTRT_AO_VARIANT selects an experimental AO kernel per launch: 9 (no first-bounce pre-test),
// 27 (no batched first bounce), 17 (no split tail rounds), 11 (no lazy shortcuts), 91-93 (timing
// ablations: bounce tests twice, culled primary tests twice, section clocks), 96/97 (section
// clocks with the first bounce split, event counts), 0/2 (the lane-per-sample kernel, LDS table /
// scalar table).  RTRT_GENERAL=1 runs every program on the unculled LDS-table kernels (the pre-plane-
// support path for scenes with planes).  RTRT_B1_MIN: least live lanes for a batched first bounce.
static bool ab_launch_ao(const FrameParams& p, FrameParams& q, hipStream_t stream, long long npix) {
  const char* ev = getenv("RTRT_AO_VARIANT");
  const int variant = ev ? atoi(ev) : 7;
  const char* eb = getenv("RTRT_B1_MIN");
  q.b1_min = eb ? atoi(eb) : 1;
  if (const char* en = getenv("RTRT_NO_CLUSTERS"); en && atoi(en) == 1) q.ncl = 0;  // A/B: no bounce-ray cluster cull
  const char* er = getenv("RTRT_POOL_ROT");
  if (er && atoi(er) == 0) q.pool_rot = 0;  // A/B: pools in plain row order
  const char* eg = getenv("RTRT_GENERAL");
  const bool general = (eg && atoi(eg) == 1) || variant == 0 || variant == 2;
  const int TP = kPool / p.spp > 0 ? kPool / p.spp : 1;
  const long long pools = (npix + TP - 1) / TP;
  const dim3 g((unsigned)pools), b(64);
  const bool tl = p.nobj <= kTailMaxObj;
  if (general) {
    const int ppb = kBlock / p.spp >= 1 ? kBlock / p.spp : 1;
    const int block = ppb * p.spp;
    const long long grid = (npix + ppb - 1) / ppb;
    const size_t sh = shapes_lds_bytes(p) + (size_t)block * sizeof(float4);
    if (variant == 2 && p.nplanes == 0)
      hipLaunchKernelGGL((ao_kernel<true, 2>), dim3((unsigned)grid), dim3(block), sh, stream, q, q.shapes);
    else
      hipLaunchKernelGGL((ao_kernel<false, 0>), dim3((unsigned)grid), dim3(block), sh, stream, q, q.shapes);
    return true;
  }
  if (variant == 7 || (p.nplanes > 0 && variant != 93)) return false;  // production
  if (variant == 93 && p.nplanes > 0) {  // section clocks of the production plane kernel
    const size_t pl_sh = (size_t)batch_lds(p.spp, kPool, tl ? p.nobj : 0).total;
    if (tl && p.spp == 16)
      hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 3, true, true, 16, true, true, true>), g, b, pl_sh, stream, q, q.sph);
    else
      hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 3, false, true, 0, false, true, true>), g, b, pl_sh, stream, q, q.sph);
    return true;
  }
  const size_t psh = (size_t)batch_lds(p.spp, kPool, (variant == 9 || variant == 27 || variant >= 93) && tl ? p.nobj : 0).total;
  if (variant == 9 && p.spp == 16 && tl)  // 7 without the per-ray first-bounce pre-test
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 0, true, true, 16, false, false>), g, b, psh, stream, q, q.sph);
  else if (variant == 27 && tl)  // 7 without the batched first bounce
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 0, true>), g, b, psh, stream, q, q.sph);
  else if (variant == 11)
    hipLaunchKernelGGL((ao_batch_kernel<7, false>), g, b, psh, stream, q, q.sph);
  else if (variant >= 101 && variant <= 110 && tl && p.spp == 16 && p.nplanes == 0 && q.ncl > 0) {
    // instruction budget (tools/sq_budget.sh): the production (d) instantiation (no counters,
    // depth 20, clusters) and its ablations, each repeating one section's work once more:
    // 101 none, 102 cluster-round tests (ABL 1), 103 culled primary tests (ABL 2), 104 the five
    // hashes (ABL 4), 105 first-bounce survivor iterations (ABL 5)
    const size_t ps = (size_t)batch_lds(16, kPool, p.nobj).total;
    if (variant == 101) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 0, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 102) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 1, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 103) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 2, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 104) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 4, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 105) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 5, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    // round 6: 106 the hit shading's arithmetic (ABL 9), 107 the primary setup after the hashes
    // (ABL 10), 108 the hand-out shuffles (ABL 11), 109 the first bounce's cone + cull (ABL 12),
    // 110 the full rounds' cluster cull (ABL 13)
    if (variant == 106) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 9, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 107) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 10, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 108) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 11, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 109) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 12, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
    if (variant == 110) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 13, true, true, 16, true, false, false, false, true, 20, true>), g, b, ps, stream, q, q.sph);
  } else if ((variant == 193 || variant == 196 || variant == 198) && !tl && p.spp == 64 && p.nplanes == 0 &&
             q.ncl > 0 && p.D == 20) {
    // section clocks of config (e)'s production instantiation (above kTailMaxObj spheres: the
    // word-by-word pre-test, rand_buffer from global memory): 193 as 93, 196 as 96, 198 as 98
    const size_t pw = (size_t)batch_lds(64, kPool, 64, false).total;
    if (variant == 193) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 3, true, true, 64, true, true, false, false, true, 20, true, true>), g, b, pw, stream, q, q.sph);
    if (variant == 196) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 6, true, true, 64, true, true, false, false, true, 20, true, true>), g, b, pw, stream, q, q.sph);
    if (variant == 198) hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 8, true, true, 64, true, true, false, false, true, 20, true, true>), g, b, pw, stream, q, q.sph);
  } else if (variant == 91)
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 1>), g, b, psh, stream, q, q.sph);
  else if (variant == 92)
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 2>), g, b, psh, stream, q, q.sph);
  else if (variant == 96 && tl && p.spp == 16)  // section clocks, first bounce split in 3
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 6, true, true, 16, true>), g, b, psh, stream, q, q.sph);
  else if (variant == 98 && tl && p.spp == 16)  // section clocks, split tail rounds apart from full rounds
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 8, true, true, 16, true>), g, b, psh, stream, q, q.sph);
  else if (variant == 97 && tl && p.spp == 16)  // first-bounce / bounce-round event counts
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 7, true, true, 16, true>), g, b, psh, stream, q, q.sph);
  else if (variant == 93 && tl && p.spp == 16)  // section clocks of the production kernel
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 3, true, true, 16, true>), g, b, psh, stream, q, q.sph);
  else if (variant == 93 && tl)
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 3, true, true>), g, b, psh, stream, q, q.sph);
  else if (variant == 93)
    hipLaunchKernelGGL((ao_batch_kernel<7, true, kPool, 3, false, true>), g, b, psh, stream, q, q.sph);
  else  // 17: without the split tail rounds
    hipLaunchKernelGGL(ao_batch_kernel<7>, g, b, psh, stream, q, q.sph);
  return true;
}
static bool ab_general() {
  const char* eg = getenv("RTRT_GENERAL");
  return eg && atoi(eg) == 1;
}

hipError_t launch_program(int program, const FrameParams& p, hipStream_t stream) {
  if (p.trace_rows <= 0) return hipSuccess;
  if (const char* es = getenv("RTRT_POST_SKIP"); es && atoi(es) == 1 && program == K_POST) return hipSuccess;  // A/B floor
  FrameParams q = launch_params(p);
  const bool pl = p.nplanes > 0;
  if (program == K_AOP || program == K_AO) {
    if (ab_launch_ao(p, q, stream, (long long)p.trace_rows * p.W)) return hipGetLastError();
    return launch_production(program, p, q, stream);
  }
  const int fpb = program == K_PHONG ? kPhongFramesPerBlock : kHybridFramesPerBlock;
  dim3 grid((p.W + 15) / 16, (p.trace_rows + 15) / 16, p.mf_n > 0 ? (p.mf_n + fpb - 1) / fpb : 1);
  if (const char* ea = getenv("RTRT_HY_ABL"); ea && program == K_HYBRID && !pl && atoi(ea) > 0) {
    const int a = atoi(ea);
    const size_t lt = tab_lds_bytes(p);  // (7: LDS tables, 8: production tables through the caches)
    if (kHyBW != 2) {  // 2x2 blocks here; the schedule's tables are sized for the production blocks
      q.tile_order = nullptr;
      q.tile_cost = nullptr;
    }
    if (a == 1) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 1>), grid, dim3(kBlock), 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    else if (a == 3) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 3>), grid, dim3(kBlock), 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    else if (a == 5) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 5>), grid, dim3(kBlock), 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    else if (a == 9) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 9>), grid, dim3(kBlock), 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    else if (a == 6) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 6>), grid, dim3(kBlock), 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    else if (a == 7) hipLaunchKernelGGL((hybrid_kernel<true, false, true, 7>), grid, dim3(kBlock), lt, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    else if (a == 8) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 7>), grid, dim3(kBlock), 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    else hipLaunchKernelGGL((hybrid_kernel<true, false, false, 2>), grid, dim3(kBlock), 0, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    return hipGetLastError();
  }
  if (const char* eb = getenv("RTRT_HY_BLK"); eb && program == K_HYBRID && !pl) {  // block shape A/B
    const int k = atoi(eb);
    auto gr = [&](int bwx, int bwy) { return dim3((p.W + 8 * bwx - 1) / (8 * bwx), (p.trace_rows + 8 * bwy - 1) / (8 * bwy)); };
    // the shim sizes the tile schedule's tables for the production blocks (kHyBW x kHyBW waves,
    // rt_shim.hip launch_sched): other shapes run in plain row order and record no costs
    const int bw = k / 10, bh = k % 10;
    if (bw != kHyBW || bh != kHyBW) {
      q.tile_order = nullptr;
      q.tile_cost = nullptr;
    }
    // (tables through the caches, as production since round 5: RT_HY_NOLT)
    if (k == 11) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, 1, 1>), gr(1, 1), dim3(64), 0, stream, q.tile_order, q.sph, q.shapes, gr(1, 1).x, q);
    else if (k == 21) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, 2, 1>), gr(2, 1), dim3(128), 0, stream, q.tile_order, q.sph, q.shapes, gr(2, 1).x, q);
    else if (k == 41) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, 4, 1>), gr(4, 1), dim3(256), 0, stream, q.tile_order, q.sph, q.shapes, gr(4, 1).x, q);
    else if (k == 42) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, 4, 2>), gr(4, 2), dim3(512), 0, stream, q.tile_order, q.sph, q.shapes, gr(4, 2).x, q);
    else if (k == 44) hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, 4, 4>), gr(4, 4), dim3(1024), 0, stream, q.tile_order, q.sph, q.shapes, gr(4, 4).x, q);
    else hipLaunchKernelGGL((hybrid_kernel<true, false, false, 0, 2, 2>), gr(2, 2), dim3(256), 0, stream, q.tile_order, q.sph, q.shapes, gr(2, 2).x, q);
    return hipGetLastError();
  }
  if (ab_general() && (program == K_PHONG || program == K_HYBRID)) {
    const size_t lds = shapes_lds_bytes(p);
    if (program == K_PHONG) hipLaunchKernelGGL((phong_kernel<false>), grid, dim3(kBlock), lds, stream, q.sph, q.shapes, q);
    else hipLaunchKernelGGL((hybrid_kernel<false>), grid, dim3(kBlock), lds, stream, q.tile_order, q.sph, q.shapes, grid.x, q);
    return hipGetLastError();
  }
  return launch_production(program, p, q, stream);
}

hipError_t launch_selftest(int fn, const float* d_in, float* d_out, size_t n, hipStream_t stream) {
  return launch_selftest_impl(fn, d_in, d_out, n, stream);
}

hipError_t launch_gbuf_convert(const GbufXfer& x, hipStream_t stream) { return launch_gbuf_convert_impl(x, stream); }

}  // namespace rt
