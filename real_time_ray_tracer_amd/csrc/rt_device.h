// rt_device.h — device-side GLSL math and ray/shape intersection for gfx950.
//
// Implements the float semantics documented in oracle/rt_oracle.h (the contract the CPU
// oracle and these kernels share): IEEE binary32, no implicit contraction (the library is
// built with -ffp-contract=off), dot() as a fused chain, IEEE sqrtf and '/', the
// deterministic binary64 sin inside random(), binary64 shadow-ray distance test.
// Reference: resources/p_compute.glsl:65-166, ao_compute.glsl:143-158.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rt {

struct f3 {
  float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator*(float s, f3 v) { return mk(s * v.x, s * v.y, s * v.z); }
__device__ __forceinline__ f3 xyz(float4 v) { return mk(v.x, v.y, v.z); }

// GLSL dot(): fmaf(a.z,b.z, fmaf(a.y,b.y, a.x*b.x))
__device__ __forceinline__ float dot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
// GLSL normalize(): v / length(v) with IEEE sqrt and division
__device__ __forceinline__ f3 normalize(f3 v) {
  float l = sqrtf(dot(v, v));
  return mk(v.x / l, v.y / l, v.z / l);
}
// GLSL 4.60 §8.3 definitions: max(x,y) = x < y ? y : x; min(x,y) = y < x ? y : x
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }

// ---- deterministic sin: binary64 Cody-Waite reduction by pi/2 + fdlibm kernels ----------
// (bit-identical to oracle/rt_oracle.c rto_sin; any finite float input)
__device__ __forceinline__ float det_sin(float xf) {
  constexpr double INV_PIO2 = 6.36619772367581382433e-01;
  constexpr double PIO2_1 = 1.57079632673412561417e+00;
  constexpr double PIO2_2 = 6.07710050630396597660e-11;
  constexpr double PIO2_3 = 2.02226624879595063154e-21;
  constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                   S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                   S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                   C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                   C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double x = (double)xf;
  if (!(fabs(x) <= 3.4028234663852886e38)) return xf - xf;
  double k = rint(x * INV_PIO2);
  double r = fma(-k, PIO2_1, x);
  r = fma(-k, PIO2_2, r);
  r = fma(-k, PIO2_3, r);
  double q4 = k - 4.0 * floor(k * 0.25);
  int q = (int)q4;
  double z = r * r;
  double ps = fma(z, fma(z, fma(z, fma(z, fma(z, S6, S5), S4), S3), S2), S1);
  double s = fma(r * z, ps, r);
  double pc = fma(z, fma(z, fma(z, fma(z, fma(z, C6, C5), C4), C3), C2), C1);
  double c = fma(z * z, pc, fma(-0.5, z, 1.0));
  double v = (q == 0) ? s : (q == 1) ? c : (q == 2) ? -s : -c;
  return (float)v;
}

// random(vec2), p_compute.glsl:65-75
__device__ __forceinline__ float grandom(float sx, float sy) {
  float d = fmaf(sy, 78.233f, sx * 12.9898f);
  float m = det_sin(d) * 43758.5453123f;
  return m - floorf(m);
}

// ---- scene tables ---------------------------------------------------------------------
// Compact per-shape table built by the host shim from simple_shapes[S][5]
// (packing: src/main.cpp:395-469):
//   geo[i]  = simple_shapes[i][0]                       (center,r | normal,dist)
//   geo2[i] = (simple_shapes[i][3].xyz, bits(int(id)))   (plane point p0 | -, shape id)
//   col[i]  = simple_shapes[i][4]                       (color, id)
//   aux[i]  = (simple_shapes[i][1].w, simple_shapes[i][3].w, 0, 0)  (emissive, reflectivity)
enum { SHAPE_SPHERE = 1, SHAPE_PLANE = 5 };

// sphere_eval_ray, p_compute.glsl:77-109
__device__ __forceinline__ float sphere_eval(f3 pos, f3 dir, float4 g) {
  f3 pmc = pos - xyz(g);
  float b = dot(dir, pmc);
  float del = fmaf(g.w, g.w, fmaf(b, b, -dot(pmc, pmc)));
  if (del < 0.0f) return -1.0f;
  if (del == 0.0f) return -1.0f * b;
  float s = sqrtf(del);
  float t1 = -1.0f * b + s;
  float t2 = -1.0f * b - s;
  if (t2 < 0.0f) return (t1 < 0.0f) ? -1.0f : t1;
  return t2;
}

// plane_eval_ray, p_compute.glsl:111-119
__device__ __forceinline__ float plane_eval(f3 pos, f3 dir, float4 g, float4 g2) {
  f3 n = xyz(g);
  float denom = dot(n, dir);
  if (denom < 0.001f && denom > -0.001f) return -1.0f;
  return dot(n, xyz(g2) - pos) / denom;
}

// eval_ray, p_compute.glsl:121-138
__device__ __forceinline__ float eval_shape(f3 pos, f3 dir, float4 g, float4 g2) {
  int id = __float_as_int(g2.w);
  if (id == SHAPE_SPHERE) return sphere_eval(pos, dir, g);
  if (id == SHAPE_PLANE) return plane_eval(pos, dir, g, g2);
  return -1.0f;
}

// Closest hit over the scene (p_compute.glsl:177-188 with thr 0; h_compute.glsl:199-210 with
// 0.001; ao_compute.glsl:183-194 with 0.0001).  The lowest index wins ties (strict '<').
// ALLSPH: every shape is a sphere (host-checked), so the id dispatch is compiled out.
// Fast path: the discriminant sign is tested first; the sqrt tail runs only for lanes whose
// ray meets the sphere, and is skipped by the whole wave when none does.
template <bool ALLSPH>
__device__ __forceinline__ int closest_hit(const float4* __restrict__ geo, const float4* __restrict__ geo2,
                                           int nobj, f3 pos, f3 dir, float thr, float& t_out) {
  float t = -1.0f;
  int ind = -1;
  for (int i = 0; i < nobj; ++i) {
    float4 g = geo[i];
    float res;
    if (ALLSPH) {
      f3 pmc = pos - xyz(g);
      float b = dot(dir, pmc);
      float del = fmaf(g.w, g.w, fmaf(b, b, -dot(pmc, pmc)));
      if (!(del >= 0.0f)) continue;  // del < 0 -> -1 (never accepted); NaN -> NaN (never accepted)
      if (del == 0.0f) {
        res = -1.0f * b;
      } else {
        float s = sqrtf(del);
        float t1 = -1.0f * b + s;
        float t2 = -1.0f * b - s;
        res = (t2 < 0.0f) ? ((t1 < 0.0f) ? -1.0f : t1) : t2;
      }
    } else {
      res = eval_shape(pos, dir, g, geo2[i]);
    }
    if (res > thr) {
      if (res < t || t < 0.0f) {
        t = res;
        ind = i;
      }
    }
  }
  t_out = t;
  return ind;
}

// shadow_ray, p_compute.glsl:145-166: any occluder with double t > 0.0001 closer than the light
template <bool ALLSPH>
__device__ __forceinline__ bool shadow_lit(const float4* __restrict__ geo, const float4* __restrict__ geo2,
                                           int nobj, f3 light, f3 pos) {
  f3 lv = light - pos;
  f3 l = normalize(lv);
  float len = sqrtf(dot(lv, lv));
  f3 np = pos + 0.01f * l;
  const double dlen = (double)len;
  for (int i = 0; i < nobj; ++i) {
    float tf = ALLSPH ? sphere_eval(np, l, geo[i]) : eval_shape(np, l, geo[i], geo2[i]);
    double t = (double)tf;
    if (t > (double)0.0001f) {
      double dx = t * (double)l.x, dy = t * (double)l.y, dz = t * (double)l.z;
      double L = sqrt(fma(dz, dz, fma(dy, dy, dx * dx)));
      if (L < dlen) return false;
    }
  }
  return true;
}

// sphere normal or stored plane normal (p_compute.glsl:140-143, 199-202)
__device__ __forceinline__ f3 shape_normal(float4 g, int id, f3 p) {
  if (id == SHAPE_SPHERE) return normalize(p - xyz(g));
  if (id == SHAPE_PLANE) return xyz(g);
  return mk(0.0f, 0.0f, 0.0f);
}

}  // namespace rt
