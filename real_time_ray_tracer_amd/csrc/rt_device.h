// rt_device.h — device-side GLSL math and ray/shape intersection for gfx950.
//
// Implements the float semantics documented in oracle/rt_oracle.h (the contract the CPU
// oracle and these kernels share): IEEE binary32, no implicit contraction (the library is
// built with -ffp-contract=off), dot() as a fused chain, normalize = v * (1/sqrtf(dot)), the
// deterministic binary32 sin inside random(), binary64 shadow-ray distance test.
// Reference: resources/p_compute.glsl:65-166, ao_compute.glsl:143-158.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_sin.h"
#include "rt_sin_table.h"

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
// 1 / sqrtf(d), correctly rounded twice (IEEE sqrt, then IEEE division), as the reference
// semantics of normalize() (below).  When every active lane has d in [2^-96, 2^126) (always,
// in practice) it is computed as sqrt_rn_core (exact there) followed by v_rcp_f32 and one
// Newton step, fma(fma(-s, y, 1), y, y): that step returns 1.0f / s exactly for every
// normal s in [2^-126, 2^126] (checked on the device for all of them:
// tests/test_gpu_parity.py::test_rcp_rn_exhaustive), and s lies in [2^-48, 2^63).  Other
// inputs (0, tiny, huge, inf, NaN) take the compiler's sequence.  About 13 instructions
// shorter than the division + scaled sqrt it replaces.
__device__ __forceinline__ float sqrt_rn_core(float x);
__device__ __forceinline__ float rcp_rn_normal(float s) {
  const float y = __builtin_amdgcn_rcpf(s);
  return fmaf(fmaf(-s, y, 1.0f), y, y);
}
__device__ __forceinline__ float inv_len_rn(float d) {
  // d in [2^-96, 2^126) as one unsigned compare on the bits (NaN and negatives fail)
  const bool ok = __float_as_uint(d) - 0x0F800000u < 0x7E800000u - 0x0F800000u;
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(!ok) == 0, 1)) return rcp_rn_normal(sqrt_rn_core(d));
  return 1.0f / sqrtf(d);
}
// a / b for a divisor b known ahead with y = 1.0f / b (correctly rounded): Markstein's
// refinement q = a*y, r = fma(-b, q, a) (exact), q' = fma(r, y, q).  By Markstein's theorem
// q' is the correctly rounded a / b whenever there is no underflow or overflow (a / b, y and
// b normal); the device sweep tools/micro/div_sweep.hip finds no mismatch for a in
// [2^-100, 2^100) with b = 6 and every configured width and height (mismatches appear only
// where a / b is subnormal).  Callers pass a = 0, NaN, or |a| in [2^-40, 2^14].  3
// instructions instead of the 11 of the IEEE division sequence.
__device__ __forceinline__ float div_rn_by(float a, float b, float y) {
  const float q = a * y;
  return fmaf(fmaf(-b, q, a), y, q);
}
// GLSL normalize(): v * (1 / length(v)) with IEEE sqrt and division (GPU GLSL compilers
// lower normalize to a reciprocal-square-root multiply; this is its correctly rounded form)
__device__ __forceinline__ f3 normalize(f3 v) {
  float il = inv_len_rn(dot(v, v));
  return mk(v.x * il, v.y * il, v.z * il);
}
// GLSL normalize(vec2)
__device__ __forceinline__ void normalize2(float& x, float& y) {
  float il = inv_len_rn(fmaf(y, y, x * x));
  x = x * il;
  y = y * il;
}
// GLSL 4.60 §8.3 definitions: max(x,y) = x < y ? y : x; min(x,y) = y < x ? y : x
__device__ __forceinline__ float gmax(float x, float y) { return x < y ? y : x; }
__device__ __forceinline__ float gmin(float x, float y) { return y < x ? y : x; }
__device__ __forceinline__ float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }

// ---- sin in random(): the correctly rounded binary32 sin (rt_sin.h), in two tiers.  Tier 1
// (det_sin_n): the binary64 reduction by pi and a degree-5 polynomial (relative error 2^-43.7),
// rounded to binary32 when that rounding is unambiguous within 2048 binary64 ulps.  The rare
// lanes — 1 in 2^17 ambiguous at tier 1, or an argument beyond the reduction's range (|x| >=
// 2^22, inf, NaN) — take det_sin_rare behind a wave-uniform branch: rt_sin.h's degree-6 /
// Payne-Hanek binary64 value, its 16-ulp ambiguity test, and the exception table.  Checked on
// all 2^32 inputs against the oracle (tests/test_gpu_parity.py::test_det_sin_exhaustive).
// Rounds 1-4 used a binary32 reduction and polynomial here (a faithful sin, 17 VALU), which a
// CPU re-execution with the math library's sin could not reproduce (round-4 review).
__device__ __noinline__ static float det_sin_rare(float x) {
  if (!(__builtin_fabsf(x) <= 0x1.fffffep127f)) return x - x;  // inf, NaN -> NaN
  const double s = sin_binary64(x);
  if (!sin_ambiguous(s)) return (float)s;
  const uint32_t b = __float_as_uint(x);
  int lo = 0, hi = kSinTableN;  // lower bound of b in the sorted table
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (kSinTableX[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  return (lo < kSinTableN && kSinTableX[lo] == b) ? __uint_as_float(kSinTableY[lo]) : (float)s;
}

// IEEE binary32 square root, correctly rounded: the value sqrtf() has under
// -fhip-fp32-correctly-rounded-divide-sqrt, written out so it stays a short straight-line
// sequence: inputs below 2^-96 are scaled by 2^32, v_sqrt_f32 (<= 1 ulp) is corrected by one
// ulp either way from the sign of the fma residuals, and the result is scaled back by 2^-16.
// 0, +inf and NaN pass through.  Checked against sqrtf on every non-negative float
// (tests/test_gpu_parity.py::test_sqrt_rn_exhaustive).
__device__ __forceinline__ float sqrt_rn(float x) {
  const bool tiny = x < 0x1p-96f;
  const float xs = tiny ? x * 0x1p32f : x;
  float s = __builtin_amdgcn_sqrtf(xs);
  const float sm = __int_as_float(__float_as_int(s) - 1);
  const float sp = __int_as_float(__float_as_int(s) + 1);
  const float rm = fmaf(-sm, s, xs);
  const float rp = fmaf(-sp, s, xs);
  s = (rm <= 0.0f) ? sm : s;
  s = (rp > 0.0f) ? sp : s;
  return tiny ? s * 0x1p-16f : s;
}

// IEEE binary32 square root for x in [2^-96, FLT_MAX], from the reciprocal square root:
// y = v_rsq_f32(x), g = x*y, h = y/2, r = fma(-g, g, x) (exact), s = fma(r, h, g) — Markstein's
// correction step.  One transcendental and 4 VALU instead of v_sqrt_f32 + the 8-instruction
// one-ulp fix-up.  Equal to sqrtf on EVERY float of that range (device sweep:
// tests/test_gpu_parity.py::test_sqrt_tail_exhaustive, RT_MATH_SQRT_TAIL_SWEEP).  Outside it:
// 0 gives NaN (0 * inf) and +inf gives NaN, so callers clamp or range-check.
__device__ __forceinline__ float sqrt_rn_core(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
  const float g = x * y, h = 0.5f * y;
  return fmaf(fmaf(-g, g, x), h, g);
}

// sqrt_rn without the tiny-input scaling, for the hit tail of sphere_candidate when the
// acceptance threshold is >= 1e-6: sqrt_rn_core of max(x, 2^-100).  Equal to sqrt_rn for x in
// [2^-96, FLT_MAX].  Below 2^-96 it returns some value in [0, 2^-47] (checked by the same
// sweep), and no caller can tell: with s < 2^-47 and |b| >= 2^-22, s is below a quarter ulp
// of b, so fl(-b + s) and fl(-b - s) are both -b whatever s is; with |b| < 2^-22 both roots
// are below 2.4e-7 in magnitude and never pass the threshold.  Accepted t and index are
// therefore unchanged.  (x = +inf, a discriminant that overflowed — |b| > 2^64 — gives NaN,
// which the caller rejects, where sqrt_rn gives +inf.)
// (The clamp is one v_max_f32 written out: fmaxf adds a canonicalising v_max in front of it,
// which buys nothing here, x being a non-negative discriminant and never NaN.)
__device__ __forceinline__ float sqrt_rn_tail(float x) {
  float xc;
  asm("v_max_f32_e32 %0, 0x0d800000, %1" : "=v"(xc) : "v"(x));  // max(x, 2^-100)
  return sqrt_rn_core(xc);
}

// sin of N arguments at once (tier 1 above), the same operations per argument: each binary64 constant is
// materialised once for the N (two s_mov_b32, or one v_mov_b64 for the polynomial's first step,
// whose two constants cannot both be SGPR operands) and the N independent chains interleave.
template <int N>
__device__ __forceinline__ void det_sin_n(const float (&x)[N], float (&y)[N]) {
  using namespace sinrn;
  double r[N], kd[N], z[N], p[N];
  const double ci = sconst(kInvPi);
#ifndef RT_SIN_MAGIC
#define RT_SIN_MAGIC 1
#endif
#if RT_SIN_MAGIC
  // k = x/pi rounded to an integer by adding 1.5*2^52 (one VGPR pair per group: a v_fma_f64 cannot
  // take two SGPR constants): k's parity is bit 0 of the sum's low word, so no v_cvt_i32_f64
  double rnd = sconst(0x1.8p52);
  asm volatile("" : "+v"(rnd));
  uint32_t par[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    r[i] = (double)x[i];
    const double t = fma(r[i], ci, rnd);
    par[i] = (uint32_t)dbits(t);
    kd[i] = t - sconst(0x1.8p52);
  }
#else
#pragma unroll
  for (int i = 0; i < N; ++i) {
    r[i] = (double)x[i];
    kd[i] = __builtin_rint(fma(r[i], ci, 0.0));
  }
#endif
  const double pa = sconst(kPiA);
#pragma unroll
  for (int i = 0; i < N; ++i) r[i] = fma(-kd[i], pa, r[i]);
  const double pb = sconst(kPiB);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    r[i] = fma(-kd[i], pb, r[i]);
    z[i] = r[i] * r[i];
  }
  const double c5 = sconst(kQ5);
  double c4 = sconst(kQ4);  // into a VGPR pair here (one v_mov_b64), not hoisted out of the loop
  asm volatile("" : "+v"(c4));
#pragma unroll
  for (int i = 0; i < N; ++i) p[i] = fma(c5, z[i], c4);
#define RT_SIN_STEP(c)                                        \
  {                                                           \
    const double cc = sconst(c);                              \
    _Pragma("unroll") for (int i = 0; i < N; ++i) p[i] = fma(p[i], z[i], cc); \
  }
  RT_SIN_STEP(kQ3) RT_SIN_STEP(kQ2) RT_SIN_STEP(kQ1) RT_SIN_STEP(kQ0)
#undef RT_SIN_STEP
  unsigned rare = 0;  // bit i: argument i goes to tier 2 (the binary64 values die here)
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const double si = r[i] * fma(z[i], p[i], 1.0);  // sin_poly
#if RT_SIN_MAGIC
    const double sv = dfrom(dbits(si) ^ ((uint64_t)par[i] << 63));
#else
    const double sv = dfrom(dbits(si) ^ ((uint64_t)(uint32_t)(int32_t)kd[i] << 63));
#endif
    y[i] = (float)sv;
    rare |= (unsigned)(!(__builtin_fabsf(x[i]) < 0x1p22f) || sin_ambiguous<kSinFastAmbUlps>(sv)) << i;
  }
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(rare != 0) != 0, 0)) {
#pragma unroll
    for (int i = 0; i < N; ++i)
      if ((rare >> i) & 1u) y[i] = det_sin_rare(x[i]);
  }
}
__device__ __forceinline__ float det_sin(float x) {
  float y[1];
  det_sin_n<1>({x}, y);
  return y[0];
}

// random(vec2), p_compute.glsl:65-75
__device__ __forceinline__ float grandom(float sx, float sy) {
  float d = fmaf(sy, 78.233f, sx * 12.9898f);
  float m = det_sin(d) * 43758.5453123f;
  return m - floorf(m);
}
// N random() calls at once (det_sin_n); the same float operations per call as grandom
#ifndef RT_SIN_WIDE
#define RT_SIN_WIDE 1
#endif
template <int N>
__device__ __forceinline__ void grandom_n(const float (&sx)[N], const float (&sy)[N], float (&out)[N]) {
  float d[N], s[N];
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = fmaf(sy[i], 78.233f, sx[i] * 12.9898f);
  if (RT_SIN_WIDE) {
    det_sin_n<N>(d, s);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] = det_sin(d[i]);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float m = s[i] * 43758.5453123f;
    out[i] = m - floorf(m);
  }
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

// sphere_eval for shadow rays, whose result is only compared with 0.0001 (p_compute.glsl:
// 145-166): the square root is sqrt_rn_tail, which by its contract (thr >= 1e-6) leaves every
// t > 0.0001 decision and every accepted t unchanged.
__device__ __forceinline__ float sphere_eval_shadow(f3 pos, f3 dir, float4 g) {
  f3 pmc = pos - xyz(g);
  float b = dot(dir, pmc);
  float del = fmaf(g.w, g.w, fmaf(b, b, -dot(pmc, pmc)));
  if (del < 0.0f) return -1.0f;
  if (del == 0.0f) return -1.0f * b;
  float s = sqrt_rn_tail(del);
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

// One ray-sphere candidate of the min-t scan: updates t/ind when sphere i becomes the closest
// hit.  Equivalent to sphere_eval + the scan's acceptance test: a miss (del < 0, or NaN) yields
// -1 / NaN in the reference, which the scan never accepts.
// The hit tail sits behind a wave-uniform branch (a ballot of del >= 0; one scalar compare and
// branch instead of an exec-mask save / branch / restore, which keeps the CU's one scalar unit
// free: config (d) -1.9% with the bounce rounds' 4-sphere groups, (c) -2.9%).  When some lane
// takes it, the tail runs on every active lane and del >= 0 joins the acceptance: a lane with a
// negative discriminant computes a finite, rejected root (the tail's square root sees
// max(del, 2^-100)); NaN fails both compares.  Accepted t and index are unchanged.
__device__ __forceinline__ void sphere_candidate(f3 pos, f3 dir, float4 g, int i, float thr, float& t, int& ind) {
  f3 pmc = pos - xyz(g);
  float b = dot(dir, pmc);
  float del = fmaf(g.w, g.w, fmaf(b, b, -dot(pmc, pmc)));
  const bool hit = del >= 0.0f;
  if (__builtin_amdgcn_ballot_w64(hit) != 0) {
    // One straight-line tail for del == 0 and del > 0: with s = sqrt(0) = 0 both roots are
    // -b, so the reference's (del == 0 ? -b : root choice) differs only in values <= 0, and
    // (t2 < 0 ? t1 : t2) differs from (t2 < 0 ? (t1 < 0 ? -1 : t1) : t2) only when t1 < 0:
    // none of these is ever accepted (thr > 0).  Accepted t and index are unchanged.
    float s = thr >= 1e-6f ? sqrt_rn_tail(del) : sqrt_rn(del);  // thr is a literal at every call
    float t1 = -1.0f * b + s;
    float t2 = -1.0f * b - s;
    // (t2 < 0 ? t1 : t2) as an unsigned min of the bits: t1 >= t2, so for t2 >= 0 both are
    // non-negative and the min is t2; a negative t2 has its sign bit set and loses to t1 >= 0;
    // the remaining cases (both negative, or t2 = -0 with t1 = +0) give a value <= 0 either
    // way, which the acceptance below rejects (thr >= 0)
    float res = __uint_as_float(min(__float_as_uint(t1), __float_as_uint(t2)));
    // (res < t || t < 0) as one unsigned compare: t is -1.0f (no hit yet, bits 0xBF800000, above
    // every positive float's bits, +inf included) or an accepted res > thr >= 0; for res > thr
    // (positive, not NaN) and positive t the float and bit orders agree
    const bool acc = hit & (res > thr) & (__float_as_uint(res) < __float_as_uint(t));  // no short-circuit branches
    t = acc ? res : t;
    ind = acc ? i : ind;
  }
}

// sphere_candidate for a ray from the camera, with the sphere's camera-relative row q = (pmc, pp)
// precomputed: pmc = cam - centre and pp = dot(pmc, pmc), the values sphere_candidate computes
// first (rt_shim pack_header, the same binary32 operations), and the radius r.  Bit for bit the
// same (t, ind) as sphere_candidate(cam, dir, g, ...).
__device__ __forceinline__ void sphere_candidate_rel(f3 dir, float4 q, float r, int i, float thr, float& t, int& ind) {
  const float b = dot(dir, xyz(q));
  const float del = fmaf(r, r, fmaf(b, b, -q.w));
  const bool hit = del >= 0.0f;
  if (__builtin_amdgcn_ballot_w64(hit) != 0) {
    // the tail of sphere_candidate (see there)
    float s = thr >= 1e-6f ? sqrt_rn_tail(del) : sqrt_rn(del);
    float t1 = -1.0f * b + s;
    float t2 = -1.0f * b - s;
    float res = __uint_as_float(min(__float_as_uint(t1), __float_as_uint(t2)));
    const bool acc = hit & (res > thr) & (__float_as_uint(res) < __float_as_uint(t));
    t = acc ? res : t;
    ind = acc ? i : ind;
  }
}

// sphere_candidate for the lanes with `on` only (the others run the arithmetic and accept nothing):
// callers branch on a wave-uniform ballot of `on` instead of masking exec per lane.
__device__ __forceinline__ void sphere_candidate_if(f3 pos, f3 dir, float4 g, int i, float thr, float& t, int& ind,
                                                    unsigned long long onm) {
  // onm: the lanes whose pre-test passed, as the wave mask (the caller's ballot).  Every
  // decision stays a scalar mask: the branch on (del >= 0) & onm, and the acceptance mask that
  // drives the two selects (VOP3 v_cndmask with an SGPR-pair mask).  With a per-lane bool
  // argument the compiler rebuilt the mask through a v_cndmask + v_cmp pair per survivor.
  f3 pmc = pos - xyz(g);
  float b = dot(dir, pmc);
  float del = fmaf(g.w, g.w, fmaf(b, b, -dot(pmc, pmc)));
  const unsigned long long hm = __builtin_amdgcn_ballot_w64(del >= 0.0f) & onm;
  if (hm != 0) {
    // One straight-line tail for del == 0 and del > 0: with s = sqrt(0) = 0 both roots are
    // -b, so the reference's (del == 0 ? -b : root choice) differs only in values <= 0, and
    // (t2 < 0 ? t1 : t2) differs from (t2 < 0 ? (t1 < 0 ? -1 : t1) : t2) only when t1 < 0:
    // none of these is ever accepted (thr > 0).  Accepted t and index are unchanged.
    float s = thr >= 1e-6f ? sqrt_rn_tail(del) : sqrt_rn(del);  // thr is a literal at every call
    float t1 = -1.0f * b + s;
    float t2 = -1.0f * b - s;
    // (t2 < 0 ? t1 : t2) as an unsigned min of the bits: t1 >= t2, so for t2 >= 0 both are
    // non-negative and the min is t2; a negative t2 has its sign bit set and loses to t1 >= 0;
    // the remaining cases (both negative, or t2 = -0 with t1 = +0) give a value <= 0 either
    // way, which the acceptance below rejects (thr >= 0)
    float res = __uint_as_float(min(__float_as_uint(t1), __float_as_uint(t2)));
    // (res < t || t < 0) as one unsigned compare: t is -1.0f (no hit yet, bits 0xBF800000, above
    // every positive float's bits, +inf included) or an accepted res > thr >= 0; for res > thr
    // (positive, not NaN) and positive t the float and bit orders agree
    const unsigned long long am = hm & __builtin_amdgcn_ballot_w64(res > thr) &
                                  __builtin_amdgcn_ballot_w64(__float_as_uint(res) < __float_as_uint(t));
    float tn;
    int in;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(tn) : "v"(t), "v"(res), "s"(am));
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(in) : "v"(ind), "v"(i), "s"(am));
    t = tn;
    ind = in;
  }
}

// The lowest set bit of a wave-uniform 64-bit mask, cleared with one s_bitset0_b64 (the
// compiler's m & (m - 1) is a 64-bit subtract and an and: three scalar instructions).
__device__ __forceinline__ int pop_lowest(unsigned long long& m) {
  const int j = __builtin_ctzll(m);
  asm("s_bitset0_b64 %0, %1" : "+s"(m) : "s"(j));
  return j;
}

// One plane of the min-t scan, tested out of index order (after the spheres): plane_eval_ray
// (p_compute.glsl:111-119) and the scan's acceptance, with the tie rule made explicit.  The
// sequential scan (`res > thr && (res < t || t < 0)`, ascending i) ends with the accepted
// candidate of least t and, among equal t, least index; that lexicographic minimum does not
// depend on the visiting order, so testing the planes after the spheres gives the same (t, ind).
// a = (normal, bits(index)), b = (p0, 0) (rt_kernels.h plane table).
__device__ __forceinline__ void plane_candidate(f3 pos, f3 dir, float4 a, float4 b, float thr, float& t, int& ind) {
  const float res = plane_eval(pos, dir, a, b);
  const int i = __float_as_int(a.w);
  const bool acc = res > thr && (t < 0.0f || res < t || (res == t && i < ind));
  t = acc ? res : t;
  ind = acc ? i : ind;
}

// All-sphere closest hit with the min-t update inside the hit branch and the geometry of 4
// spheres fetched before any of them is tested (V = 2: global table read with wave-uniform
// scalar loads; V = 0: closest_hit).  Bit-identical to closest_hit.
template <bool ALLSPH, int V>
__device__ __forceinline__ int closest_hit_v(const float4* __restrict__ geo, const float4* __restrict__ geo2,
                                             int nobj, f3 pos, f3 dir, float thr, float& t_out) {
  if (V == 0 || !ALLSPH) return closest_hit<ALLSPH>(geo, geo2, nobj, pos, dir, thr, t_out);
  float t = -1.0f;
  int ind = -1;
  int i = 0;
  for (; i + 4 <= nobj; i += 4) {
    float4 g0 = geo[i], g1 = geo[i + 1], g2 = geo[i + 2], g3 = geo[i + 3];
    sphere_candidate(pos, dir, g0, i, thr, t, ind);
    sphere_candidate(pos, dir, g1, i + 1, thr, t, ind);
    sphere_candidate(pos, dir, g2, i + 2, thr, t, ind);
    sphere_candidate(pos, dir, g3, i + 3, thr, t, ind);
  }
  for (; i < nobj; ++i) sphere_candidate(pos, dir, geo[i], i, thr, t, ind);
  t_out = t;
  return ind;
}

// All-sphere closest hit with the scalar geometry loads software-pipelined: the next 4
// spheres are requested before the current 4 are tested, so the scalar-cache latency overlaps
// the tests.  Same visiting order and acceptance as closest_hit (bit-identical).
__device__ __forceinline__ int closest_hit_pf(const float4* __restrict__ geo, int nobj, f3 pos, f3 dir, float thr,
                                              float& t_out) {
  float t = -1.0f;
  int ind = -1;
  int i = 0;
  if (nobj >= 4) {
    float4 g0 = geo[0], g1 = geo[1], g2 = geo[2], g3 = geo[3];
    for (; i + 8 <= nobj; i += 4) {
      float4 n0 = geo[i + 4], n1 = geo[i + 5], n2 = geo[i + 6], n3 = geo[i + 7];
      sphere_candidate(pos, dir, g0, i, thr, t, ind);
      sphere_candidate(pos, dir, g1, i + 1, thr, t, ind);
      sphere_candidate(pos, dir, g2, i + 2, thr, t, ind);
      sphere_candidate(pos, dir, g3, i + 3, thr, t, ind);
      g0 = n0; g1 = n1; g2 = n2; g3 = n3;
    }
    sphere_candidate(pos, dir, g0, i, thr, t, ind);
    sphere_candidate(pos, dir, g1, i + 1, thr, t, ind);
    sphere_candidate(pos, dir, g2, i + 2, thr, t, ind);
    sphere_candidate(pos, dir, g3, i + 3, thr, t, ind);
    i += 4;
  }
  for (; i < nobj; ++i) sphere_candidate(pos, dir, geo[i], i, thr, t, ind);
  t_out = t;
  return ind;
}

// closest_hit_pf over the n <= 64 spheres geo[0..n) (indices base + i) whose bit is set in the
// wave-uniform mask m: the table is still streamed 4 spheres per scalar load, prefetched one
// group ahead, and a sphere whose bit is clear is skipped by a scalar branch.  Ascending order
// with the strict '<' of sphere_candidate, so the result equals closest_hit's on the set bits.
__device__ __forceinline__ void closest_hit_pf_masked(const float4* __restrict__ geo, int n, int base,
                                                      unsigned long long m, f3 pos, f3 dir, float thr, float& t,
                                                      int& ind) {
  int i = 0;
  if (n >= 4) {
    float4 g0 = geo[0], g1 = geo[1], g2 = geo[2], g3 = geo[3];
    for (; i + 8 <= n; i += 4) {
      float4 n0 = geo[i + 4], n1 = geo[i + 5], n2 = geo[i + 6], n3 = geo[i + 7];
      const unsigned nib = (unsigned)(m >> i) & 0xfu;
      if (nib) {
        if (nib & 1u) sphere_candidate(pos, dir, g0, base + i, thr, t, ind);
        if (nib & 2u) sphere_candidate(pos, dir, g1, base + i + 1, thr, t, ind);
        if (nib & 4u) sphere_candidate(pos, dir, g2, base + i + 2, thr, t, ind);
        if (nib & 8u) sphere_candidate(pos, dir, g3, base + i + 3, thr, t, ind);
      }
      g0 = n0; g1 = n1; g2 = n2; g3 = n3;
    }
    const unsigned nib = (unsigned)(m >> i) & 0xfu;
    if (nib & 1u) sphere_candidate(pos, dir, g0, base + i, thr, t, ind);
    if (nib & 2u) sphere_candidate(pos, dir, g1, base + i + 1, thr, t, ind);
    if (nib & 4u) sphere_candidate(pos, dir, g2, base + i + 2, thr, t, ind);
    if (nib & 8u) sphere_candidate(pos, dir, g3, base + i + 3, thr, t, ind);
    i += 4;
  }
  for (; i < n; ++i)
    if ((m >> i) & 1ull) sphere_candidate(pos, dir, geo[i], base + i, thr, t, ind);
}

// closest_hit_pf with groups of 2 spheres (one s_load_dwordx8 each): half the scalar registers
// of the 4-sphere pipeline.  Same visiting order and acceptance (bit-identical).
__device__ __forceinline__ int closest_hit_pf2(const float4* __restrict__ geo, int nobj, f3 pos, f3 dir, float thr,
                                               float& t_out) {
  float t = -1.0f;
  int ind = -1;
  int i = 0;
  if (nobj >= 2) {
    float4 g0 = geo[0], g1 = geo[1];
    for (; i + 4 <= nobj; i += 2) {
      float4 n0 = geo[i + 2], n1 = geo[i + 3];
      sphere_candidate(pos, dir, g0, i, thr, t, ind);
      sphere_candidate(pos, dir, g1, i + 1, thr, t, ind);
      g0 = n0; g1 = n1;
    }
    sphere_candidate(pos, dir, g0, i, thr, t, ind);
    sphere_candidate(pos, dir, g1, i + 1, thr, t, ind);
    i += 2;
  }
  for (; i < nobj; ++i) sphere_candidate(pos, dir, geo[i], i, thr, t, ind);
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
    float tf = ALLSPH ? sphere_eval_shadow(np, l, geo[i]) : eval_shape(np, l, geo[i], geo2[i]);
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
