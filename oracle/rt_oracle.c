/*
 * rt_oracle.c — CPU restatement of the reference's five compute shaders.
 * TEST INFRASTRUCTURE ONLY (see rt_oracle.h): the checker for the HIP path and the CPU
 * baseline of bench.py.  Parity unpinned by reference artifacts (none exist); see header.
 *
 * Function-by-function restatement of
 *   resources/p_compute.glsl:65-245         (random, sphere/plane/eval_ray, shadow_ray, phong, main)
 *   resources/h_compute.glsl:168-321        (hybrid_helper, hybrid, main)
 *   resources/ao_compute.glsl:143-339       (get_pt_within_unit_sphere, ambient_occlusion*, main)
 *   resources/aop_compute.glsl:141-336      (= ao_compute without the imageStore)
 *   resources/aop_postprocessing.glsl:57-208 (spatial + temporal filter)
 * and the dispatch of src/main.cpp:553-671.  Compile with -ffp-contract=off.
 */
#include "rt_oracle.h"

#include <immintrin.h>
#include <math.h>
#include <quadmath.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/rt/layout.h"

/* ------------------------------------------------------------------------------------ */
/* float helpers                                                                        */
/* ------------------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

static inline v3 mk3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 sub3(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 add3(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 scl3(float s, v3 v) { return mk3(s * v.x, s * v.y, s * v.z); }
/* GLSL dot(): fused chain */
static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
/* GLSL normalize(): v * (1 / length(v)) — the correctly rounded form of the reciprocal-
 * square-root multiply GPU GLSL compilers emit */
static inline v3 nrm3(v3 v) {
  float il = 1.0f / sqrtf(dot3(v, v));
  return mk3(v.x * il, v.y * il, v.z * il);
}
/* GLSL min/max/clamp definitions (GLSL 4.60 §8.3): max(x,y) = x < y ? y : x, etc. */
static inline float gmax(float x, float y) { return x < y ? y : x; }
static inline float gmin(float x, float y) { return y < x ? y : x; }
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }

/* ------------------------------------------------------------------------------------ */
/* sin inside random(): the correctly rounded binary32 sin (see rt_oracle.h).            */
/* glibc's binary64 sin (error < 1 ulp) rounded once to binary32.  Where that rounding   */
/* is ambiguous — the binary64 value within 8 ulps of a binary32 midpoint, i.e. its low  */
/* 29 significand bits within 8 of 2^28, 1 input in 2^25 — quad precision (libquadmath   */
/* sinq, 113 bits) decides.  A binary64 value that is a binary32 denormal is exact here  */
/* (sin(x) rounds to x for |x| < 2^-26), so the midpoint test never misreads one.        */
/* Written independently of the kernels' sin (real_time_ray_tracer_amd/csrc/rt_sin.h:    */
/* reduction by pi, their own polynomial, Payne-Hanek, an exception table).              */
/* ------------------------------------------------------------------------------------ */
float rto_sin(float x) {
  if (!isfinite(x)) return x - x; /* NaN */
  const double s = sin((double)x);
  uint64_t u;
  memcpy(&u, &s, sizeof u);
  const uint32_t low = (uint32_t)u & 0x1FFFFFFFu;
  if (low - (0x10000000u - 8u) <= 16u) return (float)sinq((__float128)x);
  return (float)s;
}

/* exhaustive-sweep support: got[i] is the device's sin of the float whose bit pattern is
   start + i (mod 2^32); counts the i where rto_sin disagrees bit for bit (NaN == NaN) and
   records the first max_bad of those bit patterns */
int64_t rto_sin_check_range(uint32_t start, int64_t n, const float* got, uint32_t* bad, int max_bad) {
  int64_t count = 0;
#pragma omp parallel for schedule(static, 1 << 16)
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t b = start + (uint32_t)i;
    float x;
    memcpy(&x, &b, 4);
    const float want = rto_sin(x);
    uint32_t wb, gb;
    memcpy(&wb, &want, 4);
    memcpy(&gb, &got[i], 4);
    if (wb != gb && !(isnan(want) && isnan(got[i]))) {
      int64_t k;
#pragma omp atomic capture
      k = count++;
      if (k < max_bad) bad[k] = b;
    }
  }
  return count;
}

/* Contraction of random()'s argument arithmetic (measurement hook, rto_set_contraction): the
   GLSL leaves it to the compiler whether a*b+c is one fma or two roundings, and the hash
   (sin * 43758.5) amplifies either choice into a different sample.  0 = this build's semantics
   (the kernels'): dot() inside random() fused as below, the seed and jitter sums unfused, as
   written.  RTO_C_UNFUSED_DOT: dot(st, c) = st.x*c.x + st.y*c.y with both products rounded
   (ao_compute.glsl:63-73 read literally).  RTO_C_FUSED_SEEDS: the hemisphere seeds contracted as a
   GLSL compiler does by default (seed1 + xy*seed4 -> fma(xy, seed4, seed1); seed2 - xy*seed4 ->
   fma(-xy, seed4, seed2); seed3*xy + seed4 -> fma(seed3, xy, seed4); ao_compute.glsl:152-157).
   RTO_C_FUSED_JITTER: the anti-aliasing seeds likewise (seed1 + xy*seed2 - xy + seed3 ->
   (fma(xy, seed2, seed1) - xy) + seed3; seed4*xy - seed3*xy*seed2 -> fma(seed4, xy,
   -((seed3*xy)*seed2)); ao_compute.glsl:317-319). */
static int rto_contract = 0;
void rto_set_contraction(int flags) { rto_contract = flags; }
int rto_get_contraction(void) { return rto_contract; }

/* random(vec2) — p_compute.glsl:65-75: fract(sin(dot(st, vec2(12.9898,78.233))) * 43758.5453123) */
float rto_random(float sx, float sy) {
  float d = (rto_contract & RTO_C_UNFUSED_DOT) ? sx * 12.9898f + sy * 78.233f : fmaf(sy, 78.233f, sx * 12.9898f);
  float m = rto_sin(d) * 43758.5453123f;
  return m - floorf(m);
}

/* ------------------------------------------------------------------------------------ */
/* frame context                                                                        */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  const rto_dims* d;
  float* ssbo;
  const float* shapes; /* simple_shapes[S][5] vec4 */
  const float* rb;     /* rand_buffer[2*AA] vec4 */
  float* pix;          /* pixels[F][W][gh] vec4 */
  float* nrm;
  float* dep;
  int frame;
  int nobj;
  v3 horiz, vert, llc, cam, light;
  v4 bg;
  /* the sphere geometry of shapes [0, nobj) as structure-of-arrays, padded to a multiple of 8
     (NaN for non-spheres and padding: never accepted), and the indices of the planes: the
     closest-hit scan evaluates 8 (AVX2) or 16 (AVX-512) spheres per step (closest_hit below) */
  float* soa; /* [4][nsoa]: cx, cy, cz, r */
  int nsoa;
  int* planes;
  int nplanes;
} octx;

#define SH(c, i, j, k) ((c)->shapes[((size_t)(i) * 5 + (j)) * 4 + (k)])

static inline size_t gidx(const octx* c, int f, int x, int y) {
  return (((size_t)f * c->d->W + x) * c->d->gh + (size_t)(y - c->d->gy0)) * 4;
}

static int octx_init(octx* c, float* ssbo, const rto_dims* d, int frame) {
  if (!ssbo || !d || d->W <= 0 || d->H <= 0 || d->S < 0 || d->AA <= 0 || d->F <= 0 || d->D <= 0 ||
      d->gy0 < 0 || d->gh <= 0 || d->gy0 + d->gh > d->H || frame < 0 || frame >= d->F)
    return -1;
  c->d = d;
  c->ssbo = ssbo;
  c->shapes = ssbo + rt_off_shapes() / 4;
  c->rb = ssbo + rt_off_rand(d->S) / 4;
  c->pix = ssbo + rt_off_pixels(d->S, d->AA) / 4;
  c->nrm = ssbo + rt_off_normals(d->S, d->AA, d->W, d->gh, d->F) / 4;
  c->dep = ssbo + rt_off_depth(d->S, d->AA, d->W, d->gh, d->F) / 4;
  ssbo[RT_HDR_MODE * 4 + 1] = (float)frame; /* mode.y = frame_num (src/main.cpp:584) */
  c->frame = frame;
  c->nobj = (int)ssbo[RT_HDR_MODE * 4 + 2]; /* int(mode.z) */
  if (c->nobj > d->S) return -1;
  const float* h = ssbo;
  c->horiz = mk3(h[4 * RT_HDR_HORIZONTAL], h[4 * RT_HDR_HORIZONTAL + 1], h[4 * RT_HDR_HORIZONTAL + 2]);
  c->vert = mk3(h[4 * RT_HDR_VERTICAL], h[4 * RT_HDR_VERTICAL + 1], h[4 * RT_HDR_VERTICAL + 2]);
  c->llc = mk3(h[4 * RT_HDR_LLC_MINUS_CAMPOS], h[4 * RT_HDR_LLC_MINUS_CAMPOS + 1],
               h[4 * RT_HDR_LLC_MINUS_CAMPOS + 2]);
  c->cam = mk3(h[4 * RT_HDR_CAMERA_LOCATION], h[4 * RT_HDR_CAMERA_LOCATION + 1],
               h[4 * RT_HDR_CAMERA_LOCATION + 2]);
  c->light = mk3(h[4 * RT_HDR_LIGHT_POS], h[4 * RT_HDR_LIGHT_POS + 1], h[4 * RT_HDR_LIGHT_POS + 2]);
  c->bg.x = h[4 * RT_HDR_BACKGROUND];
  c->bg.y = h[4 * RT_HDR_BACKGROUND + 1];
  c->bg.z = h[4 * RT_HDR_BACKGROUND + 2];
  c->bg.w = h[4 * RT_HDR_BACKGROUND + 3];
  c->soa = NULL;
  c->planes = NULL;
  c->nsoa = c->nplanes = 0;
  return 0;
}

/* after octx_init: the structure-of-arrays sphere table and the plane list (freed by
   octx_free).  Together they are eval_ray's dispatch on int(shapes[i][4].w)
   (p_compute.glsl:121-138): id 1 = sphere_eval_ray, id 5 = plane_eval_ray, any other id
   (rectangle 3 included) returns -1, i.e. is never accepted — a NaN row here.
   Returns -1 when out of memory. */
static int octx_tables(octx* c) {
  int n8 = (c->nobj + 15) & ~15; /* a multiple of both vector widths */
  c->nsoa = n8;
  c->soa = (float*)malloc(sizeof(float) * 4 * (size_t)(n8 > 0 ? n8 : 1));
  c->planes = (int*)malloc(sizeof(int) * (size_t)(c->nobj > 0 ? c->nobj : 1));
  if (!c->soa || !c->planes) return -1;
  for (int i = 0; i < n8; i++) {
    int id = i < c->nobj ? (int)c->shapes[((size_t)i * 5 + 4) * 4 + 3] : -1;
    for (int k = 0; k < 4; k++)
      c->soa[(size_t)k * n8 + i] = id == RT_SHAPE_SPHERE ? c->shapes[(size_t)i * 5 * 4 + k] : NAN;
    if (id == RT_SHAPE_PLANE) c->planes[c->nplanes++] = i;
  }
  return 0;
}

static void octx_free(octx* c) {
  free(c->soa);
  free(c->planes);
  c->soa = NULL;
  c->planes = NULL;
}

/* ------------------------------------------------------------------------------------ */
/* intersection — p_compute.glsl:77-143                                                 */
/* ------------------------------------------------------------------------------------ */
static float sphere_eval(v3 pos, v3 dir, v3 center, float radius) {
  v3 pmc = sub3(pos, center);
  float b = dot3(dir, pmc);
  float del = fmaf(radius, radius, fmaf(b, b, -dot3(pmc, pmc)));
  if (del < 0.0f) return -1.0f;
  else if (del == 0.0f) return -1.0f * b;
  else {
    float s = sqrtf(del);
    float t1 = -1.0f * b + s;
    float t2 = -1.0f * b - s;
    if (t2 < 0.0f) {
      if (t1 < 0.0f) return -1.0f;
      else return t1;
    } else
      return t2;
  }
}

float rto_sphere_eval(const float pos[3], const float dir[3], const float center[3], float r) {
  return sphere_eval(mk3(pos[0], pos[1], pos[2]), mk3(dir[0], dir[1], dir[2]),
                     mk3(center[0], center[1], center[2]), r);
}

void rto_normalize3(const float v[3], float out[3]) {
  v3 n = nrm3(mk3(v[0], v[1], v[2]));
  out[0] = n.x; out[1] = n.y; out[2] = n.z;
}

/* the discriminant of sphere_eval above (p_compute.glsl:80-82) */
float rto_sphere_del(const float pos[3], const float dir[3], const float center[3], float r) {
  v3 pmc = sub3(mk3(pos[0], pos[1], pos[2]), mk3(center[0], center[1], center[2]));
  float b = dot3(mk3(dir[0], dir[1], dir[2]), pmc);
  return fmaf(r, r, fmaf(b, b, -dot3(pmc, pmc)));
}

static float plane_eval(const octx* c, v3 pos, v3 dir, int i) {
  v3 n = mk3(SH(c, i, 0, 0), SH(c, i, 0, 1), SH(c, i, 0, 2));
  float denom = dot3(n, dir);
  if (denom < 0.001f && denom > -0.001f) return -1.0f;
  v3 p0 = mk3(SH(c, i, 3, 0), SH(c, i, 3, 1), SH(c, i, 3, 2));
  return dot3(n, sub3(p0, pos)) / denom;
}


/* sphere_eval of spheres [i, i+8) of the SoA table, up to the values no caller accepts:
   every caller accepts only res > thr >= 0, and this returns sphere_eval's value wherever that
   is positive (del > 0: the same t2 / t1 choice; del == 0: -b - 0 = -b, and t1 = t2 when -b < 0;
   del < 0 or NaN: NaN instead of -1).  Same binary32 operations in the same order, with the
   hardware fma and IEEE sqrt, so the accepted values are bit-identical to sphere_eval's. */
static inline __m256 sphere_eval8(const octx* c, int i, __m256 px, __m256 py, __m256 pz, __m256 dx, __m256 dy,
                                  __m256 dz) {
  const float* s = c->soa;
  const size_t n = (size_t)c->nsoa;
  __m256 mx = _mm256_sub_ps(px, _mm256_loadu_ps(s + i));
  __m256 my = _mm256_sub_ps(py, _mm256_loadu_ps(s + n + i));
  __m256 mz = _mm256_sub_ps(pz, _mm256_loadu_ps(s + 2 * n + i));
  __m256 r = _mm256_loadu_ps(s + 3 * n + i);
  __m256 b = _mm256_fmadd_ps(dz, mz, _mm256_fmadd_ps(dy, my, _mm256_mul_ps(dx, mx)));
  __m256 pp = _mm256_fmadd_ps(mz, mz, _mm256_fmadd_ps(my, my, _mm256_mul_ps(mx, mx)));
  __m256 del = _mm256_fmadd_ps(r, r, _mm256_fmsub_ps(b, b, pp)); /* fmaf(b, b, -pp): one rounding */
  __m256 sq = _mm256_sqrt_ps(del);
  __m256 nb = _mm256_mul_ps(_mm256_set1_ps(-1.0f), b);
  __m256 t1 = _mm256_add_ps(nb, sq);
  __m256 t2 = _mm256_sub_ps(nb, sq);
  return _mm256_blendv_ps(t2, t1, _mm256_cmp_ps(t2, _mm256_setzero_ps(), _CMP_LT_OQ));
}

#ifdef __AVX512F__
/* the same evaluation 16 spheres at a time (the CPU-baseline build for the GPU box's Zen 5
   cores, -mavx512f): identical binary32 operations per lane */
static inline __m512 sphere_eval16(const octx* c, int i, __m512 px, __m512 py, __m512 pz, __m512 dx, __m512 dy,
                                   __m512 dz) {
  const float* s = c->soa;
  const size_t n = (size_t)c->nsoa;
  __m512 mx = _mm512_sub_ps(px, _mm512_loadu_ps(s + i));
  __m512 my = _mm512_sub_ps(py, _mm512_loadu_ps(s + n + i));
  __m512 mz = _mm512_sub_ps(pz, _mm512_loadu_ps(s + 2 * n + i));
  __m512 r = _mm512_loadu_ps(s + 3 * n + i);
  __m512 b = _mm512_fmadd_ps(dz, mz, _mm512_fmadd_ps(dy, my, _mm512_mul_ps(dx, mx)));
  __m512 pp = _mm512_fmadd_ps(mz, mz, _mm512_fmadd_ps(my, my, _mm512_mul_ps(mx, mx)));
  __m512 del = _mm512_fmadd_ps(r, r, _mm512_fmsub_ps(b, b, pp));
  __m512 sq = _mm512_sqrt_ps(del);
  __m512 nb = _mm512_mul_ps(_mm512_set1_ps(-1.0f), b);
  __m512 t1 = _mm512_add_ps(nb, sq);
  __m512 t2 = _mm512_sub_ps(nb, sq);
  return _mm512_mask_blend_ps(_mm512_cmp_ps_mask(t2, _mm512_setzero_ps(), _CMP_LT_OQ), t2, t1);
}
#endif

/* closest hit with threshold thr (p_compute.glsl:177-188; h_ 199-210; ao_ 183-194).  The
   reference's ascending scan `if (res > thr && (res < t || t < 0)) {t = res; ind = i;}` keeps,
   for thr >= 0, the smallest accepted res and among equal ones the lowest index: evaluated
   here 8 (AVX2) or 16 (AVX-512) spheres at a time (each lane keeps its own first minimum,
   lanes merged by the same rule), then the planes (scalar plane_eval), merged by that rule. */
static int closest_hit(const octx* c, v3 pos, v3 dir, float thr, float* t_out) {
  float t = -1.0f;
  int ind = -1;
  if (c->nsoa > 0) {
#ifdef __AVX512F__
    enum { VW = 16 };
    const __m512 px = _mm512_set1_ps(pos.x), py = _mm512_set1_ps(pos.y), pz = _mm512_set1_ps(pos.z);
    const __m512 dx = _mm512_set1_ps(dir.x), dy = _mm512_set1_ps(dir.y), dz = _mm512_set1_ps(dir.z);
    const __m512 vthr = _mm512_set1_ps(thr);
    __m512 bt = _mm512_set1_ps(INFINITY);
    __m512i bi = _mm512_set1_epi32(-1);
    __m512i idx = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i step = _mm512_set1_epi32(VW);
    for (int i = 0; i < c->nsoa; i += VW) {
      __m512 res = sphere_eval16(c, i, px, py, pz, dx, dy, dz);
      __mmask16 acc = _mm512_cmp_ps_mask(res, vthr, _CMP_GT_OQ);
      __mmask16 none = _mm512_cmpeq_epi32_mask(bi, _mm512_set1_epi32(-1));
      __mmask16 upd = acc & (_mm512_cmp_ps_mask(res, bt, _CMP_LT_OQ) | none);
      bt = _mm512_mask_blend_ps(upd, bt, res);
      bi = _mm512_mask_blend_epi32(upd, bi, idx);
      idx = _mm512_add_epi32(idx, step);
    }
    float lt[VW];
    int li[VW];
    _mm512_storeu_ps(lt, bt);
    _mm512_storeu_si512((void*)li, bi);
#else
    enum { VW = 8 };
    const __m256 px = _mm256_set1_ps(pos.x), py = _mm256_set1_ps(pos.y), pz = _mm256_set1_ps(pos.z);
    const __m256 dx = _mm256_set1_ps(dir.x), dy = _mm256_set1_ps(dir.y), dz = _mm256_set1_ps(dir.z);
    const __m256 vthr = _mm256_set1_ps(thr);
    __m256 bt = _mm256_set1_ps(INFINITY);
    __m256i bi = _mm256_set1_epi32(-1);
    __m256i idx = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
    const __m256i step = _mm256_set1_epi32(VW);
    for (int i = 0; i < c->nsoa; i += VW) {
      __m256 res = sphere_eval8(c, i, px, py, pz, dx, dy, dz);
      __m256 acc = _mm256_cmp_ps(res, vthr, _CMP_GT_OQ);
      __m256 none = _mm256_castsi256_ps(_mm256_cmpeq_epi32(bi, _mm256_set1_epi32(-1)));
      __m256 upd = _mm256_and_ps(acc, _mm256_or_ps(_mm256_cmp_ps(res, bt, _CMP_LT_OQ), none));
      bt = _mm256_blendv_ps(bt, res, upd);
      bi = _mm256_castps_si256(_mm256_blendv_ps(_mm256_castsi256_ps(bi), _mm256_castsi256_ps(idx), upd));
      idx = _mm256_add_epi32(idx, step);
    }
    float lt[VW];
    int li[VW];
    _mm256_storeu_ps(lt, bt);
    _mm256_storeu_si256((__m256i*)li, bi);
#endif
    for (int l = 0; l < VW; l++)
      if (li[l] >= 0 && (ind < 0 || lt[l] < t || (lt[l] == t && li[l] < ind))) {
        t = lt[l];
        ind = li[l];
      }
  }
  for (int k = 0; k < c->nplanes; k++) {
    int i = c->planes[k];
    float res = plane_eval(c, pos, dir, i);
    if (res > thr && (ind < 0 || res < t || (res == t && i < ind))) {
      t = res;
      ind = i;
    }
  }
  *t_out = t;
  return ind;
}

static v3 shape_normal(const octx* c, int ind, v3 p) {
  int id = (int)SH(c, ind, 4, 3);
  if (id == RT_SHAPE_SPHERE) return nrm3(sub3(p, mk3(SH(c, ind, 0, 0), SH(c, ind, 0, 1), SH(c, ind, 0, 2))));
  if (id == RT_SHAPE_PLANE) return mk3(SH(c, ind, 0, 0), SH(c, ind, 0, 1), SH(c, ind, 0, 2));
  return mk3(0.0f, 0.0f, 0.0f); /* unreachable: only spheres and planes are ever hit */
}

/* shadow_ray — p_compute.glsl:145-166 (double t, dvec3 length) */
static int shadow_ray(const octx* c, v3 pos) {
  v3 lv = sub3(c->light, pos);
  v3 l = nrm3(lv);
  float len = sqrtf(dot3(lv, lv));
  v3 np = add3(pos, scl3(0.01f, l));
  /* "some object occludes" does not depend on the scan order: spheres 8 or 16 at a time (the
     accepted values are sphere_eval's, see sphere_eval8), then the planes */
#ifdef __AVX512F__
  enum { VW = 16 };
  const __m512 px = _mm512_set1_ps(np.x), py = _mm512_set1_ps(np.y), pz = _mm512_set1_ps(np.z);
  const __m512 dx = _mm512_set1_ps(l.x), dy = _mm512_set1_ps(l.y), dz = _mm512_set1_ps(l.z);
  const __m512 vthr = _mm512_set1_ps(0.0001f);
#else
  enum { VW = 8 };
  const __m256 px = _mm256_set1_ps(np.x), py = _mm256_set1_ps(np.y), pz = _mm256_set1_ps(np.z);
  const __m256 dx = _mm256_set1_ps(l.x), dy = _mm256_set1_ps(l.y), dz = _mm256_set1_ps(l.z);
  const __m256 vthr = _mm256_set1_ps(0.0001f);
#endif
  for (int i = 0; i < c->nsoa; i += VW) {
    float rv[VW];
#ifdef __AVX512F__
    __m512 res = sphere_eval16(c, i, px, py, pz, dx, dy, dz);
    int m = (int)_mm512_cmp_ps_mask(res, vthr, _CMP_GT_OQ);
    if (!m) continue;
    _mm512_storeu_ps(rv, res);
#else
    __m256 res = sphere_eval8(c, i, px, py, pz, dx, dy, dz);
    int m = _mm256_movemask_ps(_mm256_cmp_ps(res, vthr, _CMP_GT_OQ));
    if (!m) continue;
    _mm256_storeu_ps(rv, res);
#endif
    for (int k = 0; k < VW; k++)
      if (m >> k & 1) {
        double t = (double)rv[k];
        double ddx = t * (double)l.x, ddy = t * (double)l.y, ddz = t * (double)l.z;
        double L = sqrt(fma(ddz, ddz, fma(ddy, ddy, ddx * ddx)));
        if (L < (double)len) return 0;
      }
  }
  for (int k = 0; k < c->nplanes; k++) {
    double t = (double)plane_eval(c, np, l, c->planes[k]);
    if (t > (double)0.0001f) {
      double ddx = t * (double)l.x, ddy = t * (double)l.y, ddz = t * (double)l.z;
      double L = sqrt(fma(ddz, ddz, fma(ddy, ddy, ddx * ddx)));
      if (L < (double)len) return 0;
    }
  }
  return 1;
}

/* primary ray direction — p_compute.glsl:233-235 */
static v3 primary_dir(const octx* c, float hp, float vp) {
  v3 a = add3(c->llc, scl3(hp, c->horiz));
  return nrm3(add3(a, scl3(vp, c->vert)));
}

void rto_primary_dir(const float* h, float hp, float vp, float out[3]) {
  octx c;
  c.horiz = mk3(h[4 * RT_HDR_HORIZONTAL], h[4 * RT_HDR_HORIZONTAL + 1], h[4 * RT_HDR_HORIZONTAL + 2]);
  c.vert = mk3(h[4 * RT_HDR_VERTICAL], h[4 * RT_HDR_VERTICAL + 1], h[4 * RT_HDR_VERTICAL + 2]);
  c.llc = mk3(h[4 * RT_HDR_LLC_MINUS_CAMPOS], h[4 * RT_HDR_LLC_MINUS_CAMPOS + 1], h[4 * RT_HDR_LLC_MINUS_CAMPOS + 2]);
  v3 d = primary_dir(&c, hp, vp);
  out[0] = d.x; out[1] = d.y; out[2] = d.z;
}

static const float RT_GAMMA = 1.0f / 2.2f; /* p_compute.glsl:240 */

static void store_out(octx* c, int x, int y, v4 col, float* image, int write_image) {
  size_t g = gidx(c, c->frame, x, y);
  c->pix[g + 0] = col.x;
  c->pix[g + 1] = col.y;
  c->pix[g + 2] = col.z;
  c->pix[g + 3] = col.w;
  if (image && write_image) {
    size_t o = ((size_t)(y - c->d->gy0) * c->d->W + x) * 4;
    image[o + 0] = col.x;
    image[o + 1] = col.y;
    image[o + 2] = col.z;
    image[o + 3] = col.w;
  }
}

static v4 gamma4(v4 r) {
  v4 o = {powf(r.x, RT_GAMMA), powf(r.y, RT_GAMMA), powf(r.z, RT_GAMMA), 0.0f};
  return o;
}

/* ------------------------------------------------------------------------------------ */
/* mode 3: p_compute.glsl:168-245                                                        */
/* ------------------------------------------------------------------------------------ */
static v4 phong(const octx* c, v3 dir) {
  v4 out;
  float t;
  int ind = closest_hit(c, c->cam, dir, 0.0f, &t);
  if (ind == -1) return c->bg;
  v3 curr = add3(c->cam, scl3(t, dir));
  int lit = shadow_ray(c, curr);
  v3 n = shape_normal(c, ind, curr);
  v3 col = mk3(SH(c, ind, 4, 0), SH(c, ind, 4, 1), SH(c, ind, 4, 2));
  if (lit) {
    v3 l = nrm3(sub3(c->light, curr));
    float spec = powf(gclamp(dot3(nrm3(sub3(l, dir)), n), 0.0f, 1.0f), 500.0f);
    float k = gclamp(dot3(n, l), 0.06f, 1.0f);
    out.x = col.x * k + spec;
    out.y = col.y * k + spec;
    out.z = col.z * k + spec;
    out.w = 0.0f + spec;
  } else {
    out.x = col.x * 0.06f;
    out.y = col.y * 0.06f;
    out.z = col.z * 0.06f;
    out.w = 0.0f;
  }
  return out;
}

static void p_main(octx* c, int x, int y, float* image) {
  float hp = (float)x / (float)c->d->W;
  float vp = (float)y / (float)c->d->H;
  v4 r = phong(c, primary_dir(c, hp, vp));
  v4 acc = {0.0f + r.x, 0.0f + r.y, 0.0f + r.z, 0.0f + r.w};
  store_out(c, x, y, gamma4(acc), image, 1);
}

/* ------------------------------------------------------------------------------------ */
/* mode 4: h_compute.glsl:186-321                                                        */
/* ------------------------------------------------------------------------------------ */
typedef struct { v4 a0; v3 pos; float stop; v3 dir; float refl; } hstate;

static void hybrid_helper(const octx* c, hstate* s, int depth) {
  if (depth <= 0) { v4 z = {0, 0, 0, 0}; s->a0 = z; } /* h_compute.glsl:188-189 (unreachable) */
  float t;
  int ind = closest_hit(c, s->pos, s->dir, 0.001f, &t);
  if (ind == -1) {
    s->a0 = c->bg;
    s->stop = 1.0f;
    return;
  }
  v4 att = {SH(c, ind, 4, 0), SH(c, ind, 4, 1), SH(c, ind, 4, 2), SH(c, ind, 4, 3)};
  v3 curr = add3(s->pos, scl3(t, s->dir));
  int lit = shadow_ray(c, curr);
  v3 n = shape_normal(c, ind, curr);
  if (lit) {
    v3 l = nrm3(sub3(c->light, curr));
    float spec = powf(gclamp(dot3(nrm3(sub3(l, s->dir)), n), 0.0f, 1.0f), 500.0f);
    float k = gclamp(dot3(n, l), 0.06f, 1.0f);
    att.x = att.x * k + spec;
    att.y = att.y * k + spec;
    att.z = att.z * k + spec;
    att.w = att.w * k + spec;
  } else {
    att.x = att.x * 0.06f;
    att.y = att.y * 0.06f;
    att.z = att.z * 0.06f;
    att.w = att.w * 0.06f;
  }
  float refl = 1.0f - SH(c, ind, 3, 3);
  if (refl < 0.001f) {
    s->stop = 1.0f;
  } else {
    float dn = dot3(s->dir, n);
    v3 R = nrm3(mk3(s->dir.x - 2.0f * (dn * n.x), s->dir.y - 2.0f * (dn * n.y),
                    s->dir.z - 2.0f * (dn * n.z)));
    s->pos = curr;
    s->dir = R;
    s->refl = refl;
  }
  s->a0 = att;
}

static v4 hybrid(const octx* c, v3 dir) {
  hstate s;
  s.pos = c->cam;
  s.stop = 0.0f;
  s.dir = dir;
  s.refl = 0.0f;
  hybrid_helper(c, &s, c->d->D);
  float cc = s.refl;
  v4 res = s.a0;
  if (s.stop == 1.0f) return res;
  int i = c->d->D - 1;
  while (i > 0) {
    hybrid_helper(c, &s, i);
    float den = 1.0f + cc;
    res.x = (res.x + cc * s.a0.x) / den;
    res.y = (res.y + cc * s.a0.y) / den;
    res.z = (res.z + cc * s.a0.z) / den;
    res.w = (res.w + cc * s.a0.w) / den;
    cc = cc * s.refl;
    if (s.stop == 1.0f) break;
    i -= 1;
  }
  return res;
}

static void h_main(octx* c, int x, int y, float* image) {
  float hp = (float)x / (float)c->d->W;
  float vp = (float)y / (float)c->d->H;
  v4 r = hybrid(c, primary_dir(c, hp, vp));
  v4 acc = {0.0f + r.x, 0.0f + r.y, 0.0f + r.z, 0.0f + r.w};
  store_out(c, x, y, gamma4(acc), image, 1);
}

/* ------------------------------------------------------------------------------------ */
/* modes 1/2 pass 1: ao_compute.glsl:143-339 (aop_compute.glsl:141-336)                  */
/* ------------------------------------------------------------------------------------ */
static v3 get_pt_within_unit_sphere(const octx* c, int aa, int x, int y) {
  const float* f = c->rb + (size_t)(2 * aa) * 4;
  const float* s = c->rb + (size_t)(2 * aa + 1) * 4;
  float px = (float)x, py = (float)y;
  float a, b, e;
  if (rto_contract & RTO_C_FUSED_SEEDS) {
    a = rto_random(fmaf(px, s[2], f[0]), fmaf(py, s[3], f[1]));
    b = rto_random(fmaf(-px, s[2], f[2]), fmaf(-py, s[3], f[3]));
    e = rto_random(fmaf(s[0], px, s[2]), fmaf(s[1], py, s[3]));
  } else {
    a = rto_random(f[0] + px * s[2], f[1] + py * s[3]); /* seed1 + xy * seed4 */
    b = rto_random(f[2] - px * s[2], f[3] - py * s[3]); /* seed2 - xy * seed4 */
    e = rto_random(s[0] * px + s[2], s[1] * py + s[3]); /* seed3 * xy + seed4 */
  }
  return nrm3(mk3(a * 2.0f - 1.0f, b * 2.0f - 1.0f, e * 2.0f - 1.0f));
}

typedef struct { v4 a0; v3 pos; float stop; v3 dir; } aostate;

static void ao_helper(octx* c, aostate* s, int depth, int aa, int x, int y, v3 hemi) {
  size_t g = gidx(c, c->frame, x, y);
  if (depth <= 0) { /* ao_compute.glsl:163-172 (unreachable: depth >= 1) */
    v4 z = {0, 0, 0, 0};
    s->a0 = z;
    s->stop = 1.0f;
    c->dep[g + 1] = (float)c->d->D;
    return;
  }
  float t;
  int ind = closest_hit(c, s->pos, s->dir, 0.0001f, &t);
  if (ind != -1) {
    v4 att = {SH(c, ind, 4, 0), SH(c, ind, 4, 1), SH(c, ind, 4, 2), SH(c, ind, 4, 3)};
    if (SH(c, ind, 1, 3) > 0.9f) { /* emissive */
      s->a0 = att;
      s->stop = 1.0f;
      c->dep[g + 1] = (float)(c->d->D - depth);
      return;
    }
    v3 curr = add3(c->cam, scl3(t, s->dir)); /* sic: camera origin, ao_compute.glsl:210 */
    v3 n = shape_normal(c, ind, curr);
    if (aa == 0 && depth == c->d->D) {
      c->nrm[g + 0] = n.x;
      c->nrm[g + 1] = n.y;
      c->nrm[g + 2] = n.z;
      c->nrm[g + 3] = 1.0f;
      c->dep[g + 0] = t;
      c->dep[g + 1] = 0.0f;
      c->dep[g + 2] = 0.0f;
      c->dep[g + 3] = 1.0f;
    }
    s->a0 = att;
    s->pos = curr;
    s->stop = 0.0f;
    float reflect = SH(c, ind, 3, 3);
    if (reflect > 0.999f) {
      s->dir = nrm3(add3(hemi, n));
    } else {
      float dn = dot3(s->dir, n);
      v3 R = nrm3(mk3(s->dir.x - 2.0f * (dn * n.x), s->dir.y - 2.0f * (dn * n.y),
                      s->dir.z - 2.0f * (dn * n.z)));
      s->dir = nrm3(add3(R, scl3(reflect, hemi)));
    }
    return;
  }
  if (aa == 0 && depth == c->d->D) {
    for (int k = 0; k < 4; k++) {
      c->nrm[g + k] = 0.0f;
      c->dep[g + k] = 0.0f;
    }
  }
  s->a0 = c->bg;
  s->stop = 1.0f;
  c->dep[g + 1] = (float)(c->d->D - depth);
}

static v4 ambient_occlusion(octx* c, v3 dir, int aa, int x, int y) {
  v4 res = {1.0f, 1.0f, 1.0f, 1.0f};
  aostate s;
  s.pos = c->cam;
  s.stop = 0.0f;
  s.dir = dir;
  /* get_pt_within_unit_sphere depends only on (aa, x, y): same value every bounce */
  v3 hemi = get_pt_within_unit_sphere(c, aa, x, y);
  int i = c->d->D;
  while (i > 0) {
    ao_helper(c, &s, i, aa, x, y, hemi);
    res.x = res.x * s.a0.x;
    res.y = res.y * s.a0.y;
    res.z = res.z * s.a0.z;
    res.w = res.w * s.a0.w;
    if ((int)s.stop == 1) break;
    i -= 1;
  }
  return res;
}

static void ao_main(octx* c, int x, int y, float* image, int write_image) {
  const int AA = c->d->AA;
  const float* rb = c->rb;
  v4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  float px = (float)x, py = (float)y;
  {
    float hp = px / (float)c->d->W;
    float vp = py / (float)c->d->H;
    v4 r = ambient_occlusion(c, primary_dir(c, hp, vp), 0, x, y);
    acc.x += r.x; acc.y += r.y; acc.z += r.z; acc.w += r.w;
  }
  for (int aa = 1; aa < AA; aa++) {
    const float* f = rb + (size_t)(2 * aa) * 4;
    const float* s = rb + (size_t)(2 * aa + 1) * 4;
    float s1x = s[0], s1y = f[1]; /* seed1 = (rb[second].x, rb[first].y) */
    float s2x = f[2], s2y = s[3]; /* seed2 = (rb[first].z, rb[second].w) */
    float s3x = f[0], s3y = s[1]; /* seed3 = (rb[first].x, rb[second].y) */
    float s4x = s[2], s4y = f[3]; /* seed4 = (rb[second].z, rb[first].w) */
    float u, w;
    if (rto_contract & RTO_C_FUSED_JITTER) {
      u = rto_random((fmaf(px, s2x, s1x) - px) + s3x, (fmaf(py, s2y, s1y) - py) + s3y);
      w = rto_random(fmaf(s4x, px, -((s3x * px) * s2x)), fmaf(s4y, py, -((s3y * py) * s2y)));
    } else {
      u = rto_random(((s1x + px * s2x) - px) + s3x, ((s1y + py * s2y) - py) + s3y);
      w = rto_random(s4x * px - (s3x * px) * s2x, s4y * py - (s3y * py) * s2y);
    }
    float il = 1.0f / sqrtf(fmaf(w, w, u * u)); /* normalize(vec2) */
    float jx = (u * il) / 6.0f - 0.08333f;
    float jy = (w * il) / 6.0f - 0.08333f;
    float hp = (px + jx) / (float)c->d->W;
    float vp = (py + jy) / (float)c->d->H;
    v4 r = ambient_occlusion(c, primary_dir(c, hp, vp), aa, x, y);
    acc.x += r.x; acc.y += r.y; acc.z += r.z; acc.w += r.w;
  }
  float fa = (float)AA;
  acc.x /= fa; acc.y /= fa; acc.z /= fa; acc.w /= fa;
  size_t g = gidx(c, c->frame, x, y);
  for (int k = 0; k < 4; k++) c->dep[g + k] /= fa; /* depth_buffer[frame][x][y] /= AA */
  store_out(c, x, y, gamma4(acc), image, write_image);
}

/* ------------------------------------------------------------------------------------ */
/* mode 1 pass 2: aop_postprocessing.glsl:57-208                                         */
/* Documented semantics: spatial neighbours read the PRE-FILTER snapshot */
/* of pixels[f] (the reference reads it while neighbours overwrite it in place); a right  */
/* neighbour exists iff x+1 < W, left iff x > 0, up iff y+1 < H, down iff y >= 2 (y = 1   */
/* keeps the reference's `y - 1 > 0`; the y = 0 unsigned wrap is treated as absent).      */
/* ------------------------------------------------------------------------------------ */
static float nbr_weight(v3 n, float nd, float nb, const float* nn, const float* dd) {
  if (nn[3] < 0.001f) return 1.0f;
  float normal_dot = dot3(n, mk3(nn[0], nn[1], nn[2]));
  float depth_diff = 1.0f - gclamp(fabsf(nd - dd[0]), 0.0f, 1.0f);
  float bounces_diff = 1.0f - gclamp(fabsf(nb - dd[1]) / 1.7f, 0.0f, 1.0f);
  return normal_dot * depth_diff * bounces_diff + 0.2f;
}

static void post_main(octx* c, const float* snap /* [W][gh] vec4 */, int x, int y, float* image) {
  const rto_dims* d = c->d;
  const int f = c->frame;
  size_t g = gidx(c, f, x, y);
  size_t sg = ((size_t)x * d->gh + (size_t)(y - d->gy0)) * 4;
  v4 color = {snap[sg], snap[sg + 1], snap[sg + 2], snap[sg + 3]};
  const float* nn = c->nrm + g;
  if (nn[3] > 0.99f) {
    v3 n = mk3(nn[0], nn[1], nn[2]);
    float nd = c->dep[g + 0], nb = c->dep[g + 1];
    /* neighbours in GLSL summation order: up, down, left, right (line 173) */
    int nx[4] = {x, x, x - 1, x + 1};
    int ny[4] = {y + 1, y - 1, y, y};
    int present[4] = {y + 1 < d->H, y >= 2, x > 0, x + 1 < d->W};
    float wsum_c[4] = {color.x, color.y, color.z, color.w};
    float den = 1.0f;
    for (int k = 0; k < 4; k++) {
      float wk = 0.0f, val[4] = {0, 0, 0, 0};
      if (present[k] && ny[k] >= d->gy0 && ny[k] < d->gy0 + d->gh) {
        size_t gk = gidx(c, f, nx[k], ny[k]);
        size_t sk = ((size_t)nx[k] * d->gh + (size_t)(ny[k] - d->gy0)) * 4;
        wk = nbr_weight(n, nd, nb, c->nrm + gk, c->dep + gk);
        for (int ch = 0; ch < 4; ch++) val[ch] = snap[sk + ch];
      }
      for (int ch = 0; ch < 4; ch++) wsum_c[ch] = wsum_c[ch] + wk * val[ch];
      den = den + wk;
    }
    color.x = wsum_c[0] / den;
    color.y = wsum_c[1] / den;
    color.z = wsum_c[2] / den;
    color.w = wsum_c[3] / den;
    /* temporal (lines 177-201) */
    float cs[4] = {0, 0, 0, 0};
    float denominator = 0.9f;
    for (int i = 1; i < d->F; i++) {
      int cf = (f + d->F - i) % d->F;
      size_t gc = gidx(c, cf, x, y);
      v3 cn = mk3(c->nrm[gc], c->nrm[gc + 1], c->nrm[gc + 2]);
      float normal_dot = dot3(n, cn);
      float depth_diff = 1.0f - gclamp(fabsf(nd - c->dep[gc]), 0.0f, 1.0f);
      float bounces_diff = 1.0f - gclamp(fabsf(nb - c->dep[gc + 1]) / 1.7f, 0.0f, 1.0f);
      float coeff = normal_dot * depth_diff * bounces_diff;
      if (coeff > 0.85f) {
        for (int ch = 0; ch < 4; ch++) cs[ch] = cs[ch] + coeff * c->pix[gc + ch];
        denominator = denominator + coeff;
      } else
        break;
    }
    color.x = (color.x * 0.9f + cs[0]) / denominator;
    color.y = (color.y * 0.9f + cs[1]) / denominator;
    color.z = (color.z * 0.9f + cs[2]) / denominator;
    color.w = (color.w * 0.9f + cs[3]) / denominator;
  }
  store_out(c, x, y, color, image, 1);
}

/* ------------------------------------------------------------------------------------ */
/* drivers                                                                               */
/* ------------------------------------------------------------------------------------ */
int rto_run_program_window(float* ssbo, const rto_dims* d, int program, int frame, float* image, int y0,
                           int y1, int x0, int x1, int nthreads) {
  octx c;
  if (octx_init(&c, ssbo, d, frame) != 0) return -1;
  if (y0 < d->gy0 || y1 > d->gy0 + d->gh || y0 > y1) return -1;
  if (x0 < 0 || x1 > d->W || x0 > x1) return -1;
  if (program < RTO_AOP_COMPUTE || program > RTO_H_COMPUTE) return -1;
#ifdef _OPENMP
  int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#else
  (void)nthreads;
#endif
  const int W = d->W;
  if (program == RTO_AOP_POSTPROCESSING) {
    size_t slot = (size_t)W * d->gh * 4;
    float* snap = (float*)malloc(slot * sizeof(float));
    if (!snap) return -1;
    memcpy(snap, c.pix + (size_t)frame * slot, slot * sizeof(float));
    /* every pixel is independent: threads share the window's pixels (chunks of 64), not rows,
       so a thin band still uses every thread */
    const long long w = x1 - x0, npx = w * (long long)(y1 - y0);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nt)
#endif
    for (long long i = 0; i < npx; i++) post_main(&c, snap, x0 + (int)(i % w), y0 + (int)(i / w), image);
    free(snap);
    return 0;
  }
  if (octx_tables(&c) != 0) {
    octx_free(&c);
    return -1;
  }
  const long long w = x1 - x0, npx = w * (long long)(y1 - y0);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nt)
#endif
  for (long long i = 0; i < npx; i++) {
    const int x = x0 + (int)(i % w), y = y0 + (int)(i / w);
    switch (program) {
      case RTO_P_COMPUTE: p_main(&c, x, y, image); break;
      case RTO_H_COMPUTE: h_main(&c, x, y, image); break;
      case RTO_AO_COMPUTE: ao_main(&c, x, y, image, 1); break;
      case RTO_AOP_COMPUTE: ao_main(&c, x, y, image, 0); break;
      default: break;
    }
  }
  octx_free(&c);
  return 0;
}

int rto_run_program(float* ssbo, const rto_dims* d, int program, int frame, float* image, int y0,
                    int y1, int nthreads) {
  return d ? rto_run_program_window(ssbo, d, program, frame, image, y0, y1, 0, d->W, nthreads) : -1;
}

int rto_dispatch(float* ssbo, const rto_dims* d, int mode, int frame, float* image, int nthreads) {
  int y0 = d->gy0, y1 = d->gy0 + d->gh, rc;
  switch (mode) {
    case 1:
      rc = rto_run_program(ssbo, d, RTO_AOP_COMPUTE, frame, image, y0, y1, nthreads);
      if (rc == 0) rc = rto_run_program(ssbo, d, RTO_AOP_POSTPROCESSING, frame, image, y0, y1, nthreads);
      break;
    case 2: rc = rto_run_program(ssbo, d, RTO_AO_COMPUTE, frame, image, y0, y1, nthreads); break;
    case 3: rc = rto_run_program(ssbo, d, RTO_P_COMPUTE, frame, image, y0, y1, nthreads); break;
    case 4: rc = rto_run_program(ssbo, d, RTO_H_COMPUTE, frame, image, y0, y1, nthreads); break;
    default: return -1;
  }
  if (rc != 0) return rc;
  return (frame + 1) % d->F;
}
