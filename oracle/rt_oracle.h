/*
 * rt_oracle.h — CPU restatement of the reference's GLSL hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code,
 * and only as the checker / CPU baseline.  The product path (real_time_ray_tracer_amd) never
 * calls it and fails loudly when its HIP library is missing.
 *
 * PARITY STATUS: parity unpinned by reference artifacts.  The reference ships no tests, no
 * golden images and no fixtures, and it cannot run here (OpenGL 4.3+ compute
 * with GLFW/GLM and a display).  This restatement is pinned instead by
 * (1) analytic known-answer tests (tests/test_oracle_kat.py), (2) an independent numpy
 * restatement (oracle/numpy_ref.py) compared on small frames, and (3) golden fixtures produced
 * by this file and committed under tests/golden/ (tests/golden/make_golden.py).
 *
 * Float semantics (the "GLSL math" both this file and the HIP kernels implement):
 *   - IEEE binary32 with round-to-nearest, denormals kept, NO implicit contraction
 *     (built with -ffp-contract=off); operations in the written GLSL order;
 *   - dot(a,b) = fmaf(a.z,b.z, fmaf(a.y,b.y, a.x*b.x)) (a fused chain, as GLSL compilers emit);
 *   - sphere discriminant = fmaf(r, r, fmaf(b, b, -dot(pmc,pmc)));
 *   - normalize(v) = v * (1.0f / sqrtf(dot(v,v))), length(v) = sqrtf(dot(v,v)), IEEE / and
 *     sqrtf (the correctly rounded form of the rsqrt-multiply GLSL compilers emit);
 *   - sin() inside random() = rto_sin(): the correctly rounded binary32 sin(x), the
 *     mathematical function (glibc's binary64 sin rounded once; quad-precision sinq where that
 *     rounding is ambiguous).  random() multiplies sin by 43758.5 before fract(), so only
 *     the exact function lets any CPU re-execution reproduce the hash: (float)sin((double)x)
 *     equals it except at the rare double-rounding inputs (round 5; rounds 1-4 used a
 *     binary32 polynomial sin that only this oracle and the kernels shared);
 *   - shadow_ray's `double t` and its dvec3 length run in binary64 (p_compute.glsl:147-163);
 *   - pow() = libm powf (outputs only; never feeds control flow), so pixels agree within
 *     the north-star tolerance |g-c| <= 1e-4*max(|g|,|c|) + 1e-6, not bit for bit.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int W, H;      /* full frame (WIDTH, HEIGHT): ray generation and post-process bounds */
  int S;         /* simple_shapes capacity (NUM_SHAPES) */
  int AA;        /* samples per pixel */
  int F;         /* NUM_FRAMES */
  int D;         /* RECURSION_DEPTH */
  int gy0, gh;   /* g-buffer covers rows [gy0, gy0+gh); full frame: 0, H */
} rto_dims;

/* programs, same numbering as include/rt/abi.h */
enum { RTO_AOP_COMPUTE = 1, RTO_AOP_POSTPROCESSING = 2, RTO_AO_COMPUTE = 3,
       RTO_P_COMPUTE = 4, RTO_H_COMPUTE = 5 };

/* Run `program` over frame rows [y0, y1) (must lie inside the g-buffer rows) on the reference-
 * layout buffer `ssbo` (header + shapes + rand + pixels/normals/depth [F][W][gh]).  `frame` is
 * written into mode.y first.  image (optional) is [gh][W] rgba32f, row 0 = gy0.
 * nthreads <= 0: OpenMP default.  Returns 0 or -1 on bad arguments. */
int rto_run_program(float* ssbo, const rto_dims* d, int program, int frame, float* image,
                    int y0, int y1, int nthreads);

/* rto_run_program over the window of columns [x0, x1) only (the g-buffer and image keep their
 * full width W).  A post-process pixel reads its left/right neighbours' pixels of the same
 * pass-1 output, so a window checked after the post-process needs pass 1 over [x0-1, x1+1). */
int rto_run_program_window(float* ssbo, const rto_dims* d, int program, int frame, float* image,
                           int y0, int y1, int x0, int x1, int nthreads);

/* compute() of src/main.cpp:553-578 for modes 1..4 over the whole g-buffer band; returns the
 * next frame slot. */
int rto_dispatch(float* ssbo, const rto_dims* d, int mode, int frame, float* image, int nthreads);

/* primitives (exported for the math self-tests) */
float rto_sin(float x);
/* counts the bit patterns start .. start+n-1 (mod 2^32) where got[i] != rto_sin (NaN == NaN),
 * recording the first max_bad of them in bad (the device sin's exhaustive sweep) */
int64_t rto_sin_check_range(uint32_t start, int64_t n, const float* got, uint32_t* bad, int max_bad);
float rto_random(float x, float y);
/* contraction variants of random()'s argument arithmetic (measurement hook; 0 = the kernels') */
enum { RTO_C_UNFUSED_DOT = 1, RTO_C_FUSED_SEEDS = 2, RTO_C_FUSED_JITTER = 4 };
void rto_set_contraction(int flags);
int rto_get_contraction(void);
float rto_sphere_eval(const float pos[3], const float dir[3], const float center[3], float r);
void rto_normalize3(const float v[3], float out[3]);
/* the sphere discriminant fmaf(r, r, fmaf(b, b, -dot(pmc, pmc))) of sphere_eval_ray, and the
 * primary direction normalize(llc + hp*horizontal + vp*vertical) of a header: used by the
 * tests to construct exactly tangent rays (del == 0) */
float rto_sphere_del(const float pos[3], const float dir[3], const float center[3], float r);
void rto_primary_dir(const float* header, float hp, float vp, float out[3]);

#ifdef __cplusplus
}
#endif
#endif
