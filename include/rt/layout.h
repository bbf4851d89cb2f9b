/*
 * rt/layout.h — byte layout of the reference's std430 `shader_data` block.
 *
 * The reference declares one SSBO (binding 0) that every compute shader shares:
 *   resources/p_compute.glsl:28-63  (identical block in h_/ao_/aop_/aop_postprocessing)
 *   src/main.cpp:49-85              (host mirror `class ssbo_data`)
 *
 *   vec4 mode;                  // .y = frame slot, .z = object count (as float)
 *   vec4 horizontal, vertical, llc_minus_campos, camera_location, light_pos, background;
 *   vec4 simple_shapes[S][5];   // 80 B per shape, packing per src/main.cpp:395-469
 *   vec4 rand_buffer[2*AA];     // src/main.cpp:535-539
 *   vec4 pixels[F][W][H];       // x-major, y fastest
 *   vec4 normals_buffer[F][W][H];
 *   vec4 depth_buffer[F][W][H];
 *
 * The reference instance is S=10, AA=4, W=440, H=330, F=8 (src/main.cpp:29-36); every
 * member is a vec4 so std430 adds no padding.  This header parameterises the block by
 * (S, AA, W, H, F).  It is plain C so the oracle, the HIP shim and the tests share it:
 * it describes a data format, not an algorithm.
 */
#ifndef RT_LAYOUT_H
#define RT_LAYOUT_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* vec4 indices of the 7 header vectors (p_compute.glsl:30-36) */
enum {
  RT_HDR_MODE = 0,
  RT_HDR_HORIZONTAL = 1,
  RT_HDR_VERTICAL = 2,
  RT_HDR_LLC_MINUS_CAMPOS = 3,
  RT_HDR_CAMERA_LOCATION = 4,
  RT_HDR_LIGHT_POS = 5,
  RT_HDR_BACKGROUND = 6,
  RT_HDR_VEC4S = 7
};

/* shape ids (p_compute.glsl:15-17; src/geom_objs/{sphere,plane,rectangle}.h) */
enum { RT_SHAPE_SPHERE = 1, RT_SHAPE_RECTANGLE = 3, RT_SHAPE_PLANE = 5 };

/* defaults (src/main.cpp:29-47, resources/<shader>.glsl:7-20) */
#define RT_REF_WIDTH 440
#define RT_REF_HEIGHT 330
#define RT_REF_AA 4
#define RT_REF_NUM_SHAPES 10
#define RT_NUM_FRAMES 8
#define RT_RECURSION_DEPTH 20

#define RT_VEC4_BYTES 16u
#define RT_SHAPE_VEC4S 5u

static inline size_t rt_off_shapes(void) { return (size_t)RT_HDR_VEC4S * RT_VEC4_BYTES; }
static inline size_t rt_off_rand(int S) { return rt_off_shapes() + (size_t)S * RT_SHAPE_VEC4S * RT_VEC4_BYTES; }
/* header = everything before pixels: 7 vec4 + shapes + rand_buffer */
static inline size_t rt_header_bytes(int S, int AA) { return rt_off_rand(S) + (size_t)2 * AA * RT_VEC4_BYTES; }
static inline size_t rt_gbuf_bytes(int W, int H, int F) { return (size_t)F * W * H * RT_VEC4_BYTES; }
static inline size_t rt_off_pixels(int S, int AA) { return rt_header_bytes(S, AA); }
static inline size_t rt_off_normals(int S, int AA, int W, int H, int F) {
  return rt_off_pixels(S, AA) + rt_gbuf_bytes(W, H, F);
}
static inline size_t rt_off_depth(int S, int AA, int W, int H, int F) {
  return rt_off_normals(S, AA, W, H, F) + rt_gbuf_bytes(W, H, F);
}
static inline size_t rt_ssbo_bytes(int S, int AA, int W, int H, int F) {
  return rt_off_depth(S, AA, W, H, F) + rt_gbuf_bytes(W, H, F);
}
/* float index of g-buffer element [f][x][y] component c (reference layout, y fastest) */
static inline size_t rt_gbuf_index(int W, int H, int f, int x, int y) {
  return (((size_t)f * W + x) * H + y) * 4u;
}

#ifdef __cplusplus
}
#endif
#endif /* RT_LAYOUT_H */
