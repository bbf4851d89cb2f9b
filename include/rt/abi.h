/*
 * rt/abi.h — C ABI of the MI355X ray-tracing hot path (librtrt.so).
 *
 * Drop-in for the GL dispatch boundary of JustinPrivitera/Real_Time_Ray_Tracer:
 *   the reference binds one std430 SSBO `shader_data` (resources/p_compute.glsl:28-63) plus
 *   an rgba32f image (src/main.cpp:389-392) and launches one of five compute programs with
 *   glDispatchCompute(WIDTH, HEIGHT, 1) from
 *     Application::compute()              src/main.cpp:553-578
 *     Application::compute_one_shader()   src/main.cpp:580-620
 *     Application::compute_two_shaders()  src/main.cpp:622-671
 *   and packs the scene / rand buffer / light with
 *     loadShapeBuffer()    src/main.cpp:395-469
 *     fill_rand_buffer()   src/main.cpp:535-539
 *     moving_light()       src/main.cpp:541-551
 *     camera basis         src/main.cpp:772-779
 *
 * Every entry point below names the reference function it replaces.  Conventions:
 *   - plain C types only; no exceptions cross the ABI;
 *   - return value 0 = RT_OK, < 0 = one of the RT_E* codes (rt_strerror() names it);
 *     functions that return a frame index return it (>= 0) on success;
 *   - one rt_ctx per (device, frame strip); a context is not thread-safe;
 *   - all GPU work is ordered on the context's HIP stream (rt_set_stream to share one).
 *
 * Host-only helpers (rt_pack_*, rt_camera_basis, rt_fill_rand_buffer, rt_moving_light,
 * rt_scenegen, rt_init_scene, rt_strerror, rt_version) never touch the GPU.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#include "layout.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

/* ---- status codes ---------------------------------------------------------------- */
enum {
  RT_OK = 0,
  RT_E_INVAL = -1,    /* bad argument (size, index, mode, program ...) */
  RT_E_NOMEM = -2,    /* host or device allocation failed */
  RT_E_HIP = -3,      /* a HIP runtime call failed; rt_last_hip_error() has the code */
  RT_E_NODEV = -4,    /* no HIP device / bad device ordinal */
  RT_E_STATE = -5     /* call order (e.g. dispatch before a header was uploaded) */
};

/* ---- compute programs (src/main.cpp:484-501, resources/<shader>.glsl) ------------------ */
enum {
  RT_PROG_AOP_COMPUTE = 1,        /* resources/aop_compute.glsl        (mode 1 pass 1) */
  RT_PROG_AOP_POSTPROCESSING = 2, /* resources/aop_postprocessing.glsl (mode 1 pass 2) */
  RT_PROG_AO_COMPUTE = 3,         /* resources/ao_compute.glsl         (mode 2)        */
  RT_PROG_P_COMPUTE = 4,          /* resources/p_compute.glsl          (mode 3)        */
  RT_PROG_H_COMPUTE = 5,          /* resources/h_compute.glsl          (mode 4)        */
  RT_PROG_COUNT = 6
};

/* ---- lighting modes (`mycam.lighting`, src/main.cpp:266-273, 553-578) -------------- */
enum { RT_MODE_AO_PP = 1, RT_MODE_AO = 2, RT_MODE_PHONG = 3, RT_MODE_PHONG_REFL = 4 };

typedef struct rt_ctx rt_ctx;

typedef struct {
  int width;      /* WIDTH  (src/main.cpp:29): full-frame width in pixels               */
  int height;     /* HEIGHT (src/main.cpp:30): full-frame height in pixels              */
  int num_shapes; /* NUM_SHAPES (src/main.cpp:34): capacity of simple_shapes[S][5]      */
  int spp;        /* AA (src/main.cpp:31): samples per pixel; rand_buffer has 2*spp vec4 */
  int num_frames; /* NUM_FRAMES (src/main.cpp:36): g-buffer ring length, normally 8     */
  int max_depth;  /* RECURSION_DEPTH (resources/ao_compute.glsl:10): path length cap, 20 (<= 65535) */
  int row_begin;  /* this context renders frame rows [row_begin, row_end);              */
  int row_end;    /*   row_begin = row_end = 0 means the whole frame                    */
} rt_config;

/* ---- context lifetime ------------------------------------------------------------- */
/* Replaces computeInitGeom()/computeInit() (src/main.cpp:471-501): allocates the device-
 * resident header, g-buffer ring (zeroed like the value-initialised ssbo_CPUMEM) and image. */
int rt_create(int device, const rt_config* cfg, rt_ctx** out);
int rt_destroy(rt_ctx* ctx);
/* Order all of the context's work on an external HIP stream (hipStream_t).  NULL is the
 * device's legacy NULL stream (e.g. torch's default stream), not "no stream". */
int rt_set_stream(rt_ctx* ctx, void* hip_stream);
/* Go back to the context's own (non-blocking) stream. */
int rt_use_own_stream(rt_ctx* ctx);
void* rt_get_stream(rt_ctx* ctx);
/* Pipelined mode 1 (on != 0): rt_dispatch(RT_MODE_AO_PP) runs consecutive frames' aop_compute
 * passes on two alternating streams (the main stream and one of the context's own), so frame
 * k+1's pass fills the tail of frame k's, and every aop_postprocessing pass on `output_stream`
 * (NULL: a stream of the context's own).  Results are bit-identical to the sequential order:
 * normals/depth/raw pixels rotate through spare buffers and the header has two device copies,
 * so no pass sees data another in-flight pass writes.  A pipelined frame's image is complete in
 * output-stream order; rt_synchronize, rt_download and every other call (each first orders
 * all streams before the main stream) see finished frames.  Off by default. */
int rt_enable_pipelining(rt_ctx* ctx, int on, void* output_stream);
void* rt_get_output_stream(rt_ctx* ctx);
/* The stream of the last launch that wrote the context's image (the output stream for a
 * pipelined mode-1 frame, the main stream for every other program); a consumer of the image
 * (a copy, a collective) orders itself after it.  The next image writer is ordered after
 * whatever was enqueued on that stream before it. */
void* rt_image_stream(rt_ctx* ctx);
/* Number of visible HIP devices (0 when none). */
int rt_device_count(void);
/* Wait for all of the context's work (both streams). */
int rt_synchronize(rt_ctx* ctx);
int rt_last_hip_error(rt_ctx* ctx);
/* Test hook: the next query of a pinned staging buffer's "consumed" event (the uploads'
 * ring, rt_upload_header / rt_upload_rand_buffer) reports hip_error instead of asking HIP, so a
 * test can check that such a fault is returned (RT_E_HIP, rt_last_hip_error() == hip_error) and
 * the buffer is not reused.  The ring's slots are queried once they have been used (after 8
 * uploads). */
int rt_debug_fail_next_event_query(rt_ctx* ctx, int hip_error);

/* ---- device-resident path (what render() drives each frame) ------------------------ */
/* Upload the SSBO prefix: 7 header vec4 + simple_shapes[S][5] + rand_buffer[2*spp],
 * byte-identical to the reference's std430 layout (bytes == rt_header_bytes(S, spp)).
 * Replaces the memcpy-in of src/main.cpp:598-602 for everything but the g-buffer. */
int rt_upload_header(rt_ctx* ctx, const void* header, size_t bytes);
/* Replace only rand_buffer[2*spp] (fill_rand_buffer, src/main.cpp:535-539); n_vec4 == 2*spp. */
int rt_upload_rand_buffer(rt_ctx* ctx, const float* rand_vec4, size_t n_vec4);
/* Run one program on frame slot `frame` (glDispatchCompute(W,H,1), src/main.cpp:604). */
int rt_run_program(rt_ctx* ctx, int program, int frame);
/* compute() (src/main.cpp:553-578) without the host-side light/rand updates:
 * mode 1 = aop_compute + aop_postprocessing, 2 = ao_compute, 3 = p_compute, 4 = h_compute.
 * Returns the next frame slot (frame+1) % num_frames, as compute_one_shader does. */
int rt_dispatch(rt_ctx* ctx, int mode, int frame);
/* n consecutive compute() calls (src/main.cpp:553-578) as the reference's render loop makes
 * them (src/main.cpp:763-781), with the host-side updates in C++: per frame k = 0..n-1,
 * fill_rand_buffer(rand_seed + k) for the AO modes (1, 2) or moving_light(light_movement) for
 * the Phong modes (3, 4); set_mode(frame slot, int(mode.z)); upload the header; dispatch.
 * header: the caller's std430 prefix (rt_header_bytes(S, spp) bytes), updated in place as the
 * host loop leaves it.  Equal, frame for frame, to n rounds of those calls made one by one.
 * Returns the next frame slot, or < 0. */
int rt_compute_frames(rt_ctx* ctx, float* header, int mode, int frame, int n, uint64_t rand_seed,
                      int light_movement);
/* rt_compute_frames renders modes 2-4 as launches of up to `max_frames` frames (at most
 * num_frames).  1 (the default) = one launch and one image write per frame, the reference's own
 * dispatch shape (src/main.cpp:604).  > 1 = multi-frame launches (opt-in): each frame writes its
 * own ring slot, the image is written only by a launch's last frame (the one the caller sees).
 * The ring, the image the caller sees and the header are identical either way. */
int rt_set_frame_batch(rt_ctx* ctx, int max_frames);
/* Mode 4 (h_compute) tile schedule, on by default: the 16x16 tiles of a launch are dispatched
 * longest first, by the bounce rounds their waves needed in recent frames (read back every 16
 * launches on a side stream; an order is taken up once its upload has landed).  Only the order
 * of the workgroups changes, never an image.  The dispatch it replaces is the one
 * glDispatchCompute(WIDTH, HEIGHT, 1) of h_compute (src/main.cpp:604), whose workgroup order
 * the GL driver chooses.  on = 0 restores row order (and frees the schedule's buffers). */
int rt_set_tile_schedule(rt_ctx* ctx, int on);
/* 0 = off, 1 = on with row order still in use (no costs read back yet), 2 = a longest-first
 * order is in use. */
int rt_tile_schedule_state(rt_ctx* ctx);
/* how many longest-first orders have been taken up since the schedule was (re)enabled: each new
 * order replaces a table that launches still in flight may read, so tests count the swaps */
int rt_tile_schedule_orders(rt_ctx* ctx);
/* Copy device state to the host in the REFERENCE layout.  Any pointer may be NULL.
 * pixels/normals/depth: [F][W][R] vec4 (x-major, y fastest; R = rows of this context),
 * image: [R][W] rgba32f (row 0 = row_begin, bottom-left origin like the GL texture). */
int rt_download(rt_ctx* ctx, float* pixels, float* normals, float* depth, float* image);
/* rt_download of the window of columns [x0, x1) x frame rows [y0, y1) (inside this context's
 * rows): pixels/normals/depth as [F][x1-x0][y1-y0] vec4 (the reference's x-major, y-fastest
 * order restricted to the window), image as [y1-y0][x1-x0] rgba32f.  Any pointer may be NULL.
 * For checking regions of large frames without copying the whole ring. */
int rt_download_rect(rt_ctx* ctx, int x0, int x1, int y0, int y1, float* pixels, float* normals, float* depth,
                     float* image);
/* Upload a reference-layout g-buffer ring ([F][W][R] vec4 each; NULL = leave as is). */
int rt_upload_gbuffer(rt_ctx* ctx, const float* pixels, const float* normals, const float* depth);
/* Device pointer of the context's image ([R][W] float4), for collectives. */
void* rt_image_device_ptr(rt_ctx* ctx);
/* Render the image into a caller-owned device buffer of R*W float4 (NULL = own buffer). */
int rt_bind_image(rt_ctx* ctx, void* device_ptr);

/* ---- host-buffer parity path (mirrors the reference call shape) -------------------- */
/* compute_one_shader(frame_num, prog) (src/main.cpp:580-620): sets mode.y = frame_num in
 * `ssbo` (a whole ssbo_data-layout host buffer of rt_ssbo_bytes(S,spp,W,R,F) bytes), copies
 * it in, runs `program`, copies the g-buffer back into `ssbo`, writes the image if non-NULL,
 * and returns (frame_num + 1) % F. */
int rt_compute_one_shader(rt_ctx* ctx, void* ssbo, int frame_num, int program, float* image);
/* compute_two_shaders(frame_num, p1, p2) (src/main.cpp:622-671). */
int rt_compute_two_shaders(rt_ctx* ctx, void* ssbo, int frame_num, int program1, int program2,
                           float* image);

/* ---- multi-device row strips (one process, n strip contexts) ------------------------ */
/* The reference renders one frame with one glDispatchCompute(WIDTH, HEIGHT, 1)
 * (src/main.cpp:604, 645-653) and blits the whole image (783-797).  A group splits that frame
 * into n contiguous row strips, strip i = rows [bounds[i], bounds[i+1]) on device devices[i]
 * (devices may repeat: several strips on one GPU), each an rt_ctx with its own g-buffer ring
 * (+ 1-row halo, so strips never exchange data), and assembles the image strips into one
 * [H][W] rgba32f frame on devices[0]: root-device strips render into their frame rows, the
 * others copy their strip over xGMI (peer access) on the stream that wrote their image
 * (rt_image_stream).  One host thread per strip enqueues its work.  Results equal a
 * whole-frame rt_ctx bit for bit. */
typedef struct rt_group rt_group;
/* cfg: the whole frame (row_begin/row_end ignored); bounds: n+1 increasing rows from 0 to H,
 * or NULL for equal strips.  Fails with RT_E_NODEV for a device ordinal that does not exist and
 * when peer access from a strip's device to devices[0] cannot be enabled (the strip copies
 * would silently go through host memory). */
int rt_group_create(int n, const int* devices, const rt_config* cfg, const int* bounds, rt_group** out);
/* Strip i's copy path: 1 = its image is copied into the frame (another device, peer access
 * on, or forced below), 0 = it renders straight into its frame rows; < 0 on a bad argument. */
int rt_group_strip_copies(rt_group* g, int i);
/* Test hook: on != 0 makes every strip but the root strip (rt_group_root_strip; strip 0 unless a
 * plan moved it) render into its own image and copy it into the frame, even on the root device
 * (the copy path of distinct devices, on one GPU). */
int rt_group_force_copies(rt_group* g, int on);
int rt_group_destroy(rt_group* g);
int rt_group_size(rt_group* g);
int rt_group_bounds(rt_group* g, int* bounds);          /* n+1 entries */
/* Re-plan the strips (the contexts are re-created: fresh rings, pipelining kept). */
int rt_group_set_bounds(rt_group* g, const int* bounds);
/* Strip i's context (kernel stats, counters, downloads of its rows); owned by the group. */
rt_ctx* rt_group_strip(rt_group* g, int i);
int rt_group_last_hip_error(rt_group* g);
/* rt_enable_pipelining on every strip (each on a stream of its own). */
int rt_group_enable_pipelining(rt_group* g, int on);
/* Assemble frames into a caller-owned device buffer of H*W float4 on devices[0] (NULL: the
 * group's own).  Waits for the frames in flight first. */
int rt_group_bind_frame(rt_group* g, void* device_ptr);
void* rt_group_frame_device_ptr(rt_group* g);
/* rt_upload_header for every strip (validated now, uploaded by the next dispatch). */
int rt_group_upload_header(rt_group* g, const void* header, size_t bytes);
/* compute() (src/main.cpp:553-578) on every strip + the strip copies; returns the next slot. */
int rt_group_dispatch(rt_group* g, int mode, int frame);
/* rt_compute_frames on every strip in parallel (the render loop's host updates per strip,
 * identical on all), each frame followed by the strip copies.  Returns the next slot. */
int rt_group_compute_frames(rt_group* g, float* header, int mode, int frame, int n, uint64_t rand_seed,
                            int light_movement);
int rt_group_synchronize(rt_group* g);
/* The assembled frame, [H][W] rgba32f (row 0 = bottom row, like the GL texture). */
int rt_group_download_image(rt_group* g, float* image);
/* Cost-balance the strips for `header`/`mode`: one probe frame with per-row work counters
 * gives the frame's cost profile, rt_plan_strips splits it; then `rounds` plans are timed
 * strip by strip (wall clock of 16 frames after 8, copy included) with rt_calibrate_row_cost
 * re-planning between them, and the best is kept (contexts re-created, rings fresh).
 * strip_ms (n entries, may be NULL): the kept plan's measured ms per frame per strip. */
int rt_group_balance(rt_group* g, const float* header, int mode, int rounds, double* strip_ms);
/* Host-only strip planner (no GPU): contiguous strips of nearly equal total row_cost
 * (row_cost[y] >= 0 for y < H); bounds gets n+1 entries, each strip >= 1 row. */
int rt_plan_strips(const double* row_cost, int H, int n, int* bounds);
/* Host-only gather-aware planner (no GPU).  The frame the reference blits whole
 * (src/main.cpp:783-797) is assembled on a root device that renders one strip, the root strip,
 * into its frame rows; every other strip's image (rows * width * 16 B) crosses one link into the
 * root each frame, overlapped with the next frame's render.  Minimises, over the bounds AND the
 * choice of root strip, the steady-state frame bound
 *   T = max( max_i render_i, max_{i != root} bytes_i / link_gbps, sum_{i != root} bytes_i / ingest_gbps )
 * with render_i = sum of row_ms over strip i (ms per row, e.g. rt_calibrate_row_cost's output).
 * link_gbps: GB/s one way over one link (<= 0: no link term); ingest_gbps: GB/s the root can take
 * from all links at once (<= 0: no ingest term).  Of the root positions that reach the bound, the
 * one whose strip has the most rows (fewest bytes on the links) is taken; the strips on either
 * side of it are balanced within the bound.  bounds: n+1 entries; root_strip: the strip the root
 * owns; bound_ms (NULL or 4 entries): T, render, link and ingest parts (rt_strip_gather_bound). */
int rt_plan_strips_gather(const double* row_ms, int H, int n, int width, double link_gbps, double ingest_gbps,
                          int* bounds, int* root_strip, double* bound_ms);
/* The same bound for a given plan: bound_ms[0..3] = T, max render, max link, ingest (ms). */
int rt_strip_gather_bound(const double* row_ms, int H, const int* bounds, int n, int root_strip, int width,
                          double link_gbps, double ingest_gbps, double* bound_ms);
/* Re-plan with a root strip: strip root_strip renders on devices[0] into its frame rows, strip
 * i < root_strip on devices[i + 1], strip i > root_strip on devices[i] (contexts re-created). */
int rt_group_set_plan(rt_group* g, const int* bounds, int root_strip);
int rt_group_root_strip(rt_group* g);
/* the device strip i renders on */
int rt_group_strip_device(rt_group* g, int i);
/* The link model rt_group_balance plans with when strips copy into the root (distinct devices or
 * forced copies): GB/s per link and into the root.  0 (the default) = measured by the next
 * rt_group_balance (each non-root strip's copy alone, then all at once) and kept.  The first
 * balance round plans the render only (its cost profile is not in ms yet); the gather-aware plan
 * and its root strip come from the second round on, so rounds >= 2. */
int rt_group_set_link_model(rt_group* g, double link_gbps, double ingest_gbps);
int rt_group_link_model(rt_group* g, double* link_gbps, double* ingest_gbps);
/* Rescale row_cost so every strip's total equals its measured time (row shape kept). */
int rt_calibrate_row_cost(double* row_cost, int H, const int* bounds, int n, const double* strip_ms);

/* ---- instrumentation --------------------------------------------------------------- */
/* When on, every kernel launch is bracketed by HIP events on the context stream. */
int rt_enable_timing(rt_ctx* ctx, int on);
/* Sum of event-measured durations of `program`'s kernel since the last reset. */
int rt_kernel_stats(rt_ctx* ctx, int program, int* launches, double* total_ms);
int rt_reset_stats(rt_ctx* ctx);
/* Host time (ms) the context's uploads spent waiting for a free pinned staging buffer — back-
 * pressure when the host runs more than 8 uploads ahead of the GPU — and how many waits,
 * since the last rt_reset_stats.  Host time per frame minus this is the enqueue cost. */
int rt_host_stats(rt_ctx* ctx, double* wait_ms, long long* waits);
/* Work counters (a separate, un-timed instrumentation mode).  on = bit 0: totals, bit 1:
 * per-row counts.  Totals, added by every trace launch: [0] primary samples, [1] closest-hit
 * segments (one scene loop each), [2] shadow rays, [3] ray-shape tests = ([1] + [2]) *
 * int(mode.z) — the algorithmic-FLOP basis of the roofline (20 FLOP per ray-sphere test,
 * SURVEY.md §8d), [4] executed lane-tests = sum over wavefronts of 64 x the shapes their scene
 * loops tested (divergence and culling: [3]/[4] is the useful fraction); post-process:
 * [5] filtered pixels (those with a primary hit, normals.w > 0.99; the others are copied),
 * [6] history slots read, [7] history slots accepted. */
int rt_enable_counters(rt_ctx* ctx, int on);
/* Read the 8 totals (synchronises); reset != 0 zeroes them afterwards. */
int rt_read_counters(rt_ctx* ctx, uint64_t out[8], int reset);
/* Per-row work of this context's rows (R = row_end - row_begin entries), collected while
 * row counters are on: segments + shadow rays (modes 3/4, simple AO kernel), or an estimate in
 * sphere-test units (pooled AO kernel: per-sample setup + culled primary tests + bounce tests).
 * The cost profile used to balance row strips across GPUs. */
int rt_read_row_counters(rt_ctx* ctx, uint64_t* rows, int reset);

/* ---- device math self-test (parity of the shared float semantics) ------------------ */
enum {
  RT_MATH_SIN = 0,       /* sin used by random(): correctly rounded binary32 (in: x)  */
  RT_MATH_RANDOM = 1,    /* random(vec2) hash, p_compute.glsl:65-75 (in: x,y pairs)    */
  RT_MATH_SQRT = 2,      /* IEEE sqrt as used by the kernels (in: x)                   */
  RT_MATH_DIV = 3,       /* IEEE a/b (in: a,b pairs)                                   */
  RT_MATH_NORMALIZE = 4, /* normalize(vec3) (in: xyz triples, out: xyz triples)        */
  RT_MATH_SPHERE = 5,    /* sphere_eval_ray (in: pos3,dir3,center3,r = 10 floats)      */
  RT_MATH_SQRT_SWEEP = 6, /* out[i] = #bit patterns in [i*in[0], (i+1)*in[0]) of the
                             non-negative floats where the kernels' sqrt != sqrtf         */
  RT_MATH_RCP_SWEEP = 7,  /* out[i] = #bit patterns in [i*in[0], (i+1)*in[0]) of the non-
                             negative floats x where the kernels' 1/sqrt (normalize) differs
                             from 1.0f/sqrtf(x), plus those of the normal x in [2^-126, 2^126]
                             where their reciprocal differs from 1.0f/x                   */
  RT_MATH_SQRT_TAIL_SWEEP = 8, /* out[i] = #bit patterns in [i*in[0], (i+1)*in[0]) of the finite
                             non-negative floats where the hit-tail sqrt breaks its contract
                             (== sqrtf on [2^-96, FLT_MAX], in [0, 2^-47] below)          */
  RT_MATH_SIN_RANGE = 9,  /* out[i] = sin(x) of random() for the float whose bit pattern is
                             bits(in[0]) + i (mod 2^32): exhaustive sweeps without inputs  */
  RT_MATH_SHADOW = 10     /* shadow_ray's occluder test (p_compute.glsl:159-161) as the
                             kernels decide it: in = (light - pos).xyz, t quads; l =
                             normalize(light - pos), len = length(light - pos); out = (l.xyz,
                             len, 1 if t > 0.0001 && length(dvec3(t * l)) < len else 0)     */,
  RT_MATH_SIN_TABLE = 11  /* the sin's exception table (rt_sin_table.h) on this build's device code:
                             out[2i] = 1 if entry i's binary64 sin is flagged ambiguous (so the
                             table decides it), 0 if not, -1 past the table; out[2i+1] = its x */
};
int rt_selftest_math(rt_ctx* ctx, int fn, const float* in, float* out, size_t n);

/* ---- host-only scene / header helpers (no GPU) ------------------------------------- */
/* loadShapeBuffer() entries (src/main.cpp:417-420, 439-442, 462-466).  `header` is the
 * SSBO prefix as float*, S its shape capacity; index i < S.  Unwritten lanes are untouched,
 * as in the reference. */
int rt_pack_sphere(float* header, int S, int i, const float center[3], float radius,
                   const float color[3], float reflectivity, int emissive);
/* plane(normal, dist, color) — p0 = dist * normal (src/geom_objs/plane.h:31-34). */
int rt_pack_plane(float* header, int S, int i, const float normal[3], float dist,
                  const float color[3], float reflectivity, int emissive);
int rt_pack_rectangle(float* header, int S, int i, const float llc[3], const float right[3],
                      const float up[3], const float color[3], float reflectivity, int emissive);
/* Camera basis of render() (src/main.cpp:772-779): w = look; u = normalize(cross(up,w));
 * v = normalize(cross(w,u)); horizontal = aspect*u; vertical = v;
 * llc_minus_campos = -0.5*(horizontal+vertical) - w; writes those + camera_location. */
int rt_camera_basis(float* header, const float location[3], const float up[3],
                    const float look_towards[3], float aspect);
/* Header fill of compute_one_shader (src/main.cpp:584-589): mode.y = frame, mode.z = n. */
int rt_set_mode(float* header, int frame, int num_objects);
/* fill_rand_buffer (src/main.cpp:535-539) with a seeded generator instead of rand():
 * splitmix64(seed), top 24 bits / 2^24 per float, 2*AA vec4. */
int rt_fill_rand_buffer(float* header, int S, int AA, uint64_t seed);
/* moving_light (src/main.cpp:541-551). */
int rt_moving_light(float* header, int light_movement);
/* Synthetic seeded scene of SURVEY §8d: ground sphere + (n_objects-1) random spheres, the
 * default camera (src/main.cpp:98-100), light (-12,8,7), SKY background, mode.z = n_objects.
 * S = capacity >= n_objects. */
int rt_scenegen(float* header, int S, int n_objects, int AA, uint64_t seed, float aspect);
/* The reference's built-in scenes 1, 5, 6 (src/scene.h:15-167) with the default camera. */
int rt_init_scene(float* header, int S, int AA, int which, float aspect);

const char* rt_strerror(int status);
int rt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_ABI_H */
