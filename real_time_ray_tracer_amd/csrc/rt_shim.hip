// rt_shim.hip — C-ABI host shim (include/rt/abi.h) over the gfx950 kernels.
//
// Replaces the GL boundary of src/main.cpp:
//   computeInitGeom / computeInit (471-501)   -> rt_create
//   compute_one_shader (580-620)              -> rt_compute_one_shader / rt_run_program
//   compute_two_shaders (622-671)             -> rt_compute_two_shaders
//   compute() (553-578)                       -> rt_dispatch
// Device layout: the g-buffer ring stays resident in HBM as per-slot row-major [rows][W]
// float4 arrays, each reached through a slot -> buffer map with spare buffers (pixels: two,
// so the post-process can write out of place and swap; normals/depth: one), instead of the
// reference's 2 x 55.76 MB host round trip per frame.  The reference [F][W][H] layout is
// produced only by rt_download / consumed by rt_upload_gbuffer.
//
// Pipelined mode 1 (rt_enable_pipelining): consecutive frames' AO passes run on two
// alternating streams (so frame k+1's AO fills the tail of frame k's), and every post-process
// runs on a third, output stream.  AO k writes its normals/depth into free buffers (a queue of
// two) and its raw pixels into one of the two spare pixel buffers, and reads its header from
// its own copy (two copies), so nothing another in-flight pass reads changes under it: the
// post-process of frame k-1 may read slot k%8's previous contents as its oldest history, and
// AO k itself reads them for the stale normal/depth of emissive first hits.  AO k waits for
// post k-2 (the last reader of the buffers it overwrites); post k waits for AO k.  The results
// are those of the sequential order, bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <new>
#include <utility>
#include <vector>

#include "../../include/rt/abi.h"
#include "rt_kernels.h"

namespace {

constexpr int kMaxShapes = 2048;
constexpr int kMaxSpp = 256;
constexpr int kMaxDepth = 65535;  // stop values are packed in 16 bits by the pooled AO kernel
constexpr int kStageSlots = 8;
// Pipelining depth D: AO k waits for post k-D, the last reader of the raw pixel buffer and the
// normals/depth buffers it overwrites (D of each rotate outside the slot map)
constexpr int kPipe = 4;  // capacity; the depth in use is rt_ctx::pipe_depth (default 3)
// AO streams: pipelined frame k's AO pass runs on AO stream k % n_ao_streams (0 = the main
// stream) and reads header copy k % n_ao_streams
constexpr int kAoStreams = 3;  // capacity; in use: rt_ctx::n_ao_streams (default 2)

struct Stage {
  void* host = nullptr;  // pinned
  size_t bytes = 0;
  hipEvent_t done = nullptr;
  bool used = false;
};

// Longest-first workgroup schedule.  A launch's time is set by its longest workgroups when they
// start late: the few hybrid tiles (mode 4) whose mirror paths bounce for many rounds.  The waves
// record their bounce rounds in d_cost; every kSchedPeriod-th launch the costs are read back on
// a side stream, and when the sorted order changes it is uploaded into the table no launch in
// flight reads, which becomes the active one once the copy has landed.  Nothing here waits on the GPU or puts a copy between two launches
// on a launch stream; the permutation only moves work between workgroups, so the images do not
// depend on it.
enum { kSchedHybrid = 0, kSchedKinds = 1 };
struct TileSched {
  int gx = 0, gy = 0, nunits = 0, per_unit = 1;  // units (tiles / pools) = gx * gy; cost slots per unit
  unsigned* d_cost = nullptr;          // [nunits * per_unit]
  unsigned* d_order[2] = {};           // [nunits] each
  unsigned* h_cost = nullptr;          // pinned
  unsigned* h_order[2] = {};           // pinned
  hipStream_t side = nullptr;
  hipEvent_t ev_launch = nullptr, ev_cost = nullptr, ev_order = nullptr;
  hipEvent_t ev_use[2][3] = {};        // per table: its last readers on each launch stream
  hipStream_t used_on[2][3] = {};      // the launch streams a table was read on
  int active = -1;                     // the table launches read (-1: the plain order)
  int pending = -1;                    // the table being uploaded
  bool cost_inflight = false;
  long long launches = 0;
  int orders_taken = 0;                // orders that became active (rt_tile_schedule_orders)
  std::vector<unsigned> cur, next;     // the active / pending order
};
constexpr int kSchedPeriod = 16;

}  // namespace

struct rt_ctx {
  int device = 0;
  int inject_query_error = 0;  // test hook (rt_debug_fail_next_event_query): the next staging query fails
  rt_config cfg{};
  int own0 = 0, own_rows = 0;    // strip rows
  int band0 = 0, band_rows = 0;  // strip + 1-row halo (post-process neighbours)
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  float4* d_shapes_buf[kAoStreams] = {};  // shape tables + rand_buffer (rt::table_vec4), one copy per AO stream
  float4* d_rb_buf[kAoStreams] = {};      // = d_shapes_buf[k] + rt::rand_table(S) (one allocation, one upload)
  float4* d_shapes = nullptr;  // the copy the next dispatch reads
  float4* d_rb = nullptr;
  std::vector<float4*> pix;    // F+pipe_depth buffers
  std::vector<int> pix_slot;   // slot -> buffer index
  int spare = 0;               // pixel buffer outside the map (sequential post-process target)
  int raw_buf[kPipe] = {};     // raw_buf[1..]: more pixel buffers outside the map (pipelined raw AO output)
  std::vector<float4*> nrm, dep;       // F+pipe_depth buffers each
  std::vector<int> nrm_slot, dep_slot;  // slot -> buffer index
  int nrm_free[kPipe] = {}, dep_free[kPipe] = {};  // buffers outside the map, oldest first
  // pipelined mode 1
  bool pipelined = false;
  hipStream_t out_stream = nullptr, own_out_stream = nullptr;
  hipStream_t ao_streams[kAoStreams] = {};  // [0] unused (the main stream); [1..] the context's own
  int pipe_depth = 3, n_ao_streams = 2;
  hipEvent_t ev_ao = nullptr, ev_post[kPipe] = {}, ev_join = nullptr, ev_seq = nullptr;
  bool post_recorded[kPipe] = {};
  long long pipe_n = 0;
  bool out_pending = false;
  float4* d_image_own = nullptr;
  float4* d_image = nullptr;
  hipStream_t img_stream = nullptr;  // the stream of the last launch that wrote the image
  std::vector<float> header;   // host copy of the SSBO prefix
  std::vector<float4> table;   // host copy of the device table (rt::table_vec4 float4)
  bool have_header = false;
  int nplanes = 0;             // planes among simple_shapes[0, nobj)
  int ncl = 0;                 // AO bounce-ray clusters of the table the next dispatch reads (build_clusters)
  float4* d_xfer = nullptr;    // rt_download / rt_upload_gbuffer: one array in the reference layout [F][W][R]
  float4* d_batch = nullptr;   // rt_compute_frames: device table copies, 2 x kBatch slots (one per distinct table)
  int batch_last = -1;         // the d_batch slot d_shapes points into after rt_compute_frames (else -1)
  TileSched sched[kSchedKinds];  // longest-first schedules (set up by the first launch of each kind)
  bool sched_on = true;          // rt_set_tile_schedule
  float4* d_mf_rb = nullptr;   // rt_compute_frames, mode 2: the rand_buffers of a multi-frame launch
  std::vector<float4> batch_host;
  std::vector<float> batch_hdr;  // the batch's host headers (camera, light: launch parameters)
  int nobj = 0;
  int mf_max = 1;  // rt_compute_frames: most frames per launch (rt_set_frame_batch; 1 = the reference's shape)
  Stage stage[kStageSlots];
  int stage_next = 0;
  // timing
  bool timing = false;
  struct Timed {
    hipEvent_t e0, e1;
    int frames;  // frames the launch rendered (multi-frame Phong/hybrid launches: up to kMaxBatch)
  };
  std::vector<Timed> pending[RT_PROG_COUNT];  // recorded on the launch stream
  std::vector<hipEvent_t> event_pool;
  double total_ms[RT_PROG_COUNT] = {};
  int launches[RT_PROG_COUNT] = {};
  unsigned long long* d_counters = nullptr;
  unsigned long long* d_row_counters = nullptr;  // [band_rows]
  bool counting = false;
  bool row_counting = false;
  int last_hip = 0;
  // host time spent waiting for a staging buffer to be free (back-pressure: the host is up to
  // kStageSlots uploads ahead of the GPU), since the last rt_reset_stats
  double host_wait_ms = 0.0;
  long long host_waits = 0;
};

namespace {

int hip_fail(rt_ctx* c, hipError_t e) {
  if (c) c->last_hip = (int)e;
  return RT_E_HIP;
}

#define RT_HIP(ctx, expr)                     \
  do {                                        \
    hipError_t _e = (expr);                   \
    if (_e != hipSuccess) return hip_fail(ctx, _e); \
  } while (0)

size_t slot_elems(const rt_ctx* c) { return (size_t)c->band_rows * c->cfg.width; }
// stride of the device shape tables (>= 1, so an empty scene still has valid pointers)
// One row per table beyond the shapes: the colour table's row -1 (the geo2 table's last row)
// holds the background, so the AO kernel's shading reads a miss's attenuation as col[-1]
// (rt_kernels_impl.h col_at) instead of keeping the background in scalar registers.
int table_stride(const rt_ctx* c) { return std::max(1, c->cfg.num_shapes) + 1; }

hipEvent_t get_event(rt_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Async H2D copy through a ring of pinned staging buffers, so callers may reuse their
// (pageable) memory as soon as the call returns and the stream never has to drain.
int staged_copy(rt_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (bytes == 0) return RT_OK;
  Stage& s = c->stage[c->stage_next];
  c->stage_next = (c->stage_next + 1) % kStageSlots;
  if (s.used) {
    // hipErrorNotReady is "the GPU has not consumed it yet" (wait, and clear that per-thread
    // error); any other failure is a fault of the copy or of the work before it on the stream:
    // reported (rt_last_hip_error), never taken as "consumed" and the buffer reused
    hipError_t q = hipEventQuery(s.done);
    if (c->inject_query_error) {
      q = (hipError_t)c->inject_query_error;
      c->inject_query_error = 0;
    }
    if (q == hipErrorNotReady) {
      (void)hipGetLastError();
      const auto t0 = std::chrono::steady_clock::now();
      RT_HIP(c, hipEventSynchronize(s.done));
      c->host_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      c->host_waits += 1;
    } else if (q != hipSuccess) {
      return hip_fail(c, q);
    }
  }
  if (s.bytes < bytes) {  // grow to a power of two >= 256 KiB: pinned allocations are slow, keep them rare
    if (s.host) RT_HIP(c, hipHostFree(s.host));
    s.host = nullptr;
    size_t cap = 256 << 10;
    while (cap < bytes) cap <<= 1;
    RT_HIP(c, hipHostMalloc(&s.host, cap, hipHostMallocDefault));
    s.bytes = cap;
  }
  if (!s.done) RT_HIP(c, hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  std::memcpy(s.host, src, bytes);
  RT_HIP(c, hipMemcpyAsync(dst, s.host, bytes, hipMemcpyHostToDevice, st));
  RT_HIP(c, hipEventRecord(s.done, st));
  s.used = true;
  return RT_OK;
}

void free_sched(TileSched& h) {
  if (h.side) (void)hipStreamSynchronize(h.side);
  if (h.d_cost) (void)hipFree(h.d_cost);
  for (int k = 0; k < 2; ++k) {
    if (h.d_order[k]) (void)hipFree(h.d_order[k]);
    if (h.h_order[k]) (void)hipHostFree(h.h_order[k]);
    for (auto e : h.ev_use[k])
      if (e) (void)hipEventDestroy(e);
  }
  if (h.h_cost) (void)hipHostFree(h.h_cost);
  for (auto e : {h.ev_launch, h.ev_cost, h.ev_order})
    if (e) (void)hipEventDestroy(e);
  if (h.side) (void)hipStreamDestroy(h.side);
  h = TileSched{};
}

void free_all(rt_ctx* c) {
  for (auto& h : c->sched) free_sched(h);
  for (auto& s : c->stage) {
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.host) (void)hipHostFree(s.host);
  }
  for (int k = 0; k < RT_PROG_COUNT; ++k)
    for (auto& pr : c->pending[k]) {
      (void)hipEventDestroy(pr.e0);
      (void)hipEventDestroy(pr.e1);
    }
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  for (auto p : c->pix) if (p) (void)hipFree(p);
  for (auto p : c->nrm) if (p) (void)hipFree(p);
  for (auto p : c->dep) if (p) (void)hipFree(p);
  if (c->d_image_own) (void)hipFree(c->d_image_own);
  for (int k = 0; k < kAoStreams; ++k) {
    if (c->d_shapes_buf[k]) (void)hipFree(c->d_shapes_buf[k]);
  }
  if (c->d_counters) (void)hipFree(c->d_counters);
  if (c->d_batch) (void)hipFree(c->d_batch);
  if (c->d_xfer) (void)hipFree(c->d_xfer);
  if (c->d_mf_rb) (void)hipFree(c->d_mf_rb);
  if (c->d_row_counters) (void)hipFree(c->d_row_counters);
  for (auto e : {c->ev_ao, c->ev_join, c->ev_seq})
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->ev_post)
    if (e) (void)hipEventDestroy(e);
  if (c->own_out_stream) (void)hipStreamDestroy(c->own_out_stream);
  for (int k = 1; k < kAoStreams; ++k)
    if (c->ao_streams[k]) (void)hipStreamDestroy(c->ao_streams[k]);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
}

// Order everything issued so far on the output stream before later work on the main stream
// (every call except a pipelined mode-1 dispatch starts with this).
int join(rt_ctx* c) {
  if (!c->out_pending) return RT_OK;
  for (int k = 1; k < c->n_ao_streams; ++k) {
    RT_HIP(c, hipEventRecord(c->ev_join, c->ao_streams[k]));
    RT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
  }
  RT_HIP(c, hipEventRecord(c->ev_join, c->out_stream));
  RT_HIP(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
  c->out_pending = false;
  for (auto& r : c->post_recorded) r = false;  // ordered by the join from now on
  c->pipe_n = 0;
  return RT_OK;
}

int sync_all(rt_ctx* c) {
  RT_HIP(c, hipStreamSynchronize(c->stream));
  for (int k = 1; k < kAoStreams; ++k)
    if (c->ao_streams[k]) RT_HIP(c, hipStreamSynchronize(c->ao_streams[k]));
  if (c->out_stream && c->out_stream != c->stream) RT_HIP(c, hipStreamSynchronize(c->out_stream));
  return RT_OK;
}

// Stream and header copy of the next header upload / AO pass: pipelined frames alternate
// between the main stream + copy 0 and the second stream + copy 1.
int hdr_copy(const rt_ctx* c) { return c->pipelined ? (int)(c->pipe_n % c->n_ao_streams) : 0; }
hipStream_t ao_stream(const rt_ctx* c) { return hdr_copy(c) ? c->ao_streams[hdr_copy(c)] : c->stream; }
// a new pipelined sequence: the other AO streams start after everything issued so far
int start_sequence(rt_ctx* c) {
  RT_HIP(c, hipEventRecord(c->ev_seq, c->stream));
  for (int k = 1; k < c->n_ao_streams; ++k) RT_HIP(c, hipStreamWaitEvent(c->ao_streams[k], c->ev_seq, 0));
  return RT_OK;
}

const float* hv(const rt_ctx* c, int v) { return c->header.data() + 4 * v; }

void fill_params(const rt_ctx* c, int frame, rt::FrameParams& p) {
  std::memset(&p, 0, sizeof(p));
  p.W = c->cfg.width;
  p.H = c->cfg.height;
  p.band_row0 = c->band0;
  p.band_rows = c->band_rows;
  p.img_row0 = c->own0;
  p.img_rows = c->own_rows;
  p.nobj = c->nobj;
  p.S = table_stride(c);
  p.nplanes = c->nplanes;
  p.ncl = c->ncl;
  p.spp = c->cfg.spp;
  p.inv_spp = 1.0f / (float)c->cfg.spp;
  p.fW = (float)c->cfg.width;
  p.inv_W = 1.0f / p.fW;
  p.fH = (float)c->cfg.height;
  p.inv_H = 1.0f / p.fH;
  p.D = c->cfg.max_depth;
  p.F = c->cfg.num_frames;
  p.frame = frame;
  const float *h = hv(c, RT_HDR_HORIZONTAL), *v = hv(c, RT_HDR_VERTICAL),
              *l = hv(c, RT_HDR_LLC_MINUS_CAMPOS), *cam = hv(c, RT_HDR_CAMERA_LOCATION),
              *L = hv(c, RT_HDR_LIGHT_POS), *bg = hv(c, RT_HDR_BACKGROUND);
  p.hx = h[0]; p.hy = h[1]; p.hz = h[2];
  p.vx = v[0]; p.vy = v[1]; p.vz = v[2];
  p.lx = l[0]; p.ly = l[1]; p.lz = l[2];
  p.cx = cam[0]; p.cy = cam[1]; p.cz = cam[2];
  p.Lx = L[0]; p.Ly = L[1]; p.Lz = L[2];
  p.bg = make_float4(bg[0], bg[1], bg[2], bg[3]);
  p.shapes = c->d_shapes;
  p.rb = c->d_rb;
  p.image = c->d_image;
  for (int s = 0; s < c->cfg.num_frames; ++s) {
    p.hist_pix[s] = c->pix[c->pix_slot[s]];
    p.hist_nrm[s] = c->nrm[c->nrm_slot[s]];
    p.hist_dep[s] = c->dep[c->dep_slot[s]];
  }
  p.nrm = c->nrm[c->nrm_slot[frame]];
  p.dep = c->dep[c->dep_slot[frame]];
  p.nrm_prev = p.nrm;
  p.dep_prev = p.dep;
  p.counters = c->counting ? c->d_counters : nullptr;
  p.row_counters = c->row_counting ? c->d_row_counters : nullptr;
}

int launch(rt_ctx* c, int program, const rt::FrameParams& p, hipStream_t st) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->timing) {
    e0 = get_event(c);
    e1 = get_event(c);
    if (!e0 || !e1) return RT_E_HIP;
    RT_HIP(c, hipEventRecord(e0, st));
  }
  hipError_t e = rt::launch_program(program, p, st);
  if (e != hipSuccess) return hip_fail(c, e);
  if (p.image) c->img_stream = st;  // consumers of the image order their reads after this stream
  if (c->timing) {
    RT_HIP(c, hipEventRecord(e1, st));
    c->pending[program].push_back(rt_ctx::Timed{e0, e1, p.mf_n > 0 ? p.mf_n : 1});
  }
  return RT_OK;
}
int launch(rt_ctx* c, int program, const rt::FrameParams& p) { return launch(c, program, p, c->stream); }

// Before a launch of schedule `kind` over gx x gy units (cost slots per_unit each): take up a
// landed order table, turn landed costs into an order, and set the launch's tile_order /
// tile_cost (see TileSched).
int sched_before(rt_ctx* c, int kind, int gx, int gy, int per_unit, rt::FrameParams& p) {
  TileSched& h = c->sched[kind];
  if (!c->sched_on || gx < 1 || gy < 1) return RT_OK;
  if (h.nunits && (h.gx != gx || h.gy != gy || h.per_unit != per_unit)) {
    RT_HIP(c, hipDeviceSynchronize());  // (never in practice: a context's launch shapes are fixed)
    free_sched(h);
  }
  if (!h.nunits) {
    if (gx >= 65536 || gy >= 65536) return RT_OK;
    h.gx = gx;
    h.gy = gy;
    h.per_unit = per_unit;
    h.nunits = gx * gy;
    const size_t nc = (size_t)h.nunits * per_unit * sizeof(unsigned), no = (size_t)h.nunits * sizeof(unsigned);
    RT_HIP(c, hipMalloc(&h.d_cost, nc));
    RT_HIP(c, hipMemsetAsync(h.d_cost, 0, nc, c->stream));
    RT_HIP(c, hipHostMalloc(&h.h_cost, nc, hipHostMallocDefault));
    for (int k = 0; k < 2; ++k) {
      RT_HIP(c, hipMalloc(&h.d_order[k], no));
      RT_HIP(c, hipHostMalloc(&h.h_order[k], no, hipHostMallocDefault));
      for (auto& e : h.ev_use[k]) RT_HIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    RT_HIP(c, hipStreamCreateWithFlags(&h.side, hipStreamNonBlocking));
    RT_HIP(c, hipEventCreateWithFlags(&h.ev_launch, hipEventDisableTiming));
    RT_HIP(c, hipEventCreateWithFlags(&h.ev_cost, hipEventDisableTiming));
    RT_HIP(c, hipEventCreateWithFlags(&h.ev_order, hipEventDisableTiming));
  }
  // has the work before event e finished?  hipErrorNotReady is "not yet" (its per-thread error
  // is cleared); any other failure is a fault of the side stream's copies or of the launches they
  // wait on, reported to the caller (rt_last_hip_error), never taken as "not yet"
  bool order_landed = false, cost_landed = false;
  auto query = [&](hipEvent_t e, bool& done) -> hipError_t {
    const hipError_t q = hipEventQuery(e);
    done = q == hipSuccess;
    if (q == hipErrorNotReady) {
      (void)hipGetLastError();
      return hipSuccess;
    }
    return q;
  };
  if (h.pending >= 0) RT_HIP(c, query(h.ev_order, order_landed));
  if (h.cost_inflight) RT_HIP(c, query(h.ev_cost, cost_landed));
  if (order_landed) {
    if (h.active >= 0)  // the launches enqueued so far are the old table's last readers
      for (int s = 0; s < 3; ++s)
        if (h.used_on[h.active][s]) RT_HIP(c, hipEventRecord(h.ev_use[h.active][s], h.used_on[h.active][s]));
    h.active = h.pending;
    h.pending = -1;
    ++h.orders_taken;
    h.cur.swap(h.next);
    for (auto& st : h.used_on[h.active]) st = nullptr;
  }
  if (cost_landed) {
    h.cost_inflight = false;
    if (h.pending < 0) {
      // longest first: a unit's cost is its slowest slot's; ties keep the plain order
      std::vector<unsigned> cost(h.nunits);
      for (int t = 0; t < h.nunits; ++t) {
        unsigned v = 0;
        for (int k = 0; k < h.per_unit; ++k) v = std::max(v, h.h_cost[(size_t)t * h.per_unit + k]);
        cost[t] = v;
      }
      std::vector<unsigned> idx(h.nunits);
      for (int t = 0; t < h.nunits; ++t) idx[t] = (unsigned)t;
      std::stable_sort(idx.begin(), idx.end(), [&](unsigned a, unsigned b) { return cost[a] > cost[b]; });
      for (auto& t : idx) t = (t % (unsigned)h.gx) | ((t / (unsigned)h.gx) << 16);  // packed x | y << 16
      const bool uniform = std::all_of(cost.begin(), cost.end(), [&](unsigned v) { return v == cost[0]; });
      if (!uniform && idx != h.cur) {
        const int x = h.active == 0 ? 1 : 0;  // the table no launch reads from now on
        std::memcpy(h.h_order[x], idx.data(), idx.size() * sizeof(unsigned));
        for (int s = 0; s < 3; ++s)
          if (h.used_on[x][s]) RT_HIP(c, hipStreamWaitEvent(h.side, h.ev_use[x][s], 0));
        RT_HIP(c, hipMemcpyAsync(h.d_order[x], h.h_order[x], idx.size() * sizeof(unsigned), hipMemcpyHostToDevice,
                                 h.side));
        RT_HIP(c, hipEventRecord(h.ev_order, h.side));
        h.pending = x;
        h.next.swap(idx);
      }
    }
  }
  p.tile_order = h.active >= 0 ? h.d_order[h.active] : nullptr;
  p.tile_cost = h.d_cost;
  return RT_OK;
}

// After a launch of schedule `kind` on stream `st`: note that the active table was read on st;
// every kSchedPeriod-th launch has its costs read back on the side stream (launches after it may
// overwrite them meanwhile: a cost is a hint, never a result).
int sched_after(rt_ctx* c, int kind, hipStream_t st) {
  TileSched& h = c->sched[kind];
  if (!c->sched_on || !h.nunits) return RT_OK;
  if (h.active >= 0) {
    hipStream_t* u = h.used_on[h.active];
    for (int s = 0; s < 3; ++s) {
      if (u[s] == st) break;
      if (!u[s]) {
        u[s] = st;
        break;
      }
    }
  }
  if (h.launches++ % kSchedPeriod == 0 && !h.cost_inflight) {
    RT_HIP(c, hipEventRecord(h.ev_launch, st));
    RT_HIP(c, hipStreamWaitEvent(h.side, h.ev_launch, 0));
    RT_HIP(c, hipMemcpyAsync(h.h_cost, h.d_cost, (size_t)h.nunits * h.per_unit * sizeof(unsigned),
                             hipMemcpyDeviceToHost, h.side));
    RT_HIP(c, hipEventRecord(h.ev_cost, h.side));
    h.cost_inflight = true;
  }
  return RT_OK;
}

// A launch of `program` with its schedule (hybrid tiles, AO pools), if it has one.
int launch_sched(rt_ctx* c, int program, rt::FrameParams& p, hipStream_t st) {
  int kind = -1, gx = 0, gy = 1, per = 1;
  if (program == RT_PROG_H_COMPUTE) {  // units: the hybrid workgroups (rt::kHyTile px square, kHyBW^2 waves)
    kind = kSchedHybrid;
    gx = (p.W + rt::kHyTile - 1) / rt::kHyTile;
    gy = (p.trace_rows + rt::kHyTile - 1) / rt::kHyTile;
    per = rt::kHyBW * rt::kHyBW;
  }
  // (AO pools in the same longest-first order by wave time measured nothing at (c) and (d): those
  // launches are not tail-bound; the kernel's bookkeeping cost registers, profiles/r04h_*)
  if (kind < 0) return launch(c, program, p, st);
  int rc = sched_before(c, kind, gx, gy, per, p);
  if (rc == RT_OK) rc = launch(c, program, p, st);
  if (rc == RT_OK) rc = sched_after(c, kind, st);
  return rc;
}

int run_program(rt_ctx* c, int program, int frame) {
  if (!c->have_header) return RT_E_STATE;
  if (frame < 0 || frame >= c->cfg.num_frames) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int jr = join(c);
  if (jr != RT_OK) return jr;
  rt::FrameParams p;
  fill_params(c, frame, p);
  switch (program) {
    case RT_PROG_P_COMPUTE:
    case RT_PROG_H_COMPUTE:
      // pixels of the strip rows only; the halo rows' pixels are never read
      p.trace_row0 = c->own0;
      p.trace_rows = c->own_rows;
      p.out_pix = c->pix[c->pix_slot[frame]];
      return launch_sched(c, program, p, c->stream);
    case RT_PROG_AO_COMPUTE:
    case RT_PROG_AOP_COMPUTE:
      // g-buffer writers trace the halo rows too, so a strip's ring evolves exactly like the
      // same rows of a whole-frame ring (post-process neighbours + stale-depth reads)
      p.trace_row0 = c->band0;
      p.trace_rows = c->band_rows;
      p.out_pix = c->pix[c->pix_slot[frame]];
      if (program == RT_PROG_AOP_COMPUTE) p.image = nullptr;  // aop_compute.glsl has no image
      return launch(c, program, p);
    case RT_PROG_AOP_POSTPROCESSING: {
      p.trace_row0 = c->own0;
      p.trace_rows = c->own_rows;
      p.raw = c->pix[c->pix_slot[frame]];
      p.out_pix = c->pix[c->spare];
      int rc = launch(c, program, p);
      if (rc != RT_OK) return rc;
      std::swap(c->pix_slot[frame], c->spare);  // filtered buffer becomes slot `frame`
      return RT_OK;
    }
    default:
      return RT_E_INVAL;
  }
}

// Frames slot0, slot0+1, ... (m <= min(kMaxBatch, F)) of one program in ONE launch: Phong /
// hybrid (gridDim.z = m, one light each) or ao_compute (gridDim.y = m, one rand_buffer each,
// from d_mf_rb).  The frames of modes 2-4 touch only their own slot (mode 2's stale-depth reads
// come from the slot's previous contents, F frames back), so they may run concurrently; the
// image, which each next frame overwrites, is written by the last frame only.
int run_program_mf(rt_ctx* c, int program, int slot0, int m, const float4* lights) {
  if (!c->have_header) return RT_E_STATE;
  if (program != RT_PROG_P_COMPUTE && program != RT_PROG_H_COMPUTE && program != RT_PROG_AO_COMPUTE) return RT_E_INVAL;
  if (m < 1 || m > rt::kMaxBatch || m > c->cfg.num_frames || slot0 < 0 || slot0 >= c->cfg.num_frames)
    return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int jr = join(c);
  if (jr != RT_OK) return jr;
  rt::FrameParams p;
  fill_params(c, slot0, p);
  const bool ao = program == RT_PROG_AO_COMPUTE;
  p.trace_row0 = ao ? c->band0 : c->own0;  // g-buffer writers trace the halo rows too (run_program)
  p.trace_rows = ao ? c->band_rows : c->own_rows;
  p.out_pix = c->pix[c->pix_slot[slot0]];
  p.mf_n = m;
  p.mf_slot0 = slot0;
  if (ao) p.mf_rb = c->d_mf_rb;
  else
    for (int j = 0; j < m; ++j) p.mf_light[j] = lights[j];
  return launch_sched(c, program, p, c->stream);
}

// One pipelined mode-1 frame (see the header comment): AO on the frame's AO stream into free
// normals/depth buffers and a raw pixel buffer, post-process on the output stream.
int pipelined_frame(rt_ctx* c, int frame) {
  if (!c->have_header) return RT_E_STATE;
  if (frame < 0 || frame >= c->cfg.num_frames) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  const int D = c->pipe_depth;
  const int nq = (int)(c->pipe_n % D);
  hipStream_t st = ao_stream(c);
  if (c->pipe_n == 0) {  // a new sequence: the other AO streams start after everything so far
    int sr = start_sequence(c);
    if (sr != RT_OK) return sr;
  }
  if (c->post_recorded[nq]) RT_HIP(c, hipStreamWaitEvent(st, c->ev_post[nq], 0));  // post k-D
  float4* raw = c->pix[nq == 0 ? c->spare : c->raw_buf[nq]];  // the sequential spare is raw buffer 0
  rt::FrameParams p;
  fill_params(c, frame, p);
  p.shapes = c->d_shapes_buf[hdr_copy(c)];
  p.rb = c->d_rb_buf[hdr_copy(c)];
  p.trace_row0 = c->band0;
  p.trace_rows = c->band_rows;
  p.out_pix = raw;
  p.image = nullptr;
  p.nrm_prev = p.nrm;  // the slot's previous contents (stale reads)
  p.dep_prev = p.dep;
  const int xn = c->nrm_free[0], xd = c->dep_free[0];
  p.nrm = c->nrm[xn];
  p.dep = c->dep[xd];
  int rc = launch(c, RT_PROG_AOP_COMPUTE, p, st);
  if (rc != RT_OK) return rc;
  // the slot now maps to the fresh buffers; its previous ones join the back of the free queue
  for (int q = 0; q + 1 < D; ++q) {
    c->nrm_free[q] = c->nrm_free[q + 1];
    c->dep_free[q] = c->dep_free[q + 1];
  }
  c->nrm_free[D - 1] = c->nrm_slot[frame];
  c->dep_free[D - 1] = c->dep_slot[frame];
  c->nrm_slot[frame] = xn;
  c->dep_slot[frame] = xd;
  RT_HIP(c, hipEventRecord(c->ev_ao, st));
  RT_HIP(c, hipStreamWaitEvent(c->out_stream, c->ev_ao, 0));
  rt::FrameParams q;
  fill_params(c, frame, q);
  q.trace_row0 = c->own0;
  q.trace_rows = c->own_rows;
  q.raw = raw;
  q.out_pix = c->pix[c->pix_slot[frame]];  // filtered in place of slot `frame`'s oldest contents
  rc = launch(c, RT_PROG_AOP_POSTPROCESSING, q, c->out_stream);
  if (rc != RT_OK) return rc;
  RT_HIP(c, hipEventRecord(c->ev_post[nq], c->out_stream));
  c->post_recorded[nq] = true;
  c->out_pending = true;
  c->pipe_n += 1;
  c->d_shapes = c->d_shapes_buf[hdr_copy(c)];  // what a sequential dispatch would read next
  c->d_rb = c->d_rb_buf[hdr_copy(c)];
  return RT_OK;
}

int resolve_timing(rt_ctx* c) {
  bool any = false;
  for (int k = 0; k < RT_PROG_COUNT; ++k) any = any || !c->pending[k].empty();
  if (!any) return RT_OK;
  int rc = sync_all(c);
  if (rc != RT_OK) return rc;
  for (int k = 0; k < RT_PROG_COUNT; ++k) {
    for (auto& pr : c->pending[k]) {
      float ms = 0.0f;
      RT_HIP(c, hipEventElapsedTime(&ms, pr.e0, pr.e1));
      c->total_ms[k] += ms;
      c->launches[k] += pr.frames;  // per frame: a multi-frame launch counts its frames
      c->event_pool.push_back(pr.e0);
      c->event_pool.push_back(pr.e1);
    }
    c->pending[k].clear();
  }
  return RT_OK;
}

// Slot layouts on the device (rt_kernels_impl.h): pixels are [band_rows][W] float4; normals are
// a [band_rows][W] xyz plane (12 B) then a w plane (4 B) (nrm_store); depth is two [band_rows][W]
// float2 planes, (x, y) then (z, w) (dep_store).
enum SlotKind { kPixels = 0, kNormals = 1, kDepth = 2 };

// The g-buffer in the reference layout ([F][W][R] vec4, y fastest) goes through one device array
// of that layout: a conversion kernel (rt::launch_gbuf_convert) between it and the slot layouts,
// and one copy of exactly the caller's bytes (no host-side transposes).
// The array holds ONE frame ([W][R] vec4): frames are converted and copied one at a time (each
// frame is an independent [W][R] block of the reference layout), so a 4K context keeps 133 MB
// for it, not the ring's F frames.
int xfer_buffer(rt_ctx* c) {
  if (!c->d_xfer) {
    hipError_t e = hipMalloc(&c->d_xfer, (size_t)c->cfg.width * c->own_rows * sizeof(float4));
    if (e == hipErrorOutOfMemory) {
      c->last_hip = (int)e;
      c->d_xfer = nullptr;
      return RT_E_NOMEM;
    }
    RT_HIP(c, e);
  }
  return RT_OK;
}
// frame f of array `kind` <-> the one-frame reference-layout array
rt::GbufXfer xfer_desc(const rt_ctx* c, int kind, int to_ref, int f) {
  rt::GbufXfer x{};
  x.W = c->cfg.width;
  x.R = c->own_rows;
  x.r0 = c->own0 - c->band0;
  x.F = 1;
  x.kind = kind;
  x.to_ref = to_ref;
  x.n = slot_elems(c);
  x.ref = c->d_xfer;
  const std::vector<float4*>& bufs = kind == kPixels ? c->pix : kind == kNormals ? c->nrm : c->dep;
  const std::vector<int>& map = kind == kPixels ? c->pix_slot : kind == kNormals ? c->nrm_slot : c->dep_slot;
  x.slot[0] = bufs[map[f]];
  return x;
}

}  // namespace

extern "C" {

int rt_version(void) { return RT_ABI_VERSION; }

const char* rt_strerror(int s) {
  switch (s) {
    case RT_OK: return "ok";
    case RT_E_INVAL: return "invalid argument";
    case RT_E_NOMEM: return "out of memory";
    case RT_E_HIP: return "HIP runtime error";
    case RT_E_NODEV: return "no HIP device";
    case RT_E_STATE: return "bad call order";
    default: return "unknown status";
  }
}

int rt_create(int device, const rt_config* cfg, rt_ctx** out) {
  if (!cfg || !out) return RT_E_INVAL;
  *out = nullptr;
  rt_config c = *cfg;
  if (c.num_frames == 0) c.num_frames = RT_NUM_FRAMES;
  if (c.max_depth == 0) c.max_depth = RT_RECURSION_DEPTH;
  if (c.row_begin == 0 && c.row_end == 0) c.row_end = c.height;
  if (c.width <= 0 || c.height <= 0 || c.num_shapes < 0 || c.num_shapes > kMaxShapes || c.spp <= 0 ||
      c.spp > kMaxSpp || c.num_frames <= 0 || c.num_frames > rt::kMaxFrames || c.max_depth <= 0 || c.max_depth > kMaxDepth ||
      c.row_begin < 0 || c.row_end > c.height || c.row_begin >= c.row_end)
    return RT_E_INVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_E_NODEV;
  if (device < 0 || device >= ndev) return RT_E_NODEV;
  rt_ctx* x = new (std::nothrow) rt_ctx();
  if (!x) return RT_E_NOMEM;
  x->device = device;
  x->cfg = c;
  x->own0 = c.row_begin;
  x->own_rows = c.row_end - c.row_begin;
  x->band0 = std::max(0, c.row_begin - 1);
  x->band_rows = std::min(c.height, c.row_end + 1) - x->band0;
  int rc = RT_OK;
  auto fail = [&](hipError_t e) {
    x->last_hip = (int)e;
    rc = (e == hipErrorOutOfMemory) ? RT_E_NOMEM : RT_E_HIP;
  };
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&x->own_stream, hipStreamNonBlocking);
  x->stream = x->own_stream;
  const size_t slot = slot_elems(x) * sizeof(float4);
  const int F = c.num_frames;
  if (e == hipSuccess) {
    const int NB = F + x->pipe_depth;
    x->pix.assign(NB, nullptr);
    x->nrm.assign(NB, nullptr);
    x->dep.assign(NB, nullptr);
    for (int k = 0; k < NB && e == hipSuccess; ++k) e = hipMalloc(&x->pix[k], slot);
    for (int k = 0; k < NB && e == hipSuccess; ++k) e = hipMalloc(&x->nrm[k], slot);
    for (int k = 0; k < NB && e == hipSuccess; ++k) e = hipMalloc(&x->dep[k], slot);
    // value-initialised ssbo_CPUMEM: the ring starts at zero
    for (int k = 0; k < NB && e == hipSuccess; ++k) e = hipMemsetAsync(x->pix[k], 0, slot, x->stream);
    for (int k = 0; k < NB && e == hipSuccess; ++k) e = hipMemsetAsync(x->nrm[k], 0, slot, x->stream);
    for (int k = 0; k < NB && e == hipSuccess; ++k) e = hipMemsetAsync(x->dep[k], 0, slot, x->stream);
    for (hipEvent_t* ev : {&x->ev_ao, &x->ev_join, &x->ev_seq})
      if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    for (auto& ev : x->ev_post)
      if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  }
  if (e == hipSuccess) e = hipMalloc(&x->d_image_own, (size_t)x->own_rows * c.width * sizeof(float4));
  if (e == hipSuccess) e = hipMemsetAsync(x->d_image_own, 0, (size_t)x->own_rows * c.width * sizeof(float4), x->stream);
  const int Sc = table_stride(x);
  for (int k = 0; k < kAoStreams; ++k) {
    if (e == hipSuccess) e = hipMalloc(&x->d_shapes_buf[k], rt::table_vec4(Sc, c.spp) * sizeof(float4));
    if (e == hipSuccess) x->d_rb_buf[k] = x->d_shapes_buf[k] + rt::rand_table(Sc);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(x->stream);
  if (e != hipSuccess) {
    fail(e);
    free_all(x);
    delete x;
    return rc;
  }
  x->d_image = x->d_image_own;
  x->pix_slot.resize(F);
  x->nrm_slot.resize(F);
  x->dep_slot.resize(F);
  for (int k = 0; k < F; ++k) x->pix_slot[k] = x->nrm_slot[k] = x->dep_slot[k] = k;
  x->spare = F;
  for (int q = 0; q < x->pipe_depth; ++q) {
    x->raw_buf[q] = F + q;  // raw buffer 0 is whichever buffer is the sequential spare
    x->nrm_free[q] = x->dep_free[q] = F + q;
  }
  x->d_shapes = x->d_shapes_buf[0];
  x->d_rb = x->d_rb_buf[0];
  x->out_stream = x->own_stream;
  x->header.assign(rt_header_bytes(c.num_shapes, c.spp) / 4, 0.0f);
  x->table.assign(rt::table_vec4(Sc, c.spp), make_float4(0, 0, 0, 0));
  *out = x;
  return RT_OK;
}

int rt_destroy(rt_ctx* c) {
  if (!c) return RT_E_INVAL;
  (void)hipSetDevice(c->device);
  (void)sync_all(c);
  free_all(c);
  delete c;
  return RT_OK;
}

int rt_set_stream(rt_ctx* c, void* s) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int rc = sync_all(c);
  if (rc != RT_OK) return rc;
  c->out_pending = false;
  for (auto& r : c->post_recorded) r = false;
  c->pipe_n = 0;
  c->img_stream = nullptr;  // everything is finished (sync_all above)
  for (auto& h : c->sched)  // no launch reads an order table any more: forget the old streams
    for (auto& u : h.used_on)
      for (auto& st : u) st = nullptr;
  c->stream = (hipStream_t)s;  // NULL = the legacy NULL stream
  if (!c->pipelined) c->out_stream = c->stream;
  // an idle own stream is released: every stream holds one of the process's few hardware
  // queues (GPU_MAX_HW_QUEUES), and busy streams that share one serialise
  if (c->own_stream && c->stream != c->own_stream && c->out_stream != c->own_stream) {
    RT_HIP(c, hipStreamDestroy(c->own_stream));
    c->own_stream = nullptr;
  }
  return RT_OK;
}

int rt_use_own_stream(rt_ctx* c) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  if (!c->own_stream) RT_HIP(c, hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
  return rt_set_stream(c, (void*)c->own_stream);
}

int rt_enable_pipelining(rt_ctx* c, int on, void* output_stream) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int rc = sync_all(c);
  if (rc != RT_OK) return rc;
  c->out_pending = false;
  for (auto& r : c->post_recorded) r = false;
  c->pipe_n = 0;
  c->img_stream = nullptr;
  c->pipelined = on != 0;
  if (!c->pipelined) {
    c->out_stream = c->stream;
    return RT_OK;
  }
  if (c->d_shapes && c->d_shapes != c->d_shapes_buf[0]) {
    // the current table sits in an rt_compute_frames slot: pipelined frames read header copy k
    RT_HIP(c, hipMemcpyAsync(c->d_shapes_buf[0], c->d_shapes, c->table.size() * sizeof(float4),
                             hipMemcpyDeviceToDevice, c->stream));
    c->d_shapes = c->d_shapes_buf[0];
    c->d_rb = c->d_rb_buf[0];
  }
  for (int k = 1; k < c->n_ao_streams; ++k)
    if (!c->ao_streams[k]) RT_HIP(c, hipStreamCreateWithFlags(&c->ao_streams[k], hipStreamNonBlocking));
  if (output_stream) {
    c->out_stream = (hipStream_t)output_stream;
  } else {
    if (!c->own_out_stream) RT_HIP(c, hipStreamCreateWithFlags(&c->own_out_stream, hipStreamNonBlocking));
    c->out_stream = c->own_out_stream;
  }
  if (c->out_stream == c->stream) c->pipelined = false;  // one stream: nothing to overlap
  return RT_OK;
}

void* rt_get_output_stream(rt_ctx* c) { return c ? (void*)c->out_stream : nullptr; }

void* rt_get_stream(rt_ctx* c) { return c ? (void*)c->stream : nullptr; }

void* rt_image_stream(rt_ctx* c) {
  if (!c) return nullptr;
  return (void*)(c->img_stream ? c->img_stream : c->stream);
}

int rt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int rt_synchronize(rt_ctx* c) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  return sync_all(c);
}

int rt_last_hip_error(rt_ctx* c) { return c ? c->last_hip : 0; }

int rt_debug_fail_next_event_query(rt_ctx* c, int hip_error) {
  if (!c || hip_error == (int)hipSuccess) return RT_E_INVAL;
  c->inject_query_error = hip_error;
  return RT_OK;
}

}  // extern "C"

namespace {

// Bounce-ray clusters of the AO kernel's later bounce rounds (rt_kernels_impl.h cluster_may_hit):
// the spheres among [0, nobj) are cut into spatial groups of at most max(kClusterSize, ceil(sqrt(nobj)))
// by recursive median splits of their centres along the widest axis (a round tests ~N/s balls and
// the members of the few it keeps: config (e), 256 spheres, AO 120.0 -> 116.0 ms per launch with
// groups of 16 instead of 8, 117.8 with 32; config (d), 64 spheres, 2.371 -> 2.395 ms with 16, so
// 8 there, profiles/r06s_*); each cluster is stored as (centre, R)
// with every member inside the ball: |c_i - centre| + |r_i| <= R (computed in double and
// rounded up).  Spheres that would inflate a cluster (radius above 8x the median, e.g. a ground
// sphere) and spheres with non-finite geometry are tested in every round instead (the always
// mask).  Non-spheres (NaN in the sphere table) are never accepted and are left out entirely.
// Returns the cluster count, 0 = off (small scenes, more than 256 objects, nothing to cluster).
constexpr int kClusterSize = 8;
constexpr int kClusterMinObj = 16;
int build_clusters(const float4* sph, int nobj, float4* ctab, unsigned long long* cmask) {
  std::memset(cmask, 0, sizeof(unsigned long long) * (1 + rt::kMaxClusters) * rt::kClusterWords);
  if (nobj < kClusterMinObj || nobj > 64 * rt::kClusterWords) return 0;
  std::vector<int> small;
  std::vector<float> radii;
  for (int i = 0; i < nobj; ++i) {
    const float4 g = sph[i];
    if (g.x != g.x) continue;  // not a sphere (NaN row): never accepted
    if (std::isfinite(g.x) && std::isfinite(g.y) && std::isfinite(g.z) && std::isfinite(g.w)) radii.push_back(std::fabs(g.w));
  }
  if (radii.size() < (size_t)kClusterSize) return 0;
  const int csize = std::max(kClusterSize, (int)std::ceil(std::sqrt((double)nobj)));
  std::nth_element(radii.begin(), radii.begin() + radii.size() / 2, radii.end());
  const double big = 8.0 * radii[radii.size() / 2];
  for (int i = 0; i < nobj; ++i) {
    const float4 g = sph[i];
    if (g.x != g.x) continue;
    const bool fin = std::isfinite(g.x) && std::isfinite(g.y) && std::isfinite(g.z) && std::isfinite(g.w);
    if (fin && std::fabs(g.w) <= big) small.push_back(i);
    else cmask[i >> 6] |= 1ull << (i & 63);  // always tested
  }
  // recursive median split into groups of <= csize
  std::vector<std::pair<int, int>> groups, work{{0, (int)small.size()}};
  while (!work.empty()) {
    auto [a, b] = work.back();
    work.pop_back();
    if (b - a <= csize) {
      groups.push_back({a, b});
      continue;
    }
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (int k = a; k < b; ++k) {
      const float4 g = sph[small[k]];
      const double v[3] = {g.x, g.y, g.z};
      for (int d = 0; d < 3; ++d) lo[d] = std::min(lo[d], v[d]), hi[d] = std::max(hi[d], v[d]);
    }
    int ax = 0;
    for (int d = 1; d < 3; ++d)
      if (hi[d] - lo[d] > hi[ax] - lo[ax]) ax = d;
    const int mid = (a + b) / 2;
    auto key = [&](int i) { const float4 g = sph[i]; return ax == 0 ? g.x : ax == 1 ? g.y : g.z; };
    std::nth_element(small.begin() + a, small.begin() + mid, small.begin() + b,
                     [&](int i, int j) { return key(i) < key(j) || (key(i) == key(j) && i < j); });
    work.push_back({mid, b});
    work.push_back({a, mid});
  }
  if ((int)groups.size() > rt::kMaxClusters) {  // too many groups: test everything every round
    std::memset(cmask, 0, sizeof(unsigned long long) * rt::kClusterWords);
    return 0;
  }
  int k = 0;
  for (auto [a, b] : groups) {
    double cx = 0, cy = 0, cz = 0;
    for (int q = a; q < b; ++q) cx += sph[small[q]].x, cy += sph[small[q]].y, cz += sph[small[q]].z;
    const float fx = (float)(cx / (b - a)), fy = (float)(cy / (b - a)), fz = (float)(cz / (b - a));
    double R = 0.0;
    for (int q = a; q < b; ++q) {
      const float4 g = sph[small[q]];
      const double dx = (double)g.x - fx, dy = (double)g.y - fy, dz = (double)g.z - fz;
      R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + std::fabs((double)g.w));
      cmask[(size_t)(1 + k) * rt::kClusterWords + (small[q] >> 6)] |= 1ull << (small[q] & 63);
    }
    ctab[k] = make_float4(fx, fy, fz, std::nextafter((float)(R * (1.0 + 1e-6)), INFINITY));
    ++k;
  }
  return k;
}

// Validate a header and pack it into the device table layout (rt::table_vec4 float4 at `tab`:
// shape tables, sphere table, plane table, clusters, rand_buffer); sets nobj / nplanes / ncl.
int pack_header(rt_ctx* c, const float* h, float4* tab, int& nobj, int& nplanes, int& ncl) {
  const int S = c->cfg.num_shapes, spp = c->cfg.spp;
  const float mz = h[RT_HDR_MODE * 4 + 2];
  if (!(mz >= 0.0f && mz < (float)(S + 1))) return RT_E_INVAL;  // int(mode.z) must be in [0, S]
  nobj = (int)mz;
  const float* sh = h + rt_off_shapes() / 4;
  const int Sc = table_stride(c);
  const float qnan = std::numeric_limits<float>::quiet_NaN();
  float4* sph = tab + rt::sphere_table(Sc);
  float4* pln = tab + rt::plane_table(Sc);
  int np = 0;
  for (int i = 0; i < S; ++i) {
    const float* s = sh + (size_t)i * 20;
    float idf = s[16 + 3];
    int id = (idf > -2147483648.0f && idf < 2147483648.0f) ? (int)idf : 0;  // int(simple_shapes[i][4].w)
    tab[i] = make_float4(s[0], s[1], s[2], s[3]);
    float4 g2 = make_float4(s[12], s[13], s[14], 0.0f);
    std::memcpy(&g2.w, &id, 4);
    tab[(size_t)Sc + i] = g2;
    tab[(size_t)2 * Sc + i] = make_float4(s[16], s[17], s[18], s[19]);
    tab[(size_t)3 * Sc + i] = make_float4(s[4 + 3], s[12 + 3], 0.0f, 0.0f);
    // sphere table: the spheres' geometry; every other shape NaN (a NaN discriminant is never
    // accepted: eval_ray's -1 for shapes it does not intersect, p_compute.glsl:121-138)
    sph[i] = id == RT_SHAPE_SPHERE ? tab[i] : make_float4(qnan, qnan, qnan, qnan);
    if (i < nobj && id == RT_SHAPE_PLANE) {  // plane table: (normal, bits(index)), (p0, 0)
      float4 a = make_float4(s[0], s[1], s[2], 0.0f);
      std::memcpy(&a.w, &i, 4);
      pln[2 * np] = a;
      pln[2 * np + 1] = make_float4(s[12], s[13], s[14], 0.0f);
      ++np;
    }
  }
  // the padding rows; the colour table's row -1 is the background (table_stride)
  for (int k = 0; k < 4; ++k) tab[(size_t)k * Sc + Sc - 1] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  tab[4 * (size_t)Sc + Sc - 1] = make_float4(qnan, qnan, qnan, qnan);  // sphere table: never accepted
  {
    const float* bg = h + RT_HDR_BACKGROUND * 4;
    tab[(size_t)2 * Sc - 1] = make_float4(bg[0], bg[1], bg[2], bg[3]);
  }
  std::memcpy(tab + rt::rand_table(Sc), h + rt_off_rand(S) / 4, (size_t)2 * spp * sizeof(float4));
  {  // camera-relative sphere rows: pmc = camera - centre, pp = dot(pmc, pmc) as the kernels'
    // sphere_candidate forms them (binary32, fmaf; this file is built with -ffp-contract=off)
    const float* cam = h + RT_HDR_CAMERA_LOCATION * 4;
    float4* crel = tab + rt::camrel_table(Sc);
    for (int i = 0; i < Sc; ++i) {
      const float4 g = sph[i];
      const float px = cam[0] - g.x, py = cam[1] - g.y, pz = cam[2] - g.z;
      crel[i] = make_float4(px, py, pz, std::fmaf(pz, pz, std::fmaf(py, py, px * px)));
    }
  }
  nplanes = np;
  ncl = build_clusters(sph, nobj, tab + rt::cluster_table(Sc), (unsigned long long*)(tab + rt::cluster_mask_table(Sc)));
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_upload_header(rt_ctx* c, const void* header, size_t bytes) {
  if (!c || !header) return RT_E_INVAL;
  const int S = c->cfg.num_shapes, spp = c->cfg.spp;
  if (bytes != rt_header_bytes(S, spp)) return RT_E_INVAL;
  const float* h = (const float*)header;
  int nobj = 0, np = 0, ncl = 0;
  {
    const float mz = h[RT_HDR_MODE * 4 + 2];
    if (!(mz >= 0.0f && mz < (float)(S + 1))) return RT_E_INVAL;
  }
  std::memcpy(c->header.data(), header, bytes);
  int rc = pack_header(c, h, c->table.data(), nobj, np, ncl);
  if (rc != RT_OK) return rc;
  RT_HIP(c, hipSetDevice(c->device));
  // pipelined: into the header copy of the next frame, on its AO stream (ordered after the AO
  // pass two frames back that read that copy); sequential: in place, on the main stream
  const int hc = hdr_copy(c);
  if (c->pipelined && c->pipe_n == 0) {  // the first frame of a sequence: order after everything
    int sr = start_sequence(c);
    if (sr != RT_OK) return sr;
  }
  // table + rand_buffer in one upload (per-frame host cost matters for small strips/frames)
  rc = staged_copy(c, c->d_shapes_buf[hc], c->table.data(), c->table.size() * sizeof(float4), ao_stream(c));
  if (rc != RT_OK) return rc;
  c->d_shapes = c->d_shapes_buf[hc];
  c->d_rb = c->d_rb_buf[hc];
  c->nobj = nobj;
  c->nplanes = np;
  c->ncl = ncl;
  c->have_header = true;
  return RT_OK;
}

int rt_upload_rand_buffer(rt_ctx* c, const float* rb, size_t n_vec4) {
  if (!c || !rb || n_vec4 != (size_t)2 * c->cfg.spp) return RT_E_INVAL;
  std::memcpy(c->header.data() + rt_off_rand(c->cfg.num_shapes) / 4, rb, n_vec4 * 16);
  std::memcpy(c->table.data() + rt::rand_table(table_stride(c)), rb, n_vec4 * 16);
  RT_HIP(c, hipSetDevice(c->device));
  const int hc = hdr_copy(c);
  int rc = staged_copy(c, c->d_rb_buf[hc], rb, n_vec4 * 16, ao_stream(c));
  if (rc != RT_OK) return rc;
  // the other copy keeps the shape table: bring it along when switching copies
  if (c->d_shapes != c->d_shapes_buf[hc])
    RT_HIP(c, hipMemcpyAsync(c->d_shapes_buf[hc], c->d_shapes, rt::rand_table(table_stride(c)) * sizeof(float4),
                             hipMemcpyDeviceToDevice, ao_stream(c)));
  c->d_shapes = c->d_shapes_buf[hc];
  c->d_rb = c->d_rb_buf[hc];
  return RT_OK;
}

int rt_run_program(rt_ctx* c, int program, int frame) {
  if (!c) return RT_E_INVAL;
  return run_program(c, program, frame);
}

int rt_dispatch(rt_ctx* c, int mode, int frame) {
  if (!c) return RT_E_INVAL;
  int rc;
  switch (mode) {
    case RT_MODE_AO_PP:
      if (c->pipelined) {
        rc = pipelined_frame(c, frame);
        break;
      }
      rc = run_program(c, RT_PROG_AOP_COMPUTE, frame);
      if (rc == RT_OK) rc = run_program(c, RT_PROG_AOP_POSTPROCESSING, frame);
      break;
    case RT_MODE_AO: rc = run_program(c, RT_PROG_AO_COMPUTE, frame); break;
    case RT_MODE_PHONG: rc = run_program(c, RT_PROG_P_COMPUTE, frame); break;
    case RT_MODE_PHONG_REFL: rc = run_program(c, RT_PROG_H_COMPUTE, frame); break;
    default: return RT_E_INVAL;
  }
  if (rc != RT_OK) return rc;
  return (frame + 1) % c->cfg.num_frames;
}

int rt_compute_frames(rt_ctx* c, float* header, int mode, int frame, int n, uint64_t rand_seed, int light_movement) {
  if (!c || !header || n < 0 || mode < RT_MODE_AO_PP || mode > RT_MODE_PHONG_REFL) return RT_E_INVAL;
  if (frame < 0 || frame >= c->cfg.num_frames) return RT_E_INVAL;
  const int S = c->cfg.num_shapes, spp = c->cfg.spp;
  const size_t bytes = rt_header_bytes(S, spp);
  // the render loop's host update of frame k (src/main.cpp:553-578), then set_mode
  auto update = [&](int k, int slot) -> int {
    int rc = (mode == RT_MODE_AO_PP || mode == RT_MODE_AO) ? rt_fill_rand_buffer(header, S, spp, rand_seed + (uint64_t)k)
                                                           : rt_moving_light(header, light_movement);
    if (rc != RT_OK) return rc;
    const float mz = header[RT_HDR_MODE * 4 + 2];
    if (!(mz >= 0.0f && mz < (float)(S + 1))) return RT_E_INVAL;
    return rt_set_mode(header, slot, (int)mz);
  };
  if ((mode == RT_MODE_PHONG || mode == RT_MODE_PHONG_REFL) && n >= 2 && c->mf_max > 1) {
    // Modes 3/4: the per-frame host update moves only the light (and mode.y), so the shape
    // table is uploaded once and up to kMaxBatch frames go in one multi-frame launch with their
    // lights (run_program_mf).  Every frame writes its own colour slot, as frame-by-frame calls
    // do; the image is written once per launch, by its last frame (the one the caller sees).
    std::vector<float4> lights(n);
    std::vector<int> slots(n);
    int f = frame;
    for (int k = 0; k < n; ++k) {
      int rc = update(k, f);
      if (rc == RT_OK && k == 0) rc = rt_upload_header(c, header, bytes);
      if (rc != RT_OK) return rc;
      const float* L = header + 4 * RT_HDR_LIGHT_POS;
      lights[k] = make_float4(L[0], L[1], L[2], L[3]);
      slots[k] = f;
      f = (f + 1) % c->cfg.num_frames;
    }
    std::memcpy(c->header.data(), header, bytes);  // as the per-frame calls leave it
    const int prog = mode == RT_MODE_PHONG ? RT_PROG_P_COMPUTE : RT_PROG_H_COMPUTE;
    // at most F frames per launch: each colour slot is written by one frame of a launch (frames
    // k and k + F of one launch would race for slot k % F)
    const int mb = std::min(std::min(rt::kMaxBatch, c->mf_max), c->cfg.num_frames);
    for (int k0 = 0; k0 < n; k0 += mb) {
      const int m = std::min(mb, n - k0);
      int rc = run_program_mf(c, prog, slots[k0], m, lights.data() + k0);
      if (rc != RT_OK) return rc;
    }
    return f;
  }
  if (mode == RT_MODE_AO && n >= 2 && !c->counting && !c->row_counting && c->mf_max > 1) {
    // Mode 2: the per-frame host update replaces only rand_buffer (fill_rand_buffer,
    // src/main.cpp:535-539) and mode.y, so the shape table is uploaded once and up to F frames
    // go in one launch, each with its own rand_buffer (run_program_mf).
    const int nrb = 2 * spp;
    std::vector<float4> rbs((size_t)n * nrb);
    std::vector<int> slots(n);
    int f = frame;
    for (int k = 0; k < n; ++k) {
      int rc = update(k, f);
      if (rc == RT_OK && k == 0) rc = rt_upload_header(c, header, bytes);
      if (rc != RT_OK) return rc;
      std::memcpy(&rbs[(size_t)k * nrb], header + rt_off_rand(S) / 4, (size_t)nrb * sizeof(float4));
      slots[k] = f;
      f = (f + 1) % c->cfg.num_frames;
    }
    RT_HIP(c, hipSetDevice(c->device));
    if (!c->d_mf_rb) RT_HIP(c, hipMalloc(&c->d_mf_rb, (size_t)rt::kMaxBatch * nrb * sizeof(float4)));
    const int mb = std::min(std::min(rt::kMaxBatch, c->mf_max), c->cfg.num_frames);
    for (int k0 = 0; k0 < n; k0 += mb) {
      const int m = std::min(mb, n - k0);
      int rc = staged_copy(c, c->d_mf_rb, &rbs[(size_t)k0 * nrb], (size_t)m * nrb * sizeof(float4), c->stream);
      if (rc == RT_OK) rc = run_program_mf(c, RT_PROG_AO_COMPUTE, slots[k0], m, nullptr);
      if (rc != RT_OK) return rc;
    }
    // leave the context as the per-frame calls would: the last header uploaded
    int rc = rt_upload_header(c, header, bytes);
    if (rc != RT_OK) return rc;
    return f;
  }
  if (c->pipelined || n < 2) {  // pipelined mode 1 rotates its own header copies per frame
    for (int k = 0; k < n; ++k) {
      int rc = update(k, frame);
      if (rc == RT_OK) rc = rt_upload_header(c, header, bytes);
      if (rc != RT_OK) return rc;
      frame = rt_dispatch(c, mode, frame);
      if (frame < 0) return frame;
    }
    return frame;
  }
  // Sequential frames in batches: the host updates of up to kBatch frames are packed into
  // device table copies with ONE upload, then the frames' programs are launched back to back,
  // each reading its own copy.  Per frame the host then only enqueues kernels, which keeps small
  // frames (config (a): a ~9 us kernel) GPU-bound.  Only DISTINCT tables are uploaded: modes 3/4
  // move the light, which travels in the kernel arguments, so their packed table never changes
  // and, after the first call, nothing is copied at all (an in-stream host-to-device copy
  // between two kernels stalls the queue for the copy's round trip: ~40 us every 8 frames of
  // config (b), 5 us per frame).  The last table stays where it is (d_batch slot batch_last)
  // as the context's current table.
  constexpr int kBatch = 32;
  const size_t tv = c->table.size();
  RT_HIP(c, hipSetDevice(c->device));
  int jr = join(c);
  if (jr != RT_OK) return jr;
  if (!c->d_batch) RT_HIP(c, hipMalloc(&c->d_batch, (size_t)2 * kBatch * tv * sizeof(float4)));
  c->batch_host.resize((size_t)kBatch * tv);
  c->batch_hdr.resize((size_t)kBatch * (bytes / sizeof(float)));
  const int Sc = table_stride(c);
  const size_t hf = bytes / sizeof(float);
  const size_t tb = tv * sizeof(float4);
  for (int k0 = 0; k0 < n; k0 += kBatch) {
    const int m = std::min(kBatch, n - k0);
    std::vector<int> nobj(m), npl(m), ncl(m), slot(m), dslot(m);
    // the context's current table, if it already sits in a d_batch slot (host copy: c->table)
    const int prev = (c->batch_last >= 0 && c->d_shapes == c->d_batch + (size_t)c->batch_last * tv) ? c->batch_last : -1;
    int nd = 0;                  // distinct new tables, packed into batch_host[0 .. nd)
    const float4* last = prev >= 0 ? c->table.data() : nullptr;  // the previous frame's table
    int f = frame;
    for (int j = 0; j < m; ++j) {
      float4* tab = c->batch_host.data() + (size_t)nd * tv;
      int rc = update(k0 + j, f);
      if (rc == RT_OK) rc = pack_header(c, header, tab, nobj[j], npl[j], ncl[j]);
      if (rc != RT_OK) return rc;
      std::memcpy(c->batch_hdr.data() + (size_t)j * hf, header, bytes);  // camera / light of frame j
      slot[j] = f;
      f = (f + 1) % c->cfg.num_frames;
      if (last && std::memcmp(tab, last, tb) == 0) {
        dslot[j] = j == 0 ? -1 : dslot[j - 1];  // -1: the previous slot `prev`
      } else {
        dslot[j] = -2 - nd;  // new table nd (its slot is fixed below)
        last = tab;
        ++nd;
      }
    }
    // new tables go to slots base .. base + nd - 1, never over `prev` if frame 0 reads it
    const bool keep_prev = dslot[0] == -1;
    const int base = keep_prev && prev + 1 + nd <= 2 * kBatch ? prev + 1 : 0;
    for (int j = 0; j < m; ++j) dslot[j] = dslot[j] == -1 ? prev : base + (-2 - dslot[j]);
    if (nd > 0) {
      int rc = staged_copy(c, c->d_batch + (size_t)base * tv, c->batch_host.data(), (size_t)nd * tb, c->stream);
      if (rc != RT_OK) return rc;
    }
    // the context's table from here on: the last frame's (host copy first: `last` may point
    // into batch_host, which the next batch reuses)
    if (last != c->table.data()) std::memcpy(c->table.data(), last, tb);
    for (int j = 0; j < m; ++j) {
      c->d_shapes = c->d_batch + (size_t)dslot[j] * tv;
      c->d_rb = c->d_shapes + rt::rand_table(Sc);
      c->nobj = nobj[j];
      c->nplanes = npl[j];
      c->ncl = ncl[j];
      c->have_header = true;
      std::memcpy(c->header.data(), c->batch_hdr.data() + (size_t)j * hf, bytes);  // launch parameters
      frame = rt_dispatch(c, mode, slot[j]);
      if (frame < 0) return frame;
    }
    c->batch_last = dslot[m - 1];
  }
  // the context is left as the per-frame calls would leave it: the last header, its table current
  std::memcpy(c->header.data(), header, bytes);
  return frame;
}

int rt_set_tile_schedule(rt_ctx* c, int on) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  RT_HIP(c, hipStreamSynchronize(c->stream));  // no launch in flight reads the tables freed here
  for (auto& h : c->sched) free_sched(h);
  c->sched_on = on != 0;
  return RT_OK;
}

int rt_tile_schedule_state(rt_ctx* c) {
  if (!c) return RT_E_INVAL;
  if (!c->sched_on) return 0;
  for (auto& h : c->sched)
    if (h.active >= 0) return 2;
  return 1;
}

int rt_tile_schedule_orders(rt_ctx* c) {
  if (!c) return RT_E_INVAL;
  int n = 0;
  for (auto& h : c->sched) n += h.orders_taken;
  return n;
}

int rt_set_frame_batch(rt_ctx* c, int max_frames) {
  if (!c || max_frames < 1) return RT_E_INVAL;
  c->mf_max = std::min(max_frames, rt::kMaxBatch);
  return RT_OK;
}

int rt_download(rt_ctx* c, float* pixels, float* normals, float* depth, float* image) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int rc = join(c);
  if (rc == RT_OK) rc = sync_all(c);
  if (rc == RT_OK && (pixels || normals || depth)) rc = xfer_buffer(c);
  if (rc != RT_OK) return rc;
  const size_t fbytes = (size_t)c->cfg.width * c->own_rows * sizeof(float4);  // one frame
  float* dst[3] = {pixels, normals, depth};
  for (int k = 0; k < 3; ++k) {
    if (!dst[k]) continue;
    for (int f = 0; f < c->cfg.num_frames; ++f) {  // stream order: frame f's copy precedes f+1's convert
      RT_HIP(c, rt::launch_gbuf_convert(xfer_desc(c, k, 1, f), c->stream));
      RT_HIP(c, hipMemcpyAsync((char*)dst[k] + (size_t)f * fbytes, c->d_xfer, fbytes, hipMemcpyDeviceToHost,
                               c->stream));
    }
  }
  if (image)
    RT_HIP(c, hipMemcpyAsync(image, c->d_image, (size_t)c->own_rows * c->cfg.width * 16, hipMemcpyDeviceToHost,
                             c->stream));
  RT_HIP(c, hipStreamSynchronize(c->stream));
  return RT_OK;
}

int rt_download_rect(rt_ctx* c, int x0, int x1, int y0, int y1, float* pixels, float* normals, float* depth,
                     float* image) {
  if (!c) return RT_E_INVAL;
  const int W = c->cfg.width;
  if (x0 < 0 || x1 > W || x0 >= x1 || y0 < c->own0 || y1 > c->own0 + c->own_rows || y0 >= y1) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int rc = join(c);
  if (rc == RT_OK) rc = sync_all(c);
  if (rc != RT_OK) return rc;
  const int w = x1 - x0, h = y1 - y0, F = c->cfg.num_frames;
  const size_t pitch = (size_t)W * sizeof(float4), row = (size_t)w * sizeof(float4);
  std::vector<float4> tmp((size_t)w * h);
  auto rect = [&](const float4* base, int r0) {  // rows [r0, r0 + h) of a [rows][W] device array
    return hipMemcpy2D(tmp.data(), row, base + (size_t)r0 * W + x0, pitch, row, h, hipMemcpyDeviceToHost);
  };
  // a plane-split slot's rect: plane a (ea floats per pixel) then plane b (4 - ea floats per
  // pixel, starting ea * n floats into the slot), interleaved into tmp
  const size_t n = slot_elems(c);
  std::vector<float> ta((size_t)w * h * 3), tb((size_t)w * h * 3);
  auto split_rect = [&](const float4* base, int r0, int ea) -> hipError_t {
    const int eb = 4 - ea;
    const float* pa = (const float*)base + ((size_t)r0 * W + x0) * ea;
    const float* pb = (const float*)base + ea * n + ((size_t)r0 * W + x0) * eb;
    hipError_t e = hipMemcpy2D(ta.data(), (size_t)w * ea * 4, pa, (size_t)W * ea * 4, (size_t)w * ea * 4, h,
                               hipMemcpyDeviceToHost);
    if (e == hipSuccess)
      e = hipMemcpy2D(tb.data(), (size_t)w * eb * 4, pb, (size_t)W * eb * 4, (size_t)w * eb * 4, h,
                      hipMemcpyDeviceToHost);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
      float* o = (float*)&tmp[i];
      for (int q = 0; q < ea; ++q) o[q] = ta[i * ea + q];
      for (int q = 0; q < eb; ++q) o[ea + q] = tb[i * eb + q];
    }
    return e;
  };
  for (int f = 0; f < F; ++f) {
    struct { float* dst; const float4* src; } items[3] = {
        {pixels, c->pix[c->pix_slot[f]]}, {normals, c->nrm[c->nrm_slot[f]]}, {depth, c->dep[c->dep_slot[f]]}};
    for (int k = 0; k < 3; ++k) {
      auto& it = items[k];
      if (!it.dst) continue;
      RT_HIP(c, (k == kPixels || (k == kNormals && !RT_NRM_PLANES)) ? rect(it.src, y0 - c->band0)
                                                                   : split_rect(it.src, y0 - c->band0, k == kNormals ? 3 : 2));
      float* out = it.dst + (size_t)f * w * h * 4;  // [w][h] vec4, y fastest (reference layout)
      for (int x = 0; x < w; ++x)
        for (int r = 0; r < h; ++r) std::memcpy(out + ((size_t)x * h + r) * 4, &tmp[(size_t)r * w + x], 16);
    }
  }
  if (image) {
    RT_HIP(c, rect(c->d_image, y0 - c->own0));
    std::memcpy(image, tmp.data(), tmp.size() * sizeof(float4));
  }
  return RT_OK;
}

int rt_upload_gbuffer(rt_ctx* c, const float* pixels, const float* normals, const float* depth) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int rc = join(c);
  if (rc == RT_OK) rc = sync_all(c);
  if (rc == RT_OK && (pixels || normals || depth)) rc = xfer_buffer(c);
  if (rc != RT_OK) return rc;
  const size_t fbytes = (size_t)c->cfg.width * c->own_rows * sizeof(float4);  // one frame
  const float* src[3] = {pixels, normals, depth};
  for (int k = 0; k < 3; ++k) {  // (the halo rows of a strip keep their contents)
    if (!src[k]) continue;
    for (int f = 0; f < c->cfg.num_frames; ++f) {
      RT_HIP(c, hipMemcpyAsync(c->d_xfer, (const char*)src[k] + (size_t)f * fbytes, fbytes, hipMemcpyHostToDevice,
                               c->stream));
      RT_HIP(c, rt::launch_gbuf_convert(xfer_desc(c, k, 0, f), c->stream));
    }
  }
  RT_HIP(c, hipStreamSynchronize(c->stream));
  return RT_OK;
}

void* rt_image_device_ptr(rt_ctx* c) { return c ? (void*)c->d_image : nullptr; }

int rt_bind_image(rt_ctx* c, void* p) {
  if (!c) return RT_E_INVAL;
  c->d_image = p ? (float4*)p : c->d_image_own;
  return RT_OK;
}

// ---- host-buffer parity path -----------------------------------------------------------
static int hostbuf_in(rt_ctx* c, void* ssbo, int frame_num) {
  if (!c || !ssbo) return RT_E_INVAL;
  if (c->own0 != 0 || c->own_rows != c->cfg.height) return RT_E_STATE;  // whole-frame contexts only
  if (frame_num < 0 || frame_num >= c->cfg.num_frames) return RT_E_INVAL;
  float* f = (float*)ssbo;
  f[RT_HDR_MODE * 4 + 1] = (float)frame_num;  // ssbo_CPUMEM.mode.y = frame_num (main.cpp:584)
  const int S = c->cfg.num_shapes, A = c->cfg.spp, W = c->cfg.width, H = c->cfg.height, F = c->cfg.num_frames;
  int rc = rt_upload_header(c, ssbo, rt_header_bytes(S, A));
  if (rc != RT_OK) return rc;
  return rt_upload_gbuffer(c, f + rt_off_pixels(S, A) / 4, f + rt_off_normals(S, A, W, H, F) / 4,
                           f + rt_off_depth(S, A, W, H, F) / 4);
}

static int hostbuf_out(rt_ctx* c, void* ssbo, float* image) {
  float* f = (float*)ssbo;
  const int S = c->cfg.num_shapes, A = c->cfg.spp, W = c->cfg.width, H = c->cfg.height, F = c->cfg.num_frames;
  return rt_download(c, f + rt_off_pixels(S, A) / 4, f + rt_off_normals(S, A, W, H, F) / 4,
                     f + rt_off_depth(S, A, W, H, F) / 4, image);
}

int rt_compute_one_shader(rt_ctx* c, void* ssbo, int frame_num, int program, float* image) {
  int rc = hostbuf_in(c, ssbo, frame_num);
  if (rc != RT_OK) return rc;
  rc = run_program(c, program, frame_num);
  if (rc != RT_OK) return rc;
  rc = hostbuf_out(c, ssbo, image);
  if (rc != RT_OK) return rc;
  return (frame_num + 1) % c->cfg.num_frames;
}

int rt_compute_two_shaders(rt_ctx* c, void* ssbo, int frame_num, int p1, int p2, float* image) {
  int rc = hostbuf_in(c, ssbo, frame_num);
  if (rc != RT_OK) return rc;
  rc = run_program(c, p1, frame_num);
  if (rc == RT_OK) rc = run_program(c, p2, frame_num);
  if (rc != RT_OK) return rc;
  rc = hostbuf_out(c, ssbo, image);
  if (rc != RT_OK) return rc;
  return (frame_num + 1) % c->cfg.num_frames;
}

// ---- instrumentation ------------------------------------------------------------------
int rt_enable_timing(rt_ctx* c, int on) {
  if (!c) return RT_E_INVAL;
  c->timing = on != 0;
  return RT_OK;
}

int rt_kernel_stats(rt_ctx* c, int program, int* launches, double* total_ms) {
  if (!c || program <= 0 || program >= RT_PROG_COUNT) return RT_E_INVAL;
  int rc = resolve_timing(c);
  if (rc != RT_OK) return rc;
  if (launches) *launches = c->launches[program];
  if (total_ms) *total_ms = c->total_ms[program];
  return RT_OK;
}

int rt_host_stats(rt_ctx* c, double* wait_ms, long long* waits) {
  if (!c) return RT_E_INVAL;
  if (wait_ms) *wait_ms = c->host_wait_ms;
  if (waits) *waits = c->host_waits;
  return RT_OK;
}

int rt_reset_stats(rt_ctx* c) {
  if (!c) return RT_E_INVAL;
  int rc = resolve_timing(c);
  if (rc != RT_OK) return rc;
  c->host_wait_ms = 0.0;
  c->host_waits = 0;
  for (int k = 0; k < RT_PROG_COUNT; ++k) {
    c->total_ms[k] = 0.0;
    c->launches[k] = 0;
  }
  return RT_OK;
}

int rt_enable_counters(rt_ctx* c, int on) {
  if (!c) return RT_E_INVAL;
  RT_HIP(c, hipSetDevice(c->device));
  int jr = join(c);
  if (jr != RT_OK) return jr;
  if (on && !c->d_counters) {
    RT_HIP(c, hipMalloc(&c->d_counters, rt::kCounters * rt::kCounterSlots * sizeof(unsigned long long)));
    RT_HIP(c, hipMemsetAsync(c->d_counters, 0, rt::kCounters * rt::kCounterSlots * sizeof(unsigned long long),
                             c->stream));
    RT_HIP(c, hipMalloc(&c->d_row_counters, (size_t)c->band_rows * sizeof(unsigned long long)));
    RT_HIP(c, hipMemsetAsync(c->d_row_counters, 0, (size_t)c->band_rows * sizeof(unsigned long long), c->stream));
  }
  c->counting = (on & 1) != 0;
  c->row_counting = (on & 2) != 0;
  return RT_OK;
}

int rt_read_counters(rt_ctx* c, uint64_t out[8], int reset) {
  if (!c || !out) return RT_E_INVAL;
  if (!c->d_counters) {
    for (int k = 0; k < rt::kCounters; ++k) out[k] = 0;
    return RT_OK;
  }
  RT_HIP(c, hipSetDevice(c->device));
  std::vector<unsigned long long> h((size_t)rt::kCounters * rt::kCounterSlots);
  int rc = sync_all(c);
  if (rc != RT_OK) return rc;
  RT_HIP(c, hipMemcpy(h.data(), c->d_counters, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  for (int k = 0; k < rt::kCounters; ++k) {
    unsigned long long sum = 0;
    for (int j = 0; j < rt::kCounterSlots; ++j) sum += h[(size_t)k * rt::kCounterSlots + j];
    out[k] = (uint64_t)sum;
  }
  if (reset) RT_HIP(c, hipMemset(c->d_counters, 0, h.size() * sizeof(unsigned long long)));
  return RT_OK;
}

int rt_read_row_counters(rt_ctx* c, uint64_t* rows, int reset) {
  if (!c || !rows) return RT_E_INVAL;
  const int R = c->own_rows;
  if (!c->d_row_counters) {
    for (int k = 0; k < R; ++k) rows[k] = 0;
    return RT_OK;
  }
  RT_HIP(c, hipSetDevice(c->device));
  std::vector<unsigned long long> h(c->band_rows);
  int rc = sync_all(c);
  if (rc != RT_OK) return rc;
  RT_HIP(c, hipMemcpy(h.data(), c->d_row_counters, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  for (int k = 0; k < R; ++k) rows[k] = (uint64_t)h[(size_t)(c->own0 - c->band0) + k];
  if (reset) RT_HIP(c, hipMemset(c->d_row_counters, 0, h.size() * sizeof(unsigned long long)));
  return RT_OK;
}

int rt_selftest_math(rt_ctx* c, int fn, const float* in, float* out, size_t n) {
  if (!c || !in || !out || fn < 0 || fn > RT_MATH_SIN_TABLE) return RT_E_INVAL;
  static const int in_w[] = {1, 2, 1, 2, 3, 10, 0, 0, 0, 0, 4, 0}, out_w[] = {1, 1, 1, 1, 3, 1, 1, 1, 1, 1, 5, 2};
  RT_HIP(c, hipSetDevice(c->device));
  float *din = nullptr, *dout = nullptr;
  const bool sweep = fn == RT_MATH_SQRT_SWEEP || fn == RT_MATH_RCP_SWEEP || fn == RT_MATH_SQRT_TAIL_SWEEP ||
                     fn == RT_MATH_SIN_RANGE || fn == RT_MATH_SIN_TABLE;  // in: one float (the count or the first bit pattern)
  size_t ib = sweep ? sizeof(float) : n * in_w[fn] * sizeof(float);
  size_t ob = n * out_w[fn] * sizeof(float);
  RT_HIP(c, hipMalloc(&din, std::max<size_t>(ib, 4)));
  hipError_t e = hipMalloc(&dout, std::max<size_t>(ob, 4));
  if (e == hipSuccess) e = hipMemcpy(din, in, ib, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = rt::launch_selftest(fn, din, dout, n, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipMemcpy(out, dout, ob, hipMemcpyDeviceToHost);
  (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  if (e != hipSuccess) return hip_fail(c, e);
  return RT_OK;
}

}  // extern "C"
