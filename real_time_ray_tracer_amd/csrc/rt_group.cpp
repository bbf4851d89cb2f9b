// rt_group.cpp — multi-device row strips behind the C ABI (include/rt/abi.h, rt_group_*).
//
// The reference renders one frame on one GPU: compute() (src/main.cpp:553-578) dispatches
// glDispatchCompute(WIDTH, HEIGHT, 1) and the blit reads the whole image (783-797).  Every
// pixel is independent, so here one process drives n strip contexts (rt_ctx, one per row
// strip, each on its own device, or several on one device) and assembles their image strips
// into one [H][W] rgba32f frame on the root device (devices[0]):
//   - a strip on the root device renders straight into its rows of the frame (rt_bind_image);
//   - a strip on another device renders into its own image and copies it into the frame with
//     one device-to-device copy over xGMI (peer access enabled), enqueued on the stream of the
//     pass that wrote the image (rt_image_stream: the post-process's output stream for a
//     pipelined mode-1 frame, the main stream otherwise), so frame k's copy follows that pass
//     and overlaps frame k+1's trace passes; the next pass that writes the image is ordered
//     after everything on that stream, the copy included.
// Each strip keeps its own g-buffer ring for its rows plus a 1-row halo (rt_create), so no
// strip reads another's data: the copies into the frame are the only transfers.
// One host thread per strip enqueues its strip's work, so the per-frame host cost does not add
// up over the strips.  Strip bounds are cost-balanced (rt_group_balance): one probe frame with
// per-row work counters, then calibration passes that time each strip and rescale the profile
// (rt_plan_strips / rt_calibrate_row_cost, the host-only planner also used by the
// torch.distributed path in real_time_ray_tracer_amd/dist.py).  When strips copy into the root
// device, the later passes plan with the copies (rt_plan_strips_gather): the bounds and the root
// strip, the one rendered on devices[0] in place, minimise max(render, per-link copy, ingest).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/rt/abi.h"

namespace {

// n persistent worker threads; run(f) calls f(i) on worker i for every i and returns the
// first error status (or RT_OK).
class Workers {
 public:
  explicit Workers(int n) : rc_(n, RT_OK) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~Workers() {
    {
      std::lock_guard<std::mutex> l(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int run(const std::function<int(int)>& f) {
    const int n = (int)th_.size();
    if (n == 1) return f(0);
    std::unique_lock<std::mutex> l(m_);
    job_ = &f;
    pending_ = n;
    ++gen_;
    cv_.notify_all();
    done_.wait(l, [&] { return pending_ == 0; });
    job_ = nullptr;
    for (int r : rc_)
      if (r < 0) return r;
    return RT_OK;
  }

 private:
  void loop(int i) {
    long seen = 0;
    std::unique_lock<std::mutex> l(m_);
    for (;;) {
      cv_.wait(l, [&] { return quit_ || gen_ != seen; });
      if (quit_) return;
      seen = gen_;
      const std::function<int(int)>* f = job_;
      l.unlock();
      const int r = (*f)(i);
      l.lock();
      rc_[i] = r;
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<int(int)>* job_ = nullptr;
  long gen_ = 0;
  int pending_ = 0;
  bool quit_ = false;
  std::vector<int> rc_;
};

bool valid_bounds(const int* b, int n, int H) {
  if (b[0] != 0 || b[n] != H) return false;
  for (int i = 0; i < n; ++i)
    if (b[i + 1] <= b[i]) return false;
  return true;
}

}  // namespace

struct rt_group {
  int n = 0;
  std::vector<int> devices;
  rt_config cfg{};
  std::vector<int> bounds;
  bool pipelined = false;
  std::vector<rt_ctx*> ctx;
  float4* frame_own = nullptr;  // [H][W] on devices[0]
  float4* frame = nullptr;      // the bound frame (own or the caller's)
  std::vector<float> header;    // the group's copy of the SSBO prefix
  std::vector<std::vector<float>> strip_header;  // per-strip copies for the worker loops
  std::vector<char> header_dirty;
  bool have_header = false;
  Workers* workers = nullptr;
  int last_hip = 0;
  bool force_copies = false;  // test hook: every strip but the root strip takes the copy path
  // the root strip: rendered on devices[0] (the frame's device) into its frame rows; strip i < root
  // runs on devices[i + 1], strip i > root on devices[i] (root 0: strip i on devices[i])
  int root = 0;
  double link_gbps = 0.0, ingest_gbps = 0.0;  // the gather-aware planner's link model (0: measure)
};

namespace {

// the device strip i renders on
int strip_dev(const rt_group* g, int i) {
  return i == g->root ? g->devices[0] : g->devices[i < g->root ? i + 1 : i];
}

// strip i renders straight into its rows of the frame (no copy)
bool on_root(const rt_group* g, int i) {
  return strip_dev(g, i) == g->devices[0] && (i == g->root || !g->force_copies);
}

void destroy_strips(rt_group* g) {
  for (auto*& c : g->ctx)
    if (c) {
      rt_destroy(c);
      c = nullptr;
    }
}

int bind_strips(rt_group* g) {
  const int W = g->cfg.width;
  for (int i = 0; i < g->n; ++i) {
    int rc = rt_bind_image(g->ctx[i], on_root(g, i) ? (void*)(g->frame + (size_t)g->bounds[i] * W) : nullptr);
    if (rc != RT_OK) return rc;
  }
  return RT_OK;
}

// (Re)create the strip contexts for g->bounds (fresh g-buffer rings).
int make_strips(rt_group* g) {
  destroy_strips(g);
  g->ctx.assign(g->n, nullptr);
  for (int i = 0; i < g->n; ++i) {
    rt_config c = g->cfg;
    c.row_begin = g->bounds[i];
    c.row_end = g->bounds[i + 1];
    int rc = rt_create(strip_dev(g, i), &c, &g->ctx[i]);
    if (rc == RT_OK && g->pipelined) rc = rt_enable_pipelining(g->ctx[i], 1, nullptr);
    if (rc != RT_OK) {
      destroy_strips(g);
      return rc;
    }
  }
  std::fill(g->header_dirty.begin(), g->header_dirty.end(), 1);
  return bind_strips(g);
}

// The image copy of strip i into its frame rows (strips off the root device), on the stream of
// the pass that wrote the image (read after write), so the next writer of the image, ordered
// after that stream's work, cannot overwrite it under the copy (write after read).
int copy_strip(rt_group* g, int i) {
  if (on_root(g, i)) return RT_OK;
  const int W = g->cfg.width;
  const size_t bytes = (size_t)(g->bounds[i + 1] - g->bounds[i]) * W * sizeof(float4);
  hipError_t e = hipSetDevice(strip_dev(g, i));
  if (e == hipSuccess)
    e = hipMemcpyAsync(g->frame + (size_t)g->bounds[i] * W, rt_image_device_ptr(g->ctx[i]), bytes,
                       hipMemcpyDeviceToDevice, (hipStream_t)rt_image_stream(g->ctx[i]));
  if (e != hipSuccess) {
    g->last_hip = (int)e;
    return RT_E_HIP;
  }
  return RT_OK;
}

// n frames of the render loop (src/main.cpp:763-781) on strip i, as rt_compute_frames does,
// each followed by the strip's copy into the frame.
int strip_frames(rt_group* g, int i, float* hdr, int mode, int frame, int n, uint64_t seed, int light) {
  const int S = g->cfg.num_shapes, spp = g->cfg.spp;
  const size_t bytes = rt_header_bytes(S, spp);
  for (int k = 0; k < n; ++k) {
    int rc = (mode == RT_MODE_AO_PP || mode == RT_MODE_AO) ? rt_fill_rand_buffer(hdr, S, spp, seed + (uint64_t)k)
                                                           : rt_moving_light(hdr, light);
    if (rc != RT_OK) return rc;
    const float mz = hdr[RT_HDR_MODE * 4 + 2];
    if (!(mz >= 0.0f && mz < (float)(S + 1))) return RT_E_INVAL;
    rc = rt_set_mode(hdr, frame, (int)mz);
    if (rc == RT_OK) rc = rt_upload_header(g->ctx[i], hdr, bytes);
    if (rc != RT_OK) return rc;
    frame = rt_dispatch(g->ctx[i], mode, frame);
    if (frame < 0) return frame;
    rc = copy_strip(g, i);
    if (rc != RT_OK) return rc;
  }
  return frame;
}

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- the gather-aware strip planner (rt_plan_strips_gather) ----------------------------------
// A frame split into n contiguous row strips is assembled on a root device, which renders one
// strip (the root strip) straight into its frame rows; every other strip's image, rows * W * 16 B,
// crosses one link into the root once per frame, overlapped with the next frame's render.  The
// steady-state frame time is then bounded by
//   T = max( max_i render_i,  max_{i != root} bytes_i / link,  sum_{i != root} bytes_i / ingest ).
// The planner minimises T over the bounds and the choice of root strip: bisection on T, each
// candidate checked for every root position j by filling the strips below j from row 0 and
// those above j from row H with as many rows as the render and link caps allow, then giving the
// root the cheapest interval that covers what they leave and satisfies the ingest bound.
struct GatherModel {
  const double* cum;  // prefix sums of the per-row render cost (ms), H + 1 entries
  int H, n;
  double rl;  // ms per row over one link (0: no link term)
  double ri;  // ms per non-root row at the root's ingest (0: no ingest term)
};

double seg_cost(const GatherModel& m, int a, int b) { return m.cum[b] - m.cum[a]; }

int link_cap(const GatherModel& m, double T, int limit) {
  if (m.rl <= 0.0) return limit;
  const double r = std::floor(T / m.rl);
  return r < (double)limit ? (int)r : limit;
}

// most rows (<= limit) a non-root strip starting at row y and growing up may take within T
int rows_up(const GatherModel& m, int y, int limit, double T) {
  const int cap = link_cap(m, T, limit);
  if (cap <= 0) return 0;
  const double* p = std::upper_bound(m.cum + y, m.cum + y + cap + 1, m.cum[y] + T);
  return (int)(p - (m.cum + y)) - 1;
}

// most rows (<= limit) a non-root strip ending at row y (exclusive) and growing down may take
int rows_down(const GatherModel& m, int y, int limit, double T) {
  const int cap = link_cap(m, T, limit);
  if (cap <= 0) return 0;
  const double* p = std::lower_bound(m.cum + y - cap, m.cum + y + 1, m.cum[y] - T);
  return y - (int)(p - m.cum);
}

// k strips covering [y0, y1) upward, each within T (rows_up caps), each >= 1 row; false if the
// caps cannot cover the range.  b receives the k - 1 inner bounds.
bool fill_up(const GatherModel& m, int y0, int y1, int k, double T, int* b) {
  int y = y0;
  for (int s = 0; s < k; ++s) {
    const int left = k - 1 - s;  // strips after this one, one row each at least
    int r = s == k - 1 ? y1 - y : std::min(rows_up(m, y, y1 - y - left, T), y1 - y - left);
    if (r < 1) return false;
    if (s == k - 1 && (seg_cost(m, y, y1) > T || (m.rl > 0.0 && r * m.rl > T))) return false;
    y += r;
    if (s < k - 1) b[s] = y;
  }
  return y == y1;
}

// the smallest per-strip bound T' <= T with which k strips still cover [y0, y1): balanced strips
bool fill_balanced(const GatherModel& m, int y0, int y1, int k, double T, int* b) {
  if (k == 0) return y0 == y1;
  if (!fill_up(m, y0, y1, k, T, b)) return false;
  double lo = 0.0, hi = T;
  for (int it = 0; it < 60; ++it) {
    const double mid = 0.5 * (lo + hi);
    std::vector<int> t(std::max(1, k - 1));
    if (fill_up(m, y0, y1, k, mid, t.data())) hi = mid; else lo = mid;
  }
  return fill_up(m, y0, y1, k, hi, b);
}

// root strip j within T: the root's interval [ra, rb), or false.  Minimises the root's render cost.
bool root_interval(const GatherModel& m, int j, double T, int& ra, int& rb) {
  const int H = m.H, n = m.n;
  int a = 0;  // rows [0, a) the j strips below the root can cover at most
  for (int s = 0; s < j; ++s) {
    const int r = rows_up(m, a, H - a - (n - 1 - s), T);
    if (r < 1) return false;
    a += r;
  }
  int b = H;  // rows [b, H) the strips above the root can cover at most
  for (int s = n - 1; s > j; --s) {
    const int r = rows_down(m, b, b - s, T);
    if (r < 1) return false;
    b -= r;
  }
  int need = 1;  // ingest: the non-root rows must cross into the root within T
  if (m.ri > 0.0) need = std::max(need, H - (int)std::min((double)H, std::floor(T / m.ri)));
  const int amax = std::min(a, H - (n - 1 - j) - 1), bmax = H - (n - 1 - j);
  double best = -1.0;
  for (int x = j; x <= amax; ++x) {
    const int y = std::max(std::max(b, x + need), x + 1);
    if (y > bmax) continue;
    const double c = seg_cost(m, x, y);
    if (best < 0.0 || c < best) best = c, ra = x, rb = y;
  }
  return best >= 0.0 && best <= T;
}

}  // namespace

extern "C" {

int rt_plan_strips(const double* row_cost, int H, int n, int* bounds) {
  if (!row_cost || !bounds || H <= 0 || n <= 0 || n > H) return RT_E_INVAL;
  double mx = 0.0;
  for (int y = 0; y < H; ++y) {
    if (!(row_cost[y] >= 0.0)) return RT_E_INVAL;  // negative or NaN
    mx = std::max(mx, row_cost[y]);
  }
  // a tiny per-row floor, so zero-cost rows still split evenly
  const double eps = 1e-9 * std::max(1.0, mx);
  std::vector<double> cum((size_t)H + 1, 0.0);
  for (int y = 0; y < H; ++y) cum[y + 1] = cum[y] + (row_cost[y] + eps);
  const double total = cum[H];
  bounds[0] = 0;
  for (int i = 1; i < n; ++i) {
    // first prefix index whose cumulative cost reaches i/n of the total
    int y = (int)(std::lower_bound(cum.begin(), cum.end(), total * i / n) - cum.begin());
    y = std::max(y, bounds[i - 1] + 1);
    y = std::min(y, H - (n - i));
    bounds[i] = y;
  }
  bounds[n] = H;
  return RT_OK;
}

int rt_strip_gather_bound(const double* row_ms, int H, const int* bounds, int n, int root_strip, int width,
                          double link_gbps, double ingest_gbps, double* bound_ms) {
  if (!row_ms || !bounds || !bound_ms || H <= 0 || n <= 0 || width <= 0 || root_strip < 0 || root_strip >= n ||
      !valid_bounds(bounds, n, H))
    return RT_E_INVAL;
  const double row_bytes = (double)width * 16.0;
  double render = 0.0, link = 0.0, rest = 0.0;
  for (int i = 0; i < n; ++i) {
    double c = 0.0;
    for (int y = bounds[i]; y < bounds[i + 1]; ++y) c += row_ms[y];
    render = std::max(render, c);
    if (i == root_strip) continue;
    const double bytes = row_bytes * (bounds[i + 1] - bounds[i]);
    rest += bytes;
    if (link_gbps > 0.0) link = std::max(link, bytes / (link_gbps * 1e6));
  }
  const double ingest = ingest_gbps > 0.0 ? rest / (ingest_gbps * 1e6) : 0.0;
  bound_ms[0] = std::max(render, std::max(link, ingest));
  bound_ms[1] = render;
  bound_ms[2] = link;
  bound_ms[3] = ingest;
  return RT_OK;
}

int rt_plan_strips_gather(const double* row_ms, int H, int n, int width, double link_gbps, double ingest_gbps,
                          int* bounds, int* root_strip, double* bound_ms) {
  if (!row_ms || !bounds || !root_strip || H <= 0 || n <= 0 || n > H || width <= 0 || !(link_gbps == link_gbps) ||
      !(ingest_gbps == ingest_gbps))
    return RT_E_INVAL;
  std::vector<double> cum((size_t)H + 1, 0.0);
  for (int y = 0; y < H; ++y) {
    if (!(row_ms[y] >= 0.0) || row_ms[y] == HUGE_VAL) return RT_E_INVAL;  // negative, NaN or inf
    cum[y + 1] = cum[y] + row_ms[y];
  }
  const double row_bytes = (double)width * 16.0;
  const GatherModel m{cum.data(), H, n, link_gbps > 0.0 ? row_bytes / (link_gbps * 1e6) : 0.0,
                      ingest_gbps > 0.0 ? row_bytes / (ingest_gbps * 1e6) : 0.0};
  // bisection on T: every root position is tried at every candidate
  double lo = 0.0, hi = cum[H] + H * (m.rl + m.ri) + 1e-9;
  auto feasible = [&](double T) {
    int ra, rb;
    for (int j = 0; j < n; ++j)
      if (root_interval(m, j, T, ra, rb)) return true;
    return false;
  };
  for (int it = 0; it < 100 && hi - lo > 1e-12 * std::max(1.0, hi); ++it) {
    const double mid = 0.5 * (lo + hi);
    if (feasible(mid)) hi = mid; else lo = mid;
  }
  // at the bound: of the feasible root positions the one whose strip keeps the most rows (fewest
  // bytes on the links), its neighbours' strips balanced within the bound
  int bj = -1, bra = 0, brb = 0;
  for (int j = 0; j < n; ++j) {
    int ra, rb;
    if (root_interval(m, j, hi, ra, rb) && (bj < 0 || rb - ra > brb - bra)) bj = j, bra = ra, brb = rb;
  }
  if (bj < 0) return RT_E_INVAL;  // (cannot happen: hi is feasible)
  bounds[0] = 0;
  bounds[n] = H;
  bounds[bj] = bra;
  bounds[bj + 1] = brb;
  if (!fill_balanced(m, 0, bra, bj, hi, bounds + 1) || !fill_balanced(m, brb, H, n - 1 - bj, hi, bounds + bj + 2))
    return RT_E_INVAL;
  *root_strip = bj;
  if (bound_ms) return rt_strip_gather_bound(row_ms, H, bounds, n, bj, width, link_gbps, ingest_gbps, bound_ms);
  return RT_OK;
}

int rt_calibrate_row_cost(double* row_cost, int H, const int* bounds, int n, const double* strip_ms) {
  if (!row_cost || !bounds || !strip_ms || H <= 0 || n <= 0 || !valid_bounds(bounds, n, H)) return RT_E_INVAL;
  for (int i = 0; i < n; ++i) {
    const int a = bounds[i], b = bounds[i + 1];
    double tot = 0.0;
    for (int y = a; y < b; ++y) tot += row_cost[y];
    for (int y = a; y < b; ++y) row_cost[y] = tot > 0.0 ? row_cost[y] * (strip_ms[i] / tot) : strip_ms[i] / (b - a);
  }
  return RT_OK;
}

int rt_group_create(int n, const int* devices, const rt_config* cfg, const int* bounds, rt_group** out) {
  if (!out) return RT_E_INVAL;
  *out = nullptr;
  if (n <= 0 || !devices || !cfg || cfg->height <= 0 || cfg->width <= 0 || n > cfg->height) return RT_E_INVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RT_E_NODEV;
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= ndev) return RT_E_NODEV;
  rt_group* g = new (std::nothrow) rt_group();
  if (!g) return RT_E_NOMEM;
  g->n = n;
  g->devices.assign(devices, devices + n);
  g->cfg = *cfg;
  g->cfg.row_begin = g->cfg.row_end = 0;
  const int H = cfg->height, W = cfg->width;
  g->bounds.resize(n + 1);
  if (bounds) {
    if (!valid_bounds(bounds, n, H)) {
      delete g;
      return RT_E_INVAL;
    }
    std::copy(bounds, bounds + n + 1, g->bounds.begin());
  } else {
    for (int i = 0; i <= n; ++i) g->bounds[i] = (int)(((long long)i * H + n / 2) / n);
  }
  g->header.assign(rt_header_bytes(std::max(0, cfg->num_shapes), std::max(1, cfg->spp)) / 4, 0.0f);
  g->strip_header.assign(n, g->header);
  g->header_dirty.assign(n, 1);
  // peer access from every other device to the root (the strip copies go over xGMI).  Without
  // it a device-to-device copy is staged through host memory: refuse instead of degrading
  // silently.
  for (int i = 1; i < n; ++i) {
    const int d = g->devices[i], r = g->devices[0];
    if (d == r) continue;
    int can = 0;
    hipError_t e = hipDeviceCanAccessPeer(&can, d, r);
    if (e == hipSuccess && !can) e = hipErrorPeerAccessUnsupported;
    if (e == hipSuccess) e = hipSetDevice(d);
    if (e == hipSuccess) {
      e = hipDeviceEnablePeerAccess(r, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) e = hipSuccess;
    }
    (void)hipGetLastError();  // no stale error for later launches to report
    if (e != hipSuccess) {
      delete g;
      return RT_E_NODEV;
    }
  }
  hipError_t e = hipSetDevice(g->devices[0]);
  if (e == hipSuccess) e = hipMalloc(&g->frame_own, (size_t)H * W * sizeof(float4));
  if (e == hipSuccess) e = hipMemset(g->frame_own, 0, (size_t)H * W * sizeof(float4));
  if (e != hipSuccess) {
    if (g->frame_own) (void)hipFree(g->frame_own);
    delete g;
    return e == hipErrorOutOfMemory ? RT_E_NOMEM : RT_E_HIP;
  }
  g->frame = g->frame_own;
  int rc = make_strips(g);
  if (rc != RT_OK) {
    (void)hipFree(g->frame_own);
    delete g;
    return rc;
  }
  g->workers = new (std::nothrow) Workers(n);
  if (!g->workers) {
    rt_group_destroy(g);
    return RT_E_NOMEM;
  }
  *out = g;
  return RT_OK;
}

int rt_group_destroy(rt_group* g) {
  if (!g) return RT_E_INVAL;
  for (auto* c : g->ctx)
    if (c) (void)rt_synchronize(c);
  delete g->workers;
  destroy_strips(g);
  if (g->frame_own) {
    (void)hipSetDevice(g->devices[0]);
    (void)hipFree(g->frame_own);
  }
  delete g;
  return RT_OK;
}

int rt_group_size(rt_group* g) { return g ? g->n : RT_E_INVAL; }

int rt_group_strip_copies(rt_group* g, int i) {
  if (!g || i < 0 || i >= g->n) return RT_E_INVAL;
  return on_root(g, i) ? 0 : 1;
}

int rt_group_force_copies(rt_group* g, int on) {
  if (!g) return RT_E_INVAL;
  for (auto* c : g->ctx) {  // the frame rows may still be written
    int rc = rt_synchronize(c);
    if (rc != RT_OK) return rc;
  }
  g->force_copies = on != 0;
  return bind_strips(g);
}

int rt_group_bounds(rt_group* g, int* bounds) {
  if (!g || !bounds) return RT_E_INVAL;
  std::copy(g->bounds.begin(), g->bounds.end(), bounds);
  return RT_OK;
}

int rt_group_set_bounds(rt_group* g, const int* bounds) {
  if (!g || !bounds || !valid_bounds(bounds, g->n, g->cfg.height)) return RT_E_INVAL;
  for (auto* c : g->ctx) {
    int rc = rt_synchronize(c);
    if (rc != RT_OK) return rc;
  }
  std::copy(bounds, bounds + g->n + 1, g->bounds.begin());
  return make_strips(g);
}

rt_ctx* rt_group_strip(rt_group* g, int i) { return (g && i >= 0 && i < g->n) ? g->ctx[i] : nullptr; }

int rt_group_last_hip_error(rt_group* g) {
  if (!g) return 0;
  if (g->last_hip) return g->last_hip;
  for (auto* c : g->ctx)
    if (c && rt_last_hip_error(c)) return rt_last_hip_error(c);
  return 0;
}

int rt_group_enable_pipelining(rt_group* g, int on) {
  if (!g) return RT_E_INVAL;
  g->pipelined = on != 0;
  for (auto* c : g->ctx) {
    int rc = rt_enable_pipelining(c, on, nullptr);
    if (rc != RT_OK) return rc;
  }
  return RT_OK;
}

int rt_group_bind_frame(rt_group* g, void* device_ptr) {
  if (!g) return RT_E_INVAL;
  for (auto* c : g->ctx) {  // the frame in use may still be written
    int rc = rt_synchronize(c);
    if (rc != RT_OK) return rc;
  }
  g->frame = device_ptr ? (float4*)device_ptr : g->frame_own;
  return bind_strips(g);
}

void* rt_group_frame_device_ptr(rt_group* g) { return g ? (void*)g->frame : nullptr; }

int rt_group_upload_header(rt_group* g, const void* header, size_t bytes) {
  if (!g || !header) return RT_E_INVAL;
  const int S = g->cfg.num_shapes;
  if (bytes != rt_header_bytes(S, g->cfg.spp)) return RT_E_INVAL;
  const float mz = ((const float*)header)[RT_HDR_MODE * 4 + 2];
  if (!(mz >= 0.0f && mz < (float)(S + 1))) return RT_E_INVAL;
  std::memcpy(g->header.data(), header, bytes);
  std::fill(g->header_dirty.begin(), g->header_dirty.end(), 1);
  g->have_header = true;
  return RT_OK;
}

int rt_group_dispatch(rt_group* g, int mode, int frame) {
  if (!g) return RT_E_INVAL;
  if (!g->have_header) return RT_E_STATE;
  if (mode < RT_MODE_AO_PP || mode > RT_MODE_PHONG_REFL || frame < 0 || frame >= g->cfg.num_frames)
    return RT_E_INVAL;
  const size_t bytes = g->header.size() * sizeof(float);
  int rc = g->workers->run([&](int i) -> int {
    if (g->header_dirty[i]) {
      int r = rt_upload_header(g->ctx[i], g->header.data(), bytes);
      if (r != RT_OK) return r;
      g->header_dirty[i] = 0;
    }
    int f = rt_dispatch(g->ctx[i], mode, frame);
    if (f < 0) return f;
    return copy_strip(g, i);
  });
  if (rc != RT_OK) return rc;
  return (frame + 1) % g->cfg.num_frames;
}

int rt_group_compute_frames(rt_group* g, float* header, int mode, int frame, int n, uint64_t rand_seed,
                            int light_movement) {
  if (!g || !header || n < 0 || mode < RT_MODE_AO_PP || mode > RT_MODE_PHONG_REFL) return RT_E_INVAL;
  if (frame < 0 || frame >= g->cfg.num_frames) return RT_E_INVAL;
  const size_t nf = g->header.size();
  std::vector<int> next(g->n, frame);
  int rc = g->workers->run([&](int i) -> int {
    std::vector<float>& h = g->strip_header[i];
    std::memcpy(h.data(), header, nf * sizeof(float));
    int f = strip_frames(g, i, h.data(), mode, frame, n, rand_seed, light_movement);
    if (f < 0) return f;
    next[i] = f;
    return RT_OK;
  });
  if (rc != RT_OK) return rc;
  std::memcpy(header, g->strip_header[0].data(), nf * sizeof(float));  // as the host loop leaves it
  std::memcpy(g->header.data(), header, nf * sizeof(float));
  std::fill(g->header_dirty.begin(), g->header_dirty.end(), 0);  // every strip holds this header
  g->have_header = true;
  return next[0];
}

int rt_group_synchronize(rt_group* g) {
  if (!g) return RT_E_INVAL;
  for (auto* c : g->ctx) {
    int rc = rt_synchronize(c);
    if (rc != RT_OK) return rc;
  }
  return RT_OK;
}

int rt_group_download_image(rt_group* g, float* image) {
  if (!g || !image) return RT_E_INVAL;
  int rc = rt_group_synchronize(g);
  if (rc != RT_OK) return rc;
  hipError_t e = hipSetDevice(g->devices[0]);
  if (e == hipSuccess)
    e = hipMemcpy(image, g->frame, (size_t)g->cfg.height * g->cfg.width * sizeof(float4), hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    g->last_hip = (int)e;
    return RT_E_HIP;
  }
  return RT_OK;
}

}  // extern "C"

namespace {

// Links into the root device, measured: each non-root strip's image copied into its frame rows
// alone (the per-link rate, the slowest link kept) and all at once (the root's ingest rate), by
// wall clock over 4 copies after one.  Strips on the root device do not copy and are skipped.
int probe_links(rt_group* g, double& link_gbps, double& ingest_gbps) {
  std::vector<int> cp;
  double all_bytes = 0.0;
  for (int i = 0; i < g->n; ++i)
    if (!on_root(g, i)) cp.push_back(i), all_bytes += (double)(g->bounds[i + 1] - g->bounds[i]) * g->cfg.width * 16.0;
  link_gbps = ingest_gbps = 0.0;
  if (cp.empty()) return RT_OK;
  auto run = [&](const std::vector<int>& which, int reps) -> double {
    for (int i : which)
      if (rt_synchronize(g->ctx[i]) != RT_OK) return -1.0;
    const double t0 = now_ms();
    for (int k = 0; k < reps; ++k)
      for (int i : which)
        if (copy_strip(g, i) != RT_OK) return -1.0;
    for (int i : which)
      if (rt_synchronize(g->ctx[i]) != RT_OK) return -1.0;
    return (now_ms() - t0) / reps;
  };
  double slow = -1.0;
  for (int i : cp) {
    if (run({i}, 1) < 0.0) return RT_E_HIP;
    const double ms = run({i}, 4);
    if (ms < 0.0) return RT_E_HIP;
    const double gbps = (double)(g->bounds[i + 1] - g->bounds[i]) * g->cfg.width * 16.0 / (std::max(ms, 1e-6) * 1e6);
    slow = slow < 0.0 ? gbps : std::min(slow, gbps);
  }
  if (run(cp, 1) < 0.0) return RT_E_HIP;
  const double ms = run(cp, 4);
  if (ms < 0.0) return RT_E_HIP;
  link_gbps = slow;
  ingest_gbps = all_bytes / (std::max(ms, 1e-6) * 1e6);
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_group_set_plan(rt_group* g, const int* bounds, int root_strip) {
  if (!g || !bounds || root_strip < 0 || root_strip >= g->n || !valid_bounds(bounds, g->n, g->cfg.height))
    return RT_E_INVAL;
  for (auto* c : g->ctx) {
    int rc = rt_synchronize(c);
    if (rc != RT_OK) return rc;
  }
  std::copy(bounds, bounds + g->n + 1, g->bounds.begin());
  g->root = root_strip;
  return make_strips(g);
}

int rt_group_root_strip(rt_group* g) { return g ? g->root : RT_E_INVAL; }

int rt_group_strip_device(rt_group* g, int i) {
  if (!g || i < 0 || i >= g->n) return RT_E_INVAL;
  return strip_dev(g, i);
}

int rt_group_set_link_model(rt_group* g, double link_gbps, double ingest_gbps) {
  if (!g || !(link_gbps >= 0.0) || !(ingest_gbps >= 0.0)) return RT_E_INVAL;
  g->link_gbps = link_gbps;
  g->ingest_gbps = ingest_gbps;
  return RT_OK;
}

int rt_group_link_model(rt_group* g, double* link_gbps, double* ingest_gbps) {
  if (!g || !link_gbps || !ingest_gbps) return RT_E_INVAL;
  *link_gbps = g->link_gbps;
  *ingest_gbps = g->ingest_gbps;
  return RT_OK;
}

int rt_group_balance(rt_group* g, const float* header, int mode, int rounds, double* strip_ms) {
  if (!g || !header || mode < RT_MODE_AO_PP || mode > RT_MODE_PHONG_REFL || rounds < 0) return RT_E_INVAL;
  const int H = g->cfg.height, W = g->cfg.width, n = g->n;
  const size_t nf = g->header.size();
  std::vector<float> h(header, header + nf);
  // 1. one probe frame with per-row work counters on every strip -> the frame's cost profile
  std::vector<double> cost(H, 0.0);
  int rc = g->workers->run([&](int i) -> int {
    std::vector<float> hh(h);
    int r = rt_enable_counters(g->ctx[i], 2);
    if (r != RT_OK) return r;
    int f = strip_frames(g, i, hh.data(), mode, 0, 1, 7000, 0);
    if (f < 0) return f;
    std::vector<uint64_t> rows(g->bounds[i + 1] - g->bounds[i]);
    r = rt_read_row_counters(g->ctx[i], rows.data(), 1);
    if (r == RT_OK) r = rt_enable_counters(g->ctx[i], 0);
    for (size_t k = 0; k < rows.size(); ++k) cost[g->bounds[i] + k] = (double)rows[k];
    return r;
  });
  if (rc != RT_OK) return rc;
  std::vector<int> b(n + 1);
  rc = rt_plan_strips(cost.data(), H, n, b.data());
  if (rc != RT_OK) return rc;
  int root = 0;
  // the gather-aware plan when strips copy into the root (distinct devices, or the copy path
  // forced): the root strip is chosen with the bounds, so the largest-byte strip stays on the root
  // device.  The first plan is render-only (the counter profile is not in ms yet); every later one
  // re-plans the calibrated (ms) profile with the link model, measured here unless set.
  bool gather = g->force_copies;
  for (int i = 1; i < n; ++i) gather = gather || g->devices[i] != g->devices[0];
  // 2. calibration: time every strip of the plan alone, as the frame loop renders it (wall
  // clock of 16 frames after 8, gather copy included), rescale the profile so each strip's
  // total is its time, re-plan; keep the plan with the smallest bound (measured render, the link
  // model's copy times)
  std::vector<int> best = b;
  int best_root = 0;
  double best_ms = -1.0;
  std::vector<double> best_t(n, 0.0), t(n, 0.0);
  for (int it = 0; it < std::max(1, rounds); ++it) {
    rc = rt_group_set_plan(g, b.data(), root);
    if (rc != RT_OK) return rc;
    if (gather && it == 0 && g->link_gbps <= 0.0) {
      rc = probe_links(g, g->link_gbps, g->ingest_gbps);
      if (rc != RT_OK) return rc;
    }
    for (int i = 0; i < n && rc == RT_OK; ++i) {  // one strip at a time (strips may share a device)
      std::vector<float> hh(h);
      int f = strip_frames(g, i, hh.data(), mode, 0, 8, 7000, 0);
      if (f >= 0) f = rt_synchronize(g->ctx[i]) == RT_OK ? f : RT_E_HIP;
      const double t0 = now_ms();
      if (f >= 0) f = strip_frames(g, i, hh.data(), mode, f, 16, 7008, 0);
      if (f >= 0 && rt_synchronize(g->ctx[i]) != RT_OK) f = RT_E_HIP;
      if (f < 0) rc = f;
      t[i] = (now_ms() - t0) / 16.0;
    }
    if (rc != RT_OK) return rc;
    double mx = *std::max_element(t.begin(), t.end());
    if (gather) {
      double bound[4];
      std::vector<double> per_row(H, 0.0);  // the measured strip times spread over their rows
      for (int i = 0; i < n; ++i)
        for (int y = b[i]; y < b[i + 1]; ++y) per_row[y] = t[i] / (b[i + 1] - b[i]);
      rc = rt_strip_gather_bound(per_row.data(), H, b.data(), n, root, W, g->link_gbps, g->ingest_gbps, bound);
      if (rc != RT_OK) return rc;
      mx = bound[0];
    }
    if (best_ms < 0.0 || mx < best_ms) {
      best_ms = mx;
      best = b;
      best_root = root;
      best_t = t;
    }
    if (it + 1 < rounds) {
      rc = rt_calibrate_row_cost(cost.data(), H, b.data(), n, t.data());
      if (rc == RT_OK)
        rc = gather ? rt_plan_strips_gather(cost.data(), H, n, W, g->link_gbps, g->ingest_gbps, b.data(), &root,
                                            nullptr)
                    : rt_plan_strips(cost.data(), H, n, b.data());
      if (rc != RT_OK) return rc;
    }
  }
  if (strip_ms) std::copy(best_t.begin(), best_t.end(), strip_ms);
  return rt_group_set_plan(g, best.data(), best_root);  // fresh rings on the chosen plan
}

}  // extern "C"
