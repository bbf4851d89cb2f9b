// rt_kernels.hip — the production launcher of the gfx950 kernels (rt_kernels_impl.h) behind the
// launch interface of rt_kernels.h.  No experiment switches: the A/B variants and their
// environment selection live in the tools-only library (tools/ab/rt_kernels_ab.hip, make ablib).
#include "rt_kernels_impl.h"

namespace rt {

hipError_t launch_program(int program, const FrameParams& p, hipStream_t stream) {
  if (p.trace_rows <= 0) return hipSuccess;
  return launch_production(program, p, launch_params(p), stream);
}

hipError_t launch_selftest(int fn, const float* d_in, float* d_out, size_t n, hipStream_t stream) {
  return launch_selftest_impl(fn, d_in, d_out, n, stream);
}

hipError_t launch_gbuf_convert(const GbufXfer& x, hipStream_t stream) { return launch_gbuf_convert_impl(x, stream); }

}  // namespace rt
