// Microbenchmark: sustained issue rate of the binary64 VALU instructions a double-precision
// sin would use (v_fma_f64, v_mul_f64, v_add_f64, v_cvt_f64_f32, v_cvt_f32_f64, v_rndne_f64)
// against v_fma_f32, wave64 on gfx950, 8 waves per SIMD, 8 independent chains per lane.
// Prints wave-instructions per ns per form and the ratio to v_fma_f32: the cost of one f64
// instruction in f32-FMA issue slots.  A mixed stream (1 f64 : 1 f32) shows whether the two
// share the issue slot.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(stmt) \
  _Pragma("unroll") for (int j = 0; j < 8; ++j) { stmt; }

template <int FORM>
__global__ __launch_bounds__(256) void k_rate(float* out, int iters, float a, float b) {
  float x[8];
  double d[8];
  for (int j = 0; j < 8; ++j) {
    x[j] = threadIdx.x * 1e-3f + j;
    d[j] = threadIdx.x * 1e-3 + j;
  }
  const double da = a, db = b;
  for (int i = 0; i < iters; ++i) {
    if (FORM == 0) CHAIN8(asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[j]) : "v"(a), "v"(b)))
    if (FORM == 1) CHAIN8(asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[j]) : "v"(da), "v"(db)))
    if (FORM == 2) CHAIN8(asm volatile("v_mul_f64 %0, %1, %0" : "+v"(d[j]) : "v"(da)))
    if (FORM == 3) CHAIN8(asm volatile("v_add_f64 %0, %1, %0" : "+v"(d[j]) : "v"(db)))
    if (FORM == 4) CHAIN8(asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d[j]) : "v"(x[j])))
    if (FORM == 5) CHAIN8(asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(x[j]) : "v"(d[j])))
    if (FORM == 6) CHAIN8(asm volatile("v_rndne_f64 %0, %0" : "+v"(d[j])))
    if (FORM == 7) {
      CHAIN8(asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[j]) : "v"(da), "v"(db)))
      CHAIN8(asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[j]) : "v"(a), "v"(b)))
    }
  }
  float s = 0;
  for (int j = 0; j < 8; ++j) s += x[j] + (float)d[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(float*, int, float, float);

int main() {
  float* out;
  const int blocks = 256 * 4 * 8 / 4;  // 8 waves per SIMD (4 waves per block)
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 50000;
  const char* names[] = {"v_fma_f32", "v_fma_f64", "v_mul_f64", "v_add_f64", "v_cvt_f64_f32",
                         "v_cvt_f32_f64", "v_rndne_f64", "mixed fma f64+f32"};
  kfn fns[] = {k_rate<0>, k_rate<1>, k_rate<2>, k_rate<3>, k_rate<4>, k_rate<5>, k_rate<6>, k_rate<7>};
  double base = 0;
  for (int form = 0; form < 8; ++form) {
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      fns[form]<<<blocks, 256>>>(out, iters, 1.0000001f, 1e-7f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double insts = (double)blocks * 4 * iters * 8 * (form == 7 ? 2 : 1);  // wave-instructions
    const double rate = insts / (best * 1e6);                                     // per ns
    if (form == 0) base = rate;
    printf("%-18s %8.3f ms  %7.2f wave-inst/ns  %.3f f32-FMA slots per instruction\n", names[form], best, rate,
           base / rate);
  }
  return 0;
}
