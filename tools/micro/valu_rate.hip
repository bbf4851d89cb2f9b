// Microbenchmark: sustained issue rate of v_fma_f32 vs v_pk_fma_f32 (wave64, gfx950),
// many waves per SIMD, 8 independent chains per lane.  Prints TFLOP/s per form.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float a, float b) {
  float x[8];
  for (int j = 0; j < 8; ++j) x[j] = threadIdx.x * 1e-3f + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[j]) : "v"(a), "v"(b));
  }
  float s = 0;
  for (int j = 0; j < 8; ++j) s += x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk(float* out, int iters, float a, float b) {
  f2 x[8];
  f2 av = {a, a}, bv = {b, b};
  for (int j = 0; j < 8; ++j) x[j] = f2{threadIdx.x * 1e-3f + j, (float)j};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x[j]) : "v"(av), "v"(bv));
  }
  float s = 0;
  for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// packed with the scalar-broadcast form the sphere test would use: one operand from an
// SGPR pair (2 spheres' coordinate), one VGPR lane value broadcast to both halves.
__global__ __launch_bounds__(256) void k_pk_bcast(float* out, int iters, f2 c) {
  f2 x[8];
  float p = threadIdx.x * 1e-3f;
  f2 pv = {p, 0.0f};
  for (int j = 0; j < 8; ++j) x[j] = f2{p + j, (float)j};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(x[j]) : "v"(pv), "s"(c));
  }
  float s = 0;
  for (int j = 0; j < 8; ++j) s += x[j].x + x[j].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  const int blocks = 256 * 4 * 8 / 4;  // 8 waves per SIMD (4 waves per block)
  hipMalloc(&out, sizeof(float) * blocks * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 200000;
  for (int form = 0; form < 3; ++form) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (form == 0) k_fma<<<blocks, 256>>>(out, iters, 1.0000001f, 1e-7f);
      if (form == 1) k_pk<<<blocks, 256>>>(out, iters, 1.0000001f, 1e-7f);
      if (form == 2) k_pk_bcast<<<blocks, 256>>>(out, iters, f2{1e-7f, 2e-7f});
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      double lanes_fma = (double)blocks * 256 * iters * 8 * (form == 0 ? 1 : 2);
      printf("%s rep %d: %.3f ms  %.1f TFLOP/s\n", form == 0 ? "v_fma_f32   " : form == 1 ? "v_pk_fma_f32" : "v_pk_bcast  ",
             rep, ms, 2 * lanes_fma / ms / 1e9);
    }
  }
  return 0;
}
