#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(float b, unsigned lo, unsigned hi, unsigned* bad, unsigned* first) {
  const float y = 1.0f / b;
  for (unsigned long long u = lo + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; u < hi; u += (unsigned long long)gridDim.x * blockDim.x) {
    float a = __uint_as_float((unsigned)u);
    float q = a * y;
    float r = fmaf(-b, q, a);
    float q1 = fmaf(r, y, q);
    if (__float_as_uint(q1) != __float_as_uint(a / b)) { atomicAdd(bad, 1u); atomicMin(first, (unsigned)u); }
  }
}
// Markstein's refinement with a variable divisor: y = RN(1/b) (as the kernels get it), for
// pseudo-random normal b (every mantissa pattern class, exponents in [-60, 60]) and random a in
// [2^-60, 2^60): count q' != a / b.
__device__ unsigned hash32(unsigned long long x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (unsigned)x;
}
__global__ void kr(unsigned long long n, unsigned* bad) {
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (unsigned long long)gridDim.x * blockDim.x) {
    const unsigned hb = hash32(2 * i + 1), ha = hash32(2 * i + 2);
    const float b = __uint_as_float(((67u + (hb >> 25)) << 23 | (hb & 0x7fffffu)) ^ ((hb & 0x400000u) << 9));  // exp 2^-60..2^67, random sign
    const float a = __uint_as_float((67u + (ha >> 25)) << 23 | (ha & 0x7fffffu));
    const float y = 1.0f / b;
    const float q = a * y;
    const float r = fmaf(-b, q, a);
    const float q1 = fmaf(r, y, q);
    if (__float_as_uint(q1) != __float_as_uint(a / b)) atomicAdd(bad, 1u);
  }
}
int main() {
  float bs[] = {6.0f, 1.7f, 3840.f, 2160.f, 1920.f, 1080.f, 640.f, 480.f, 7680.f, 4320.f, 1000.f, 1234.f};
  unsigned *d; hipMalloc(&d, 8);
  struct R { const char* n; unsigned lo, hi; } rs[] = {{"all normal", 0x00800000u, 0x7f800000u},
     {"[2^-100, 2^100)", 0x0d800000u, 0x71800000u}, {"[2^-40, 2^14)", 0x2b800000u, 0x46800000u}};
  for (auto& R : rs) for (float b : bs) {
    unsigned h[2] = {0, 0xffffffffu}; hipMemcpy(d, h, 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, b, R.lo, R.hi, d, d + 1);
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("%-18s b=%-6g bad=%u first=%a\n", R.n, b, h[0], h[1] == 0xffffffffu ? 0.0f : *(float*)&h[1]);
  }
  {
    unsigned h[2] = {0, 0}; hipMemcpy(d, h, 8, hipMemcpyHostToDevice);
    const unsigned long long n = 1ull << 32;
    hipLaunchKernelGGL(kr, dim3(16384), dim3(256), 0, 0, n, d);
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("random b, a (2^32 pairs, |b| in [2^-60, 2^68), a in [2^-60, 2^68)) bad=%u\n", h[0]);
  }
  return 0;
}
