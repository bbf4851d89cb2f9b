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
int main() {
  float bs[] = {6.0f, 3840.f, 2160.f, 1920.f, 1080.f, 640.f, 480.f, 7680.f, 4320.f, 1000.f, 1234.f};
  unsigned *d; hipMalloc(&d, 8);
  struct R { const char* n; unsigned lo, hi; } rs[] = {{"all normal", 0x00800000u, 0x7f800000u},
     {"[2^-100, 2^100)", 0x0d800000u, 0x71800000u}, {"[2^-40, 2^14)", 0x2b800000u, 0x46800000u}};
  for (auto& R : rs) for (float b : bs) {
    unsigned h[2] = {0, 0xffffffffu}; hipMemcpy(d, h, 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, b, R.lo, R.hi, d, d + 1);
    hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
    printf("%-18s b=%-6g bad=%u first=%a\n", R.n, b, h[0], h[1] == 0xffffffffu ? 0.0f : *(float*)&h[1]);
  }
  return 0;
}
