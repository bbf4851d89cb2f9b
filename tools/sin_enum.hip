// tools/sin_enum.hip — host-side enumeration for the kernels' sin (csrc/rt_sin.h): runs the
// same binary64 evaluation the device runs (sin_binary64: fast path or Payne-Hanek) on every
// finite binary32 bit pattern and prints, one per line in hex, the patterns whose binary64
// value is within kSinAmbUlps ulps of a binary32 rounding boundary (sin_ambiguous).  Those are
// the inputs rt_sin_table.h must hold; tools/gen_sin_table.py computes their correctly
// rounded values with mpmath.  `sin_enum eval` reads hex bit patterns on stdin and prints
// each one's binary64 value (the error checks of tests/test_sin_cpu.py).  Host-only program (hipcc for the __host__ __device__ header).
//   build: hipcc -O2 -std=c++17 -fopenmp -ffp-contract=off -Ireal_time_ray_tracer_amd/csrc tools/sin_enum.hip
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "rt_sin.h"

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'e') {  // "eval": hex bit patterns on stdin -> hex binary64 values
    unsigned b;
    while (scanf("%x", &b) == 1) {
      const double s = rt::sin_binary64(__builtin_bit_cast(float, b));
      printf("%08x %016llx\n", b, (unsigned long long)rt::dbits(s));
    }
    return 0;
  }
  unsigned nt = std::thread::hardware_concurrency();
  if (argc > 1) nt = (unsigned)atoi(argv[1]);
  if (nt == 0) nt = 1;
  std::vector<std::vector<uint32_t>> found(nt);
  std::vector<std::thread> th;
  const uint64_t N = 1ull << 32;
  for (unsigned t = 0; t < nt; ++t) {
    th.emplace_back([&, t] {
      const uint64_t a = N * t / nt, b = N * (t + 1) / nt;
      for (uint64_t u = a; u < b; ++u) {
        const uint32_t bits = (uint32_t)u;
        if ((bits & 0x7F800000u) == 0x7F800000u) continue;  // inf, NaN
        const float x = __builtin_bit_cast(float, bits);
        if (rt::sin_ambiguous(rt::sin_binary64(x))) found[t].push_back(bits);
      }
    });
  }
  for (auto& x : th) x.join();
  size_t n = 0;
  for (auto& f : found)
    for (uint32_t b : f) {
      printf("%08x\n", b);
      ++n;
    }
  fprintf(stderr, "sin_enum: %zu ambiguous bit patterns of 2^32 (window %u ulps)\n", n, rt::kSinAmbUlps);
  return 0;
}
