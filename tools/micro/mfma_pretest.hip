// The batched first bounce's per-ray pre-test (dot(d, q) >= K for 64 rays x 64 spheres) on the
// f32 MFMA (v_mfma_f32_16x16x4_f32), checked bit for bit against the kernels' fmaf chain.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/mfma_pretest.hip -o build/mfma_pretest && build/mfma_pretest
// 1. v_permlane16_swap / v_permlane32_swap lane maps (printed for lanes 0..63);
// 2. the 4x4 row-group transpose built from them;
// 3. C = fma(-1, K, fma(dz, qz, fma(dy, qy, fma(dx, qx, 0)))) from the MFMA equals the host fmaf
//    chain minus K for every (ray, sphere) pair (up to the sign of zero), and the per-sphere
//    "some ray passes" mask equals the host's, over many random batches (including NaN, +-inf,
//    zero-length and near-threshold rows).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ void transpose4(float& r0, float& r1, float& r2, float& r3) {
  // afterwards r_j, lane 16k + p = (before) r_k, lane 16j + p
  auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(r0), __float_as_uint(r2), false, false);
  r0 = __uint_as_float(s[0]); r2 = __uint_as_float(s[1]);
  s = __builtin_amdgcn_permlane32_swap(__float_as_uint(r1), __float_as_uint(r3), false, false);
  r1 = __uint_as_float(s[0]); r3 = __uint_as_float(s[1]);
  s = __builtin_amdgcn_permlane16_swap(__float_as_uint(r0), __float_as_uint(r1), false, false);
  r0 = __uint_as_float(s[0]); r1 = __uint_as_float(s[1]);
  s = __builtin_amdgcn_permlane16_swap(__float_as_uint(r2), __float_as_uint(r3), false, false);
  r2 = __uint_as_float(s[0]); r3 = __uint_as_float(s[1]);
}

__global__ void k_swaps(unsigned* o) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
  auto s = __builtin_amdgcn_permlane32_swap(l, 100u + l, false, false);
  o[l] = r[0]; o[64 + l] = r[1]; o[128 + l] = s[0]; o[192 + l] = s[1];
  float a = (float)l, b = 100.0f + l, c = 200.0f + l, d = 300.0f + l;
  transpose4(a, b, c, d);
  o[256 + l] = (unsigned)a; o[320 + l] = (unsigned)b; o[384 + l] = (unsigned)c; o[448 + l] = (unsigned)d;
}

typedef float v4f __attribute__((ext_vector_type(4)));
// rays: [batch][64] float3 (+pad), rows: [batch][64] float4 (q.xyz, K); out: C [batch][64 ray][64 sphere], mask [batch]
__global__ void k_pretest(const float4* rays, const float4* rows, float* cout, unsigned long long* mout) {
  const int l = threadIdx.x, b = blockIdx.x;
  const float4 d = rays[b * 64 + l], q = rows[b * 64 + l];
  float a0 = d.x, a1 = d.y, a2 = d.z, a3 = -1.0f;
  transpose4(a0, a1, a2, a3);
  float b0 = q.x, b1 = q.y, b2 = q.z, b3 = q.w;
  transpose4(b0, b1, b2, b3);
  const float A[4] = {a0, a1, a2, a3}, B[4] = {b0, b1, b2, b3};
  unsigned long long any = 0;
#pragma unroll
  for (int sb = 0; sb < 4; ++sb) {
    float mx = -INFINITY;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const v4f c = __builtin_amdgcn_mfma_f32_16x16x4f32(A[rb], B[sb], (v4f){0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // C[row = 4 (l >> 4) + r][col = l & 15] of block (rb, sb)
        cout[((size_t)b * 64 + rb * 16 + 4 * (l >> 4) + r) * 64 + sb * 16 + (l & 15)] = c[r];
      }
      mx = fmaxf(mx, fmaxf(fmaxf(c[0], c[1]), fmaxf(c[2], c[3])));
    }
    const unsigned long long bal = __ballot(mx >= 0.0f);
    const unsigned long long g = (bal | bal >> 16 | bal >> 32 | bal >> 48) & 0xffffull;
    any |= g << (16 * sb);
  }
  if (l == 0) mout[b] = any;
}

int main() {
  unsigned* dsw;
  CHECK(hipMalloc(&dsw, 512 * 4));
  k_swaps<<<1, 64>>>(dsw);
  unsigned hsw[512];
  CHECK(hipMemcpy(hsw, dsw, sizeof hsw, hipMemcpyDeviceToHost));
  const char* names[8] = {"pl16 r0", "pl16 r1", "pl32 r0", "pl32 r1", "T r0", "T r1", "T r2", "T r3"};
  for (int t = 0; t < 8; ++t) {
    printf("%-8s", names[t]);
    for (int l = 0; l < 64; l += 4) printf(" %3u", hsw[t * 64 + l]);
    printf("\n");
  }
  int tbad = 0;
  for (int j = 0; j < 4; ++j)
    for (int l = 0; l < 64; ++l)
      tbad += hsw[256 + j * 64 + l] != (unsigned)(100 * (l >> 4) + 16 * j + (l & 15));
  printf("transpose4 mismatches: %d\n", tbad);

  const int NB = 4096;
  std::mt19937 rng(12345);
  std::uniform_real_distribution<float> U(-1.0f, 1.0f);
  std::vector<float4> rays(NB * 64), rows(NB * 64);
  for (int b = 0; b < NB; ++b)
    for (int l = 0; l < 64; ++l) {
      float x = U(rng), y = U(rng), z = U(rng);
      float n = 1.0f / sqrtf(x * x + y * y + z * z);
      rays[b * 64 + l] = make_float4(x * n, y * n, z * n, 0.0f);
      float qx = U(rng), qy = U(rng), qz = U(rng);
      float m = 1.0f / sqrtf(qx * qx + qy * qy + qz * qz);
      float K = 0.6f + 0.4f * U(rng);
      rows[b * 64 + l] = make_float4(qx * m, qy * m, qz * m, K);
    }
  // near-threshold rows: K = the exact chain value of ray 0 (and its neighbours in ulps)
  for (int b = 0; b < NB; b += 3)
    for (int l = 0; l < 64; l += 5) {
      const float4 d = rays[b * 64 + (l * 7) % 64];
      float4& q = rows[b * 64 + l];
      float s = fmaf(d.z, q.z, fmaf(d.y, q.y, d.x * q.x));
      int du = (int)(rng() % 5) - 2;
      unsigned u;
      memcpy(&u, &s, 4);
      u += du;
      memcpy(&q.w, &u, 4);
    }
  // special rows
  rows[5 * 64 + 3].w = NAN; rows[6 * 64 + 4].w = INFINITY; rows[7 * 64 + 5].w = -INFINITY;
  rows[8 * 64 + 6] = make_float4(0, 0, 0, 0.0f); rows[9 * 64 + 7] = make_float4(NAN, 0, 0, 0.5f);
  rays[10 * 64 + 8] = make_float4(0, 0, 0, 0);
  float4 *drays, *drows;
  float* dc;
  unsigned long long* dm;
  CHECK(hipMalloc(&drays, NB * 64 * 16));
  CHECK(hipMalloc(&drows, NB * 64 * 16));
  CHECK(hipMalloc(&dc, (size_t)NB * 64 * 64 * 4));
  CHECK(hipMalloc(&dm, NB * 8));
  CHECK(hipMemcpy(drays, rays.data(), NB * 64 * 16, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(drows, rows.data(), NB * 64 * 16, hipMemcpyHostToDevice));
  k_pretest<<<NB, 64>>>(drays, drows, dc, dm);
  CHECK(hipDeviceSynchronize());
  std::vector<float> c((size_t)NB * 64 * 64);
  std::vector<unsigned long long> m(NB);
  CHECK(hipMemcpy(c.data(), dc, c.size() * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(m.data(), dm, NB * 8, hipMemcpyDeviceToHost));
  long long cbad = 0, mbad = 0, passes = 0;
  for (int b = 0; b < NB; ++b) {
    unsigned long long want = 0;
    for (int r = 0; r < 64; ++r)
      for (int s = 0; s < 64; ++s) {
        const float4 d = rays[b * 64 + r], q = rows[b * 64 + s];
        const float chain = fmaf(d.z, q.z, fmaf(d.y, q.y, d.x * q.x));
        const float ref = fmaf(-1.0f, q.w, chain);
        const float got = c[((size_t)b * 64 + r) * 64 + s];
        const bool same = (std::isnan(ref) && std::isnan(got)) || ref == got;
        if (!same) {
          if (cbad < 5) printf("C mismatch b %d ray %d sphere %d: %a vs %a\n", b, r, s, got, ref);
          ++cbad;
        }
        if ((got >= 0.0f) != (chain >= q.w)) ++cbad;
        if (chain >= q.w) want |= 1ull << s;
      }
    passes += __builtin_popcountll(want);
    if (want != m[b]) {
      if (mbad < 5) printf("mask mismatch b %d: %016llx vs %016llx\n", b, m[b], want);
      ++mbad;
    }
  }
  printf("batches %d, C mismatches %lld, mask mismatches %lld, mean spheres passed %.2f\n", NB, cbad, mbad,
         (double)passes / NB);
  return (tbad || cbad || mbad) ? 1 : 0;
}
