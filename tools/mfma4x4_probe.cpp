// v_mfma_f32_4x4x1f32 (16 blocks): operand / result lane layout and
// arithmetic, measured.  Assumed layout: lane l = 4 b + t (block b = l / 4,
// t = l % 4); A[i = t][0] of block b from lane l; B[0][j = t] of block b from
// lane l; D[i][j = t] of block b in lane l, register i.  A chain of 9 MFMAs
// from zero (a_k, b_k per lane) must then equal, bit for bit, the fma chain
// d[i] = fma(a_k of lane 4b + i, b_k of lane l, d[i]) for k = 0..8 — the
// operation order of block 1's VALU conv1 (conv_wino.hip).
//   usage: mfma4x4_probe   (exit 0 when every element matches)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const float* a, const float* b, float* d, int n) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < n; ++k) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[k * 64 + l], b[k * 64 + l], acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) d[l * 4 + i] = acc[i];
}

int main() {
  const int n = 9, trials = 200;
  std::mt19937 rng(5);
  std::normal_distribution<float> nd(0.f, 1.f);
  float *da, *db, *dd;
  hipMalloc(&da, n * 64 * 4);
  hipMalloc(&db, n * 64 * 4);
  hipMalloc(&dd, 64 * 4 * 4);
  size_t bad = 0, total = 0;
  for (int t = 0; t < trials; ++t) {
    std::vector<float> a(n * 64), b(n * 64), d(256);
    for (auto& v : a) v = nd(rng) * (t % 3 ? 1.f : 1e3f);
    for (auto& v : b) v = nd(rng) * (t % 5 ? 1.f : 1e-3f);
    hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, dd, n);
    hipMemcpy(d.data(), dd, d.size() * 4, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
      const int blk = l / 4;
      for (int i = 0; i < 4; ++i) {
        float e = 0.f;
        for (int k = 0; k < n; ++k) e = std::fmaf(a[k * 64 + 4 * blk + i], b[k * 64 + l], e);
        uint32_t u1, u2;
        memcpy(&u1, &e, 4);
        memcpy(&u2, &d[l * 4 + i], 4);
        bad += u1 != u2;
        ++total;
        if (u1 != u2 && bad <= 5)
          printf("trial %d lane %d reg %d: mfma %.9g fma-chain %.9g\n", t, l, i, d[l * 4 + i], e);
      }
    }
  }
  printf("v_mfma_f32_4x4x1f32 vs the fma chain with the assumed layout: %zu of %zu elements differ (%s)\n", bad,
         total, hipGetErrorString(hipGetLastError()));
  return bad ? 1 : 0;
}
