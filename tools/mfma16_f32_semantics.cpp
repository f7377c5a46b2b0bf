// Is v_mfma_f32_16x16x4_f32 an fma chain over k = 0..3?  D(i,j) = C(i,j) +
// sum_k A(i,k) B(k,j); candidates evaluated with IEEE fmaf on the host.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(const float* A, const float* Bm, const float* C, float* D, int tiles) {
  const int lane = threadIdx.x, t = blockIdx.x;
  if (t >= tiles) return;
  const float* a = A + t * 64;   // [16 i][4 k]
  const float* b = Bm + t * 64;  // [4 k][16 j]
  const float* c = C + t * 256;  // [16][16]
  float* d = D + t * 256;
  const int i = lane & 15, k = lane >> 4;
  f32x4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = c[(4 * k + r) * 16 + i];
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i * 4 + k], b[k * 16 + i], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[(4 * k + r) * 16 + i] = acc[r];
}

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 16384;
  std::mt19937 rng(7);
  const char* names[] = {"chain k0..k3", "chain k3..k0", "((c+p0)+p1)+.. rounded products", "pairs (p0+p1)+(p2+p3) fma-free"};
  for (int spread = 0; spread < 4; ++spread) {
    std::vector<float> A(tiles * 64), Bv(tiles * 64), C(tiles * 256), D(tiles * 256);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::uniform_int_distribution<int> e(-spread * 8, spread * 8);
    for (auto& x : A) x = std::ldexp(u(rng), e(rng));
    for (auto& x : Bv) x = std::ldexp(u(rng), e(rng));
    for (auto& x : C) x = std::ldexp(u(rng), e(rng));
    if (spread == 3)
      for (int t = 0; t < tiles; ++t)
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            float p = 0;
            for (int k = 0; k < 4; ++k) p += A[t * 64 + i * 4 + k] * Bv[t * 64 + k * 16 + j];
            C[t * 256 + i * 16 + j] = -p * (1.0f + std::ldexp(u(rng), -20));
          }
    float *dA, *dB, *dC, *dD;
    (void)hipMalloc(&dA, A.size() * 4); (void)hipMalloc(&dB, Bv.size() * 4);
    (void)hipMalloc(&dC, C.size() * 4); (void)hipMalloc(&dD, D.size() * 4);
    (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, Bv.data(), Bv.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(tiles), dim3(64), 0, 0, dA, dB, dC, dD, tiles);
    (void)hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    long mism[4] = {0};
    for (int t = 0; t < tiles; ++t)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          float a[4], b[4];
          for (int k = 0; k < 4; ++k) { a[k] = A[t * 64 + i * 4 + k]; b[k] = Bv[t * 64 + k * 16 + j]; }
          const float c = C[t * 256 + i * 16 + j], d = D[t * 256 + i * 16 + j];
          float cand[4];
          cand[0] = c; for (int k = 0; k < 4; ++k) cand[0] = fmaf(a[k], b[k], cand[0]);
          cand[1] = c; for (int k = 3; k >= 0; --k) cand[1] = fmaf(a[k], b[k], cand[1]);
          { volatile float s = c; for (int k = 0; k < 4; ++k) { volatile float p = a[k] * b[k]; s = s + p; } cand[2] = s; }
          { volatile float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2], p3 = a[3] * b[3];
            volatile float s01 = p0 + p1, s23 = p2 + p3; volatile float s = s01 + s23; cand[3] = c + s; }
          for (int h = 0; h < 4; ++h) mism[h] += memcmp(&cand[h], &d, 4) != 0;
        }
    printf("spread %d (%d elements):", spread, tiles * 256);
    for (int h = 0; h < 4; ++h) printf("  [%s] %ld", names[h], mism[h]);
    printf("\n");
    (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dC); (void)hipFree(dD);
  }
  return 0;
}
