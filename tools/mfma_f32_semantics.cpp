// Which VALU expression reproduces v_mfma_f32_32x32x2_f32 bit for bit?
// D(i,j) = C(i,j) + A(i,0) B(0,j) + A(i,1) B(1,j).  Random operands over
// several exponent spreads (incl. cancellation); candidates evaluated on the
// host with IEEE fmaf / float ops; mismatch counts per candidate printed.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void mfma_probe(const float* A, const float* Bm, const float* C, float* D, int tiles) {
  const int lane = threadIdx.x, t = blockIdx.x;
  if (t >= tiles) return;
  const float* a = A + t * 64;   // [32 i][2 k]
  const float* b = Bm + t * 64;  // [2 k][32 j]
  const float* c = C + t * 1024; // [32][32]
  float* d = D + t * 1024;
  const int i = lane & 31, k = lane >> 5;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = c[((r & 3) + 8 * (r >> 2) + 4 * k) * 32 + i];
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i * 2 + k], b[k * 32 + i], acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) d[((r & 3) + 8 * (r >> 2) + 4 * k) * 32 + i] = acc[r];
}

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? atoi(argv[1]) : 4096;
  std::mt19937 rng(7);
  const char* names[] = {"fma(a1,b1,fma(a0,b0,c))", "fma(a0,b0,fma(a1,b1,c))", "c+(a0b0+a1b1) 1 rounding",
                         "(a0b0+a1b1)_f32 + c", "fma(a0,b0,c)+a1b1_f32", "(c+a0b0)_r + a1b1 (2 product roundings)"};
  for (int spread = 0; spread < 4; ++spread) {
    std::vector<float> A(tiles * 64), Bv(tiles * 64), C(tiles * 1024), D(tiles * 1024);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::uniform_int_distribution<int> e(-spread * 8, spread * 8);
    for (auto& x : A) x = std::ldexp(u(rng), e(rng));
    for (auto& x : Bv) x = std::ldexp(u(rng), e(rng));
    for (auto& x : C) x = std::ldexp(u(rng), e(rng));
    if (spread == 3)   // cancellation: c ~ -(a0b0 + a1b1)
      for (int t = 0; t < tiles; ++t)
        for (int i = 0; i < 32; ++i)
          for (int j = 0; j < 32; ++j) {
            const float p = A[t * 64 + i * 2] * Bv[t * 64 + j] + A[t * 64 + i * 2 + 1] * Bv[t * 64 + 32 + j];
            C[t * 1024 + i * 32 + j] = -p * (1.0f + std::ldexp(u(rng), -20));
          }
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, Bv.size() * 4); hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, Bv.data(), Bv.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mfma_probe, dim3(tiles), dim3(64), 0, 0, dA, dB, dC, dD, tiles);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    long mism[6] = {0};
    for (int t = 0; t < tiles; ++t)
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          const float a0 = A[t * 64 + i * 2], a1 = A[t * 64 + i * 2 + 1];
          const float b0 = Bv[t * 64 + j], b1 = Bv[t * 64 + 32 + j];
          const float c = C[t * 1024 + i * 32 + j], d = D[t * 1024 + i * 32 + j];
          float cand[6];
          cand[0] = fmaf(a1, b1, fmaf(a0, b0, c));
          cand[1] = fmaf(a0, b0, fmaf(a1, b1, c));
          {  // exact a0b0 + a1b1 + c rounded once (long double holds the products exactly; sum of 3 may round
             // in 64-bit mantissa only far beyond fp32 precision)
            long double s = (long double)a0 * b0 + (long double)a1 * b1 + (long double)c;
            cand[2] = (float)s;
          }
          cand[3] = (float)(a0 * b0 + a1 * b1) + c;
          { volatile float p1 = a1 * b1; cand[4] = fmaf(a0, b0, c) + p1; }
          { volatile float p0 = a0 * b0, p1 = a1 * b1; volatile float s = c + p0; cand[5] = s + p1; }
          for (int h = 0; h < 6; ++h) mism[h] += memcmp(&cand[h], &d, 4) != 0;
        }
    printf("spread %d (%d elements):", spread, tiles * 1024);
    for (int h = 0; h < 6; ++h) printf("  [%s] %ld", names[h], mism[h]);
    printf("\n");
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
  }
  return 0;
}
