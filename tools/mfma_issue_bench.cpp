// Issue cost of the two fp32 MFMA shapes with VALU work interleaved, as the
// Winograd chunk step uses them: per "chunk" either 16 v_mfma_f32_32x32x2_f32
// (16 accumulator tiles of 16 registers... 8 here, as a row wave) or 32
// v_mfma_f32_16x16x4_f32 (same FLOPs), each variant with NV dependent-free
// VALU ops spread between the MFMAs.  Two waves per SIMD (512-thread
// workgroups, one per CU), 256 workgroups; time per chunk per SIMD in cycles
// at the measured clock, against the matrix pipe's 2048 cycles per chunk.
//   usage: mfma_issue_bench
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NV>
__global__ __launch_bounds__(512, 1) void k32(float* out, int iters) {
  f32x16 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x16{};
  float a = threadIdx.x * 1e-3f, b = 0.5f, v[NV > 0 ? NV : 1];
  for (int i = 0; i < (NV > 0 ? NV : 1); ++i) v[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      acc[j & 7] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j & 7], 0, 0, 0);
      if constexpr (NV > 0) {
#pragma unroll
        for (int q = 0; q < NV / 16; ++q) {
          const int i = (j * (NV / 16) + q) % NV;
          v[i] = v[i] * 1.0001f + 0.5f;
          asm volatile("" : "+v"(v[i]));
        }
      }
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0];
  for (int i = 0; i < (NV > 0 ? NV : 1); ++i) s += v[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int NV>
__global__ __launch_bounds__(512, 1) void k16(float* out, int iters) {
  f32x4 acc[32];
  for (int i = 0; i < 32; ++i) acc[i] = f32x4{};
  float a = threadIdx.x * 1e-3f, b = 0.5f, v[NV > 0 ? NV : 1];
  for (int i = 0; i < (NV > 0 ? NV : 1); ++i) v[i] = a + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
      if constexpr (NV > 0) {
        if (j % 2 == 0) {
#pragma unroll
          for (int q = 0; q < NV / 16; ++q) {
            const int i = ((j / 2) * (NV / 16) + q) % NV;
            v[i] = v[i] * 1.0001f + 0.5f;
            asm volatile("" : "+v"(v[i]));
          }
        }
      }
    }
  }
  float s = 0.f;
  for (int i = 0; i < 32; ++i) s += acc[i][0];
  for (int i = 0; i < (NV > 0 ? NV : 1); ++i) s += v[i];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <typename K>
static float run(K kern, float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, iters);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, out, iters);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  const int iters = 4000;
  // per chunk per SIMD: 2 waves x 16 x 64 cycles = 2048 matrix-pipe cycles
  auto report = [&](const char* name, float ms) {
    const double cyc = ms * 1e-3 * 2.4e9 / iters;   // at 2.4 GHz
    printf("%-34s %.3f ms  %.0f cycles per chunk per SIMD (pipe-bound 2048) -> %.3f of the pipe\n", name, ms, cyc,
           2048.0 / cyc);
  };
  report("32x32x2 x16, no VALU", run(k32<0>, out, iters));
  report("32x32x2 x16, 16 VALU", run(k32<16>, out, iters));
  report("32x32x2 x16, 32 VALU", run(k32<32>, out, iters));
  report("32x32x2 x16, 64 VALU", run(k32<64>, out, iters));
  report("16x16x4 x32, no VALU", run(k16<0>, out, iters));
  report("16x16x4 x32, 16 VALU", run(k16<16>, out, iters));
  report("16x16x4 x32, 32 VALU", run(k16<32>, out, iters));
  report("16x16x4 x32, 64 VALU", run(k16<64>, out, iters));
  printf("(%s)\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
