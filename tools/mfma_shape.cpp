// Micro-benchmark for the next conv core: the x3 split-bf16 tap body in three
// MFMA forms at equal MACs per CU, with every fragment read from LDS
// (ds_read_b128, conflict-free lane-linear images of random bf16) and one
// barrier per 3 taps, as in conv_x3.hip:
//   V0  32x32x16, 8 waves, 64x64 wave tile: per tap 4 A + 4 B reads, 12 MFMAs
//       (hi*hi, hi*lo, lo*hi per 32x32 block)  -- the current kernel
//   V1  16x16x32, 8 waves, 64x64 wave tile: per tap 4 A + 4 B reads and 16
//       MFMAs on [hiA|loA]x[hiB|hiB]; per tap pair 4 more B reads ([loB t|loB t+1])
//       and 16 MFMAs whose A side [hiA t|hiA t+1] is built by v_permlane32_swap
//   V2  32x32x16, 4 waves (one per SIMD), 128x64 wave tile: per tap 8 A + 4 B
//       reads, 24 MFMAs
//   V3  32x32x16, 4 waves, 128x128 wave tile, half the tap count per launch
//       (equal MACs): per tap 8 A + 8 B reads, 48 MFMAs
// Prints TF/s (useful x3 MACs: 1/3 of the bf16 MFMA work) and the in-kernel
// clock (s_memtime / s_memrealtime).  Random operands: the clock the chip
// holds depends on data (MI355X_MICROARCH.md, DVFS notes).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ unsigned long long g_clk[2];

__device__ __forceinline__ bf16x8 bf(uint4 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ uint4 swap_lo(uint4 x, uint4 y) {   // [x lanes 0-31 | y lanes 0-31]
  auto a = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
  auto b = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
  auto c = __builtin_amdgcn_permlane32_swap(x.z, y.z, false, false);
  auto d = __builtin_amdgcn_permlane32_swap(x.w, y.w, false, false);
  return make_uint4(a[0], b[0], c[0], d[0]);
}

constexpr int LDS_U4 = 8192;   // 128 KB: one workgroup per CU

template <int V>
__global__ __launch_bounds__(V >= 2 ? 256 : 512) void body(const uint4* __restrict__ src, float* out,
                                                           int iters) {
  __shared__ uint4 lds[LDS_U4];
  constexpr int NT = V >= 2 ? 256 : 512;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < LDS_U4; i += NT) lds[i] = src[(blockIdx.x * 977 + i) & (LDS_U4 * 4 - 1)];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  // fragment f of tap t: 64 lanes x 16 B at a tap/fragment dependent offset
  auto rd = [&](int t, int f) { return lds[((t * 13 + f * 5 + wave * 3) & 127) * 64 + lane]; };
  float sink = 0.f;
  if constexpr (V == 0) {
    f32x16 acc[2][2] = {};
    uint4 fa[2][4], fb[2][4];
#pragma unroll
    for (int f = 0; f < 4; ++f) { fa[0][f] = rd(0, f); fb[0][f] = rd(0, 4 + f); }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        const int c = t & 1, n = c ^ 1, tt = it * 6 + t + 1;
#pragma unroll
        for (int f = 0; f < 4; ++f) { fa[n][f] = rd(tt, f); fb[n][f] = rd(tt, 4 + f); }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m]), bf(fb[c][2 * q]), acc[m][q], 0, 0, 0);
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m]), bf(fb[c][2 * q + 1]), acc[m][q], 0, 0, 0);
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m + 1]), bf(fb[c][2 * q]), acc[m][q], 0, 0, 0);
          }
        if (t % 3 == 2) __syncthreads();
      }
    }
    for (int m = 0; m < 2; ++m)
      for (int q = 0; q < 2; ++q)
        for (int r = 0; r < 16; ++r) sink += acc[m][q][r];
  } else if constexpr (V == 1) {
    f32x4 acc[4][4] = {};
    uint4 fa[2][4], fb[2][4], fl[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) { fa[0][f] = rd(0, f); fb[0][f] = rd(0, 4 + f); }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        const int c = t & 1, n = c ^ 1, tt = it * 6 + t + 1;
#pragma unroll
        for (int f = 0; f < 4; ++f) { fa[n][f] = rd(tt, f); fb[n][f] = rd(tt, 4 + f); }
        if (c == 1) {
#pragma unroll
          for (int f = 0; f < 4; ++f) fl[f] = rd(tt, 8 + f);   // [loB t-1 | loB t]
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(fa[c][m]), bf(fb[c][q]), acc[m][q], 0, 0, 0);
        if (c == 1) {   // hi*lo of taps t-1, t: A side from the two hi halves in registers
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const uint4 ap = swap_lo(fa[0][m], fa[1][m]);
#pragma unroll
            for (int q = 0; q < 4; ++q)
              acc[m][q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf(ap), bf(fl[q]), acc[m][q], 0, 0, 0);
          }
        }
        if (t % 3 == 2) __syncthreads();
      }
    }
    for (int m = 0; m < 4; ++m)
      for (int q = 0; q < 4; ++q)
        for (int r = 0; r < 4; ++r) sink += acc[m][q][r];
  } else if constexpr (V == 3) {
    f32x16 acc[4][4] = {};
    uint4 fa[2][8], fb[2][8];
#pragma unroll
    for (int f = 0; f < 8; ++f) { fa[0][f] = rd(0, f); fb[0][f] = rd(0, 8 + f); }
    for (int it = 0; it < iters / 2; ++it) {
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        const int c = t & 1, n = c ^ 1, tt = it * 6 + t + 1;
#pragma unroll
        for (int f = 0; f < 8; ++f) { fa[n][f] = rd(tt, f); fb[n][f] = rd(tt, 8 + f); }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m]), bf(fb[c][2 * q]), acc[m][q], 0, 0, 0);
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m]), bf(fb[c][2 * q + 1]), acc[m][q], 0, 0, 0);
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m + 1]), bf(fb[c][2 * q]), acc[m][q], 0, 0, 0);
          }
        if (t % 3 == 2) __syncthreads();
      }
    }
    for (int m = 0; m < 4; ++m)
      for (int q = 0; q < 4; ++q)
        for (int r = 0; r < 16; ++r) sink += acc[m][q][r];
  } else {
    f32x16 acc[4][2] = {};
    uint4 fa[2][8], fb[2][4];
#pragma unroll
    for (int f = 0; f < 8; ++f) fa[0][f] = rd(0, f);
#pragma unroll
    for (int f = 0; f < 4; ++f) fb[0][f] = rd(0, 8 + f);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        const int c = t & 1, n = c ^ 1, tt = it * 6 + t + 1;
#pragma unroll
        for (int f = 0; f < 8; ++f) fa[n][f] = rd(tt, f);
#pragma unroll
        for (int f = 0; f < 4; ++f) fb[n][f] = rd(tt, 8 + f);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m]), bf(fb[c][2 * q]), acc[m][q], 0, 0, 0);
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m]), bf(fb[c][2 * q + 1]), acc[m][q], 0, 0, 0);
            acc[m][q] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf(fa[c][2 * m + 1]), bf(fb[c][2 * q]), acc[m][q], 0, 0, 0);
          }
        if (t % 3 == 2) __syncthreads();
      }
    }
    for (int m = 0; m < 4; ++m)
      for (int q = 0; q < 2; ++q)
        for (int r = 0; r < 16; ++r) sink += acc[m][q][r];
  }
  if (tid == 0) {
    atomicAdd(&g_clk[0], __builtin_amdgcn_s_memtime() - t0);
    atomicAdd(&g_clk[1], __builtin_amdgcn_s_memrealtime() - r0);
  }
  out[blockIdx.x * NT + tid] = sink;
}

template <int V>
static void run(const uint4* src, float* out, int ncu, int iters, int reps) {
  const int nt = V >= 2 ? 256 : 512;
  hipLaunchKernelGGL(body<V>, dim3(ncu), dim3(nt), 0, 0, src, out, iters);   // warm
  (void)hipDeviceSynchronize();
  unsigned long long z[2] = {0, 0};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_clk), z, sizeof(z));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(body<V>, dim3(ncu), dim3(nt), 0, 0, src, out, iters);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipMemcpyFromSymbol(z, HIP_SYMBOL(g_clk), sizeof(z));
  // useful MACs per CU per tap: 64x64 wave tile x 16 channels x 8 waves
  const double macs = (double)ncu * reps * iters * 6 * 8 * 64 * 64 * 16;
  printf("V%d  %.3f ms/launch  %.1f TF/s (x3-useful)  clock %.2f GHz  err=%s\n", V, ms / reps,
         2 * macs / (ms * 1e-3) / 1e12, (double)z[0] / (double)z[1] * 0.1, hipGetErrorString(hipGetLastError()));
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  std::vector<unsigned> h(LDS_U4 * 4 * 4);
  srand(7);
  for (auto& v : h) v = ((rand() & 0x7fff) | 0x3c00u) * 0x10001u ^ (rand() & 0x80008000u);
  uint4* src;
  float* out;
  (void)hipMalloc(&src, h.size() * 4);
  (void)hipMalloc(&out, (size_t)ncu * 512 * 4);
  (void)hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  for (int k = 0; k < 2; ++k) {
    run<0>(src, out, ncu, iters, reps);
    run<1>(src, out, ncu, iters, reps);
    run<2>(src, out, ncu, iters, reps);
    run<3>(src, out, ncu, iters, reps);
  }
  return 0;
}
