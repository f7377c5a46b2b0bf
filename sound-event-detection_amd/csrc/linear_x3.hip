// C = act(A W^T + b) on bf16 MFMA with the 3-term split (same arithmetic as
// conv_x3.hip: x = hi + lo, hi*hi + hi*lo + lo*hi accumulated in fp32).
// Used by the x3 precision mode for the GRU input projection (both
// directions), MHA q|k|v and fc + ReLU, and the AttBlock att|cla 1x1 convs
// (pytorch/models.py:614-615, :823-877, :161-175).
//
// Block = 256 threads (4 waves, 2 x 2), tile 128 x BN (BN 128: 64 x 64 wave
// tiles; BN 64: 64 x 32).  K in chunks of 32 (two 16-k MFMA steps): A (fp32,
// row-major [M][K]) is split to hi/lo in registers and written to LDS as 80-B
// row records per k-step (conflict-free A-fragment reads); W is pre-split and
// pre-swizzled on the host ([N/BN][K/16][BN][64 B], slot c at c ^ ((n>>2)&3),
// the conv weight layout with one tap).  Double-buffered LDS, next chunk
// prefetched in registers, one barrier per chunk.
#include "sedx_internal.h"

namespace sedx {

typedef float lx_f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 lx_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 lx_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void lx_split2(float x0, float x1, uint32_t& hi, uint32_t& lo) {
  const lx_bf16x2 h = {(__bf16)x0, (__bf16)x1};
  hi = __builtin_bit_cast(uint32_t, h);
  const lx_bf16x2 l = {(__bf16)(x0 - __uint_as_float(hi << 16)), (__bf16)(x1 - __uint_as_float(hi & 0xFFFF0000u))};
  lo = __builtin_bit_cast(uint32_t, l);
}

template <int BN, int ACT>
__global__ __launch_bounds__(256) void linear_x3_kernel(const float* __restrict__ A, int M, int K,
                                                        const uint4* __restrict__ Wp, int N,
                                                        const float* __restrict__ bias,
                                                        float* __restrict__ C) {
  constexpr int BM = 128;
  constexpr int NT = BN / 64;                  // 32-col MFMA tiles per wave (wave cols = BN/2)
  constexpr int A_U4 = 2 * BM * 5;             // two k-steps of 80-B row records
  constexpr int W_U4 = 2 * BN * 4;             // two k-steps of 64-B column records
  __shared__ uint4 lds[2 * (A_U4 + W_U4)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5;
  const int m0 = blockIdx.x * BM, nb = blockIdx.y;
  const int nk = K / 32;

  // A staging: thread -> (row, 8-float group g of the 32-k chunk); 2 items
  float4 ra[2][2];
  int arow[2], ag[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + 256 * i;             // 512 = 128 rows x 4 groups
    arow[i] = idx >> 2;
    ag[i] = idx & 3;
  }
  const uint4* wsrc = Wp + (int64_t)nb * (K / 16) * BN * 4;
  constexpr int NW = W_U4 / 256;               // uint4 per thread per chunk (2 or 4)

  // staged in named registers (an indexed array here ended up in scratch)
  uint4 rw0, rw1, rw2, rw3;
#define LX_LOAD(kc)                                                                     \
  {                                                                                     \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                     \
      const int m = min(m0 + arow[i], M - 1);                                           \
      const float4* p = reinterpret_cast<const float4*>(A + (int64_t)m * K + (kc) * 32 + 8 * ag[i]); \
      ra[i][0] = p[0];                                                                  \
      ra[i][1] = p[1];                                                                  \
    }                                                                                   \
    const uint4* w_ = wsrc + (int64_t)(kc) * W_U4 + tid;                                \
    rw0 = w_[0];                                                                        \
    rw1 = w_[256];                                                                      \
    if (NW > 2) {                                                                       \
      rw2 = w_[512];                                                                    \
      rw3 = w_[768];                                                                    \
    }                                                                                   \
    asm volatile("" ::: "memory");                                                      \
  }
#define LX_STORE(buf)                                                                   \
  {                                                                                     \
    uint4* As_ = lds + (buf) * (A_U4 + W_U4);                                           \
    uint4* Ws_ = As_ + A_U4;                                                            \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                     \
      const int ks = ag[i] >> 1, hh = ag[i] & 1;                                        \
      uint4 hi, lo;                                                                     \
      lx_split2(ra[i][0].x, ra[i][0].y, hi.x, lo.x);                                    \
      lx_split2(ra[i][0].z, ra[i][0].w, hi.y, lo.y);                                    \
      lx_split2(ra[i][1].x, ra[i][1].y, hi.z, lo.z);                                    \
      lx_split2(ra[i][1].z, ra[i][1].w, hi.w, lo.w);                                    \
      const int rec = (ks * BM + arow[i]) * 5;                                          \
      As_[rec + hh] = hi;                                                               \
      As_[rec + 2 + hh] = lo;                                                           \
    }                                                                                   \
    Ws_[tid] = rw0;                                                                     \
    Ws_[tid + 256] = rw1;                                                               \
    if (NW > 2) {                                                                       \
      Ws_[tid + 512] = rw2;                                                             \
      Ws_[tid + 768] = rw3;                                                             \
    }                                                                                   \
  }

  lx_f32x16 acc[2][NT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

  LX_LOAD(0);
  LX_STORE(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    if (kc + 1 < nk) LX_LOAD(kc + 1);
    const uint4* As = lds + (kc & 1) * (A_U4 + W_U4);
    const uint4* Ws = As + A_U4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      lx_bf16x8 ahi[2], alo[2], bhi[NT], blo[NT];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int rec = (ks * BM + wm * 64 + mt * 32 + (lane & 31)) * 5;
        ahi[mt] = __builtin_bit_cast(lx_bf16x8, As[rec + h]);
        alo[mt] = __builtin_bit_cast(lx_bf16x8, As[rec + 2 + h]);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = wn * (BN / 2) + nt * 32 + (lane & 31);
        const int sw = (n >> 2) & 3;
        bhi[nt] = __builtin_bit_cast(lx_bf16x8, Ws[(ks * BN + n) * 4 + (h ^ sw)]);
        blo[nt] = __builtin_bit_cast(lx_bf16x8, Ws[(ks * BN + n) * 4 + ((2 + h) ^ sw)]);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[mt], bhi[nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi[mt], blo[nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo[mt], bhi[nt], acc[mt][nt], 0, 0, 0);
        }
    }
    if (kc + 1 < nk) LX_STORE((kc + 1) & 1);
    __syncthreads();
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = nb * BN + wn * (BN / 2) + nt * 32 + (lane & 31);
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) {
          float v = acc[mt][nt][r] + bv;
          if (ACT == 1) v = fmaxf(v, 0.f);
          C[(int64_t)m * N + n] = v;
        }
      }
  }
#undef LX_LOAD
#undef LX_STORE
}

void launch_linear_x3(const float* A, int M, int K, const void* Wp, int N, int BN, const float* bias,
                      float* C, int act, hipStream_t s) {
  const uint4* w = static_cast<const uint4*>(Wp);
  const dim3 grid((M + 127) / 128, N / BN);
  if (BN == 128) {
    if (act)
      launch_kernel(linear_x3_kernel<128, 1>, grid, 256, s, A, M, K, w, N, bias, C);
    else
      launch_kernel(linear_x3_kernel<128, 0>, grid, 256, s, A, M, K, w, N, bias, C);
  } else {
    if (act)
      launch_kernel(linear_x3_kernel<64, 1>, grid, 256, s, A, M, K, w, N, bias, C);
    else
      launch_kernel(linear_x3_kernel<64, 0>, grid, 256, s, A, M, K, w, N, bias, C);
  }
}

}  // namespace sedx
