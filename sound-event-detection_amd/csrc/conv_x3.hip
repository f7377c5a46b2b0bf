// 3x3 conv + folded BN + ReLU (+ pool / freq-mean) on bf16 MFMA with a
// 3-term split: every fp32 operand x = hi + lo (hi = bf16(x), lo = bf16(x - hi)),
// and each 32x32x16 tile accumulates hi*hi + hi*lo + lo*hi in fp32
// (v_mfma_f32_32x32x16_bf16 x3).  Operand representation error <= 2^-17 |x|,
// product error ~2^-16: fp32-class results (parity tests: |d| ~1e-6) at
// 16/3 the fp32-MFMA rate.  Same data layout and epilogues as conv.hip
// (ConvBlock, pytorch/models.py:98-141).
//
// Block = 512 threads (8 waves), output tile 256 pixels x BN channels,
// wave tile 64x64 (BN=128) or 32x64 (BN=64).  K loop = (16-channel chunk,
// tap) units.  Per chunk the (TT+2) x (F+2) halo of the fp32 input is loaded
// to registers, split to bf16 hi/lo and written once to LDS as 64-B pixel
// records [hi k0-7 | hi k8-15 | lo k0-7 | lo k8-15] with the 16-B slots
// XOR-swizzled by position (conflict analysis: DESIGN.md); all 9 taps read it
// with shifted positions.  Weights are pre-split + pre-swizzled on the host
// in the exact LDS image, [ntile][chunk][tap][BN][64 B], and streamed one
// (chunk, tap) unit at a time through a 2-slot LDS ring, prefetched two units
// ahead in registers.  The MFMA row -> pixel map is chosen per epilogue so
// that 2x2 pooling (and the 8-bin freq mean) is an in-lane register sum.
#include "sedx_internal.h"

namespace sedx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t bf16_rne(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

__device__ __forceinline__ void split8(const float4 a, const float4 b, uint4& hi, uint4& lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t hh[8], ll[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    hh[i] = bf16_rne(v[i]);
    ll[i] = bf16_rne(v[i] - __uint_as_float(hh[i] << 16));
  }
  hi = make_uint4(hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16), hh[4] | (hh[5] << 16), hh[6] | (hh[7] << 16));
  lo = make_uint4(ll[0] | (ll[1] << 16), ll[2] | (ll[3] << 16), ll[4] | (ll[5] << 16), ll[6] | (ll[7] << 16));
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// MFMA row R (0..255 of the block tile) -> (t_local, f)
template <int F, int EPI>
__device__ __forceinline__ void rowmap(int R, int& tl, int& f) {
  if (EPI == EPI_POOL2) {            // R = 4q + e: a 2x2 pool group in one lane's regs 4g..4g+3
    const int q = R >> 2, e = R & 3;
    const int tp = q / (F / 2), fp = q % (F / 2);
    tl = 2 * tp + (e >> 1);
    f = 2 * fp + (e & 1);
  } else if (EPI == EPI_FMEAN) {     // F == 8: the 8 bins of a t in regs {4g + 2j + (0,1)}
    const int tile = R >> 5, r = R & 31;
    const int hh = (r >> 2) & 1, i = r & 3, g = r >> 3;
    tl = 4 * tile + 2 * hh + (i >> 1);
    f = 2 * g + (i & 1);
  } else {
    tl = R / F;
    f = R % F;
  }
}

template <int F, int BN, int EPI>
__global__ __launch_bounds__(512) void conv3x3_x3_kernel(const float* __restrict__ in, int T,
                                                         int Cin, int Cout,
                                                         const uint4* __restrict__ wsp,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out) {
  constexpr int BM = 256, TT = BM / F, RT = TT + 2, CS = F + 2;
  // LDS halo image: 80-B pixel records (5 x 16 B) on rows of CSP positions;
  // CSP per (F, epilogue) from the bank-conflict search: every
  // ds_read_b128 of an A fragment is conflict-free and every tap offset is a
  // compile-time immediate.
  constexpr int CSP = (EPI == EPI_POOL2) ? (F == 64 ? 72 : F == 32 ? 40 : 24)
                                         : (F == 64 ? 66 : F == 32 ? 34 : F == 16 ? 32 : 24);
  constexpr int NPOS = RT * CSP;
  constexpr int WAVES_N = BN / 64, WAVES_M = 8 / WAVES_N, WM = BM / WAVES_M;
  constexpr int MT = WM / 32, NT = 2;
  constexpr int A_U4 = NPOS * 5;
  constexpr int W_U4 = BN * 4;
  constexpr int A_ITEMS = RT * CS * 2;
  constexpr int NA = (A_ITEMS + 511) / 512;

  __shared__ uint4 lds[A_U4 + 9 * W_U4];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int h = lane >> 5;
  const int tiles_t = (T + TT - 1) / TT;
  const int b = blockIdx.x / tiles_t;
  const int t0 = (blockIdx.x - b * tiles_t) * TT;
  const int n0 = blockIdx.y * BN;

  int pbase[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int tl, f;
    rowmap<F, EPI>(wm * WM + mt * 32 + (lane & 31), tl, f);
    pbase[mt] = (tl * CSP + f) * 5;
  }
  int bhi[NT], blo[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = wn * 64 + nt * 32 + (lane & 31);
    const int s = (n >> 2) & 3;
    bhi[nt] = n * 4 + (h ^ s);
    blo[nt] = n * 4 + ((2 + h) ^ s);
  }

  f32x16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;

  const float* in_b = in + (int64_t)b * T * F * Cin;
  const int nchunks = Cin >> 4;
  const int nunits = nchunks * 9;
  const uint4* wbase = wsp + (int64_t)blockIdx.y * nunits * W_U4;

  float4 ra[NA][2];

#define SEDX_LOAD_A(chunk)                                                              \
  {                                                                                     \
    const int c0_ = (chunk) * 16;                                                       \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                    \
      const int idx = tid + i * 512;                                                    \
      float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;                             \
      if (idx < A_ITEMS) {                                                              \
        const int pos = idx >> 1, hh = idx & 1;                                         \
        const int r = pos / CS, c = pos - r * CS;                                       \
        const int t = t0 - 1 + r, f = c - 1;                                            \
        if (t >= 0 && t < T && f >= 0 && f < F) {                                       \
          const float4* src = reinterpret_cast<const float4*>(                          \
              in_b + ((int64_t)t * F + f) * Cin + c0_ + 8 * hh);                        \
          v0 = src[0];                                                                  \
          v1 = src[1];                                                                  \
        }                                                                               \
      }                                                                                 \
      ra[i][0] = v0;                                                                    \
      ra[i][1] = v1;                                                                    \
    }                                                                                   \
  }
#define SEDX_STORE_A(buf)                                                               \
  {                                                                                     \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                    \
      const int idx = tid + i * 512;                                                    \
      if (idx < A_ITEMS) {                                                              \
        const int pos = idx >> 1, hh = idx & 1;                                         \
        const int r = pos / CS, c = pos - r * CS;                                       \
        const int rec = (r * CSP + c) * 5;                                              \
        uint4 hi, lo;                                                                   \
        split8(ra[i][0], ra[i][1], hi, lo);                                             \
        (buf)[rec + hh] = hi;                                                           \
        (buf)[rec + 2 + hh] = lo;                                                       \
      }                                                                                 \
    }                                                                                   \
  }

  // LDS: one A halo image + the whole chunk's weights (9 taps); the next
  // chunk is prefetched into registers while this one's 9 x 12 MFMAs run.
  constexpr int WC_U4 = 9 * W_U4;
  constexpr int NW = (WC_U4 + 511) / 512;
  uint4* Abuf = lds;
  uint4* Wbuf = lds + A_U4;
  uint4 rw[NW];
#define SEDX_LOAD_W(chunk)                                                              \
  {                                                                                     \
    const uint4* src_ = wbase + (int64_t)(chunk) * WC_U4;                               \
    _Pragma("unroll") for (int i = 0; i < NW; ++i) {                                    \
      const int idx = tid + i * 512;                                                    \
      rw[i] = (idx < WC_U4) ? src_[idx] : make_uint4(0, 0, 0, 0);                       \
    }                                                                                   \
  }
#define SEDX_STORE_W()                                                                  \
  {                                                                                     \
    _Pragma("unroll") for (int i = 0; i < NW; ++i) {                                    \
      const int idx = tid + i * 512;                                                    \
      if (idx < WC_U4) Wbuf[idx] = rw[i];                                               \
    }                                                                                   \
  }

  SEDX_LOAD_A(0);
  SEDX_LOAD_W(0);
  SEDX_STORE_A(Abuf);
  SEDX_STORE_W();
  __syncthreads();
  if (nchunks > 1) {
    SEDX_LOAD_A(1);
    SEDX_LOAD_W(1);
  }
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    // software pipeline over the 9 taps: fragments of tap t+1 are read from
    // LDS (two register sets, static indices) while tap t's 12 MFMAs issue.
    bf16x8 fa[2][2 * MT], fb[2][2 * NT];
#define SEDX_READ_FRAGS(set, tap_)                                                      \
    {                                                                                   \
      const int toff_ = ((tap_) / 3) * CSP + ((tap_) % 3);                              \
      const uint4* W_ = Wbuf + (tap_) * W_U4;                                           \
      _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                               \
        const uint4* Ap = Abuf + pbase[mt] + toff_ * 5;                                 \
        fa[set][2 * mt] = as_bf16x8(Ap[h]);                                             \
        fa[set][2 * mt + 1] = as_bf16x8(Ap[2 + h]);                                     \
      }                                                                                 \
      _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                               \
        fb[set][2 * nt] = as_bf16x8(W_[bhi[nt]]);                                       \
        fb[set][2 * nt + 1] = as_bf16x8(W_[blo[nt]]);                                   \
      }                                                                                 \
      __builtin_amdgcn_sched_barrier(0);                                                \
    }
#define SEDX_MFMAS(set)                                                                 \
    {                                                                                   \
      _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                 \
      _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                               \
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * mt], fb[set][2 * nt], acc[mt][nt], 0, 0, 0);     \
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * mt], fb[set][2 * nt + 1], acc[mt][nt], 0, 0, 0); \
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * mt + 1], fb[set][2 * nt], acc[mt][nt], 0, 0, 0); \
      }                                                                                 \
    }
    SEDX_READ_FRAGS(0, 0);
    SEDX_READ_FRAGS(1, 1);
    SEDX_MFMAS(0);
    SEDX_READ_FRAGS(0, 2);
    SEDX_MFMAS(1);
    SEDX_READ_FRAGS(1, 3);
    SEDX_MFMAS(0);
    SEDX_READ_FRAGS(0, 4);
    SEDX_MFMAS(1);
    SEDX_READ_FRAGS(1, 5);
    SEDX_MFMAS(0);
    SEDX_READ_FRAGS(0, 6);
    SEDX_MFMAS(1);
    SEDX_READ_FRAGS(1, 7);
    SEDX_MFMAS(0);
    SEDX_READ_FRAGS(0, 8);
    SEDX_MFMAS(1);
    SEDX_MFMAS(0);
#undef SEDX_READ_FRAGS
#undef SEDX_MFMAS
    if (chunk + 1 < nchunks) {
      __syncthreads();
      SEDX_STORE_A(Abuf);
      SEDX_STORE_W();
      __syncthreads();
      if (chunk + 2 < nchunks) {
        SEDX_LOAD_A(chunk + 2);
        SEDX_LOAD_W(chunk + 2);
      }
    }
  }
#undef SEDX_LOAD_W
#undef SEDX_STORE_W
#undef SEDX_LOAD_A
#undef SEDX_STORE_A

  // ---- epilogue straight from the accumulators ----
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = n0 + wn * 64 + nt * 32 + (lane & 31);
    const float bv = bias[n];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int Rbase = wm * WM + mt * 32;
      float r[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = fmaxf(acc[mt][nt][i] + bv, 0.0f);
      if (EPI == EPI_STORE) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          int tl, f;
          rowmap<F, EPI>(Rbase + (i & 3) + 8 * (i >> 2) + 4 * h, tl, f);
          const int t = t0 + tl;
          if (t < T) out[(((int64_t)b * T + t) * F + f) * Cout + n] = r[i];
        }
      } else if (EPI == EPI_POOL2) {
        constexpr int FO = F / 2;
        const int To = T / 2;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int q = (Rbase + 8 * g + 4 * h) >> 2;
          const int tp = q / FO, fp = q % FO;
          const int to = t0 / 2 + tp;
          const float v = (((r[4 * g] + r[4 * g + 1]) + r[4 * g + 2]) + r[4 * g + 3]) * 0.25f;
          if (to < To) out[(((int64_t)b * To + to) * FO + fp) * Cout + n] = v;
        }
      } else {  // EPI_FMEAN, F == 8
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float s = 0.f;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            s += r[4 * g + 2 * j];
            s += r[4 * g + 2 * j + 1];
          }
          const int t = t0 + 4 * (Rbase >> 5) + 2 * h + j;
          if (t < T) out[((int64_t)b * T + t) * Cout + n] = s * 0.125f;
        }
      }
    }
  }
}

template <int F, int BN>
static void launch_x3(const float* in, int B, int T, int Cin, int Cout, const uint4* wp,
                      const float* bias, float* out, int epi, hipStream_t s) {
  constexpr int TT = 256 / F;
  dim3 grid(B * ((T + TT - 1) / TT), Cout / BN);
  if (epi == EPI_STORE)
    hipLaunchKernelGGL((conv3x3_x3_kernel<F, BN, EPI_STORE>), grid, dim3(512), 0, s, in, T, Cin, Cout, wp, bias, out);
  else if (epi == EPI_POOL2)
    hipLaunchKernelGGL((conv3x3_x3_kernel<F, BN, EPI_POOL2>), grid, dim3(512), 0, s, in, T, Cin, Cout, wp, bias, out);
  else
    hipLaunchKernelGGL((conv3x3_x3_kernel<8, BN, EPI_FMEAN>), grid, dim3(512), 0, s, in, T, Cin, Cout, wp, bias, out);
}

void launch_conv3x3_x3(const float* in, int B, int T, int F, int Cin, int Cout, const void* wp,
                       const float* bias, float* out, int epi, hipStream_t s) {
  const uint4* w = static_cast<const uint4*>(wp);
  switch (F) {
    case 64:   // block 1 conv2 (Cout 64)
      launch_x3<64, 64>(in, B, T, Cin, Cout, w, bias, out, epi, s);
      break;
    case 32:
      launch_x3<32, 128>(in, B, T, Cin, Cout, w, bias, out, epi, s);
      break;
    case 16:
      launch_x3<16, 128>(in, B, T, Cin, Cout, w, bias, out, epi, s);
      break;
    case 8:
      launch_x3<8, 128>(in, B, T, Cin, Cout, w, bias, out, epi, s);
      break;
    default: break;
  }
}

}  // namespace sedx
