// 9-layer CNN conv kernels for gfx950 (ConvBlock, pytorch/models.py:98-141).
//
// Activations are channels-last: [B][T][F][C].  Every 3x3 conv (pad 1, no
// bias) is followed by eval-BN (folded into the weights + a per-channel bias
// at load time) and ReLU, then an epilogue:
//   EPI_STORE  full resolution (conv1 of blocks 2..4)
//   EPI_POOL2  avg_pool2d(2x2), floor on odd T (conv2 of blocks 1..3)
//   EPI_FMEAN  pool 1x1 + torch.mean over the 8 freq bins (conv2 of block 4,
//              models.py:666-668)
//
// conv3x3_kernel is an implicit GEMM: M = output pixels (a tile = TT rows of
// t x all F freq bins = 128 pixels), N = output channels (BN), K = 9 taps x Cin.
// Per 8-channel chunk the (TT+2) x (F+2) halo of the input is staged in LDS
// once (k-major planes, zero halo) and re-read by all 9 taps; the packed
// weight slab [9][8][BN] is staged beside it; the next chunk is prefetched
// into registers while the MFMAs of the current one run.  Math is exact fp32
// on v_mfma_f32_32x32x2_f32 (lane l: A[pixel l&31][k l>>5], B[k l>>5][n l&31]).
#include "sedx_internal.h"

namespace sedx {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// block-1 conv1 (Cin = 1): pure streaming, 64 output channels per pixel.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_c1_kernel(const float* __restrict__ x0, int B, int T,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias,
                                                      float* __restrict__ out) {
  const int cg = threadIdx.x & 15;  // channels 4cg .. 4cg+3
  float wr[4][9], br[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    br[c] = bias[4 * cg + c];
#pragma unroll
    for (int k = 0; k < 9; ++k) wr[c][k] = w[(4 * cg + c) * 9 + k];
  }
  const int64_t npix = (int64_t)B * T * 64;
  for (int64_t pix = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4; pix < npix;
       pix += ((int64_t)gridDim.x * 256) >> 4) {
    const int f = (int)(pix & 63);
    const int64_t bt = pix >> 6;
    const int t = (int)(bt % T);
    const float* row = x0 + (bt - t) * 64;   // start of this clip
    float xin[9];
#pragma unroll
    for (int dt = 0; dt < 3; ++dt) {
#pragma unroll
      for (int df = 0; df < 3; ++df) {
        const int tt = t + dt - 1, ff = f + df - 1;
        xin[dt * 3 + df] = (tt >= 0 && tt < T && ff >= 0 && ff < 64) ? row[(int64_t)tt * 64 + ff] : 0.0f;
      }
    }
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < 9; ++k) acc = fmaf(wr[c][k], xin[k], acc);
      o[c] = fmaxf(acc + br[c], 0.0f);
    }
    *reinterpret_cast<float4*>(out + pix * 64 + 4 * cg) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

void launch_conv_c1(const float* x0, int B, int T, const float* w, const float* bias, float* out,
                    hipStream_t s) {
  const int64_t threads = (int64_t)B * T * 64 * 16;
  int64_t blocks = (threads + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(conv_c1_kernel, dim3(blocks), dim3(256), 0, s, x0, B, T, w, bias, out);
}

// ---------------------------------------------------------------------------
// 3x3 conv, implicit GEMM on fp32 MFMA
// ---------------------------------------------------------------------------
template <int F, int BN, int EPI>
__global__ __launch_bounds__(256, 2) void conv3x3_kernel(const float* __restrict__ in, int T,
                                                         int Cin, int Cout,
                                                         const float* __restrict__ wp,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out) {
  constexpr int BM = 128, TT = BM / F, RT = TT + 2, CS = F + 2, KC = 8;
  constexpr int PL = RT * CS;           // one channel plane of the halo tile
  constexpr int A_SZ = KC * PL;
  constexpr int W_SZ = 9 * KC * BN;
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = 4 / WAVES_N;
  constexpr int WM = BM / WAVES_M;
  constexpr int MT = WM / 32, NT = 2;   // 32x32 MFMA tiles per wave
  constexpr int CPAD = BN + 4;
  constexpr int LDS_MAIN = A_SZ + W_SZ, LDS_EPI = BM * CPAD;
  constexpr int LDS_FLOATS = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;
  constexpr int A_ITEMS = PL * 2;       // (pixel, channel quad) pairs per chunk
  constexpr int NA = (A_ITEMS + 255) / 256;
  constexpr int W_ITEMS = W_SZ / 4;
  constexpr int NW = (W_ITEMS + 255) / 256;

  __shared__ __attribute__((aligned(16))) float smem[LDS_FLOATS];
  float* As = smem;
  float* Ws = smem + A_SZ;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int tiles_t = (T + TT - 1) / TT;
  const int b = blockIdx.x / tiles_t;
  const int t0 = (blockIdx.x - b * tiles_t) * TT;
  const int n0 = blockIdx.y * BN;
  const int khalf = lane >> 5;

  int a_off[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = wm * WM + mt * 32 + (lane & 31);
    a_off[mt] = (p / F) * CS + (p % F) + khalf * PL;
  }
  int b_off[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) b_off[nt] = khalf * BN + wn * 64 + nt * 32 + (lane & 31);

  f32x16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;

  const float* in_b = in + (int64_t)b * T * F * Cin;
  float4 ra[NA], rw[NW];

#define SEDX_LOAD_CHUNK(chunk_) \
  { \
    const int c0 = (chunk_) * KC;                                                                \
_Pragma("unroll")                                                                                \
    for (int i = 0; i < NA; ++i) {                                                               \
      const int idx = tid + i * 256;                                                             \
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);                                                \
      if (idx < A_ITEMS) {                                                                       \
        const int pix = idx >> 1, q = idx & 1;                                                   \
        const int r = pix / CS, c = pix - r * CS;                                                \
        const int t = t0 - 1 + r, f = c - 1;                                                     \
        if (t >= 0 && t < T && f >= 0 && f < F)                                                  \
          v = *reinterpret_cast<const float4*>(in_b + ((int64_t)t * F + f) * Cin + c0 + 4 * q);  \
      }                                                                                          \
      ra[i] = v;                                                                                 \
    }                                                                                            \
    const float* wsrc = wp + (int64_t)(chunk_) * 9 * KC * Cout + n0;                             \
_Pragma("unroll")                                                                                \
    for (int i = 0; i < NW; ++i) {                                                               \
      const int idx = tid + i * 256;                                                             \
      if (idx < W_ITEMS) {                                                                       \
        const int row = idx / (BN / 4), c4 = idx - row * (BN / 4);                               \
        rw[i] = *reinterpret_cast<const float4*>(wsrc + (int64_t)row * Cout + 4 * c4);          \
      } else {                                                                                   \
        rw[i] = make_float4(0.f, 0.f, 0.f, 0.f);           \
      }                                                                                          \
    }                                                                                            \
  }
#define SEDX_STORE_CHUNK() \
  { \
_Pragma("unroll")                                                                                \
    for (int i = 0; i < NA; ++i) {                                                               \
      const int idx = tid + i * 256;                                                             \
      if (idx < A_ITEMS) {                                                                       \
        const int pix = idx >> 1, q = idx & 1;                                                   \
        float* dst = As + (4 * q) * PL + pix;                                                    \
        dst[0] = ra[i].x;                                                                        \
        dst[PL] = ra[i].y;                                                                       \
        dst[2 * PL] = ra[i].z;                                                                   \
        dst[3 * PL] = ra[i].w;                                                                   \
      }                                                                                          \
    }                                                                                            \
_Pragma("unroll")                                                                                \
    for (int i = 0; i < NW; ++i) {                                                               \
      const int idx = tid + i * 256;                                                             \
      if (idx < W_ITEMS) *reinterpret_cast<float4*>(Ws + 4 * idx) = rw[i];                       \
    }                                                                                            \
  }

  const int nchunks = Cin / KC;
  SEDX_LOAD_CHUNK(0);
  SEDX_STORE_CHUNK();
  __syncthreads();
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    if (chunk + 1 < nchunks) SEDX_LOAD_CHUNK(chunk + 1);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int toff = (tap / 3) * CS + (tap % 3);
#pragma unroll
      for (int ks = 0; ks < KC / 2; ++ks) {
        float a[MT], bb[NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) a[mt] = As[a_off[mt] + toff + 2 * ks * PL];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bb[nt] = Ws[(tap * KC + 2 * ks) * BN + b_off[nt]];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mt], bb[nt], acc[mt][nt], 0, 0, 0);
      }
    }
    __syncthreads();
    if (chunk + 1 < nchunks) {
      SEDX_STORE_CHUNK();
      __syncthreads();
    }
  }

#undef SEDX_LOAD_CHUNK
#undef SEDX_STORE_CHUNK
  // ---- epilogue: bias + ReLU into LDS, then store / pool / freq-mean ----
  float* Cs = smem;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = wn * 64 + nt * 32 + (lane & 31);
    const float bv = bias[n0 + col];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        Cs[row * CPAD + col] = fmaxf(acc[mt][nt][r] + bv, 0.0f);
      }
  }
  __syncthreads();
  constexpr int NQ = BN / 4;
  if (EPI == EPI_STORE) {
    for (int i = tid; i < BM * NQ; i += 256) {
      const int row = i / NQ, c4 = i - row * NQ;
      const int t = t0 + row / F, f = row % F;
      if (t < T) {
        const float4 v = *reinterpret_cast<const float4*>(Cs + row * CPAD + 4 * c4);
        *reinterpret_cast<float4*>(out + (((int64_t)b * T + t) * F + f) * Cout + n0 + 4 * c4) = v;
      }
    }
  } else if (EPI == EPI_POOL2) {
    constexpr int FO = F / 2;
    const int To = T / 2;
    for (int i = tid; i < (TT / 2) * FO * NQ; i += 256) {
      const int c4 = i % NQ;
      const int pp = i / NQ;
      const int tp = pp / FO, fp = pp % FO;
      const int to = t0 / 2 + tp;
      if (to < To) {
        const int r00 = (2 * tp) * F + 2 * fp;
        const float4 a = *reinterpret_cast<const float4*>(Cs + r00 * CPAD + 4 * c4);
        const float4 bq = *reinterpret_cast<const float4*>(Cs + (r00 + 1) * CPAD + 4 * c4);
        const float4 c = *reinterpret_cast<const float4*>(Cs + (r00 + F) * CPAD + 4 * c4);
        const float4 d = *reinterpret_cast<const float4*>(Cs + (r00 + F + 1) * CPAD + 4 * c4);
        float4 v;
        v.x = (((a.x + bq.x) + c.x) + d.x) * 0.25f;
        v.y = (((a.y + bq.y) + c.y) + d.y) * 0.25f;
        v.z = (((a.z + bq.z) + c.z) + d.z) * 0.25f;
        v.w = (((a.w + bq.w) + c.w) + d.w) * 0.25f;
        *reinterpret_cast<float4*>(out + (((int64_t)b * To + to) * FO + fp) * Cout + n0 + 4 * c4) = v;
      }
    }
  } else {  // EPI_FMEAN
    for (int i = tid; i < TT * NQ; i += 256) {
      const int tl = i / NQ, c4 = i % NQ;
      const int t = t0 + tl;
      if (t < T) {
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int f = 0; f < F; ++f) {
          const float4 v = *reinterpret_cast<const float4*>(Cs + (tl * F + f) * CPAD + 4 * c4);
          s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        const float inv = 1.0f / F;
        s.x *= inv; s.y *= inv; s.z *= inv; s.w *= inv;
        *reinterpret_cast<float4*>(out + ((int64_t)b * T + t) * Cout + n0 + 4 * c4) = s;
      }
    }
  }
}

template <int F, int BN>
static void launch_f_bn(const float* in, int B, int T, int Cin, int Cout, const float* wp,
                        const float* bias, float* out, int epi, hipStream_t s) {
  constexpr int TT = 128 / F;
  dim3 grid(B * ((T + TT - 1) / TT), Cout / BN);
  if (epi == EPI_STORE)
    launch_excl(conv3x3_kernel<F, BN, EPI_STORE>, grid, 256, s, in, T, Cin, Cout, wp, bias, out);
  else if (epi == EPI_POOL2)
    launch_excl(conv3x3_kernel<F, BN, EPI_POOL2>, grid, 256, s, in, T, Cin, Cout, wp, bias, out);
  else
    launch_excl(conv3x3_kernel<F, BN, EPI_FMEAN>, grid, 256, s, in, T, Cin, Cout, wp, bias, out);
}

void launch_conv3x3(const float* in, int B, int T, int F, int Cin, int Cout, const float* wp,
                    const float* bias, float* out, int epi, hipStream_t s) {
  // F is 64/32/16/8 on this path (mel_bins=64 halved by each 2x2 pool)
  const bool bn128 = (Cout % 128) == 0;
  switch (F) {
    case 64:
      if (bn128) launch_f_bn<64, 128>(in, B, T, Cin, Cout, wp, bias, out, epi, s);
      else launch_f_bn<64, 64>(in, B, T, Cin, Cout, wp, bias, out, epi, s);
      break;
    case 32:
      if (bn128) launch_f_bn<32, 128>(in, B, T, Cin, Cout, wp, bias, out, epi, s);
      else launch_f_bn<32, 64>(in, B, T, Cin, Cout, wp, bias, out, epi, s);
      break;
    case 16:
      launch_f_bn<16, 128>(in, B, T, Cin, Cout, wp, bias, out, epi, s);
      break;
    case 8:
      launch_f_bn<8, 128>(in, B, T, Cin, Cout, wp, bias, out, epi, s);
      break;
    default: break;
  }
}

}  // namespace sedx
