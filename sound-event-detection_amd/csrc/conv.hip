// 9-layer CNN conv kernel for gfx950 in exact fp32 (ConvBlock,
// pytorch/models.py:98-141): the reference's arithmetic, fp32 operands on
// v_mfma_f32_32x32x2_f32 with fp32 accumulation.
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
// t x all F freq bins = 256 pixels; 512 in block 1), N = output channels
// (BN), K = 9 taps x Cin, walked in chunks of KC = 4 input channels; 8 waves,
// each a 64 x 64 output tile.  Per chunk the (TT+2) x (F+2) halo of the input
// ([pixel][channel], zero border) and the weight slab [9][KC][BN] are copied
// global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no ds_write)
// into a ring of three buffers, two chunks ahead; one raw barrier per chunk
// behind a counted vmcnt wait keeps the next chunk's DMA in flight across
// it.  Inside a chunk the A / B fragments of tap t+1 are read while tap t's
// MFMAs run (lane l: A[pixel l&31][k l>>5], B[k l>>5][n l&31]; the slab holds
// each lane's two k-steps side by side, one 8-byte read).
// FUSE (block 1): the input is the zero-bordered bn0 output X0 [B][T+2][66]
// (Cin 1) and the kernel computes conv1 (Cin 1 -> 64, BN folded, ReLU) for
// the KC channels of each chunk while staging the halo (36 FMAs per halo
// pixel and chunk, VALU beside the MFMAs): conv1's 64-channel activation
// never exists in HBM.  conv2's zero padding applies to conv1's output, so
// halo pixels outside the clip stage zeros.
#include "sedx_internal.h"

namespace sedx {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// WAVES (8, or 4 for grids too small to fill the chip) waves per workgroup,
// each owning a 64 x 64 output tile: WAVES / (BN / 64) along M
template <int F, int BN, bool FUSE, int WAVES>
struct ExactGeom {
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int BM = 64 * (WAVES / (BN / 64)), TT = BM / F, RT = TT + 2, CS = F + 2, KC = 4;
  static constexpr int PL = RT * CS;                 // halo pixels
  static constexpr int PLP = (PL + 63) / 64 * 64;    // padded to whole 64-pixel DMA units
  static constexpr int A_SZ = KC * PLP;              // floats: [pixel][channel]
  static constexpr int W_SZ = 9 * KC * BN;           // floats: [tap][khalf][n][ks]
  static constexpr int BUF = A_SZ + W_SZ;            // one chunk's staging buffer
  static constexpr int NBUF = 3;                     // ring: DMA two chunks ahead
  static constexpr int W1_OFF = NBUF * BUF;          // FUSE: conv1 weights + bias
  static constexpr int MAIN = W1_OFF + (FUSE ? 64 * 9 + 64 : 0);
  static constexpr int EC = BN / 2;                  // epilogue pass: half of the n-tile
  static constexpr int CPAD = EC + 4;
  static constexpr int LDS_EPI = BM * CPAD;
  static constexpr int LDS_FLOATS = MAIN > LDS_EPI ? MAIN : LDS_EPI;
  // LDS-DMA units (one wave-instruction = 64 lanes x 16 B = 1 KiB) per chunk
  static constexpr int UW = W_SZ / 256;              // weight slab
  static constexpr int UA = FUSE ? 0 : PLP / 64;     // halo (FUSE computes it instead)
  static constexpr int U = UW + UA;
  static constexpr int UPW = (U + WAVES - 1) / WAVES;   // units per wave (at most)
  static constexpr int VM_MIN = U / WAVES;              // units of the wave with the fewest
  static constexpr int NA = (PL + THREADS - 1) / THREADS;   // FUSE: halo pixels per thread
};

template <int F, int BN, int EPI, bool FUSE, int WAVES>
__global__ __launch_bounds__(64 * WAVES, WAVES == 8 ? 2 : 1) void conv3x3_kernel(const float* __restrict__ in, int T, int Cin,
                                                                int Cout, const float* __restrict__ wp,
                                                                const float* __restrict__ bias,
                                                                float* __restrict__ out,
                                                                const float* __restrict__ w1,
                                                                const float* __restrict__ b1,
                                                                const float* __restrict__ zero16) {
  using G = ExactGeom<F, BN, FUSE, WAVES>;
  constexpr int EX_THREADS = G::THREADS;
  constexpr int BM = G::BM, TT = G::TT, CS = G::CS, KC = G::KC, PL = G::PL;
  constexpr int WAVES_N = BN / 64;
  constexpr int WAVES_M = WAVES / WAVES_N;
  constexpr int WM = BM / WAVES_M;
  constexpr int MT = WM / 32, NT = 2;   // 32x32 MFMA tiles per wave

  // ALL LDS in one array (a second __shared__ object can make hipcc drain
  // vmcnt before the fragment reads)
  __shared__ __attribute__((aligned(16))) float smem[G::LDS_FLOATS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int tiles_t = (T + TT - 1) / TT;
  const int b = blockIdx.x / tiles_t;
  const int t0 = (blockIdx.x - b * tiles_t) * TT;
  const int n0 = blockIdx.y * BN;
  const int khalf = lane >> 5;

  // fragment offsets (floats): A pixel p -> [p][khalf], [p][2 + khalf] =
  // (ks 0, ks 1); B [tap][khalf][n][ks]
  int a_off[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = wm * WM + mt * 32 + (lane & 31);
    a_off[mt] = ((p / F) * CS + (p % F)) * KC + khalf;
  }
  int b_off[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) b_off[nt] = (khalf * BN + wn * 64 + nt * 32 + (lane & 31)) * 2;

  f32x16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;

  // ---- this wave's LDS-DMA units (unit u -> wave u % 8): per unit a lane's
  // source pointer at chunk 0, its per-chunk stride and the unit's LDS offset.
  // Weight unit u: 1 KiB of the [tap][khalf][n][ks] slab, rows of 2 BN floats.
  // Halo unit: 64 pixels x 16 B; pixels outside the clip (and the padding
  // past PL) read 16 zero bytes, so every DMA is unconditional. ----
  const float* dsrc[G::UPW];
  int64_t dstep[G::UPW];
  int dlds[G::UPW];
#pragma unroll
  for (int k = 0; k < G::UPW; ++k) {
    const int u = wv + WAVES * k;
    dsrc[k] = zero16;
    dstep[k] = 0;
    dlds[k] = 0;
    if (u < G::UW) {
      constexpr int LPR = BN / 2;                     // lanes per slab row (16 B each)
      const int row = u * (64 / LPR) + lane / LPR;    // (tap, khalf)
      dsrc[k] = wp + 2 * n0 + (int64_t)row * 2 * Cout + 4 * (lane % LPR);
      dstep[k] = (int64_t)9 * KC * Cout;
      dlds[k] = G::A_SZ + 256 * u;
    } else if (u < G::U) {
      const int pix = 64 * (u - G::UW) + lane;
      const int r = pix / CS, c = pix - (pix / CS) * CS;
      const int t = t0 - 1 + r, f = c - 1;
      if (pix < PL && t >= 0 && t < T && f >= 0 && f < F) {
        dsrc[k] = in + (((int64_t)b * T + t) * F + f) * Cin;
        dstep[k] = KC;
      }
      dlds[k] = 256 * (u - G::UW);
    }
  }
#define SEDX_EX_DMA(chunk_, buf_)                                                                      \
  {                                                                                                    \
    _Pragma("unroll") for (int k = 0; k < G::UPW; ++k) {                                               \
      if (wv + WAVES * k < G::U) {                                                                         \
        const uint32_t m0_ = (uint32_t)(size_t)(__attribute__((address_space(3))) float*)(             \
            smem + (buf_) * G::BUF + dlds[k]);                                                         \
        sedx_glds16(dsrc[k] + (int64_t)(chunk_) * dstep[k], __builtin_amdgcn_readfirstlane(m0_));      \
      }                                                                                                \
    }                                                                                                  \
    asm volatile("" ::: "memory");                                                                     \
  }

  // ---- FUSE: conv1 weights in LDS, the 3x3 X0 window of each staged pixel in
  // registers; conv1 (BN folded + ReLU) of a chunk's 4 channels computed into
  // the halo image while the previous chunk's MFMAs run ----
  bool pin[G::NA];
  float xw[FUSE ? G::NA : 1][9];
  if constexpr (FUSE) {
    for (int i = tid; i < 64 * 9 + 64; i += EX_THREADS)
      smem[G::W1_OFF + i] = i < 64 * 9 ? w1[i] : b1[i - 64 * 9];
#pragma unroll
    for (int i = 0; i < G::NA; ++i) {
      const int pix = tid + EX_THREADS * i;
      const int r = pix / CS, c = pix - (pix / CS) * CS;
      const int t = t0 - 1 + r, f = c - 1;
      pin[i] = pix < PL && t >= 0 && t < T && f >= 0 && f < F;
      // X0pad [B][T+2][66]: (t, f) of X0 at (t+1, f+1); window corner (t, f)
      const int64_t src = pin[i] ? ((int64_t)b * (T + 2) + t) * 66 + f : 0;
#pragma unroll
      for (int k = 0; k < 9; ++k) xw[i][k] = pin[i] ? in[src + (k / 3) * 66 + (k % 3)] : 0.0f;
    }
    __syncthreads();   // w1 / b1 in LDS; no DMA in flight yet
  }
#define SEDX_EX_CONV1(chunk_, buf_)                                                                    \
  {                                                                                                    \
    float* As_ = smem + (buf_) * G::BUF;                                                               \
    const float* w1s_ = smem + G::W1_OFF + (chunk_) * KC * 9;                                          \
    const float* b1s_ = smem + G::W1_OFF + 64 * 9 + (chunk_) * KC;                                     \
    _Pragma("unroll") for (int i = 0; i < G::NA; ++i) {                                                \
      const int pix = tid + EX_THREADS * i;                                                            \
      if (pix < PL) {                                                                                  \
        float v_[KC];                                                                                  \
        _Pragma("unroll") for (int c = 0; c < KC; ++c) {                                               \
          float s_ = 0.0f;                                                                             \
          _Pragma("unroll") for (int k = 0; k < 9; ++k) s_ = fmaf(w1s_[c * 9 + k], xw[i][k], s_);     \
          v_[c] = pin[i] ? fmaxf(s_ + b1s_[c], 0.0f) : 0.0f;                                           \
        }                                                                                              \
        *reinterpret_cast<float4*>(As_ + pix * KC) = make_float4(v_[0], v_[1], v_[2], v_[3]);          \
      }                                                                                                \
    }                                                                                                  \
  }
  // chunk barrier: this wave's DMAs older than its n_ youngest VMEM ops have
  // landed and its LDS operations are done, then the workgroup barrier (raw:
  // __syncthreads() would drain every DMA in flight)
#define SEDX_EX_BAR(n_) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(n_) : "memory")

  const int nchunks = Cin / KC;
  SEDX_EX_DMA(0, 0);
  if (nchunks > 1) SEDX_EX_DMA(1, 1);
  if constexpr (FUSE) SEDX_EX_CONV1(0, 0);
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    // chunk's DMAs (issued two chunks ago) landed for every wave; buffer
    // (chunk + 2) % 3 was last read in chunk - 1, finished by every wave
    if (chunk + 1 < nchunks)
      SEDX_EX_BAR(G::VM_MIN);
    else
      SEDX_EX_BAR(0);
    const int buf = chunk % 3;
    if (chunk + 2 < nchunks) SEDX_EX_DMA(chunk + 2, (chunk + 2) % 3);
    const float* As = smem + buf * G::BUF;
    const float* Ws = As + G::A_SZ;
    float2 a[2][MT], bb[2][NT];   // [slot][.]: (.x, .y) = (ks 0, ks 1)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) a[0][mt] = make_float2(As[a_off[mt]], As[a_off[mt] + 2]);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bb[0][nt] = *reinterpret_cast<const float2*>(Ws + b_off[nt]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int cur = tap & 1, nxt = cur ^ 1;
      if (tap < 8) {
        const int tn = tap + 1;
        const int toff = ((tn / 3) * CS + (tn % 3)) * KC;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          a[nxt][mt] = make_float2(As[a_off[mt] + toff], As[a_off[mt] + toff + 2]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          bb[nxt][nt] = *reinterpret_cast<const float2*>(Ws + tn * KC * BN + b_off[nt]);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][mt].x, bb[cur][nt].x, acc[mt][nt], 0, 0, 0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][mt].y, bb[cur][nt].y, acc[mt][nt], 0, 0, 0);
    }
    // FUSE: the next chunk's halo (its buffer was last read in chunk - 2)
    if constexpr (FUSE)
      if (chunk + 1 < nchunks) SEDX_EX_CONV1(chunk + 1, (chunk + 1) % 3);
  }
  SEDX_EX_BAR(0);   // every wave's fragment reads done before the epilogue reuses the LDS
#undef SEDX_EX_DMA
#undef SEDX_EX_CONV1
#undef SEDX_EX_BAR

  // ---- epilogue: bias + ReLU into LDS, then store / pool / freq-mean, in two
  // passes over halves of the n-tile (pass h: columns wn*64 + h*32 + j of each
  // wave; local column c = wn*32 + j), so the staging fits three workgroups
  // per CU ----
  constexpr int CPAD = G::CPAD, EC = G::EC;
  constexpr int NQ = EC / 4;
  float* Cs = smem;
#pragma unroll
  for (int h = 0; h < NT; ++h) {
    {
      const int col = wn * 32 + (lane & 31);
      const float bv = bias[n0 + wn * 64 + h * 32 + (lane & 31)];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
          Cs[row * CPAD + col] = fmaxf(acc[mt][h][r] + bv, 0.0f);
        }
    }
    __syncthreads();
    // global channel of local float4 group c4 (4 consecutive columns)
    auto gch = [&](int c4) { return n0 + (c4 / 8) * 64 + h * 32 + (c4 % 8) * 4; };
    if (EPI == EPI_STORE) {
      for (int i = tid; i < BM * NQ; i += EX_THREADS) {
        const int row = i / NQ, c4 = i - row * NQ;
        const int t = t0 + row / F, f = row % F;
        if (t < T) {
          const float4 v = *reinterpret_cast<const float4*>(Cs + row * CPAD + 4 * c4);
          *reinterpret_cast<float4*>(out + (((int64_t)b * T + t) * F + f) * Cout + gch(c4)) = v;
        }
      }
    } else if (EPI == EPI_POOL2) {
      constexpr int FO = F / 2;
      const int To = T / 2;
      for (int i = tid; i < (TT / 2) * FO * NQ; i += EX_THREADS) {
        const int c4 = i % NQ;
        const int pp = i / NQ;
        const int tp = pp / FO, fp = pp % FO;
        const int to = t0 / 2 + tp;
        if (to < To) {
          const int r00 = (2 * tp) * F + 2 * fp;
          const float4 a0 = *reinterpret_cast<const float4*>(Cs + r00 * CPAD + 4 * c4);
          const float4 a1 = *reinterpret_cast<const float4*>(Cs + (r00 + 1) * CPAD + 4 * c4);
          const float4 a2 = *reinterpret_cast<const float4*>(Cs + (r00 + F) * CPAD + 4 * c4);
          const float4 a3 = *reinterpret_cast<const float4*>(Cs + (r00 + F + 1) * CPAD + 4 * c4);
          float4 v;
          v.x = (((a0.x + a1.x) + a2.x) + a3.x) * 0.25f;
          v.y = (((a0.y + a1.y) + a2.y) + a3.y) * 0.25f;
          v.z = (((a0.z + a1.z) + a2.z) + a3.z) * 0.25f;
          v.w = (((a0.w + a1.w) + a2.w) + a3.w) * 0.25f;
          *reinterpret_cast<float4*>(out + (((int64_t)b * To + to) * FO + fp) * Cout + gch(c4)) = v;
        }
      }
    } else {  // EPI_FMEAN
      for (int i = tid; i < TT * NQ; i += EX_THREADS) {
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
          *reinterpret_cast<float4*>(out + ((int64_t)b * T + t) * Cout + gch(c4)) = s;
        }
      }
    }
    if (h + 1 < NT) __syncthreads();
  }
}

template <int F, int BN, bool FUSE, int WAVES>
static void launch_f_bn_w(const float* in, int B, int T, int Cin, int Cout, const float* wp,
                          const float* bias, float* out, int epi, const float* w1, const float* b1,
                          const float* zero16, hipStream_t s) {
  constexpr int TT = ExactGeom<F, BN, FUSE, WAVES>::TT;
  constexpr int NT = 64 * WAVES;
  dim3 grid(B * ((T + TT - 1) / TT), Cout / BN);
  if (epi == EPI_STORE)
    launch_kernel(conv3x3_kernel<F, BN, EPI_STORE, FUSE, WAVES>, grid, NT, s, in, T, Cin, Cout, wp, bias, out, w1, b1, zero16);
  else if (epi == EPI_POOL2)
    launch_kernel(conv3x3_kernel<F, BN, EPI_POOL2, FUSE, WAVES>, grid, NT, s, in, T, Cin, Cout, wp, bias, out, w1, b1, zero16);
  else
    launch_kernel(conv3x3_kernel<F, BN, EPI_FMEAN, FUSE, WAVES>, grid, NT, s, in, T, Cin, Cout, wp, bias, out, w1, b1, zero16);
}

// 8-wave tiles when they make at least two workgroups per CU of the chip,
// else 4-wave tiles (half the pixels per tile: twice the workgroups)
template <int F, int BN, bool FUSE>
static void launch_f_bn(const float* in, int B, int T, int Cin, int Cout, const float* wp,
                        const float* bias, float* out, int epi, const float* w1, const float* b1,
                        const float* zero16, hipStream_t s) {
  constexpr int TT8 = ExactGeom<F, BN, FUSE, 8>::TT;
  const int64_t tiles8 = (int64_t)B * ((T + TT8 - 1) / TT8) * (Cout / BN);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (tiles8 >= 2 * (int64_t)ncu)
    launch_f_bn_w<F, BN, FUSE, 8>(in, B, T, Cin, Cout, wp, bias, out, epi, w1, b1, zero16, s);
  else
    launch_f_bn_w<F, BN, FUSE, 4>(in, B, T, Cin, Cout, wp, bias, out, epi, w1, b1, zero16, s);
}

void launch_conv3x3(const float* in, int B, int T, int F, int Cin, int Cout, const float* wp,
                    const float* bias, float* out, int epi, const float* zero16, hipStream_t s) {
  // F is 64/32/16/8 on this path (mel_bins=64 halved by each 2x2 pool); the
  // instantiated (F, epilogue) pairs are the model's
  if (Cin % 4 != 0) return note_launch_error(hipErrorInvalidValue);
  switch (F) {
    case 32:
      if (Cout % 128 == 0) launch_f_bn<32, 128, false>(in, B, T, Cin, Cout, wp, bias, out, epi, nullptr, nullptr, zero16, s);
      break;
    case 16:
      if (Cout % 128 == 0) launch_f_bn<16, 128, false>(in, B, T, Cin, Cout, wp, bias, out, epi, nullptr, nullptr, zero16, s);
      break;
    case 8:
      if (Cout % 128 == 0) launch_f_bn<8, 128, false>(in, B, T, Cin, Cout, wp, bias, out, epi, nullptr, nullptr, zero16, s);
      break;
    default:
      note_launch_error(hipErrorInvalidValue);
      break;
  }
}

void launch_block1_exact(const float* xpad, int B, int T, const float* w1, const float* b1, const float* wp,
                         const float* bias, float* out, const float* zero16, hipStream_t s) {
  launch_f_bn<64, 64, true>(xpad, B, T, 64, 64, wp, bias, out, EPI_POOL2, w1, b1, zero16, s);
}

}  // namespace sedx
