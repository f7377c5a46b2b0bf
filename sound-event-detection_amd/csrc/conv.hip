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

#include <type_traits>

namespace sedx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifdef SEDX_EXACT_STAMPS
// diagnostic build (tools/conv_exact_bench.cpp): per-wave s_memtime sums —
// [0] wave cycles, [1] barrier waits, [2] FUSE conv1, [3] epilogue, [4] waves,
// [5] wave realtime (100 MHz)
__device__ unsigned long long g_exact_stamps[8];
#define SEDX_XS_DECL                                                                    \
  unsigned long long xs_bar = 0, xs_c1 = 0, xs_epi = 0, xs_x = 0;                       \
  const unsigned long long xs_t0 = __builtin_amdgcn_s_memtime();                        \
  const unsigned long long xs_r0 = __builtin_amdgcn_s_memrealtime();
#define SEDX_XS_BEGIN() xs_x = __builtin_amdgcn_s_memtime()
#define SEDX_XS_END(a) a += __builtin_amdgcn_s_memtime() - xs_x
#define SEDX_XS_FLUSH()   /* sampled: every 16th workgroup (few atomics) */         \
  if (lane == 0 && (blockIdx.x & 15) == 0) {                                            \
    atomicAdd(&g_exact_stamps[0], __builtin_amdgcn_s_memtime() - xs_t0);                \
    atomicAdd(&g_exact_stamps[1], xs_bar);                                              \
    atomicAdd(&g_exact_stamps[2], xs_c1);                                               \
    atomicAdd(&g_exact_stamps[3], xs_epi);                                              \
    atomicAdd(&g_exact_stamps[4], 1ull);                                                \
    atomicAdd(&g_exact_stamps[5], __builtin_amdgcn_s_memrealtime() - xs_r0);            \
  }
void exact_stamps_rw(unsigned long long* out8, bool reset) {
  (void)hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_exact_stamps), 8 * sizeof(unsigned long long));
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_exact_stamps), z, sizeof(z));
  }
}
#else
#define SEDX_XS_DECL
#define SEDX_XS_BEGIN()
#define SEDX_XS_END(a)
#define SEDX_XS_FLUSH()
#endif

// WAVES waves per workgroup, each owning a WT x WT output tile (WT = 64:
// 2 x 2 MFMA tiles; WT = 32: one; WT = 16: one v_mfma_f32_16x16x4_f32
// tile), BN / WT of them along N and the rest along M.  WT = 64 with 8 waves
// (4 for grids too small to fill the chip) is the throughput shape; WT = 32
// and WT = 16 are the small-batch shapes: a quarter (a sixteenth) of the
// MFMA work per wave per chunk, so that much shorter a serial K chain and
// that many more waves.  fp32 MFMAs on gfx950 are in-order fma chains over k
// (32x32x2: two k per instruction, 16x16x4: four;
// tools/mfma_f32_semantics.cpp, tools/mfma16_f32_semantics.cpp), and every
// shape walks chunk, tap, channel in the same order, so all three give
// bit-identical outputs.
template <int F, int BN, bool FUSE, int WAVES, int WT>
struct ExactGeom {
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int WAVES_N = BN / WT, WAVES_M = WAVES / WAVES_N;
  static constexpr int BM = WT * WAVES_M, TT = BM / F, RT = TT + 2, CS = F + 2, KC = 4;
  static constexpr int PL = RT * CS;                 // halo pixels
  static constexpr int PLP = (PL + 63) / 64 * 64;    // padded to whole 64-pixel DMA units
  static constexpr int A_SZ = KC * PLP;              // floats: [pixel][channel]
  static constexpr int W_SZ = 9 * KC * BN;           // floats: [tap][khalf][n][ks]
  static constexpr int BUF = A_SZ + W_SZ;            // one chunk's staging buffer
  // ring: DMA NBUF - 1 chunks ahead (deeper for the small-batch shape, whose
  // one or two waves per SIMD cannot hide a DMA behind other waves' MFMAs)
  static constexpr int NBUF = WT <= 32 ? 5 : 3;
  static constexpr int MAIN = NBUF * BUF;
  static constexpr int EC = WT == 16 ? BN : BN / (WT / 32);   // epilogue pass: one MFMA tile column block per wave
  static constexpr int CPAD = EC + 4;
  static constexpr int LDS_EPI = BM * CPAD;
  static constexpr int W1_OFF = MAIN > LDS_EPI ? MAIN : LDS_EPI;   // FUSE: conv1 weights + bias
  static constexpr int LDS_FLOATS = W1_OFF + (FUSE ? 64 * 9 + 64 : 0);
  // LDS-DMA units (one wave-instruction = 64 lanes x 16 B = 1 KiB) per chunk
  static constexpr int UW = W_SZ / 256;              // weight slab
  static constexpr int UA = FUSE ? 0 : PLP / 64;     // halo (FUSE computes it instead)
  static constexpr int U = UW + UA;
  static constexpr int UPW = (U + WAVES - 1) / WAVES;   // units per wave (at most)
  static constexpr int VM_MIN = U / WAVES;              // units of the wave with the fewest
  static constexpr int NA = (PL + THREADS - 1) / THREADS;   // FUSE: halo pixels per thread
};

template <int F, int BN, int EPI, bool FUSE, int WAVES, int WT>
__global__ __launch_bounds__(64 * WAVES, WAVES == 8 && WT == 64 ? 2 : 1) void conv3x3_kernel(const float* __restrict__ in, int T, int Cin,
                                                                int Cout, const float* __restrict__ wp,
                                                                const float* __restrict__ bias,
                                                                float* __restrict__ out,
                                                                const float* __restrict__ w1,
                                                                const float* __restrict__ b1,
                                                                const float* __restrict__ zero16) {
  using G = ExactGeom<F, BN, FUSE, WAVES, WT>;
  constexpr int EX_THREADS = G::THREADS;
  constexpr int BM = G::BM, TT = G::TT, CS = G::CS, KC = G::KC, PL = G::PL;
  constexpr int WAVES_N = G::WAVES_N;
  constexpr int WM = WT;
  constexpr int MT = WT == 16 ? 1 : WT / 32, NT = MT;   // MFMA tiles per wave (each dimension)
  constexpr int NR = WT == 16 ? 4 : 16;                 // accumulator registers per MFMA tile
  using accv = typename std::conditional<WT == 16, f32x4, f32x16>::type;
  // WT = 32 pooled: a wave's 32 rows are 2 t-rows x 16 bins, so a 2x2
  // window is registers r, r+1, r+8, r+9 of one lane (as at F = 16)
  constexpr bool SEG16 = WT == 32 && EPI == EPI_POOL2;
  // WT = 16: a wave's 16 rows are 2 t-rows x 8 bins; lane quarter q holds rows
  // 4q..4q+3 (t-row q >> 1, bins 4 (q & 1) + r): a 2x2 window spans lanes l
  // and l + 32, an 8-bin mean lanes l and l ^ 16
  constexpr bool SEG8 = WT == 16;
  static_assert(TT * F == BM && (EPI != EPI_POOL2 || TT % 2 == 0), "tile = whole (pairs of) t-rows");

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
  // A row m of MFMA tile mt of wave wm is tile pixel (t, f) = pix_t / pix_f:
  // row-major (pixel WT wm + 32 mt + m) except at WT = 64, F = 64, where a
  // wave covers two t-rows x 32 bins, so every 2x2 pooling window lies in one
  // lane's accumulators (bins m, m+1 in registers r, r+1; rows in mt 0, 1),
  // and SEG16 (above)
  auto pix_t = [&](int mt, int m) {
    if constexpr (SEG8) return 2 * (wm / (F / 8)) + (m >> 3);
    if constexpr (SEG16) return 2 * (wm / (F / 16)) + (m >> 4);
    return (F == 64 && WT == 64) ? 2 * (wm >> 1) + mt : (wm * WM + mt * 32 + m) / F;
  };
  auto pix_f = [&](int mt, int m) {
    if constexpr (SEG8) return 8 * (wm % (F / 8)) + (m & 7);
    if constexpr (SEG16) return 16 * (wm % (F / 16)) + (m & 15);
    return (F == 64 && WT == 64) ? 32 * (wm & 1) + m : (wm * WM + mt * 32 + m) % F;
  };
  // WT = 16: lane supplies A[pixel lane & 15][channel lane >> 4] and
  // B[channel lane >> 4][n lane & 15] (channel c = 2 ks + khalf in the slab)
  int a_off[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    a_off[mt] = WT == 16 ? (pix_t(0, lane & 15) * CS + pix_f(0, lane & 15)) * KC + (lane >> 4)
                         : (pix_t(mt, lane & 31) * CS + pix_f(mt, lane & 31)) * KC + khalf;
  int b_off[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    b_off[nt] = WT == 16 ? (((lane >> 4) & 1) * BN + wn * 16 + (lane & 15)) * 2 + (lane >> 5)
                         : (khalf * BN + wn * WT + nt * 32 + (lane & 31)) * 2;
  // MFMA row m held in accumulator register r of this lane
  [[maybe_unused]] auto drow = [&](int r) { return WT == 16 ? 4 * (lane >> 4) + r : (r & 3) + 8 * (r >> 2) + 4 * khalf; };

  accv acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[mt][nt][r] = 0.0f;

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

  // ---- FUSE: the 3x3 X0 window of each staged pixel in registers; conv1
  // (BN folded + ReLU) of a chunk's 4 channels computed into the halo image
  // while the previous chunk's MFMAs run, on the matrix pipe:
  // v_mfma_f32_4x4x1f32 (16 blocks of 4 pixels x 4 channels, one tap per
  // instruction) over taps 0..8 from zero is bit for bit the fma chain
  // s = fma(w_k, x_k, s) (fp32 MFMAs on gfx950 are in-order fma chains:
  // tools/mfma_f32_semantics.cpp, tools/mfma16_f32_semantics.cpp), so it
  // equals the VALU conv1 it replaces (14.8 % of b1c2's wave time, s_memtime).
  // Lane l supplies pixel 64 g + l's tap value (A) and w1[channel l & 3][tap]
  // (B); it receives pixels 64 g + 4 (l >> 2) + r, r = 0..3, channel l & 3. ----
  float xw[FUSE ? G::NA : 1][9];
  float omask[FUSE ? G::NA : 1][4];   // validity of the 4 output pixels of each group
  if constexpr (FUSE) {
    for (int i = tid; i < 64 * 9 + 64; i += EX_THREADS) smem[G::W1_OFF + i] = i < 576 ? w1[i] : b1[i - 576];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < G::NA; ++i) {
      const int pix = tid + EX_THREADS * i;
      const int r = pix / CS, c = pix - (pix / CS) * CS;
      const int t = t0 - 1 + r, f = c - 1;
      const bool pin = pix < PL && t >= 0 && t < T && f >= 0 && f < F;
      // X0pad [B][T+2][66]: (t, f) of X0 at (t+1, f+1); window corner (t, f)
      const int64_t src = pin ? ((int64_t)b * (T + 2) + t) * 66 + f : 0;
#pragma unroll
      for (int k = 0; k < 9; ++k) xw[i][k] = in[src + (k / 3) * 66 + (k % 3)];   // masked via omask
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int po = EX_THREADS * i + 64 * wv + 4 * (lane >> 2) + q;
        const int ro = po / CS, co = po - ro * CS;
        const int to = t0 - 1 + ro, fo = co - 1;
        omask[i][q] = (po < PL && to >= 0 && to < T && fo >= 0 && fo < F) ? 1.0f : 0.0f;
      }
    }
    // the window loads retire here, on every path, so the compiler's wait
    // tracking does not carry them into the chunk loop, where a wait for them
    // would drain the LDS-DMAs in flight (vmcnt 0; expcnt, lgkmcnt untouched)
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
#define SEDX_EX_CONV1(chunk_, buf_)                                                                    \
  {                                                                                                    \
    float* As_ = smem + (buf_) * G::BUF;                                                               \
    const int ch_ = (chunk_) * KC + (lane & 3);                                                        \
    float wv_[9];                                                                                      \
    _Pragma("unroll") for (int k = 0; k < 9; ++k) wv_[k] = smem[G::W1_OFF + ch_ * 9 + k];             \
    const float bv_ = smem[G::W1_OFF + 576 + ch_];                                                     \
    _Pragma("unroll") for (int i = 0; i < G::NA; ++i) {                                                \
      if (G::NA * EX_THREADS == PL || EX_THREADS * i + 64 * wv < PL) {   /* wave-uniform */            \
        f32x4 d_ = {0.0f, 0.0f, 0.0f, 0.0f};                                                           \
        _Pragma("unroll") for (int k = 0; k < 9; ++k)                                                  \
            d_ = __builtin_amdgcn_mfma_f32_4x4x1f32(xw[i][k], wv_[k], d_, 0, 0, 0);                    \
        const int p0_ = EX_THREADS * i + 64 * wv + 4 * (lane >> 2);                                    \
        _Pragma("unroll") for (int q = 0; q < 4; ++q)                                                  \
            As_[(p0_ + q) * KC + (lane & 3)] = fmaxf(d_[q] + bv_, 0.0f) * omask[i][q];                 \
      }                                                                                                \
    }                                                                                                  \
  }
  // chunk barrier: this wave's DMAs older than its n_ youngest VMEM ops have
  // landed and its LDS operations are done, then the workgroup barrier (raw:
  // __syncthreads() would drain every DMA in flight)
#define SEDX_EX_BAR(n_) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(n_) : "memory")

  SEDX_XS_DECL
  const int nchunks = Cin / KC;
  constexpr int NB = G::NBUF;
#pragma unroll
  for (int c = 0; c < NB - 1; ++c)
    if (c < nchunks) SEDX_EX_DMA(c, c);
  if constexpr (FUSE) SEDX_EX_CONV1(0, 0);
  int buf = 0;
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    // chunk's DMAs (issued NB - 1 chunks ago) landed for every wave: at most
    // the younger chunks' DMAs (up to NB - 2 of them) still in flight; buffer
    // (chunk + NB - 1) % NB was last read in chunk - 1, finished by every wave
    const int younger = min(NB - 2, nchunks - 1 - chunk);
    SEDX_XS_BEGIN();
    if (younger >= 3 && NB > 4)
      SEDX_EX_BAR(3 * G::VM_MIN);
    else if (younger == 2 && NB > 3)
      SEDX_EX_BAR(2 * G::VM_MIN);
    else if (younger >= 1)
      SEDX_EX_BAR(G::VM_MIN);
    else
      SEDX_EX_BAR(0);
    SEDX_XS_END(xs_bar);
    const int dbuf = buf == 0 ? NB - 1 : buf - 1;   // (chunk + NB - 1) % NB
    if (chunk + NB - 1 < nchunks) SEDX_EX_DMA(chunk + NB - 1, dbuf);
    const float* As = smem + buf * G::BUF;
    const float* Ws = As + G::A_SZ;
    if constexpr (WT == 16) {
      // one 16x16x4 MFMA per tap: k = the chunk's 4 channels in order
      float a1[2], b1v[2];
      a1[0] = As[a_off[0]];
      b1v[0] = Ws[b_off[0]];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int cur = tap & 1, nxt = cur ^ 1;
        if (tap < 8) {
          const int tn = tap + 1;
          a1[nxt] = As[a_off[0] + ((tn / 3) * CS + (tn % 3)) * KC];
          b1v[nxt] = Ws[tn * KC * BN + b_off[0]];
        }
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[cur], b1v[cur], acc[0][0], 0, 0, 0);
      }
    } else {
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
    }
    const int nbuf = buf + 1 == NB ? 0 : buf + 1;
    // FUSE: the next chunk's halo (its buffer's A region was last read in
    // chunk + 1 - NB)
    if constexpr (FUSE) {
      SEDX_XS_BEGIN();
      if (chunk + 1 < nchunks) SEDX_EX_CONV1(chunk + 1, nbuf);
      SEDX_XS_END(xs_c1);
    }
    buf = nbuf;
  }
  SEDX_XS_BEGIN();
  SEDX_EX_BAR(0);   // every wave's fragment reads done before the epilogue reuses the LDS
  SEDX_XS_END(xs_bar);
  SEDX_XS_BEGIN();
#undef SEDX_EX_DMA
#undef SEDX_EX_CONV1
#undef SEDX_EX_BAR

  // ---- epilogue.  Lane l holds output channel n = wn*64 + nt*32 + (l&31) of
  // rows m = (r&3) + 8(r>>2) + 4(l>>5) of each 32-row tile (MFMA C layout).
  // EPI_POOL2 / EPI_FMEAN: bias + ReLU, then the 2x2 average / the 8-bin mean
  // in registers (plus one lane-32 swap for the mean) and 128-B row stores;
  // EPI_STORE: through LDS in two passes (float4 stores). ----
  if constexpr (EPI == EPI_POOL2 && WT == 16) {
    // rows (t, f), (t, f+1) in registers r, r+1; t-row t+1 in lane l + 32
    constexpr int FO = F / 2;
    const int To = T / 2;
    const int n = n0 + wn * 16 + (lane & 15);
    const float bv = bias[n];
    float v4[4], p4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v4[r] = fmaxf(acc[0][0][r] + bv, 0.0f);
#pragma unroll
    for (int r = 0; r < 4; ++r) p4[r] = __shfl_xor(v4[r], 32);
    if (lane < 32)
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const float v = (((v4[r] + v4[r + 1]) + p4[r]) + p4[r + 1]) * 0.25f;
        const int m = drow(r);
        const int to = t0 / 2 + (pix_t(0, m) >> 1), fo = pix_f(0, m) >> 1;
        if (to < To) out[(((int64_t)b * To + to) * FO + fo) * Cout + n] = v;
      }
  } else if constexpr (EPI == EPI_FMEAN && WT == 16) {
    // a lane's 4 bins of one t-row; the other 4 bins in lane l ^ 16
    static_assert(F == 8, "freq-mean epilogue: F = 8");
    const int n = n0 + wn * 16 + (lane & 15);
    const float bv = bias[n];
    float s4 = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s4 += fmaxf(acc[0][0][j] + bv, 0.0f);
    const float o4 = __shfl_xor(s4, 16);
    const int q = lane >> 4;
    const float v = ((q & 1) ? o4 + s4 : s4 + o4) * (1.0f / F);
    const int t = t0 + pix_t(0, 4 * q);
    if ((q & 1) == 0 && t < T) out[((int64_t)b * T + t) * Cout + n] = v;
  } else if constexpr (EPI == EPI_POOL2) {
    static_assert(F >= 16, "pooled epilogue: F in {16, 32, 64}");
    constexpr int FO = F / 2;
    const int To = T / 2;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + wn * WT + nt * 32 + (lane & 31);
      const float bv = bias[n];
      auto rl = [&](int mt, int r) { return fmaxf(acc[mt][nt][r] + bv, 0.0f); };
      if constexpr (F == 16 || SEG16) {
        // rows m, m+1 (bins), m+16 (next t-row): registers r, r+1, r+8, r+9
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 8; r += 2) {
            const float v = (((rl(mt, r) + rl(mt, r + 1)) + rl(mt, r + 8)) + rl(mt, r + 9)) * 0.25f;
            const int m = (r & 3) + 8 * (r >> 2) + 4 * khalf;
            const int to = t0 / 2 + (pix_t(mt, m) >> 1), fo = pix_f(mt, m) >> 1;
            if (to < To) out[(((int64_t)b * To + to) * FO + fo) * Cout + n] = v;
          }
      } else {
        // rows m, m+1 (bins) in registers r, r+1; t-rows in mt 0, 1
        static_assert(MT == 2, "pooled epilogue: two MFMA row tiles per wave");
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const float v = (((rl(0, r) + rl(0, r + 1)) + rl(1, r)) + rl(1, r + 1)) * 0.25f;
          const int m = (r & 3) + 8 * (r >> 2) + 4 * khalf;
          const int to = t0 / 2 + (pix_t(0, m) >> 1), fo = pix_f(0, m) >> 1;
          if (to < To) out[(((int64_t)b * To + to) * FO + fo) * Cout + n] = v;
        }
      }
    }
  } else if constexpr (EPI == EPI_FMEAN) {
    static_assert(F == 8, "freq-mean epilogue: F = 8");
    // a 32-row tile = 4 t-rows x 8 bins: bins (r&3) + 4 khalf, t-row r>>2;
    // sum the lane's 4 bins, add the other half-wave's 4 (lane ^ 32)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + wn * WT + nt * 32 + (lane & 31);
      const float bv = bias[n];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float s4 = 0.0f;
#pragma unroll
          for (int j = 0; j < 4; ++j) s4 += fmaxf(acc[mt][nt][4 * q + j] + bv, 0.0f);
          const float o4 = __shfl_xor(s4, 32);
          // torch.mean over the 8 bins: ((b0 + b1 + ... + b7) / 8, bins in order)
          const float v = (khalf ? o4 + s4 : s4 + o4) * (1.0f / F);
          const int t = t0 + pix_t(mt, 8 * q);
          if (khalf == (q & 1) && t < T) out[((int64_t)b * T + t) * Cout + n] = v;
        }
    }
  } else {
    constexpr int CPAD = G::CPAD, EC = G::EC;
    constexpr int NQ = EC / 4;
    float* Cs = smem;
#pragma unroll
    for (int h = 0; h < NT; ++h) {
      {
        const int col = WT == 16 ? wn * 16 + (lane & 15) : wn * 32 + (lane & 31);
        const float bv = bias[WT == 16 ? n0 + col : n0 + wn * WT + h * 32 + (lane & 31)];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            const int m = drow(r);
            const int row = pix_t(mt, m) * F + pix_f(mt, m);
            Cs[row * CPAD + col] = fmaxf(acc[mt][h][r] + bv, 0.0f);
          }
      }
      __syncthreads();
      // global channel of local float4 group c4 (4 consecutive columns)
      auto gch = [&](int c4) { return WT == 16 ? n0 + 4 * c4 : n0 + (c4 / 8) * WT + h * 32 + (c4 % 8) * 4; };
      for (int i = tid; i < BM * NQ; i += EX_THREADS) {
        const int row = i / NQ, c4 = i - row * NQ;
        const int t = t0 + row / F, f = row % F;
        if (t < T) {
          const float4 v = *reinterpret_cast<const float4*>(Cs + row * CPAD + 4 * c4);
          *reinterpret_cast<float4*>(out + (((int64_t)b * T + t) * F + f) * Cout + gch(c4)) = v;
        }
      }
      if (h + 1 < NT) __syncthreads();
    }
  }
  SEDX_XS_END(xs_epi);
  SEDX_XS_FLUSH();
}

template <int F, int BN, bool FUSE, int WAVES, int WT>
static void launch_f_bn_w(const float* in, int B, int T, int Cin, int Cout, const float* wp,
                          const float* bias, float* out, int epi, const float* w1, const float* b1,
                          const float* zero16, hipStream_t s) {
  constexpr int TT = ExactGeom<F, BN, FUSE, WAVES, WT>::TT;
  constexpr int NT = 64 * WAVES;
  dim3 grid(B * ((T + TT - 1) / TT), Cout / BN);
#define SEDX_EX_LAUNCH(E)                                                                              \
  return launch_kernel(conv3x3_kernel<F, BN, E, FUSE, WAVES, WT>, grid, NT, s, in, T, Cin, Cout, wp, bias, out, \
                       w1, b1, zero16)
  // only the model's (F, epilogue) pairs are instantiated
  if constexpr (F != 64 && F != 8) {
    if (epi == EPI_STORE) SEDX_EX_LAUNCH(EPI_STORE);
  }
  if constexpr (F == 8) {
    if (epi == EPI_STORE) SEDX_EX_LAUNCH(EPI_STORE);
    if (epi == EPI_FMEAN) SEDX_EX_LAUNCH(EPI_FMEAN);
  } else {
    if (epi == EPI_POOL2) SEDX_EX_LAUNCH(EPI_POOL2);
  }
#undef SEDX_EX_LAUNCH
  note_launch_error(hipErrorInvalidValue);
}

static int device_cus() {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return ncu;
}

// Shape by grid size: 8-wave 64x64 wave tiles when they make at least two
// workgroups per CU of the chip; 4-wave ones likewise (one workgroup per CU
// and a half-empty second round measured slower than the small shapes);
// below that (small batches) 32x32 wave tiles over whole pairs
// of t-rows (F = 64: 8 waves, F = 32: 4), or at F = 16 / 8 16x16 wave tiles
// over pairs of t-rows (8 / 4 waves), BN = 64.  All give bit-identical
// outputs.
template <int F, int BN, bool FUSE>
static void launch_f_bn(const float* in, int B, int T, int Cin, int Cout, const float* wp,
                        const float* bias, float* out, int epi, const float* w1, const float* b1,
                        const float* zero16, hipStream_t s) {
  const int64_t ncu = device_cus();
  constexpr int TT8 = ExactGeom<F, BN, FUSE, 8, 64>::TT, TT4 = ExactGeom<F, BN, FUSE, 4, 64>::TT;
  const int64_t tiles8 = (int64_t)B * ((T + TT8 - 1) / TT8) * (Cout / BN);
  const int64_t tiles4 = (int64_t)B * ((T + TT4 - 1) / TT4) * (Cout / BN);
  constexpr int SW = (F == 8 ? 32 : 2 * F) / 32 * 2;   // WT = 32 shape: (BM / 32) x (64 / 32) waves
  if (tiles8 >= 2 * ncu)
    launch_f_bn_w<F, BN, FUSE, 8, 64>(in, B, T, Cin, Cout, wp, bias, out, epi, w1, b1, zero16, s);
  else if (tiles4 >= 2 * ncu)
    launch_f_bn_w<F, BN, FUSE, 4, 64>(in, B, T, Cin, Cout, wp, bias, out, epi, w1, b1, zero16, s);
  else if constexpr (F <= 16)   // WT = 16: 2 t-rows x F bins, BN = 64 -> (2F / 16) x 4 waves
    launch_f_bn_w<F, 64, FUSE, F / 2, 16>(in, B, T, Cin, Cout, wp, bias, out, epi, w1, b1, zero16, s);
  else
    launch_f_bn_w<F, 64, FUSE, SW, 32>(in, B, T, Cin, Cout, wp, bias, out, epi, w1, b1, zero16, s);
}

void launch_conv3x3(const float* in, int B, int T, int F, int Cin, int Cout, const float* wp,
                    const float* bias, float* out, int epi, const float* zero16, hipStream_t s) {
  // F is 64/32/16/8 on this path (mel_bins=64 halved by each 2x2 pool); the
  // instantiated (F, epilogue) pairs are the model's
  if (Cin % 4 != 0) return note_launch_error(hipErrorInvalidValue);
  switch (F) {
    case 32:
      if (Cout % 128 == 0) launch_f_bn<32, 128, false>(in, B, T, Cin, Cout, wp, bias, out, epi, nullptr, nullptr, zero16, s);
      else note_launch_error(hipErrorInvalidValue);   // never leave the output unwritten silently
      break;
    case 16:
      if (Cout % 128 == 0) launch_f_bn<16, 128, false>(in, B, T, Cin, Cout, wp, bias, out, epi, nullptr, nullptr, zero16, s);
      else note_launch_error(hipErrorInvalidValue);   // never leave the output unwritten silently
      break;
    case 8:
      if (Cout % 128 == 0) launch_f_bn<8, 128, false>(in, B, T, Cin, Cout, wp, bias, out, epi, nullptr, nullptr, zero16, s);
      else note_launch_error(hipErrorInvalidValue);   // never leave the output unwritten silently
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
