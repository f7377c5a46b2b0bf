// 3x3 conv of the 9-layer CNN (ConvBlock, pytorch/models.py:98-141) as fp32
// Winograd F(2x2, 3x3) on v_mfma_f32_32x32x2_f32: every operand, product and
// sum is fp32 (no narrower type anywhere), 16 multiplies per 2x2 output tile
// instead of 36 (2.25x fewer matrix-pipe FLOPs than the direct conv.hip).
//
// Per output tile (2 t x 2 f) and input channel c the 4x4 input patch d
// (rows t-1..t+2, cols f-1..f+2, zero outside the clip) is transformed to
// V = B^T d B; the folded 3x3 weights g (BN scale applied) to U = G g G^T
// (host, float64, rounded once to fp32); the 16 element-wise positions
// p = 4 i + j are 16 independent GEMMs  M_p[tile][n] = sum_c V_p[tile][c] U_p[c][n]
// and the output is Y = A^T M A, then + bias, ReLU and the block's epilogue
// (Lavin & Gray 2016; B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],
// G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1], A^T = [1 1 1 0; 0 1 -1 -1]).
//
// Waves (round 4: "row waves"): a tile group = 32 tiles x 32 NT output
// channels (NT = 2 channel tiles, 1 for small grids), computed by FOUR waves,
// wave ROW owning the 4 positions of V row ROW for every channel tile
// (4 NT MFMA accumulator tiles, 128 registers at NT = 2): one V fragment
// feeds NT MFMAs, so the in-lane input transform and the patch reads are
// paid once per 64 channels (round 3's layout — a wave pair per 32 channels,
// each wave two V rows — computed every V twice per 64 channels: block 1's
// two channel groups, blocks 2-4's consecutive channel-group items).
// The input transform is in-lane: lane (tile m, k-half kh) reads the 2 patch
// rows its V row needs (8 pixels, channels 2 kh and 2 kh + 1 of a 4-channel
// chunk: 8 ds_read_b64) and its 4 transformed values per channel ARE its A
// fragments — V never exists in LDS or HBM.  The output transform: a lane's
// register r holds the same (tile, channel) in all of its position tiles, so
// each wave reduces its row to z = (M A)_ROW in registers; Y = A^T M A then
// sums the four rows' z — the row waves swap their z through LDS, one channel
// tile per round, and each finishes a quarter of the registers.
// A workgroup is TG tile groups (4 TG waves) x 32 NT channels; per 4-channel
// chunk the raw halo ([pixel][4 ch], 16 B per pixel, four parity planes) and
// the chunk's U slab ([p][h][n][ks]) are copied global -> LDS by LDS-DMA into
// a 3-buffer ring, NBUF - 1 chunks ahead, one counted-vmcnt barrier per chunk
// (the exact kernel's pipeline); the next chunk's reads and transform are
// spread between the current chunk's MFMAs.
//
// Workgroup -> (tile block, channel group) is XCD-aware: the channel groups
// of one tile block are consecutive workgroups of one XCD (same halo, one
// L2), so the halo comes from HBM once per layer.
//
// Every shape (TG = 2 / 1, NT = 2 / 1) performs the same operations in the
// same order for each (tile, channel), so outputs do not depend on the batch
// size or the shape chosen.
#include <type_traits>

#include "sedx_internal.h"

namespace sedx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4w __attribute__((ext_vector_type(4)));

// TG tile groups (32 tiles each) x 32 NT channels per workgroup, 4 TG waves.
// C1 (block 1, F = 64): the input is the bn0 output X0 [B][T][64] and conv1
// (Cin 1 -> 64, BN folded, ReLU) is computed into each chunk's halo image in
// LDS (below): conv1's 64-channel activation never exists in HBM.
template <int F, int TG, int NT = 2, bool C1 = false>
struct WinoGeom {
  static constexpr int WAVES = 4 * TG;               // row waves 0..3 of each tile group
  static constexpr int THREADS = 64 * WAVES;
  static constexpr int NCH = 32 * NT;                // output channels per workgroup
  static constexpr int P = 32 * TG;                  // tiles per workgroup
  static constexpr int FT = F / 2;                   // tiles per tile row
  static constexpr int TRW = P / FT;                 // tile rows per workgroup
  static constexpr int RT = 2 * TRW + 2, CS = F + 2, KC = 4;
  static constexpr int PL = RT * CS;                 // halo pixels
  static constexpr int PLP = (PL + 63) / 64 * 64;    // whole 64-pixel DMA units
  // floats: [pixel][4 ch] (C1: a 64-pixel conv1 group for every wave; the
  // groups past the halo write zeros into the padding)
  static constexpr int A_SZ = KC * (C1 && PLP < 64 * WAVES ? 64 * WAVES : PLP);
  static constexpr int W_SZ = 16 * KC * NCH;         // floats: [p][h][n NCH][ks]
  static constexpr int BUF = A_SZ + W_SZ;
#ifndef SEDX_WINO_NBUF
#define SEDX_WINO_NBUF 3
#endif
  static constexpr int NBUF = SEDX_WINO_NBUF;        // ring depth
  static constexpr int UW = W_SZ / 256;              // 1-KiB DMA units per chunk
  static constexpr int UA = C1 ? 0 : PLP / 64;       // halo units (C1 computes the halo instead)
  static constexpr int U = UW + UA;
  static constexpr int UPW = (U + WAVES - 1) / WAVES;
  static constexpr int VM_MIN = U / WAVES;           // units of the wave with the fewest
  // epilogue exchange, one channel tile per round: per tile group
  // [finisher row 4][other row 3][register 4][z 2][lane 64] floats
  static constexpr int XTG = 4 * 3 * 4 * 2 * 64;
  static constexpr int XCH = TG * XTG;
  // C1: an item's X0 rows t0 - 2 .. t0 + RT - 1 ([row][F], zero rows outside
  // the clip), two buffers by item parity, in 1-KiB DMA units; the conv1
  // halo pixels in 64-pixel groups, one group per wave
  static constexpr int XROWS = RT + 2;
  static constexpr int UX = C1 ? (XROWS * F + 255) / 256 : 0;
  static constexpr int X0_SZ = 256 * UX;
  static constexpr int XA_OFF = NBUF * BUF + XCH;
  // the layer's biases (Cout <= 512), LDS-DMA'd once in the prologue: read
  // from LDS, the epilogue's bias needs no vmcnt wait (which would also wait
  // for the next item's DMAs in flight)
  static constexpr int BIAS_OFF = XA_OFF + 2 * X0_SZ, BIAS_MAX = 512;
  // C1 with conv1 on the matrix pipe: conv1's weights [64 ch][9] (3 DMA
  // units, zero-padded) and biases (1 unit), LDS-DMA'd in the prologue
  static constexpr int W1_OFF = BIAS_OFF + BIAS_MAX, W1_SZ = C1 ? 1024 : 0;
  static constexpr int LDS_BYTES = 4 * (W1_OFF + W1_SZ);   // ring, epilogue exchange, X0 tiles, biases, conv1 weights
  static constexpr int WG_PER_CU = WAVES == 8 || LDS_BYTES > 80 * 1024 ? 1 : 2;
  static_assert(NT == 1 || NT == 2, "channel tiles per wave");
  static_assert(P % FT == 0, "whole tile rows per workgroup");
  static_assert(VM_MIN * (NBUF - 1) <= 63, "vmcnt field");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS per workgroup");
  static_assert(!C1 || (F == 64 && NT == 2 && PLP <= 64 * WAVES && UX <= WAVES && NBUF >= 3), "C1: block 1 (64 bins), a conv1 group per wave");
};

// Diagnostic builds only (tools/wino_b1_bench.cpp, tools/gpu_r04d.sh; never
// the library): SEDX_WINO_STAMPS accumulates per-wave s_memtime intervals by
// phase, from every wave of every 16th workgroup, into g_wino_stamps:
//   [0] prologue  [1] item top (chunk 0 reads + transform, next item's DMA
//   sources)  [2] chunk steps (MFMAs with the next chunk's LDS reads,
//   transform and C1's conv1 interleaved)  [3] barrier waits  [4] DMA issue
//   (+ C1's X0 tile)  [5] C1's window load  [6] epilogue  [7] whole wave
//   [8] waves sampled
// SEDX_WINO_ABL (a bit mask) removes one piece of work — results WRONG,
// timing only: 1 conv1, 2 the input transform, 4 the patch LDS reads, 8 the U
// LDS reads, 16 the DMAs of the chunk operands.
#ifndef SEDX_WINO_ABL
#define SEDX_WINO_ABL 0
#endif
// block 1's conv1 on the matrix pipe (v_mfma_f32_4x4x1f32, 16 blocks) instead
// of VALU fma chains: the same fma chain per (pixel, channel)
#ifndef SEDX_WINO_C1MFMA
#define SEDX_WINO_C1MFMA 0
#endif
// VALU instructions per MFMA in the second half of a chunk step (tuning builds)
#ifndef SEDX_WINO_VG
#define SEDX_WINO_VG 3
#endif
#ifndef SEDX_WINO_VG1
#define SEDX_WINO_VG1 9
#endif
#ifdef SEDX_WINO_STAMPS
__device__ unsigned long long g_wino_stamps[16];
#define WS_DECL                                      \
  unsigned long long ws_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long ws_t = __builtin_amdgcn_s_memtime();  \
  const unsigned long long ws_t0 = ws_t;
#define WS_MARK(i)                                           \
  {                                                          \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
    ws_acc[i] += n_ - ws_t;                                  \
    ws_t = n_;                                               \
  }
#define WS_FLUSH()                                                           \
  if (lane == 0 && (blockIdx.x & 15) == 0) {                                 \
    ws_acc[7] = __builtin_amdgcn_s_memtime() - ws_t0;                        \
    for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_wino_stamps[i_], ws_acc[i_]); \
    atomicAdd(&g_wino_stamps[8], 1ull);                                      \
  }
#else
#define WS_DECL
#define WS_MARK(i)
#define WS_FLUSH()
#endif

// raw workgroup barrier behind "this wave's DMAs older than its N youngest
// VMEM ops landed, its LDS operations done" (__syncthreads() would drain
// every DMA in flight); N = VM x y for y = min(younger, Y) chunks in flight
template <int N>
__device__ __forceinline__ void wino_bar_n() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
// S: this wave's epilogue stores issued after the awaited chunk's DMA (a
// persistent workgroup's previous tile; every store is issued, so the count
// is exact)
template <int VM, int Y, int S = 0>
__device__ __forceinline__ void wino_bar(int younger) {
  if constexpr (Y > 0) {
    if (younger >= Y) {
      wino_bar_n<VM * Y + S>();
      return;
    }
    wino_bar<VM, Y - 1, S>(younger);
  } else {
    wino_bar_n<S>();
  }
}

// 4-point column pass of B^T d B: (x0 - x2, x1 + x2, x2 - x1, x1 - x3)
__device__ __forceinline__ void wino_bt4(float* x) {
  const float e0 = x[0] - x[2], e1 = x[1] + x[2], e2 = x[2] - x[1], e3 = x[1] - x[3];
  x[0] = e0; x[1] = e1; x[2] = e2; x[3] = e3;
}

// the kernel body for V row ROW (wave-uniform; a template parameter so the
// transform, the U rows and the patch offsets are static per wave)
// C4O (block 1 only): the pooled output in the chunk-of-4 layout
// [B][Cout/4][T/2][F/2][4] that the F(4x4,3x3) layers read (conv_wino43.hip)
template <int F, int EPI, int TG, int NT, int ROW, bool C1, bool C4O = false>
__device__ __forceinline__ void wino_body(const float* __restrict__ in, int B, int T, int Cin, int Cout,
                                          const float* __restrict__ U, const float* __restrict__ bias,
                                          float* __restrict__ out, const float* __restrict__ zero16,
                                          float* __restrict__ trash, int tb_per_clip, int ngroups,
                                          const float* __restrict__ w1, const float* __restrict__ b1,
                                          int order2d = 0) {
  using G = WinoGeom<F, TG, NT, C1>;
  constexpr int WAVES = G::WAVES;
  constexpr int CS = G::CS, KC = G::KC, FT = G::FT;
  extern __shared__ __attribute__((aligned(16))) float smem[];   // G::LDS_BYTES (dynamic: > 64 KiB)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  WS_DECL
  // unit u = wv + WAVES k of this wave: a weight unit, a halo unit, or none.
  // Folded at compile time where k alone decides (k < UW / WAVES weight,
  // k >= ceil(UW / WAVES) halo; k < U / WAVES always present), so the
  // per-chunk DMA issue has no branches but the last unit's presence check
  // (and, when UW is not a multiple of WAVES, one wave-uniform test)
  auto is_w = [&](int k) {
    if ((k + 1) * WAVES <= G::UW) return true;
    if (k * WAVES >= G::UW) return false;
    return wv + WAVES * k < G::UW;
  };
  auto present = [&](int k, int wv_) { return (k + 1) * WAVES <= G::U || wv_ + WAVES * k < G::U; };
  // tile group of the wave: waves tg, tg + TG, tg + 2 TG, tg + 3 TG are its
  // V rows 0..3
  const int tg = wv % TG;
  // Persistent: workgroup g takes items g, g + gridDim.x, ... (gridDim.x a
  // multiple of 8, so every item of a workgroup is on its XCD).  XCD-aware
  // item decode: item -> XCD id & 7; on one XCD, tile blocks in order, each
  // with its channel groups consecutive.  Padding items (tile blocks rounded
  // up to a multiple of 8) come last on their XCD.
  // order2d = G > 0 (launcher: more than G channel groups, whole rounds of
  // 32 items per XCD, no padding tile blocks): each round of 32 consecutive
  // items on an XCD — the ones its 32 resident workgroups run together — is
  // 32 / G tile blocks x G channel groups instead of 32 / ngroups x ngroups,
  // so per round the XCD's L2 streams G weight slabs (at most ~8 MB) instead
  // of all of them (fewer L2 misses on the 512-input-channel layers; a
  // workgroup's successive items keep their slot in the round)
  auto decode = [&](int item, int& b_, int& t0_, int& n0_) -> bool {
    const int xcd = item & 7, j = item >> 3;
    int jb, cgi;
    if (order2d) {
      const int tbr = 32 / order2d;                // tile blocks per round
      const int idx = j & 31, r = j >> 5, ncg = ngroups / order2d;
      const int tbg = r / ncg;
      jb = tbr * tbg + idx % tbr;
      cgi = order2d * (r - tbg * ncg) + idx / tbr;
    } else {
      jb = j / ngroups;
      cgi = j - jb * ngroups;
    }
    const int tb = jb * 8 + xcd;
    if (tb >= B * tb_per_clip) return false;
    b_ = tb / tb_per_clip;
    t0_ = 2 * (tb - b_ * tb_per_clip) * G::TRW;   // first row (2 x first tile row)
    n0_ = cgi * G::NCH;
    return true;
  };
  // this workgroup's 128 trash floats (spread: the dummy and out-of-range
  // stores of different workgroups do not pile onto one cache line)
  float* const tr_lane = trash + (blockIdx.x & 63) * 128 + lane;
  int item = blockIdx.x;
  int b = 0, t0 = 0, n0 = 0;
  if (!decode(item, b, t0, n0)) return;   // uniform
  const int khalf = lane >> 5;

  // A side: this lane's tile (lane & 31) and channel pair (2 khalf, 2 khalf + 1).
  // Halo image in LDS: 16 B per pixel ([4 ch]) in four parity planes, slot
  // (r, c) -> ((r & 1) 2 + (c & 1)) Q + (r >> 1) HC + (c >> 1): a patch pixel
  // (2 tr + i, 2 tf + j) of the 32 tiles of a wave is then one plane at
  // consecutive slots along tf, so a fragment read spreads over all banks
  // (row-major pixels put the tiles 8 floats apart: 4-way conflicts)
  constexpr int HC = CS / 2, Q = G::PL / 4;
  const int pt = 32 * tg + (lane & 31);
  const int a_base = ((pt / FT) * HC + (pt % FT)) * KC + 2 * khalf;
  auto a_off = [&](int i, int jj) { return ((((i & 1) << 1) | (jj & 1)) * Q + (i >> 1) * HC + (jj >> 1)) * KC; };
  // B side: U slab [p][h][n NCH][ks], lane (h = khalf, n = 32 nt + (lane & 31)),
  // this wave's positions 4 ROW .. 4 ROW + 3 (rows of 2 NCH floats)
  const int b_base = G::A_SZ + 4 * ROW * 4 * G::NCH + khalf * 2 * G::NCH + 2 * (lane & 31);

  // ---- LDS-DMA units of this wave (unit u -> wave u % WAVES): LDS offsets
  // fixed, sources per item ----
  int dlds[G::UPW];
#pragma unroll
  for (int k = 0; k < G::UPW; ++k) {
    const int u = wv + WAVES * k;
    dlds[k] = is_w(k) ? G::A_SZ + 256 * u : 256 * (u - G::UW);
  }
  // a unit's source as a 32-bit element offset (from U + 2 n0 for weight
  // units, from in for halo units; -1: a pixel outside the clip, read from
  // the zero block): one VGPR per unit (the launcher checks B T F Cin < 2^31)
  auto desc = [&](int b_, int t0_, int (&off)[G::UPW]) {
#pragma unroll
    for (int k = 0; k < G::UPW; ++k) {
      const int u = wv + WAVES * k;
      off[k] = -1;
      if (is_w(k)) {
        constexpr int LPR = G::NCH / 2;   // lanes per (p, h) row of 2 NCH floats
        const int row = (64 / LPR) * u + lane / LPR;
        off[k] = row * 2 * Cout + 4 * (lane % LPR);
      } else if (present(k, wv)) {
        const int slot = 64 * (u - G::UW) + lane;
        const int q = slot / Q, rem = slot - q * Q;
        const int r = 2 * (rem / HC) + (q >> 1), c = 2 * (rem % HC) + (q & 1);
        const int t = t0_ - 1 + r, f = c - 1;
        if (slot < G::PL && t >= 0 && t < T && f >= 0 && f < F) off[k] = ((b_ * T + t) * F + f) * Cin;
      }
    }
  };
  auto dma = [&](const int (&off)[G::UPW], int n0_, int chunk_, int buf_) {
#pragma unroll
    for (int k = 0; k < G::UPW; ++k) {
      if (present(k, wv)) {
        const uint32_t m0_ =
            (uint32_t)(size_t)(__attribute__((address_space(3))) float*)(smem + buf_ * G::BUF + dlds[k]);
        const float* src = is_w(k) ? U + 2 * n0_ + off[k] + (int64_t)chunk_ * (64 * Cout)
                                     : (off[k] >= 0 ? in + off[k] + chunk_ * KC : zero16);
        if constexpr (!(SEDX_WINO_ABL & 16)) sedx_glds16(src, __builtin_amdgcn_readfirstlane(m0_));
      }
    }
    asm volatile("" ::: "memory");
  };
  // the current item's unit sources at chunk 0 (a chunk adds a uniform step:
  // 64 Cout floats for weight units, KC for halo units — a halo lane outside
  // the clip steps through the zero block, >= Cin + 4 floats)
  const float* dptr[G::UPW];
  auto ptrs = [&](const int (&off)[G::UPW], int n0_) {
#pragma unroll
    for (int k = 0; k < G::UPW; ++k) {
      dptr[k] = is_w(k) ? U + 2 * n0_ + off[k] : (off[k] >= 0 ? in + off[k] : zero16);
    }
  };
  auto dma_cur = [&](int chunk_, int buf_) {
#pragma unroll
    for (int k = 0; k < G::UPW; ++k) {
      if (present(k, wv)) {
        const uint32_t m0_ =
            (uint32_t)(size_t)(__attribute__((address_space(3))) float*)(smem + buf_ * G::BUF + dlds[k]);
        const int64_t stp = is_w(k) ? (int64_t)64 * Cout : KC;
        if constexpr (!(SEDX_WINO_ABL & 16)) sedx_glds16(dptr[k] + chunk_ * stp, __builtin_amdgcn_readfirstlane(m0_));
      }
    }
    asm volatile("" ::: "memory");
  };
  {
    int doff[G::UPW];
    desc(b, t0, doff);
    ptrs(doff, n0);
  }

  // ---- C1: conv1 into the halo images.  Wave wv owns halo slots 64 wv +
  // lane (one pixel per lane, the parity-plane slot order of the halo DMA;
  // slots past the halo compute into the padding, so no wave branches).  Per item its 3x3 X0 window sits in 9 registers, read from the
  // item's X0 tile in LDS (LDS-DMA'd with the previous item's last chunk, or
  // in the prologue); per chunk it computes its pixel's 4 channels of the
  // chunk c + 2 (two ahead: chunk c + 1 is read during chunk c) into that
  // chunk's ring buffer, one 16-byte LDS write.  Per channel the 9 taps are
  // one fma chain in tap order from 0, then + bias and ReLU — the operation
  // order of conv1_nhwc_kernel (and of the direct kernel's fused conv1), so
  // the outputs are bit-identical to the unfused Winograd block 1.  conv2's
  // zero padding: halo pixels outside the clip store 0. ----
  [[maybe_unused]] float xw[C1 ? 9 : 1];
  [[maybe_unused]] bool c1_ov = false;
  [[maybe_unused]] const int pslot = 64 * wv + lane;
  [[maybe_unused]] int pr = 0, pc = 0;
  if constexpr (C1) {
    const int sl = pslot < G::PL ? pslot : 0;
    const int q = sl / Q, rem = sl - q * Q;
    pr = 2 * (rem / HC) + (q >> 1);
    pc = 2 * (rem % HC) + (q & 1);
  }
  // X0 rows t0_ - 2 + xr of clip b_ -> X0 tile xb (unit x: wave x; 16 lanes a row)
  [[maybe_unused]] auto x0_dma = [&](int b_, int t0_, int xb) {
    if (wv < G::UX) {   // wave-uniform
      const int xr = 4 * wv + (lane >> 4);
      const int t = t0_ - 2 + xr;
      const float* src = (xr < G::XROWS && t >= 0 && t < T) ? in + ((b_ * T + t) * F + 4 * (lane & 15)) : zero16;
      const uint32_t m0_ =
          (uint32_t)(size_t)(__attribute__((address_space(3))) float*)(smem + G::XA_OFF + xb * G::X0_SZ + 256 * wv);
      sedx_glds16(src, __builtin_amdgcn_readfirstlane(m0_));
    }
    asm volatile("" ::: "memory");
  };
  // the lane's window from X0 tile xb (columns outside the bins read as 0;
  // rows outside the clip are zero rows of the tile) and its pixel's validity
  [[maybe_unused]] auto load_window = [&](int t0_, int xb) {
    {
      const float* xa = smem + G::XA_OFF + xb * G::X0_SZ;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int col = pc - 2 + dx;
          const float v = xa[(pr + dy) * F + min(max(col, 0), F - 1)];
          xw[dy * 3 + dx] = (col >= 0 && col < F) ? v : 0.0f;
        }
      const int t = t0_ - 1 + pr;
      c1_ov = pslot < G::PL && t >= 0 && t < T && pc >= 1 && pc <= F;
    }
  };
  // channels 4 cc .. 4 cc + 3 of the lane's pixel -> ring buffer cb
  // (the chunk's 36 weights + 4 biases are wave-uniform: scalar loads; issued
  // at the top of the chunk instead, the launch measured 2 % slower)
  [[maybe_unused]] auto c1_weights = [&](int cc, float (&wq)[40]) {
#pragma unroll
    for (int i = 0; i < 36; ++i) wq[i] = w1[36 * cc + i];
#pragma unroll
    for (int i = 0; i < 4; ++i) wq[36 + i] = b1[4 * cc + i];
  };
  [[maybe_unused]] auto conv1w = [&](const float (&wq)[40], int cb) {
    float y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = 0.0f;
#pragma unroll
      for (int k = 0; k < 9; ++k) a = fmaf(xw[k], wq[9 * i + k], a);
      const float v = fmaxf(a + wq[36 + i], 0.0f);
      y[i] = c1_ov ? v : 0.0f;
    }
    *reinterpret_cast<float4*>(smem + cb * G::BUF + 4 * pslot) = make_float4(y[0], y[1], y[2], y[3]);
  };
  // on the matrix pipe: v_mfma_f32_4x4x1f32 (16 blocks of 4 x 4, K = 1;
  // tools/mfma4x4_probe.cpp): lane l = 4 b + t supplies A[t][0] of block b
  // (the weight of channel 4 cc + t for tap k, from LDS) and B[0][t] (tap k
  // of its own pixel) and receives D[0..3][t] of block b — channels 4 cc ..
  // 4 cc + 3 of its pixel, i.e. the chunk's [pixel][4 ch] halo slot.  Nine
  // MFMAs from zero are the VALU form's fma chain over the taps in order
  [[maybe_unused]] auto conv1m = [&](int cc, int cb) {
    const float* wl = smem + G::W1_OFF + 9 * (4 * cc + (lane & 3));
    f32x4w d = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int k = 0; k < 9; ++k) d = __builtin_amdgcn_mfma_f32_4x4x1f32(wl[k], xw[k], d, 0, 0, 0);
    const float4 bq = *reinterpret_cast<const float4*>(smem + G::W1_OFF + 768 + 4 * cc);
    const float y0 = fmaxf(d[0] + bq.x, 0.0f), y1 = fmaxf(d[1] + bq.y, 0.0f);
    const float y2 = fmaxf(d[2] + bq.z, 0.0f), y3 = fmaxf(d[3] + bq.w, 0.0f);
    *reinterpret_cast<float4*>(smem + cb * G::BUF + 4 * pslot) =
        c1_ov ? make_float4(y0, y1, y2, y3) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  };
  [[maybe_unused]] auto conv1 = [&](int cc, int cb) {
    if constexpr (SEDX_WINO_C1MFMA) {
      conv1m(cc, cb);
    } else {
      float wq[40];
      c1_weights(cc, wq);
      conv1w(wq, cb);
    }
  };

  f32x16 acc[4][NT];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][nt][r] = 0.0f;

  // a chunk's operands in registers: V of this wave's 4 positions (both
  // k-steps) and the U fragments; two sets, ping-pong
  float va[2][4], vb[2][4];
  float2 ua[4][NT], ubv[4][NT];
  // V row ROW of B^T d from patch rows RA, RB:
  //   ROW 0: d0 - d2   1: d1 + d2   2: d2 - d1   3: d1 - d3
  constexpr int RA = ROW == 0 ? 0 : 1;
  constexpr int RB = ROW == 3 ? 3 : 2;
  // read chunk's patch rows + U fragments from LDS buffer buf (issue only)
  auto issue_reads = [&](int buf, float2 (&pd)[2][4], float2 (&un)[4][NT]) {
    const float* sm = smem + buf * G::BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        if constexpr (SEDX_WINO_ABL & 4) {
          float2 z = make_float2((float)i, (float)jj);
          asm volatile("" : "+v"(z.x), "+v"(z.y));
          pd[i][jj] = z;
        } else {
          pd[i][jj] = *reinterpret_cast<const float2*>(sm + a_base + a_off(i ? RB : RA, jj));
        }
      }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        if constexpr (SEDX_WINO_ABL & 8) {
          float2 z = make_float2((float)j, (float)nt);
          asm volatile("" : "+v"(z.x), "+v"(z.y));
          un[j][nt] = z;
        } else {
          un[j][nt] = *reinterpret_cast<const float2*>(sm + b_base + j * 4 * G::NCH + 64 * nt);
        }
      }
  };
  auto transform = [&](const float2 (&pd)[2][4], float (&vn)[2][4]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float a = ks ? pd[0][jj].y : pd[0][jj].x;   // patch row RA
        const float b = ks ? pd[1][jj].y : pd[1][jj].x;   // patch row RB
        if constexpr (SEDX_WINO_ABL & 2)
          vn[ks][jj] = a;
        else if constexpr (ROW == 1)
          vn[ks][jj] = a + b;
        else if constexpr (ROW == 2)
          vn[ks][jj] = b - a;
        else
          vn[ks][jj] = a - b;
      }
      if constexpr (!(SEDX_WINO_ABL & 2)) wino_bt4(&vn[ks][0]);
    }
    // pin V here: otherwise the compiler sinks each value's transform to the
    // MFMA that consumes it (next chunk), a VALU -> MFMA chain in front of
    // every matrix instruction
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(vn[ks][q]));
  };
  // the 8 NT MFMAs of one chunk from (vc, uc) — k-step 0 (channel 2 khalf) then
  // k-step 1 (2 khalf + 1), one V fragment per position for all NT channel
  // tiles — with the next chunk's LDS reads spread over the first half and
  // its transform over the second.  C1: then conv1 of channel chunk cc into
  // ring buffer cb
  auto mfmas = [&](const float (&vc)[2][4], const float2 (&uc)[4][NT]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[j][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(vc[ks][j], ks ? uc[j][nt].y : uc[j][nt].x, acc[j][nt], 0, 0, 0);
  };
  auto step = [&](const float (&vc)[2][4], const float2 (&uc)[4][NT], int nbuf, float (&vn)[2][4],
                  float2 (&un)[4][NT], int cc = -1, int cb = 0) {
    mfmas(vc, uc);
    float2 pd[2][4];
    issue_reads(nbuf, pd, un);
    transform(pd, vn);
    if constexpr (C1 && !(SEDX_WINO_ABL & 1)) conv1(cc, cb);
    // (round 3, measured slower: every LDS read ahead of the MFMAs, -10 %:
    // the transform then waits at the end of the chunk with nothing to
    // overlap; C1's conv1 beside the first MFMAs with its weights loaded a
    // chunk ahead, b1c2 +5 %: the reads then issue late)
    constexpr int NM = 8 * NT, NR = 8 + 4 * NT;
#pragma unroll
    for (int i = 0; i < NM / 2; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                        // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, (NR + NM / 2 - 1) / (NM / 2), 0);   // LDS reads
    }
#pragma unroll
    for (int i = 0; i < NM / 2; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                        // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, C1 ? SEDX_WINO_VG1 : (NT == 2 ? SEDX_WINO_VG : 5), 0);   // VALU (C1: + conv1's)
    }
  };

  const int nchunks = Cin / KC;   // even (Cin % 8 == 0, checked by the launcher)
  constexpr int NB = G::NBUF;
  // epilogue stores per wave (all issued: out-of-range ones go to trash)
  constexpr int S = NT * (EPI == EPI_FMEAN ? 2 : EPI == EPI_POOL2 ? 4 : 16);
  static_assert(G::VM_MIN * (NB - 2) + S <= 63, "vmcnt field");
  static_assert(!C1 || G::VM_MIN * NB + S <= 63, "vmcnt field");
  int xpar = 0;   // C1: the current item's X0 tile
  // the biases (oldest DMA of the prologue: covered by its first wait); unit
  // u = wave u, lanes past Cout read the zero block
  if (wv < G::BIAS_MAX / 256) {   // wave-uniform
    const int i = 256 * wv + 4 * lane;
    const uint32_t m0_ =
        (uint32_t)(size_t)(__attribute__((address_space(3))) float*)(smem + G::BIAS_OFF + 256 * wv);
    sedx_glds16(i < Cout ? bias + i : zero16, __builtin_amdgcn_readfirstlane(m0_));
    asm volatile("" ::: "memory");
  }
  if constexpr (C1 && SEDX_WINO_C1MFMA) {
    // conv1's weights (units 0-2: waves 2-4) and biases (wave 5), before the
    // ring: covered by the prologue's first wait like the biases
    if (wv >= 2 && wv < 6) {   // wave-uniform
      const int i = 256 * (wv - 2) + 4 * lane;
      const float* src = wv < 5 ? (i < 576 ? w1 + i : zero16) : (4 * lane < 64 ? b1 + 4 * lane : zero16);
      const uint32_t m0_ =
          (uint32_t)(size_t)(__attribute__((address_space(3))) float*)(smem + G::W1_OFF + 256 * (wv - 2));
      sedx_glds16(src, __builtin_amdgcn_readfirstlane(m0_));
      asm volatile("" ::: "memory");
    }
  }
  if constexpr (C1) x0_dma(b, t0, 0);
#pragma unroll
  for (int c = 0; c < NB; ++c) dma_cur(c, c);   // nchunks >= 8 (launcher)
  // S stores to trash: every item, the first included, then has S stores
  // between its chunk NB - 1 and chunk NB DMAs (a later item: the previous
  // item's epilogue), so all items wait alike
  {
    float* const vt = tr_lane;   // inline asm: exactly S global stores (never merged)
    const float zf = 0.0f;
#pragma unroll
    for (int i = 0; i < S; ++i) asm volatile("global_store_dword %0, %1, off" ::"v"(vt), "v"(zf) : "memory");
  }
  if constexpr (C1) {
    // the first item's X0 tile landed (the NB chunks' DMAs and the S stores
    // may be in flight): its window, then conv1 of chunks 0 and 1
    wino_bar_n<G::VM_MIN * NB + S>();
    load_window(t0, 0);
    conv1(0, 0);
    conv1(1, 1);
  }
  // chunk 0 landed: younger chunks 1 .. NB - 1 and the S stores may be in flight
  wino_bar<G::VM_MIN, NB - 1, S>(NB - 1);
  WS_MARK(0)

  // ---- epilogue pieces.  Register r of every position tile = MFMA row
  // m = (r & 3) + 8 (r >> 2) + 4 khalf (tile 32 tg + m), column lane & 31 of
  // channel tile nt.  This wave holds V row ROW of M: per register its row of
  // M A, z = (m0 + m1 + m2, m1 - m2 - m3) (A^T = [1 1 1 0; 0 1 -1 -1]), and
  // Y = A^T M A sums the rows: Y[0] = z_0 + z_1 + z_2, Y[1] = z_1 - z_2 - z_3
  // (in that order).  Wave ROW finishes registers 4 ROW .. 4 ROW + 3 of each
  // channel tile; the four row waves of a tile group hand each other their z
  // through LDS (an exchange area after the ring, so the next item's chunks
  // can already be landing), one channel tile per round.
  auto zrow = [&](int nt, int r, float (&z)[2]) {
    const float m0 = acc[0][nt][r], m1 = acc[1][nt][r], m2 = acc[2][nt][r], m3 = acc[3][nt][r];
    z[0] = (m0 + m1) + m2;
    z[1] = (m1 - m2) - m3;
  };
  // this tile group's exchange area: [finisher row f][other row][register k][z c][lane]
  float* const xg = smem + NB * G::BUF + tg * G::XTG;
  auto xslot = [](int f, int src) { return (f * 3 + (src < f ? src : src - 1)) * (4 * 2 * 64); };

  // top of chunk c: chunk c + 1 landed (c + 2 .. c + NB - 1 of the item
  // sequence may be in flight) and every wave has consumed chunk c's buffer
  // (its reads were waited for in the previous step), which then receives
  // chunk c + NB — of this item, or of the next one over the last chunks.
  // The next item's chunk 0 is read and transformed after the epilogue.
  int buf = 0;
  for (;;) {
    const int nitem = item + (int)gridDim.x;
    int nb_ = 0, nt0 = 0, nn0 = 0;
    const bool has_next = decode(nitem, nb_, nt0, nn0);
    {   // the item's chunk 0 (landed: the previous barrier waited for it)
      float2 pd[2][4];
      issue_reads(buf, pd, ua);
      transform(pd, va);
    }
    WS_MARK(1)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][nt][r] = 0.0f;
    auto issue = [&](int g, int bf) {
      if (g < nchunks) {
        dma_cur(g, bf);
      } else if (has_next) {
        int noff[G::UPW];
        desc(nb_, nt0, noff);
        dma(noff, nn0, g - nchunks, bf);
      }
    };
    // one chunk pair; LAST: the item's final pair, whose second step runs
    // the MFMAs only (the next item's chunk 0 is read at the next item's top)
    // MID: both DMAs of the pair are of this item and NB - 2 chunks are in
    // flight behind each awaited one (no branches: the steady state)
    auto pair = [&](int chunk, auto first_tag, auto last_tag, auto mid_tag) {
      constexpr bool FIRST = decltype(first_tag)::value, LAST = decltype(last_tag)::value;
      constexpr bool MID = decltype(mid_tag)::value;
      const int b1 = buf == NB - 1 ? 0 : buf + 1, b2 = b1 == NB - 1 ? 0 : b1 + 1;
      // chunks 1 and 2 of an item: the S stores (previous epilogue, or the
      // prologue's) were issued after their DMAs
      // C1: conv1 runs two chunks ahead — chunk + 2 into b2, chunk + 3 into
      // buf; over the last pair those are the next item's chunks 0 and 1,
      // from its window (its X0 tile was DMA'd with chunk nchunks - 1)
      WS_MARK(2)
      if constexpr (MID) {
        wino_bar_n<G::VM_MIN * (NB - 2) + (FIRST ? S : 0)>();
        WS_MARK(3)
        dma_cur(chunk + NB, buf);
      } else {
        wino_bar<G::VM_MIN, NB - 2, FIRST ? S : 0>(has_next ? NB - 2 : max(0, min(NB - 2, nchunks - chunk - 2)));
        WS_MARK(3)
        issue(chunk + NB, buf);
        // (without a next item: the current item's tile again, unused — the
        // pipeline stays branch-free; so are the window and conv1 below)
        if constexpr (C1 && !LAST && !(SEDX_WINO_ABL & 16)) x0_dma(has_next ? nb_ : b, has_next ? nt0 : t0, xpar ^ 1);
      }
      WS_MARK(4)
      if constexpr (C1 && LAST) load_window(has_next ? nt0 : t0, xpar ^ 1);
      WS_MARK(5)
      step(va, ua, b1, vb, ubv, C1 ? (LAST ? 0 : chunk + 2) : -1, b2);
      WS_MARK(2)
      if constexpr (MID) {
        wino_bar_n<G::VM_MIN * (NB - 2) + (FIRST ? S : 0)>();
        WS_MARK(3)
        dma_cur(chunk + 1 + NB, b1);
      } else {
        wino_bar<G::VM_MIN, NB - 2, FIRST ? S : 0>(has_next ? NB - 2 : max(0, min(NB - 2, nchunks - chunk - 3)));
        WS_MARK(3)
        issue(chunk + 1 + NB, b1);
      }
      WS_MARK(4)
      if constexpr (!LAST) {
        step(vb, ubv, b2, va, ua, C1 ? chunk + 3 : -1, buf);
      } else {
        mfmas(vb, ubv);
        if constexpr (C1 && !(SEDX_WINO_ABL & 1)) conv1(1, buf);
      }
      buf = b2;
    };
    // nchunks >= 8 (launcher): pair 0 and the middle pairs keep both DMAs in
    // this item; the last two pairs reach into the next one
    pair(0, std::true_type{}, std::false_type{}, std::true_type{});
    for (int chunk = 2; chunk < nchunks - 4; chunk += 2)
      pair(chunk, std::false_type{}, std::false_type{}, std::true_type{});
    pair(nchunks - 4, std::false_type{}, std::false_type{}, std::false_type{});
    pair(nchunks - 2, std::false_type{}, std::true_type{}, std::false_type{});
    WS_MARK(2)

    // ---- epilogue ----
    const int tr0 = t0 / 2;
    // the item's first output row as a 64-bit base; every store adds a
    // 32-bit offset within the item (no per-store 64-bit index math)
    float* const ob = EPI == EPI_FMEAN ? out + ((int64_t)b * T + t0) * Cout
                      : EPI == EPI_POOL2 ? out + ((int64_t)b * (T / 2) + tr0) * (F / 2) * Cout
                                         : out + ((int64_t)b * T + t0) * F * Cout;
    // an opaque copy of the lane index: the store offsets below are computed
    // here instead of being hoisted out of the item loop as live registers
    int le = lane;
    asm volatile("" : "+v"(le));
    const int khe = le >> 5;
    // registers 4 ROW + k: tiles 32 tg + 8 ROW + 4 khalf + k (k = 0..3)
    const int pt0 = 32 * tg + 8 * ROW + 4 * khe;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      // LDS-only barriers (__syncthreads() would drain the next item's DMAs):
      // the previous round's reads are done before this round's writes
      if (nt > 0) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int f = 0; f < 4; ++f) {   // the other rows' registers
        if (f == ROW) continue;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float z[2];
          zrow(nt, 4 * f + k, z);
          xg[xslot(f, ROW) + (2 * k) * 64 + lane] = z[0];
          xg[xslot(f, ROW) + (2 * k + 1) * 64 + lane] = z[1];
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const int n = n0 + 32 * nt + (le & 31);
      const float bv = smem[G::BIAS_OFF + n];
      // full Y of register 4 ROW + k (+ bias, ReLU), as y[a][b]
      auto outtile = [&](int k, float (&y)[2][2]) {
        float z[4][2];
        zrow(nt, 4 * ROW + k, z[ROW]);
#pragma unroll
        for (int src = 0; src < 4; ++src) {
          if (src == ROW) continue;
          z[src][0] = xg[xslot(ROW, src) + (2 * k) * 64 + lane];
          z[src][1] = xg[xslot(ROW, src) + (2 * k + 1) * 64 + lane];
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          y[0][c] = fmaxf(((z[0][c] + z[1][c]) + z[2][c]) + bv, 0.0f);
          y[1][c] = fmaxf(((z[1][c] - z[2][c]) - z[3][c]) + bv, 0.0f);
        }
      };
      if constexpr (EPI == EPI_FMEAN) {
        // F = 8: the 4 registers are the 4 tiles (bins 0-7) of tile row
        // 8 tg + 2 ROW + khalf; torch.mean over the 8 bins
        static_assert(F == 8, "freq-mean epilogue: F = 8");
        float y[4][2][2];
#pragma unroll
        for (int k = 0; k < 4; ++k) outtile(k, y[k]);
        const int trl = pt0 / FT;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          float sum = 0.0f;
#pragma unroll
          for (int k = 0; k < 4; ++k) sum = (sum + y[k][a][0]) + y[k][a][1];
          const int t = t0 + 2 * trl + a;
          float* dst = t < T ? ob + (2 * trl + a) * Cout + n : tr_lane;
          *dst = sum * (1.0f / F);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int ptile = pt0 + k;
          const int trl = ptile / FT, tf = ptile % FT;
          float y[2][2];
          outtile(k, y);
          if constexpr (EPI == EPI_POOL2) {
            const int To = T / 2;
            const int to = tr0 + trl;
            const float pv = (((y[0][0] + y[0][1]) + y[1][0]) + y[1][1]) * 0.25f;
            float* dst;
            if constexpr (C4O)
              dst = to < To ? out + ((((int64_t)b * (Cout / 4) + (n >> 2)) * To + to) * (F / 2) + tf) * 4 + (n & 3)
                            : tr_lane;
            else
              dst = to < To ? ob + (trl * (F / 2) + tf) * Cout + n : tr_lane;
            *dst = pv;
          } else {
#pragma unroll
            for (int a = 0; a < 2; ++a) {
              const int t = t0 + 2 * trl + a;
              float* o = t < T ? ob + ((2 * trl + a) * F + 2 * tf) * Cout + n : tr_lane;
              const int64_t o1 = t < T ? Cout : 64;
              o[0] = y[a][0];
              o[o1] = y[a][1];
            }
          }
        }
      }
    }
    WS_MARK(6)
    if (!has_next) break;
    // the other rows' reads of this item's exchange slots finish before the
    // next item's epilogue overwrites them: many barriers lie between
    item = nitem;
    xpar ^= 1;
    b = nb_;
    t0 = nt0;
    n0 = nn0;
    {
      int doff[G::UPW];
      desc(b, t0, doff);
      ptrs(doff, n0);
    }
  }
  WS_FLUSH()
}

// the V row of a wave (wave-uniform): one body instantiation per row
#define SEDX_WINO_ROWS(F_, EPI_, TG_, NT_, C1_, ...)                                    \
  SEDX_WINO_ROWS4(F_, EPI_, TG_, NT_, C1_, false, __VA_ARGS__)
#define SEDX_WINO_ROWS4(F_, EPI_, TG_, NT_, C1_, C4O_, ...)                             \
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) / TG_) {                    \
    case 0: wino_body<F_, EPI_, TG_, NT_, 0, C1_, C4O_>(__VA_ARGS__); break;           \
    case 1: wino_body<F_, EPI_, TG_, NT_, 1, C1_, C4O_>(__VA_ARGS__); break;           \
    case 2: wino_body<F_, EPI_, TG_, NT_, 2, C1_, C4O_>(__VA_ARGS__); break;           \
    default: wino_body<F_, EPI_, TG_, NT_, 3, C1_, C4O_>(__VA_ARGS__); break;          \
  }

template <int F, int EPI, int TG, int NT>
__global__ __launch_bounds__(256 * TG, (WinoGeom<F, TG, NT>::WG_PER_CU)) void conv3x3_wino_kernel(
    const float* __restrict__ in, int B, int T, int Cin, int Cout, const float* __restrict__ U,
    const float* __restrict__ bias, float* __restrict__ out, const float* __restrict__ zero16,
    float* __restrict__ trash, int tb_per_clip, int ngroups, int order2d) {
  SEDX_WINO_ROWS(F, EPI, TG, NT, false, in, B, T, Cin, Cout, U, bias, out, zero16, trash, tb_per_clip, ngroups,
                 nullptr, nullptr, order2d)
}

// Block 1 in one launch: conv1 (computed into the halo images) + Winograd
// conv2 + 2x2 pool, TG tile groups x 64 channels per workgroup (the conv1
// halo serves all 64 output channels)
template <int TG, bool C4O = false>
__global__ __launch_bounds__(256 * TG, (WinoGeom<64, TG, 2, true>::WG_PER_CU)) void wino_block1_kernel(
    const float* __restrict__ x0, int B, int T, const float* __restrict__ U, const float* __restrict__ bias,
    float* __restrict__ out, const float* __restrict__ zero16, float* __restrict__ trash, int tb_per_clip,
    const float* __restrict__ w1, const float* __restrict__ b1) {
  SEDX_WINO_ROWS4(64, EPI_POOL2, TG, 2, true, C4O, x0, B, T, 64, 64, U, bias, out, zero16, trash, tb_per_clip, 1, w1,
                  b1, 0)
}
#undef SEDX_WINO_ROWS
#undef SEDX_WINO_ROWS4

static int wino_device_cus() {
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return ncu;
}

#ifndef SEDX_WINO_ITEMS
#define SEDX_WINO_ITEMS 4
#endif
constexpr int WINO_ITEMS = SEDX_WINO_ITEMS;
// block 1's one-launch kernel: ~8 items per workgroup (isolated 0.731-0.733
// ms against 0.735-0.744 at 4 and 0.748-0.752 at 2; the two-stream headline
// the same within noise over four alternating rounds, tools/gpu_ab_iso.sh)
#ifndef SEDX_WINO_ITEMS_B1
#define SEDX_WINO_ITEMS_B1 8
#endif
constexpr int WINO_ITEMS_B1 = SEDX_WINO_ITEMS_B1;

template <int F, int TG, int NT>
static void launch_wino_w(const float* in, int B, int T, int Cin, int Cout, const float* U, const float* bias,
                          float* out, int epi, const float* zero16, float* trash, int order, hipStream_t s) {
  using G = WinoGeom<F, TG, NT>;
  // tile rows of a clip: POOL2 drops an odd last row (floor), the others keep it
  const int trows = epi == EPI_POOL2 ? T / 2 : (T + 1) / 2;
  const int tb_per_clip = (trows + G::TRW - 1) / G::TRW;
  const int ngroups = Cout / G::NCH;
  const int64_t tblocks = (int64_t)B * tb_per_clip;
  const int64_t nitems = (tblocks + 7) / 8 * 8 * ngroups;
  if (nitems > INT32_MAX || tblocks <= 0 || (int64_t)B * T * F * Cin >= INT32_MAX)   // 32-bit DMA offsets
    return note_launch_error(hipErrorInvalidValue);
  // persistent workgroups: as many as are resident, a multiple of 8
  // (XCD-aware item decode); each walks its items with
  // the next item's first chunks landing during the current one's last
  // ~WINO_ITEMS items per workgroup, but at least one resident round: the
  // hardware dispatcher still balances the workgroups over the CUs (a CU
  // shared with another stream's kernel finishes its workgroups later)
  const int64_t resident = (int64_t)wino_device_cus() * G::WG_PER_CU / 8 * 8;
  const int64_t per = (nitems + WINO_ITEMS - 1) / WINO_ITEMS;
  const int64_t nwg = std::min<int64_t>(nitems, std::max<int64_t>(std::max<int64_t>(8, resident), (per + 7) / 8 * 8));
  dim3 grid((unsigned)nwg);
  // rounds of 32 / G tile blocks x G channel groups: the G (< ngroups,
  // dividing it) whose round streams the fewest bytes through the XCD's L2 —
  // G weight slabs (16 Cin NCH floats each) + 32 / G halos (PL Cin floats) —
  // with whole rounds of tile blocks per XCD, no padding, and a grid of whole
  // 32-item rounds per XCD (a workgroup keeps its slot in the round from item
  // to item).  (b4c2: 4 slabs of 2 MB + 8 halos of 0.7 MB instead of 8 + 4.)
  int order2d = 0;
  if (order && nwg % 256 == 0 && (nitems / 8) % 32 == 0) {
    const int64_t slab = (int64_t)16 * Cin * G::NCH * 4, halo = (int64_t)G::PL * Cin * 4;
    int64_t best = (int64_t)ngroups * slab + (32 / std::min(ngroups, 32)) * halo;   // the default order
    for (int gr = 1; gr <= 8 && gr < ngroups; gr *= 2) {
      const int64_t bytes = gr * slab + (32 / gr) * halo;
      if (ngroups % gr == 0 && tblocks % (8 * (32 / gr)) == 0 && bytes < best) {
        best = bytes;
        order2d = gr;
      }
    }
  }
#define SEDX_WG_LAUNCH(E)                                                                              \
  {                                                                                                    \
    auto* k_ = conv3x3_wino_kernel<F, E, TG, NT>;                                                      \
    if (!launch_info(reinterpret_cast<const void*>(k_), G::THREADS, G::LDS_BYTES).ok) return;          \
    hipLaunchKernelGGL(k_, grid, dim3(G::THREADS), G::LDS_BYTES, s, in, B, T, Cin, Cout, U, bias, out, zero16, \
                       trash, tb_per_clip, ngroups, order2d);                                          \
    return;                                                                                            \
  }
  if constexpr (F == 8) {
    if (epi == EPI_STORE) SEDX_WG_LAUNCH(EPI_STORE);
    if (epi == EPI_FMEAN) SEDX_WG_LAUNCH(EPI_FMEAN);
  } else {
    if (epi == EPI_STORE) SEDX_WG_LAUNCH(EPI_STORE);
    if (epi == EPI_POOL2) SEDX_WG_LAUNCH(EPI_POOL2);
  }
#undef SEDX_WG_LAUNCH
  note_launch_error(hipErrorInvalidValue);
}


// 2 tile groups x 64 channels (8 waves) when that gives every CU a
// workgroup, else 1 x 64, else 1 x 32: the same per-(tile, channel) work,
// bit-identical outputs
template <int F>
static void launch_wino_f(const float* in, int B, int T, int Cin, int Cout, const float* U, const float* bias,
                          float* out, int epi, const float* zero16, float* trash, int order, hipStream_t s) {
  const int64_t ncu = wino_device_cus();
  const int trows = epi == EPI_POOL2 ? T / 2 : (T + 1) / 2;
  auto wgs = [&](int trw, int nch) { return (int64_t)B * ((trows + trw - 1) / trw) * (Cout / nch); };
#ifdef SEDX_WINO_TG3
  if (wgs(WinoGeom<F, 3, 1>::TRW, 32) >= ncu)
    launch_wino_w<F, 3, 1>(in, B, T, Cin, Cout, U, bias, out, epi, zero16, trash, order, s);
  else
#endif
#ifdef SEDX_WINO_TG4
  if (wgs(WinoGeom<F, 4, 1>::TRW, 32) >= ncu)
    launch_wino_w<F, 4, 1>(in, B, T, Cin, Cout, U, bias, out, epi, zero16, trash, order, s);
  else
#endif
  if (wgs(WinoGeom<F, 2, 2>::TRW, 64) >= ncu)
    launch_wino_w<F, 2, 2>(in, B, T, Cin, Cout, U, bias, out, epi, zero16, trash, order, s);
  else if (wgs(WinoGeom<F, 1, 2>::TRW, 64) >= ncu)
    launch_wino_w<F, 1, 2>(in, B, T, Cin, Cout, U, bias, out, epi, zero16, trash, order, s);
  else
    launch_wino_w<F, 1, 1>(in, B, T, Cin, Cout, U, bias, out, epi, zero16, trash, order, s);
}

void launch_conv3x3_wino(const float* in, int B, int T, int F, int Cin, int Cout, const float* U,
                         const float* bias, float* out, int epi, const float* zero16, float* trash, hipStream_t s,
                         int order) {
  // halo lanes outside the clip step through the zero block by the chunk's
  // channel offset: it must hold Cin + 4 floats
  if (Cin % 8 != 0 || Cin < 32 || Cout % 64 != 0 || Cout > 512 || B <= 0 || T <= 0 || Cin + 4 > ZERO_BLOCK_FLOATS)
    return note_launch_error(hipErrorInvalidValue);
  // the kernel's DMA offsets are 32-bit: batches whose input passes 2^31
  // elements run as several launches over whole clips (same per-clip work,
  // so the outputs do not depend on the split)
  const int64_t in_clip = (int64_t)T * F * Cin;
  const int64_t out_clip = epi == EPI_STORE ? (int64_t)T * F * Cout
                           : epi == EPI_POOL2 ? (int64_t)(T / 2) * (F / 2) * Cout : (int64_t)T * Cout;
  const int64_t bmax = (INT32_MAX - 1) / in_clip;
  if (bmax < 1) return note_launch_error(hipErrorInvalidValue);
  for (int64_t b0 = 0; b0 < B; b0 += bmax) {
    const int bs = (int)std::min<int64_t>(bmax, B - b0);
    const float* in_s = in + b0 * in_clip;
    float* out_s = out + b0 * out_clip;
    switch (F) {
      case 64: launch_wino_f<64>(in_s, bs, T, Cin, Cout, U, bias, out_s, epi, zero16, trash, order, s); break;
      case 32: launch_wino_f<32>(in_s, bs, T, Cin, Cout, U, bias, out_s, epi, zero16, trash, order, s); break;
      case 16: launch_wino_f<16>(in_s, bs, T, Cin, Cout, U, bias, out_s, epi, zero16, trash, order, s); break;
      case 8: launch_wino_f<8>(in_s, bs, T, Cin, Cout, U, bias, out_s, epi, zero16, trash, order, s); break;
      default: return note_launch_error(hipErrorInvalidValue);
    }
  }
}

template <int TG>
static void launch_block1_w(const float* x0, int B, int T, const float* U, const float* bias, float* out,
                            const float* w1, const float* b1, const float* zero16, float* trash, bool c4,
                            hipStream_t s) {
  using G = WinoGeom<64, TG, 2, true>;
  const int tb_per_clip = (T / 2 + G::TRW - 1) / G::TRW;   // pooled: an odd last t-row is dropped
  const int64_t tblocks = (int64_t)B * tb_per_clip;
  const int64_t nitems = (tblocks + 7) / 8 * 8;           // one channel group (64 channels) per item
  if (nitems > INT32_MAX || tblocks <= 0 || (int64_t)B * T * 64 >= INT32_MAX) return note_launch_error(hipErrorInvalidValue);
  const int64_t resident = (int64_t)wino_device_cus() * G::WG_PER_CU / 8 * 8;
  const int64_t per = (nitems + WINO_ITEMS_B1 - 1) / WINO_ITEMS_B1;
  const int64_t nwg = std::min<int64_t>(nitems, std::max<int64_t>(std::max<int64_t>(8, resident), (per + 7) / 8 * 8));
  auto* k_ = c4 ? wino_block1_kernel<TG, true> : wino_block1_kernel<TG, false>;
  if (!launch_info(reinterpret_cast<const void*>(k_), G::THREADS, G::LDS_BYTES).ok) return;
  hipLaunchKernelGGL(k_, dim3((unsigned)nwg), dim3(G::THREADS), G::LDS_BYTES, s, x0, B, T, U, bias, out, zero16, trash,
                     tb_per_clip, w1, b1);
}

void launch_block1_wino(const float* x0, int B, int T, const float* w1, const float* b1, const float* U,
                        const float* bias, float* out, const float* zero16, float* trash, hipStream_t s, bool c4) {
  if (B <= 0 || T < 2) return note_launch_error(hipErrorInvalidValue);
  // 32-bit X0 offsets: batches past 2^31 floats run as several launches over
  // whole clips (same per-clip work)
  const int64_t in_clip = (int64_t)T * 64, out_clip = (int64_t)(T / 2) * 32 * 64;
  const int64_t bmax = (INT32_MAX - 1) / in_clip;
  for (int64_t b0 = 0; b0 < B; b0 += bmax) {
    const int bs = (int)std::min<int64_t>(bmax, B - b0);
    // 2 tile groups x 64 channels (64 tiles, 8 waves) at every batch size
    // (with 1 tile group the 4 waves would not cover the halo's conv1 pixel
    // groups)
    launch_block1_w<2>(x0 + b0 * in_clip, bs, T, U, bias, out + b0 * out_clip, w1, b1, zero16, trash, c4, s);
  }
}

// Block 1's conv1 (Cin = 1, BN folded, ReLU) as its own launch for the
// Winograd block 1: X0 [B][T][64 bins] -> [B][T][64 bins][64 ch] NHWC, the
// conv2 input.  A workgroup writes C1_ROWS whole t-rows of one clip (16 KB
// each, contiguous): the X0 rows it needs (zero-bordered) and the weights
// sit in LDS, a thread owns one pixel x 4 channels per step (one 16-byte
// store; 16 consecutive threads write a pixel's 256 bytes).  Per channel the
// 9 taps are one fma chain in tap order from 0, then + bias and ReLU — the
// operation order of the direct kernel's fused conv1.
constexpr int C1_ROWS = 4;
__global__ __launch_bounds__(256) void conv1_nhwc_kernel(const float* __restrict__ x0, int T, int rb_per_clip,
                                                         const float* __restrict__ w1, const float* __restrict__ b1,
                                                         float* __restrict__ out) {
  __shared__ float s_w[64 * 9], s_b[64];
  __shared__ float s_x[C1_ROWS + 2][66];
  const int b = blockIdx.x / rb_per_clip;
  const int t0 = (blockIdx.x - b * rb_per_clip) * C1_ROWS;
  for (int i = threadIdx.x; i < 64 * 9; i += 256) s_w[i] = w1[i];
  if (threadIdx.x < 64) s_b[threadIdx.x] = b1[threadIdx.x];
  const float* xb = x0 + (int64_t)b * T * 64;
  for (int i = threadIdx.x; i < (C1_ROWS + 2) * 66; i += 256) {
    const int r = i / 66, c = i - r * 66;
    const int t = t0 - 1 + r, f = c - 1;
    s_x[r][c] = (t >= 0 && t < T && f >= 0 && f < 64) ? xb[t * 64 + f] : 0.0f;
  }
  __syncthreads();
  const int cq = threadIdx.x & 15;
  float wr[4][9], br[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int k = 0; k < 9; ++k) wr[c][k] = s_w[(4 * cq + c) * 9 + k];
    br[c] = s_b[4 * cq + c];
  }
  float* ob = out + ((int64_t)b * T + t0) * 64 * 64 + 4 * cq;
#pragma unroll
  for (int it = 0; it < C1_ROWS * 4; ++it) {
    const int pxl = it * 16 + (threadIdx.x >> 4);   // pixel within the rows: row pxl >> 6, bin pxl & 63
    const int r = pxl >> 6, f = pxl & 63;
    if (t0 + r >= T) break;
    float xv[9];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) xv[dy * 3 + dx] = s_x[r + dy][f + dx];
    float y[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < 9; ++k) acc = fmaf(xv[k], wr[c][k], acc);
      y[c] = fmaxf(acc + br[c], 0.0f);
    }
    *reinterpret_cast<float4*>(ob + (int64_t)pxl * 64) = make_float4(y[0], y[1], y[2], y[3]);
  }
}

void launch_conv1_nhwc(const float* x0, int B, int T, const float* w1, const float* b1, float* out, hipStream_t s) {
  const int rb = (T + C1_ROWS - 1) / C1_ROWS;
  const int64_t blocks = (int64_t)B * rb;
  if (B <= 0 || T <= 0 || blocks > INT32_MAX || (int64_t)T * 64 > INT32_MAX) return note_launch_error(hipErrorInvalidValue);
  hipLaunchKernelGGL(conv1_nhwc_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x0, T, rb, w1, b1, out);
}

// Block 1's conv1 into the chunk-of-4 layout [B][16][T][64][4] (the F(4x4,3x3)
// block-1 conv2's input, conv_wino43.hip): a workgroup computes C1_ROWS
// t-rows of one clip for all 16 chunks, a thread one pixel x 4 channels per
// chunk (consecutive threads: consecutive bins, one 16-byte store each, so a
// chunk's rows are one contiguous run).  Per channel the same fma chain as
// conv1_nhwc_kernel: the two layouts hold bit-identical values.
__global__ __launch_bounds__(256) void conv1_c4_kernel(const float* __restrict__ x0, int T, int rb_per_clip,
                                                       const float* __restrict__ w1, const float* __restrict__ b1,
                                                       float* __restrict__ out) {
  __shared__ float s_w[64 * 9], s_b[64];
  __shared__ float s_x[C1_ROWS + 2][66];
  const int b = blockIdx.x / rb_per_clip;
  const int t0 = (blockIdx.x - b * rb_per_clip) * C1_ROWS;
  for (int i = threadIdx.x; i < 64 * 9; i += 256) s_w[i] = w1[i];
  if (threadIdx.x < 64) s_b[threadIdx.x] = b1[threadIdx.x];
  const float* xb = x0 + (int64_t)b * T * 64;
  for (int i = threadIdx.x; i < (C1_ROWS + 2) * 66; i += 256) {
    const int r = i / 66, c = i - r * 66;
    const int t = t0 - 1 + r, f = c - 1;
    s_x[r][c] = (t >= 0 && t < T && f >= 0 && f < 64) ? xb[t * 64 + f] : 0.0f;
  }
  __syncthreads();
  static_assert(C1_ROWS * 64 == 256, "a thread per pixel");
  const int r = threadIdx.x >> 6, f = threadIdx.x & 63;
  if (t0 + r >= T) return;
  float xv[9];
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) xv[dy * 3 + dx] = s_x[r + dy][f + dx];
  float* ob = out + (((int64_t)b * 16 * T + t0 + r) * 64 + f) * 4;
  for (int cc = 0; cc < 16; ++cc) {
    float y[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < 9; ++k) acc = fmaf(xv[k], s_w[(4 * cc + c) * 9 + k], acc);
      y[c] = fmaxf(acc + s_b[4 * cc + c], 0.0f);
    }
    *reinterpret_cast<float4*>(ob + (int64_t)cc * T * 256) = make_float4(y[0], y[1], y[2], y[3]);
  }
}

void launch_conv1_c4(const float* x0, int B, int T, const float* w1, const float* b1, float* out, hipStream_t s) {
  const int rb = (T + C1_ROWS - 1) / C1_ROWS;
  const int64_t blocks = (int64_t)B * rb;
  if (B <= 0 || T <= 0 || blocks > INT32_MAX || (int64_t)T * 64 > INT32_MAX) return note_launch_error(hipErrorInvalidValue);
  hipLaunchKernelGGL(conv1_c4_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x0, T, rb, w1, b1, out);
}

#ifdef SEDX_WINO_STAMPS
// diagnostic builds: the stamp sums (host side, this translation unit)
void wino_stamps_rw(unsigned long long* h, bool reset) {
  if (reset) {
    static const unsigned long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wino_stamps), z, sizeof(z));
  } else {
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_wino_stamps), 16 * sizeof(unsigned long long));
  }
}
#endif

// U = G g G^T per (input channel, output channel) in float64 from the
// BN-folded weights, rounded once to fp32, packed [Cin/4][16 p][2 h][Cout][2 ks]
// with channel 4 chunk + 2 h + ks (one 8-byte LDS read gives a lane both
// k-steps of a position).
void pack_conv_wino(const double* wf, int Cin, int Cout, float* Up) {
  static const double Gm[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  for (int o = 0; o < Cout; ++o)
    for (int i = 0; i < Cin; ++i) {
      const double* g = wf + ((size_t)o * Cin + i) * 9;
      double tmp[4][3];
      for (int a = 0; a < 4; ++a)
        for (int y = 0; y < 3; ++y) tmp[a][y] = Gm[a][0] * g[0 * 3 + y] + Gm[a][1] * g[1 * 3 + y] + Gm[a][2] * g[2 * 3 + y];
      const int chunk = i / 4, h = (i % 4) >> 1, ks = i & 1;
      for (int a = 0; a < 4; ++a)
        for (int c = 0; c < 4; ++c) {
          const double u = tmp[a][0] * Gm[c][0] + tmp[a][1] * Gm[c][1] + tmp[a][2] * Gm[c][2];
          const int p = 4 * a + c;
          Up[((((size_t)chunk * 16 + p) * 2 + h) * Cout + o) * 2 + ks] = (float)u;
        }
    }
}

}  // namespace sedx
