// 3x3 conv of the 9-layer CNN (ConvBlock, pytorch/models.py:98-141; blocks
// 2-4, models.py:663-666) as fp32 Winograd F(4x4, 3x3) on
// v_mfma_f32_16x16x4_f32: every operand, product and sum is fp32, 36
// multiplies per 4x4 output tile instead of F(2x2,3x3)'s 64 (conv_wino.hip)
// and the direct conv's 144 (conv.hip).
//
// Per output tile (4 t x 4 f) and input channel c the 6x6 input patch d (rows
// t-1..t+4, cols f-1..f+4, zero outside the clip) becomes V = B^T d B, the
// BN-folded 3x3 weights g become U = G g G^T (host, float64, rounded once to
// fp32), the 36 positions p = 6 i + j are 36 independent GEMMs
// M_p[n][tile] = sum_c U_p[n][c] V_p[c][tile], and the output is
// Y = A^T M A, then + bias, ReLU and the block's epilogue (store / 2x2 avg pool
// / freq mean).  Interpolation points 0, 1, -1, 2, -2 (Lavin & Gray 2016):
//   B^T = [4 0 -5 0 1 0; 0 -4 -4 1 1 0; 0 4 -4 -1 1 0; 0 -2 -1 2 1 0;
//          0 2 -1 -2 1 0; 0 4 0 -5 0 1]
//   G   = [1/4 0 0; -1/6 -1/6 -1/6; -1/6 1/6 -1/6; 1/24 1/12 1/6;
//          1/24 -1/12 1/6; 0 0 1]
//   A^T = [1 1 1 1 1 0; 0 1 -1 2 -2 0; 0 1 1 4 4 0; 0 1 -1 8 -8 1]
// (fp32 error study: tools/wino_f43/err.py -> profiles/r04_wino_f43_error.txt.)
//
// Work: an item = 32 tiles (two tile groups of 16) x 64 output channels.
// The workgroup is 12 waves (3 per SIMD): wave w = 2 ROW + tg owns V row ROW
// (positions 6 ROW .. 6 ROW + 5) of tile group tg for all 64 channels — 6
// positions x 4 channel tiles of v_mfma_f32_16x16x4_f32 (M = 16 output
// channels, N = 16 tiles, K = the 4 input channels of a chunk), 96
// accumulator registers.  Lane l supplies B[k = l >> 4][n = l & 15]: the
// transformed value of tile n, input channel k — computed in-lane from the
// patch rows its V row needs (3 or 4 rows of 6 pixels, 3 ds_read_b64 per
// row), so one V value feeds the 4 channel tiles' MFMAs; U fragments
// (A[m][k] = U_p[16 nt + m][k], one ds_read_b128 gives a lane its 4 channel
// tiles) are read from LDS just before their MFMAs.
//
// Staging (per 4-channel chunk): the U slab (36 x 4 x 64 floats, 36 KiB,
// [p][k][m][nt] so a lane's fragment read is 16 B at 16 l) by 36
// buffer_load_dwordx4 ... lds, and the halo of the 32 tiles as four channel
// planes ([k][row][RS]: one patch row of a lane is 6 consecutive floats) by
// buffer_load_dword ... lds — the DMA's lane -> pixel gather does the NHWC ->
// planar transpose, and the buffer range check writes the zeros of pixels
// outside the clip (the lane's offset is set out of range).  The row stride RS
// makes a lane's ds_read_b64 of its patch conflict-free: the 16 tiles of a
// tile group hit 16 distinct even bank pairs and the odd plane stride puts
// channels k and k + 1 on the odd ones.  Two rings of 3: the U slab of chunk c
// is read during step c and the halo of chunk c + 1 (for V of the next chunk)
// during step c, so during step c the workgroup issues U(c + 2) and
// halo(c + 3) into the slots freed by step c - 1 — two steps of DMA lead for
// both — behind one counted-vmcnt barrier per step.  The DMAs are issued
// between the step's first MFMA positions, not at its top (round 6: with all
// twelve waves issuing them right after the barrier the matrix pipes waited
// on the DMA issue; blocks 1-4 2.27 -> 2.14 ms).
//
// Output transform: per register (channel, tile) a wave holds row ROW of M, so
// z = (M A)_ROW is in-lane; Y = A^T M A sums the six rows' z across waves
// through LDS (the U slot freed by the item's last step), two registers per
// round; waves 0-3 finish (a 2x2 output block each, or one output row for the
// freq mean) and store 16-byte groups of 4 channels.
//
// Persistent workgroups walk items g, g + grid, ... (grid a multiple of 8:
// every item of a workgroup on its XCD, the XCD-aware decode of
// conv_wino.hip); the last steps of an item DMA the next item's first chunks.
// Every item performs the same operations in the same order for each (tile,
// channel): outputs do not depend on the batch size or the grid.
#include <type_traits>

#include "sedx_internal.h"

namespace sedx {

typedef float w43_f32x4 __attribute__((ext_vector_type(4)));

// Ablation builds (tools/wino43_bench.cpp only, results WRONG, timing only):
// SEDX_W43_ABL bit 1 drops the halo DMAs, 2 the U DMAs, 4 the epilogue's
// exchange and output transform (stores kept), 8 the epilogue's barriers,
// 16 the STORE epilogue's scatter (every store to one coalesced 1 KiB run),
// 32 the POOL2 epilogue's
#ifndef SEDX_W43_ABL
#define SEDX_W43_ABL 0
#endif
// where a step issues its LDS-DMAs (A/B builds; see the step)
#ifndef SEDX_W43_PRIO
#define SEDX_W43_PRIO 2   // static s_setprio: waves 4-7 at 1, 8-11 at 2 (the later-dispatched waves of each SIMD)
#endif
#ifndef SEDX_W43_EPI2
#define SEDX_W43_EPI2 0
#endif
#ifndef SEDX_W43_USEL
#define SEDX_W43_USEL 1
#endif
#ifndef SEDX_W43_DMA_SPLIT
#define SEDX_W43_DMA_SPLIT 5
#endif
// Item claims (SEDX_W43_CLAIM 1, the default; launches with more items than
// CUs): a persistent grid, one workgroup per CU, whose workgroups claim their
// items from the counter of their XCD lane x = blockIdx & 7 (items 8 v + x,
// the static decode's XCD mapping), so a workgroup that starts late — its CU
// held by the other batch's GRU — takes fewer items instead of costing a
// whole extra round.  The first two items come in one claim at the top; the
// item after next is claimed at an item's epilogue by its last wave (not a
// finisher) and lands in LDS before the epilogue's last round, read by every
// wave at the next item's top.  Counters (sched): 8 ints 128 B apart + a
// done count at [255], zero at launch; the last workgroup to finish zeroes
// them again.  0: the static grid-stride order of round 5 (A/B builds).
#ifndef SEDX_W43_CLAIM
#define SEDX_W43_CLAIM 1
#endif

// Diagnostic builds only (SEDX_W43_STAMPS, tools/wino43_bench.cpp): per-wave
// s_memtime intervals summed over every wave of every 16th workgroup:
// [0] item top (chunk-0 transform) [1] steps [2] epilogue [3] whole wave [4] items
#ifdef SEDX_W43_STAMPS
__device__ unsigned long long g_w43_stamps[8];
#define W43_MARK(i)                                            \
  {                                                            \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
    w43_st[i] += n_ - w43_t;                                   \
    w43_t = n_;                                                \
  }
#else
#define W43_MARK(i)
#endif

// TG: tile groups per item — 2 (32 tiles, 12 waves; every full-size launch)
// or 1 (16 tiles, 6 waves: the one-clip grids of the 16-channel items at
// F = 16 / 8, twice the items of 2 for the same work)
template <int F, int TG = 2>
struct W43Geom {
  static constexpr int WAVES = 6 * TG, THREADS = 64 * WAVES;
  static constexpr int NT = 4, NCH = 64;             // channel tiles / output channels per item
  static constexpr int TILES = 16 * TG;              // TG tile groups of 16
  static constexpr int FT = F / 4;                   // tiles per tile row
  static constexpr int TRW = TILES / FT;             // tile rows per item
  // a tile group is TRG tile rows x TFG tile columns (lane n = tr TFG + tf)
  static constexpr int TFG = F == 8 ? 2 : F == 64 ? 16 : 4;
  static constexpr int TRG = 16 / TFG;
  static constexpr int RT = 4 * TRW + 2, CS = F + 2; // halo rows / columns
  // halo row stride: (4 tr RS + 4 tf) / 2 over the 16 tiles of a group must
  // take the 16 even values mod 32 (b64 bank pairs): 2 RS = 8 (mod 32) for
  // 4 x 4 groups, 2 RS = 20 (mod 32) for 8 x 2
  // (F = 64, block 1: one tile row of 16 per group, 2 tf = 0, 2, .., 30 for any even RS)
  static constexpr int RS = F == 64 ? 66 : F == 32 ? 36 : F == 16 ? 20 : 10;
  // a plane's halo in 64-dword DMA blocks, one per wave 0..HB-1 (RT RS <= 704
  // for every F); wave 11 issues its four halo DMAs into an LDS trash block,
  // so every wave has the same DMA count per step (TG 1: RT RS <= 384, a
  // block per wave, no trash wave)
  static constexpr int HB = TG == 2 ? 11 : 6;
  static constexpr int PS = 64 * HB + 2;             // plane stride, = 2 mod 4 (odd bank pairs for odd k)
  static constexpr int HALO = 4 * PS;                // dwords per halo slot
  static constexpr int USZ1 = 36 * 4 * 16;           // NT 1: one 16-channel tile's slab ([p][k][m]), 9 KiB
  static constexpr int NB = 3;                       // ring depth (U and halo)
  // epilogue exchange per round, per tile group, in the U slot freed by the
  // item's last step: STORE [row 6][reg 2][kc 4][16 tiles + 4 pad][4 z] (the
  // pad: a finisher's reads of 4 kc x 16 consecutive (tile, column) words
  // hit 64 banks), else [row 6][reg 2][z pair 2][lane 64][2] (a finisher's
  // ds_read_b64 of its own pair: conflict-free)
  static constexpr int XRS = 4 * 80;
  static constexpr int XTG = 6 * 2 * XRS;
  // dwords per U slot: the 64-channel slab ([p][k][m][nt]); TG 1 (NT 1 only):
  // its 9 KiB slab or one tile group's exchange, the larger
  static constexpr int USZ = TG == 2 ? 36 * 4 * NCH : (USZ1 > XTG ? USZ1 : XTG);
  static constexpr int U_OFF = 0, H_OFF = NB * USZ, BIAS_OFF = H_OFF + NB * HALO, BIAS_MAX = 512;
  static constexpr int HTRASH_OFF = BIAS_OFF + BIAS_MAX;   // 64 dwords: wave 11's halo DMAs
  // a second exchange area (SEDX_W43_EPI2, pooled / freq-mean epilogues): one
  // tile group's [row 6][reg 2][z pair 2][lane 64][2] for registers 2, 3
  static constexpr int X2_OFF = HTRASH_OFF + 64, X2 = SEDX_W43_EPI2 && TG == 2 ? 3072 : 0;
  static constexpr int CL_OFF = X2_OFF + X2;         // item claims: the landed claim ([0]) and the first item ([1])
  static constexpr int LDS_BYTES = 4 * (CL_OFF + (SEDX_W43_CLAIM ? 4 : 0));
  static constexpr int VM = 7;                       // DMAs per wave per step (3 U units + 4 halo planes)

  static_assert(F == 64 || F == 32 || F == 16 || F == 8, "F");
  static_assert(RT * RS <= 64 * HB, "halo plane fits its DMA blocks");
  static_assert(TG == 1 || TG == 2, "TG");
  static_assert(TG == 1 ? HB == WAVES : HB == WAVES - 1, "halo blocks: one per wave (TG 2: wave 11 trash)");
  static_assert(TG == 1 || 36 % WAVES == 0, "U units per wave");
  static_assert(TG * XTG <= USZ, "the tile groups' exchange fits one U slot");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS per workgroup");
  static_assert(FT * TRW == TILES && TFG * TRG == 16, "tile groups");
};

// raw workgroup barrier behind "this wave's DMAs and stores older than its N
// youngest VMEM ops landed, its LDS operations done" (__syncthreads() would
// drain every DMA in flight)
template <int N>
__device__ __forceinline__ void w43_bar() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
__device__ __forceinline__ void w43_lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA through a buffer resource (M0 = LDS byte address of lane 0; out of
// range offsets write zeros).  m0 and soff wave-uniform.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void w43_dma16(uint32_t voff, __amdgpu_buffer_rsrc_t r, uint32_t soff, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds" ::"v"(voff), "s"(r), "s"(m0),
               "s"(soff)
               : "memory", "m0");
}
// (no instruction offset: an LDS-DMA's inst_offset moves the LDS destination
// as well as the source — measured, tools/oob_lds_probe.cpp — so the channel
// step goes into soffset)
__device__ __forceinline__ void w43_dma4(uint32_t voff, __amdgpu_buffer_rsrc_t r, uint32_t soff, uint32_t m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, %3 offen lds" ::"v"(voff), "s"(r),
               "s"(m0), "s"(soff)
               : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ uint32_t w43_lds_addr(const float* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) float*)p;
}

// v = e B (the 6-point transform of one V row)
__device__ __forceinline__ void w43_colt(const float (&e)[6], float (&v)[6]) {
  v[0] = fmaf(4.0f, e[0], fmaf(-5.0f, e[2], e[4]));
  const float a = fmaf(-4.0f, e[2], e[4]), b = fmaf(-4.0f, e[1], e[3]);
  v[1] = a + b;
  v[2] = a - b;
  const float c = e[4] - e[2], t = e[3] - e[1];
  v[3] = fmaf(2.0f, t, c);
  v[4] = fmaf(-2.0f, t, c);
  v[5] = fmaf(4.0f, e[1], fmaf(-5.0f, e[3], e[5]));
}
// z = m A (A^T applied to a row of six positions), and the same combination
// of six rows' z for Y = A^T z
__device__ __forceinline__ void w43_at(const float (&m)[6], float (&z)[4]) {
  const float s12 = m[1] + m[2], d12 = m[1] - m[2], s34 = m[3] + m[4], d34 = m[3] - m[4];
  z[0] = (m[0] + s12) + s34;
  z[1] = fmaf(2.0f, d34, d12);
  z[2] = fmaf(4.0f, s34, s12);
  z[3] = fmaf(8.0f, d34, d12) + m[5];
}

// C4: activations in the chunk-of-4 layout [B][C/4][T][F][4] (input and
// output; the freq-mean output is [B][T][C] either way), else NHWC
// [B][T][F][C].  A chunk's halo plane is then a dense run of 16-byte pixels
// (a halo DMA of 64 lanes touches ~9 cache lines instead of 64).
//
// NT: channel tiles per item.  4 (64 channels) on full grids; 1 (16 channels,
// the launcher's choice when the 64-channel items would leave CUs idle,
// e.g. one clip): four times the items, each tile's accumulation chain the
// same instructions in the same order — bit-identical to NT 4.  An NT 1 item
// DMAs only its 16 channels' U slab (9 KiB per chunk, from the second,
// [Cout/16][Cin/4][36][4][16] pack that follows the NT 4 pack): one 1 KiB
// unit per wave (waves 9-11 read out of range into the slot's unused tail),
// 5 DMAs per wave per step instead of 7.  NT 1 items are dealt over all
// eight XCDs (channel tile g on XCD g mod 8, every tile block of it there):
// at one clip the 512-channel layers have 2 tile blocks, which the tile
// block-major decode put on two XCDs.
template <int F, int EPI, int ROW, bool C4, int NT, int TG>
__device__ __forceinline__ void w43_body(const float* __restrict__ in, int B, int T, int Cin, int Cout,
                                         const float* __restrict__ U, int u_bytes, const float* __restrict__ bias,
                                         float* __restrict__ out, float* __restrict__ trash, int tb_per_clip,
                                         int ngroups, int order2d, int* __restrict__ sched, int wv) {
  using G = W43Geom<F, TG>;
  constexpr int RS = G::RS, PS = G::PS;
  static_assert(TG == 2 || (NT == 1 && (F == 16 || F == 8)), "16-tile items: 16-channel, F = 16 / 8 only");
  static_assert(NT == 4 || NT == 1, "channel tiles per item");
  // a U fragment: the lane's words of its NT channel tiles
  using UF = typename std::conditional<NT == 4, w43_f32x4, float>::type;
  // DMAs per wave per step: U units + 4 halo planes (NT 1: 9 units over
  // the waves, TG 1: two per wave)
  constexpr int VM = NT == 4 ? G::VM : TG == 2 ? 5 : 6;
  extern __shared__ __attribute__((aligned(16))) float smem[];   // G::LDS_BYTES (dynamic)

  // the lane from mbcnt (rematerialised where needed) and the wave from one
  // readfirstlane: the workitem id itself is dead after these two, so it is
  // neither kept live nor spilled (a 4-byte scratch spill of it in the
  // 168-VGPR POOL2 builds put vmcnt(0) drains in the prologue)
  // (wv: the wave, wave-uniform, read once by the kernel entry)
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int tg = TG == 2 ? wv & 1 : 0;
  const int kk = lane >> 4, nn = lane & 15;

  // XCD-aware item decode (conv_wino.hip): item -> XCD id & 7; on one XCD,
  // tile blocks in order with their channel groups consecutive, or (order2d)
  // rounds of 32 / order2d tile blocks x order2d channel groups
  auto decode = [&](int item, int& b_, int& t0_, int& g_) -> bool {
    const int xcd = item & 7, j = item >> 3;
    int jb, cgi;
    if constexpr (NT == 1) {   // channel tile 8 gi + xcd, tile block j mod tblocks
      const int tbl = B * tb_per_clip, gi = j / tbl, tb = j - gi * tbl;
      g_ = 8 * gi + xcd;
      if (g_ >= ngroups) return false;
      b_ = tb / tb_per_clip;
      t0_ = 4 * G::TRW * (tb - b_ * tb_per_clip);
      return true;
    }
    if (order2d > 0) {
      const int tbr = 32 / order2d;
      const int idx = j & 31, r = j >> 5, ncg = ngroups / order2d;
      const int tbg = r / ncg;
      jb = tbr * tbg + idx % tbr;
      cgi = order2d * (r - tbg * ncg) + idx / tbr;
    } else {
      jb = j / ngroups;
      cgi = j - jb * ngroups;
    }
    // order2d -1 (block 1, SEDX_TUNE_WINO_ORDER 2): each XCD a contiguous
    // range of tile blocks, so the halo rows two neighbouring items share are
    // fetched once into that XCD's L2; else tile block jb * 8 + xcd
    const int tbx = (B * tb_per_clip + 7) / 8;
    if (order2d < 0 && jb >= tbx) return false;
    const int tb = order2d < 0 ? xcd * tbx + jb : jb * 8 + xcd;
    if (tb >= B * tb_per_clip) return false;
    b_ = tb / tb_per_clip;
    t0_ = 4 * G::TRW * (tb - b_ * tb_per_clip);   // first output row of the item
    g_ = cgi;
    return true;
  };
  int item = blockIdx.x;
  int b = 0, t0 = 0, grp = 0;
  // item claims (sched non-null, wave-uniform); static grid-stride otherwise
  const bool claims = SEDX_W43_CLAIM && sched != nullptr;
  int* const cl = reinterpret_cast<int*>(smem + G::CL_OFF);
  const int clx = blockIdx.x & 7;
  // the workgroup's end: after its last claim landed; the last workgroup
  // zeroes the counters for the next launch on them
  auto claim_done = [&]() {
    if constexpr (SEDX_W43_CLAIM && ROW == 5) {
      if (claims && wv == G::WAVES - 1 && lane == 0 && atomicAdd(&sched[255], 1) == (int)gridDim.x - 1) {
#pragma unroll
        for (int x = 0; x < 8; ++x) __hip_atomic_store(&sched[32 * x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sched[255], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };
  if (claims) {
    // the first two items in one claim; all waves wait for it (once per workgroup)
    if (wv == G::WAVES - 1 && lane == 0) {
      const int v = atomicAdd(&sched[32 * clx], 2);
      cl[1] = 8 * v + clx;
      cl[0] = 8 * (v + 1) + clx;
    }
    __syncthreads();
    item = __builtin_amdgcn_readfirstlane(cl[1]);
  }
  if (!decode(item, b, t0, grp)) {   // uniform
    claim_done();
    return;
  }

  // this lane's tile within the item
  const int tr = (F == 16 ? 4 * tg : F == 8 ? 8 * tg : F == 64 ? tg : 0) + nn / G::TFG;
  const int tf = (F == 32 ? 4 * tg : 0) + nn % G::TFG;

  // ---- DMA sources.  Buffer resources: the input (pixels outside the clip
  // read out of range: zeros) and the U packs. ----
  const __amdgpu_buffer_rsrc_t r_in =
      __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, (int)((int64_t)B * T * F * Cin * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t r_u = __builtin_amdgcn_make_buffer_rsrc((void*)U, 0, u_bytes, 0x00020000);
  const int nchunks = Cin / 4;
  // halo block wv of each plane: LDS positions q = 64 wv + lane of [row][RS]
  auto halo_off = [&](int b_, int t0_) -> uint32_t {
    const int q = 64 * wv + lane;
    const int row = q / RS, col = q - (q / RS) * RS;
    const int t = t0_ - 1 + row, f = col - 1;
    const bool ok = row < G::RT && col < G::CS && t >= 0 && t < T && f >= 0 && f < F;
    if constexpr (C4)   // chunk 0 of clip b_; a chunk adds T F 16 bytes (soffset)
      return ok ? (uint32_t)((((b_ * (Cin / 4) * T + t) * F + f) * 16)) : 0x80000000u;
    return ok ? (uint32_t)((((b_ * T + t) * F + f) * Cin) * 4) : 0x80000000u;
  };
  const uint32_t u_voff = 16 * lane + 1024 * wv;
  // NT 1: waves 9-11 have no unit (out of range: zeros into the slot's tail)
  const uint32_t u_voff1 = wv < 9 ? u_voff : 0x80000000u;
  const uint32_t u_voff2 = wv + 6 < 9 ? u_voff + 6144 : 0x80000000u;   // TG 1
  const uint32_t bytes_per_chunk_u = 4 * G::USZ;
  // DMAs of chunk cc of an item (halo offsets hof, channel group g_) into
  // the given slots: U units Q0 .. Q1 - 1 of wv, wv + 12, wv + 24 (NT 1: the
  // wave's one or two units of the 16-channel slab, with Q0 = 0) and halo
  // planes P0 .. P1 - 1 of this wave's halo block
  auto dma_u_units = [&](int g_, int cc, int uslot, auto q0_tag, auto q1_tag) {
    if constexpr (SEDX_W43_ABL & 2) return;
    constexpr int Q0 = decltype(q0_tag)::value, Q1 = decltype(q1_tag)::value;
    if constexpr (NT == 1) {
      if constexpr (Q0 == 0) {
        const uint32_t so = __builtin_amdgcn_readfirstlane(
            (uint32_t)(u_bytes / 2 + (g_ * nchunks + cc) * (4 * G::USZ1)));
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(w43_lds_addr(smem + G::U_OFF + uslot * G::USZ + 256 * wv));
        w43_dma16(u_voff1, r_u, so, m0);
        if constexpr (TG == 1) w43_dma16(u_voff2, r_u, so, m0 + 6144);
      }
      return;
    }
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)((g_ * nchunks + cc) * bytes_per_chunk_u));
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(w43_lds_addr(smem + G::U_OFF + uslot * G::USZ + 256 * wv));
#pragma unroll
    for (int q = Q0; q < Q1; ++q) w43_dma16(u_voff, r_u, so + q * 12288, m0 + q * 12288);
  };
  auto dma_u = [&](int g_, int cc, int uslot) {
    dma_u_units(g_, cc, uslot, std::integral_constant<int, 0>{}, std::integral_constant<int, 3>{});
  };
  // planes P0 .. P1 - 1 of the halo DMA of chunk cc
  auto dma_h_planes = [&](uint32_t hof, int cc, int hslot, auto p0_tag, auto p1_tag) {
    if constexpr (SEDX_W43_ABL & 1) return;
    constexpr int P0 = decltype(p0_tag)::value, P1 = decltype(p1_tag)::value;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(16 * (C4 ? cc * T * F : cc)));
    // wave 11 (no block: its lanes' offsets are all out of range, halo_off)
    // writes its four zero DMAs into the trash block — a select, not a branch
    const bool tw = wv == G::HB;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(
        w43_lds_addr(tw ? smem + G::HTRASH_OFF : smem + G::H_OFF + hslot * G::HALO + 64 * wv));
    const uint32_t pstep = tw ? 0u : 4u * PS;
#pragma unroll
    for (int q = P0; q < P1; ++q) w43_dma4(hof, r_in, so + 4 * q, m0 + q * pstep);
  };
  auto dma_h = [&](uint32_t hof, int cc, int hslot) {
    dma_h_planes(hof, cc, hslot, std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{});
  };

  // epilogue stores per wave per item (all issued: out-of-range ones go to
  // this workgroup's trash); finisher waves 0-3 only
  constexpr int S = ROW >= 4 ? 0 : (EPI == EPI_STORE ? 4 : 1) * NT;
  float* const tr_lane = trash + (blockIdx.x & 31) * 256 + 4 * lane;
  // 4-channel group n .. n + 3 of output pixel (t, f) (rows To x cols Fo)
  auto opix = [&](int t, int f, int n, int To, int Fo) -> float* {
    if constexpr (C4) return out + ((((int64_t)b * (Cout / 4) + n / 4) * To + t) * Fo + f) * 4;
    return out + (((int64_t)b * To + t) * Fo + f) * Cout + n;
  };

  // ---- prologue: biases (oldest; covered by the first wait), halo(0), then
  // the groups of steps -2 and -1: {U(0), halo(1)}, {U(1), halo(2)} ----
  if (wv < G::BIAS_MAX / 256) {   // wave-uniform
    const int i = 256 * wv + 4 * lane;
    const __amdgpu_buffer_rsrc_t r_b = __builtin_amdgcn_make_buffer_rsrc((void*)bias, 0, Cout * 4, 0x00020000);
    w43_dma16(i < Cout ? 4 * i : 0x80000000u, r_b, 0,
              __builtin_amdgcn_readfirstlane(w43_lds_addr(smem + G::BIAS_OFF + 256 * wv)));
  }
  uint32_t hof = halo_off(b, t0);
  dma_h(hof, 0, 0);
  dma_u(grp, 0, 0);
  dma_h(hof, 1, 1);
  dma_u(grp, 1, 1);
  dma_h(hof, 2, 2);
  if constexpr (S > 0) {
    float* const vt = tr_lane;   // exactly S stores (never merged), as the epilogue's
    const float zf = 0.0f;
#pragma unroll
    for (int i = 0; i < S; ++i) asm volatile("global_store_dword %0, %1, off" ::"v"(vt), "v"(zf) : "memory");
  }

  // the lane's patch in a halo slot: plane kk, tile (tr, tf)
  const int p_base = kk * PS + 4 * tr * RS + 4 * tf;
  // e = (B^T d)_ROW as a fold over the patch rows, in the order they are
  // read: e = init(row PA[, row PB]), e = fma(CC, row PC, e), e = fma(CD, row PD, e)
  //   ROW 0: d4;      -5 d2, 4 d0      ROW 1: d3 + d4; -4 d2, -4 d1
  //   ROW 2: d4 - d3; -4 d2, 4 d1      ROW 3: d4 - d2;  2 d3, -2 d1
  //   ROW 4: d4 - d2; -2 d3, 2 d1      ROW 5: d5;      -5 d3, 4 d1
  constexpr int PA = ROW == 0 ? 4 : ROW == 5 ? 5 : ROW <= 2 ? 3 : 2;
  constexpr int PB = (ROW == 0 || ROW == 5) ? -1 : 4;
  constexpr int PC = ROW == 0 ? 2 : (ROW == 3 || ROW == 4 || ROW == 5) ? 3 : 2;
  constexpr int PD = ROW == 0 ? 0 : 1;
  constexpr float CC = ROW == 0 ? -5.0f : ROW == 1 ? -4.0f : ROW == 2 ? -4.0f : ROW == 3 ? 2.0f : ROW == 4 ? -2.0f : -5.0f;
  constexpr float CD = ROW == 0 ? 4.0f : ROW == 1 ? -4.0f : ROW == 2 ? 4.0f : ROW == 3 ? -2.0f : ROW == 4 ? 2.0f : 4.0f;
  // LDS reads of the main loop are inline asm with counted waits: the
  // compiler would merge the patch reads into ds_read2_b64 (banked per 16
  // lanes, where the 16 tiles' even bank pairs collide 2-way, and twice the
  // LDS cycles of two ds_read_b64) — and with every LDS read hidden from it,
  // the waits below are exact.  A wait names every register its consumers
  // read, so no consumer is scheduled above it.
  typedef float f2v __attribute__((ext_vector_type(2)));
  // one patch row R (6 floats, 3 ds_read_b64) at LDS byte address a (the halo
  // slot's patch base of the lane)
  auto read_row = [](uint32_t a, auto r_tag, f2v (&x)[3]) {
    constexpr int R = decltype(r_tag)::value;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(x[0]) : "v"(a), "n"(4 * (R * RS)));
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(x[1]) : "v"(a), "n"(4 * (R * RS + 2)));
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(x[2]) : "v"(a), "n"(4 * (R * RS + 4)));
  };
  // U fragment of position 6 ROW + J (byte address a of the lane in the U slot)
  auto read_u = [](uint32_t a, auto j_tag, UF& u) {
    constexpr int J = decltype(j_tag)::value;
    if constexpr (NT == 4)
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(u) : "v"(a), "n"(4 * (6 * ROW + J) * 256));
    else
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(u) : "v"(a), "n"(4 * (6 * ROW + J) * 64));
  };
  auto wait_u = [](auto n_tag, UF& u) {
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(u) : "n"(decltype(n_tag)::value));
  };
  auto wait_r = [](auto n_tag, f2v (&x)[3], UF& u) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(u) : "n"(decltype(n_tag)::value));
  };
  auto wait_rr = [](auto n_tag, f2v (&x)[3], f2v (&y)[3], UF& u) {
    asm volatile("s_waitcnt lgkmcnt(%7)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(u)
                 : "n"(decltype(n_tag)::value));
  };
  // a row's 6 floats as opaque scalars: the compiler would otherwise pair
  // element-wise operations on two rows' halves into packed FP32
  // (v_pk_add_f32), which this library bans (sedx_internal.h)
  auto scal = [](const f2v (&x)[3], float (&d)[6]) {
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      d[c] = x[c >> 1][c & 1];
      asm volatile("" : "+v"(d[c]));
    }
  };
  auto init_e = [&](const f2v (&xa)[3], const f2v (&xb)[3], float (&e)[6]) {
    float a[6], b[6];
    scal(xa, a);
    if constexpr (PB >= 0) scal(xb, b);
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      if constexpr (PB < 0) e[c] = a[c];
      else if constexpr (ROW == 1) e[c] = a[c] + b[c];
      else e[c] = b[c] - a[c];
    }
  };
  auto fold_e = [&](float coef, const f2v (&x)[3], float (&e)[6]) {
    float d[6];
    scal(x, d);
#pragma unroll
    for (int c = 0; c < 6; ++c) e[c] = fmaf(coef, d[c], e[c]);
  };
  auto pin6 = [](float (&v)[6]) {
#pragma unroll
    for (int q = 0; q < 6; ++q) asm volatile("" : "+v"(v[q]));
  };
  using IPA = std::integral_constant<int, PA>;
  using IPB = std::integral_constant<int, (PB < 0 ? 0 : PB)>;
  using IPC = std::integral_constant<int, PC>;
  using IPD = std::integral_constant<int, PD>;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I5 = std::integral_constant<int, 5>;
  const uint32_t h_lane = w43_lds_addr(smem + G::H_OFF + p_base);     // + slot * 4 HALO
  // + slot * 4 USZ; NT 4: the lane's 4 channel tiles' words, NT 1: its word
  const uint32_t u_lane = w43_lds_addr(smem + G::U_OFF + (NT == 1 ? lane : 4 * lane));
  // V of the lane's 6 positions for the chunk in halo slot hs_ (item top: no
  // MFMAs to hide behind)
  auto transform = [&](int hs_, float (&v)[6]) {
    const uint32_t a = h_lane + hs_ * (4 * G::HALO);
    f2v xa[3], xb[3], xc[3], xd[3];
    UF dummy = {};
    read_row(a, IPA{}, xa);
    if constexpr (PB >= 0) read_row(a, IPB{}, xb);
    read_row(a, IPC{}, xc);
    read_row(a, IPD{}, xd);
    wait_rr(I0{}, xa, xb, dummy);
    wait_rr(I0{}, xc, xd, dummy);
    float e[6];
    init_e(xa, xb, e);
    fold_e(CC, xc, e);
    fold_e(CD, xd, e);
    w43_colt(e, v);
    pin6(v);
  };

  w43_f32x4 acc[6][NT];
  float va[6], vb[6];
  int us = 0, hs = 0;   // slots of the current chunk's U and halo

  auto fence = []() { __builtin_amdgcn_sched_barrier(0); };
  auto mfma4 = [&](int j, const UF& u, float v) {
    if constexpr (NT == 1) {
      acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(u, v, acc[j][0], 0, 0, 0);
    } else {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[j][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(u[nt], v, acc[j][nt], 0, 0, 0);
    }
  };

  // the first item's chunk 0: halo(0) landed (younger: the groups of steps
  // -2, -1 and the S dummy stores)
  w43_bar<2 * VM + S>();
#ifdef SEDX_W43_STAMPS
  unsigned long long w43_st[5] = {0, 0, 0, 0, 0};
  unsigned long long w43_t = __builtin_amdgcn_s_memtime();
  const unsigned long long w43_t0 = w43_t;
#endif
  for (;;) {
    // V of the item's chunk 0.  A later item's halo(0) was DMA'd with the
    // previous item's step n - 3 and every wave waited for it before that
    // item's last step's barrier: no wait here
    transform(hs, va);
    int nitem = item + (int)gridDim.x;
    if (claims) {   // landed by the previous epilogue (or the kernel top)
      fence();
      nitem = __builtin_amdgcn_readfirstlane(*reinterpret_cast<volatile int*>(cl));
      fence();
    }
    int nb_ = 0, nt0 = 0, ng = 0;
    const bool has_next = decode(nitem, nb_, nt0, ng);
    const uint32_t nhof = has_next ? halo_off(nb_, nt0) : hof;
    if (!has_next) {
      nb_ = b;
      nt0 = t0;
      ng = grp;
    }
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[j][nt] = w43_f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    // step c: MFMAs of chunk c with V (vc) and U(c) read just in time (at most
    // two positions ahead); V of chunk c + 1 from halo(c + 1) into vn, its
    // patch rows folded as they arrive (not in the last step: V of the next
    // item's chunk 0 is computed after the epilogue, which keeps its registers
    // free).  LDS reads in issue order: U0 U1 | U2 PA PB | U3 PC | U4 PD | U5
    // — the counts below are the reads younger than the awaited one.
    auto step = [&](const float (&vc)[6], float (&vn)[6], int c, auto first_tag, auto last_tag) {
      constexpr bool FIRST = decltype(first_tag)::value, LASTSTEP = decltype(last_tag)::value;
      constexpr int NP0 = LASTSTEP ? 0 : (PB >= 0 ? 6 : 3), NP = LASTSTEP ? 0 : 3;
      // U(c) and halo(c + 1) landed: issued two steps ago; younger: the
      // previous step's group (+ the epilogue stores over an item's first two steps)
      w43_bar<VM + (FIRST ? S : 0)>();
      const int us1 = us == 2 ? 0 : us + 1, us2 = us1 == 2 ? 0 : us1 + 1;
      const int hs1 = hs == 2 ? 0 : hs + 1;
      const uint32_t ua = u_lane + us * (4 * G::USZ);
      const uint32_t ha = h_lane + hs1 * (4 * G::HALO);
      UF u0, u1, u2, u3, u4, u5;
      f2v xa[3], xb[3], xc[3], xd[3];
      float e[6];
      read_u(ua, I0{}, u0);
      read_u(ua, I1{}, u1);
      // group of step c: U(c + 2) -> the U slot of c - 1, halo(c + 3) -> the
      // halo slot of c (read during step c - 1); SEDX_W43_DMA_SPLIT places
      // them between the step's MFMA positions (5, default: U after position
      // 0, halo planes 0-1 after 1 and 2-3 after 2; 0: all at the step top,
      // round 5; 1, 2, 6, 11: the other measured placements, DESIGN.md §4
      // Step schedule).  Any placement inside the step keeps VM DMAs per
      // wave between two barriers.  (Placements after positions 3-4 spill.)
      // (uniform branches on "this item / the next", not selects: a select
      // of the per-lane halo offsets costs a VGPR the main loop does not have)
      auto du = [&](auto q0, auto q1) {
        // SEDX_W43_USEL: the U source by scalar selects (group and chunk are
        // wave-uniform) instead of two branch arms — not in the freq-mean
        // build, whose allocation spills with it
        if constexpr (SEDX_W43_USEL && EPI != EPI_FMEAN) {
          const bool cur = c + 2 < nchunks;
          dma_u_units(cur ? grp : ng, cur ? c + 2 : c + 2 - nchunks, us2, q0, q1);
        } else {
          if (c + 2 < nchunks) dma_u_units(grp, c + 2, us2, q0, q1);
          else dma_u_units(ng, c + 2 - nchunks, us2, q0, q1);
        }
      };
      auto dh = [&](auto p0, auto p1) {
        if (c + 3 < nchunks) dma_h_planes(hof, c + 3, hs, p0, p1);
        else dma_h_planes(nhof, c + 3 - nchunks, hs, p0, p1);
      };
      auto dmas_at = [&](auto ph_tag) {
        constexpr int PH = decltype(ph_tag)::value;   // -1 top, j: after position j
        using Z = std::integral_constant<int, 0>;
        using O = std::integral_constant<int, 1>;
        using W = std::integral_constant<int, 2>;
        using H = std::integral_constant<int, 3>;
        using Q = std::integral_constant<int, 4>;
        if constexpr (SEDX_W43_DMA_SPLIT == 0) {
          if constexpr (PH == -1) {
            du(Z{}, H{});
            dh(Z{}, Q{});
          }
        } else if constexpr (SEDX_W43_DMA_SPLIT == 1) {
          if constexpr (PH == 0) du(Z{}, H{});
          if constexpr (PH == 1) dh(Z{}, Q{});
        } else if constexpr (SEDX_W43_DMA_SPLIT == 5) {
          if constexpr (PH == 0) du(Z{}, H{});
          if constexpr (PH == 1) dh(Z{}, W{});
          if constexpr (PH == 2) dh(W{}, Q{});
        } else if constexpr (SEDX_W43_DMA_SPLIT == 11) {
          if constexpr (PH == 0) du(Z{}, W{});
          if constexpr (PH == 1) {
            du(W{}, H{});
            dh(Z{}, O{});
          }
          if constexpr (PH == 2) dh(O{}, H{});
          if constexpr (PH == 3) dh(H{}, Q{});
        } else if constexpr (SEDX_W43_DMA_SPLIT == 6) {
          if constexpr (PH == 0) dh(Z{}, Q{});
          if constexpr (PH == 1) du(Z{}, H{});
        } else {
          if constexpr (PH == 0) du(Z{}, O{});
          if constexpr (PH == 1) du(O{}, W{});
          if constexpr (PH == 2) du(W{}, H{});
          if constexpr (PH == 3) dh(Z{}, W{});
          if constexpr (PH == 4) dh(W{}, Q{});
        }
      };
      dmas_at(std::integral_constant<int, -1>{});
      fence();
      // position 0
      read_u(ua, I2{}, u2);
      if constexpr (!LASTSTEP) {
        read_row(ha, IPA{}, xa);
        if constexpr (PB >= 0) read_row(ha, IPB{}, xb);
      }
      wait_u(std::integral_constant<int, 2 + NP0>{}, u0);
      mfma4(0, u0, vc[0]);
      dmas_at(std::integral_constant<int, 0>{});
      fence();
      // position 1; e from PA (, PB)
      read_u(ua, I3{}, u3);
      if constexpr (!LASTSTEP) read_row(ha, IPC{}, xc);
      wait_u(std::integral_constant<int, 2 + NP0 + NP>{}, u1);
      mfma4(1, u1, vc[1]);
      dmas_at(std::integral_constant<int, 1>{});
      fence();
      if constexpr (!LASTSTEP) {
        wait_rr(std::integral_constant<int, 1 + NP>{}, xa, xb, u2);
        init_e(xa, xb, e);
      } else {
        wait_u(I1{}, u2);
      }
      // position 2; fold PC
      read_u(ua, I4{}, u4);
      if constexpr (!LASTSTEP) read_row(ha, IPD{}, xd);
      mfma4(2, u2, vc[2]);
      dmas_at(std::integral_constant<int, 2>{});
      fence();
      if constexpr (!LASTSTEP) {
        wait_r(std::integral_constant<int, 1 + NP>{}, xc, u3);
        fold_e(CC, xc, e);
      } else {
        wait_u(I1{}, u3);
      }
      // position 3; fold PD
      read_u(ua, I5{}, u5);
      mfma4(3, u3, vc[3]);
      dmas_at(std::integral_constant<int, 3>{});
      fence();
      if constexpr (!LASTSTEP) {
        wait_r(I1{}, xd, u4);
        fold_e(CD, xd, e);
      } else {
        wait_u(I1{}, u4);
      }
      // positions 4, 5; the column transform
      mfma4(4, u4, vc[4]);
      dmas_at(std::integral_constant<int, 4>{});
      fence();
      if constexpr (!LASTSTEP) {
        w43_colt(e, vn);
        pin6(vn);
      }
      wait_u(I0{}, u5);
      mfma4(5, u5, vc[5]);
      us = us1;
      hs = hs1;
    };
    // steps in pairs (ping-pong V); nchunks even (launcher: Cin % 8 == 0, >= 16)
    W43_MARK(0)
    step(va, vb, 0, std::true_type{}, std::false_type{});
    step(vb, va, 1, std::true_type{}, std::false_type{});
    for (int c = 2; c < nchunks - 2; c += 2) {
      step(va, vb, c, std::false_type{}, std::false_type{});
      step(vb, va, c + 1, std::false_type{}, std::false_type{});
    }
    step(va, vb, nchunks - 2, std::false_type{}, std::false_type{});
    step(vb, va, nchunks - 1, std::false_type{}, std::true_type{});

    W43_MARK(1)
    // ---- epilogue.  Exchange area: the U slot of the last step (us + 2 now);
    // every wave's reads of it are done at the first barrier below. ----
    float* const xfree = smem + G::U_OFF + (us == 0 ? 2 : us - 1) * G::USZ;
    // item claims: the item after next, claimed here and landed before the last round
    int claim_v = 0;
    if constexpr (SEDX_W43_CLAIM && ROW == 5) {
      if (claims && has_next && wv == G::WAVES - 1 && lane == 0) claim_v = atomicAdd(&sched[32 * clx], 1);
    }
    // SEDX_W43_EPI2 (pooled / freq-mean epilogues, two tile groups): all
    // four registers of a channel tile per exchange round — half the rounds
    // and barriers.  Registers 0, 1 of tile group tg at xfree + 3072 tg,
    // registers 2, 3 at xfree + 6144 (tg 0) and in the area past the halo
    // ring (tg 1); the U slot holds exactly the first three.
    constexpr bool E2 = SEDX_W43_EPI2 && EPI != EPI_STORE && TG == 2 && !(SEDX_W43_ABL & 4);
    constexpr int QS = E2 ? 2 : 1, NSR = E2 ? 4 : 2;   // rounds advance by QS; registers per round
    float* const xbuf0 = E2 ? xfree + tg * 3072 : xfree + tg * G::XTG;
    float* const xbuf1 = E2 ? (tg == 0 ? xfree + 6144 : smem + G::X2_OFF) : xbuf0;
    // output element base of the item: first output row t0 of clip b
    int le = lane;
    asm volatile("" : "+v"(le));   // opaque: offsets computed here, not hoisted as live registers
    const int kc = le >> 4;
    // STORE: z of (row, register s) of lane (kc', tile n') = 4 words at
    // xs(row, s) + 80 kc' + 4 n'; else pair bp of this lane at xp(row, s, bp)
    auto xs = [&](int row, int s) { return (row * 2 + s) * G::XRS; };
    const int xl = 80 * kc + 4 * (le & 15);   // this lane's STORE entry
    auto xp = [&](int row, int s, int bp) { return ((row * 2 + s) * 2 + bp) * 128 + 2 * le; };
    const int trg = t0 / 4 + tr;   // the lane's tile row in the clip
    w43_f32x4 ost[NT];             // POOL2 / FMEAN: one 4-channel group per channel tile
    w43_f32x4 ost2[4];             // STORE: the 2 x 2 pixels of the current channel tile
#pragma unroll
    for (int q = 0; q < 2 * NT; q += QS) {
      const int nt = q >> 1;
      if constexpr (SEDX_W43_ABL & 4) {   // timing build: no exchange / output transform
        if constexpr (ROW < 4) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int r = 2 * (q & 1) + s;
            // every position's accumulator feeds the stores (no MFMA is dead code)
            const float v = ((acc[0][nt][r] + acc[1][nt][r]) + (acc[2][nt][r] + acc[3][nt][r])) +
                            (acc[4][nt][r] + acc[5][nt][r]);
            ost[nt][r] = v;
#pragma unroll
            for (int i = 0; i < 4; ++i) ost2[i][r] = v;
          }
          if constexpr (EPI != EPI_STORE) {
            if (q & 1) *reinterpret_cast<w43_f32x4*>(tr_lane) = ost[nt];
          }
          if constexpr (EPI == EPI_STORE) {
            if (q & 1) {
              const int n = grp * 16 * NT + 16 * nt + 4 * kc;
#pragma unroll
              for (int a = 0; a < 2; ++a) {
                const int t = 4 * trg + 2 * (ROW >> 1) + a;
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                  const int f = 4 * tf + 2 * (ROW & 1) + c;
                  float* dst = t < T ? opix(t, f, n, T, F) : tr_lane;
                  *reinterpret_cast<w43_f32x4*>(dst) = ost2[2 * a + c];
                }
              }
            }
          }
        }
        continue;
      }
      // round q writes buffer q & 1: the reads of round q - 2 (same buffer)
      // finished before round q - 1's barrier; at q = 0 the last step's U reads
      // (double-buffering the rounds by parity, one barrier per round, cost
      // 20-80 spilled VGPRs in the compiler's allocation: one buffer, two
      // barriers per round)
      if constexpr (SEDX_W43_CLAIM && ROW == 5) {
        if (claims && q == 2 * NT - QS && has_next && wv == G::WAVES - 1 && lane == 0) *reinterpret_cast<volatile int*>(cl) = 8 * claim_v + clx;
      }
      if constexpr (!(SEDX_W43_ABL & 8)) w43_lds_bar();
#pragma unroll
      for (int s4 = 0; s4 < NSR; ++s4) {
        const int s = s4 & 1;
        float* const xb = s4 < 2 ? xbuf0 : xbuf1;
        const int r = E2 ? s4 : 2 * (q & 1) + s;
        float m[6], z[4];
#pragma unroll
        for (int j = 0; j < 6; ++j) m[j] = acc[j][nt][r];
        w43_at(m, z);
        if constexpr (EPI == EPI_STORE) {
          *reinterpret_cast<float4*>(xb + xs(ROW, s) + xl) = make_float4(z[0], z[1], z[2], z[3]);
        } else {
          *reinterpret_cast<float2*>(xb + xp(ROW, s, 0)) = make_float2(z[0], z[1]);
          *reinterpret_cast<float2*>(xb + xp(ROW, s, 1)) = make_float2(z[2], z[3]);
        }
      }
      if constexpr (!(SEDX_W43_ABL & 8)) w43_lds_bar();
      if constexpr (ROW < 4) {
        const int n = grp * 16 * NT + 16 * nt + 4 * kc;   // first of the lane's 4 channels
#pragma unroll
        for (int s4 = 0; s4 < NSR; ++s4) {
          const int s = s4 & 1;
          const float* const xb = s4 < 2 ? xbuf0 : xbuf1;
          const int r = E2 ? s4 : 2 * (q & 1) + s;
          const float bv = smem[G::BIAS_OFF + n + r];
          if constexpr (EPI == EPI_FMEAN) {
            // output row a = ROW of the tile: Y[ROW][0..3], ReLU, sum over
            // the 4 columns, + the other tile of the row (lane ^ 1)
            float z[6][4];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              const float2 lo = *reinterpret_cast<const float2*>(xb + xp(i, s, 0));
              const float2 hi = *reinterpret_cast<const float2*>(xb + xp(i, s, 1));
              z[i][0] = lo.x; z[i][1] = lo.y; z[i][2] = hi.x; z[i][3] = hi.y;
            }
            float sum = 0.0f;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              float col[6], y[4];
#pragma unroll
              for (int i = 0; i < 6; ++i) col[i] = z[i][c];
              w43_at(col, y);
              sum += fmaxf(y[ROW] + bv, 0.0f);
            }
            const float other = __shfl_xor(sum, 1);
            ost[nt][r] = ((tf & 1) ? other + sum : sum + other) * (1.0f / F);
          } else if constexpr (EPI == EPI_STORE) {
            // output row a = ROW; for store j the lane computes column
            // c = lane & 3 of tile 4 j + ((lane >> 2) & 3) — another lane's
            // z — so the 16 lanes of a kc hold 16 consecutive pixels of a
            // tile-group row (256 contiguous bytes of a 4-channel group, or
            // two 128-byte rows at F = 8) per store instruction
            const int c = le & 3;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float* src = xb + 80 * kc + 4 * (4 * j + ((le >> 2) & 3)) + c;
              float col[6], yy[4];
#pragma unroll
              for (int i = 0; i < 6; ++i) col[i] = src[xs(i, s)];
              w43_at(col, yy);
              ost2[j][r] = fmaxf(yy[ROW] + bv, 0.0f);
              // (claim builds: one store's chain at a time, else the allocator spills)
              if constexpr (SEDX_W43_CLAIM) __builtin_amdgcn_sched_barrier(0);
            }
          } else {
            // POOL2: the 2 x 2 block (2A, 2A + 1) x (2B, 2B + 1) of the tile
            constexpr int A = ROW >> 1, Bc = ROW & 1;
            float z[6][2];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
              const float2 w = *reinterpret_cast<const float2*>(xb + xp(i, s, Bc));
              z[i][0] = w.x;
              z[i][1] = w.y;
            }
            float y[2][2];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              float col[6], yy[4];
#pragma unroll
              for (int i = 0; i < 6; ++i) col[i] = z[i][c];
              w43_at(col, yy);
              y[0][c] = fmaxf(yy[2 * A] + bv, 0.0f);
              y[1][c] = fmaxf(yy[2 * A + 1] + bv, 0.0f);
            }
            ost[nt][r] = (((y[0][0] + y[0][1]) + y[1][0]) + y[1][1]) * 0.25f;
          }
        }
        if constexpr (EPI == EPI_STORE) {
          if (q & 1) {   // the channel tile's 4 registers done: 4 tiles' pixels x 4 channels
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int tj = 4 * j + ((le >> 2) & 3);   // the tile of store j
              const int trj = (F == 16 ? 4 * tg : F == 8 ? 8 * tg : F == 64 ? tg : 0) + tj / G::TFG;
              const int tfj = (F == 32 ? 4 * tg : 0) + tj % G::TFG;
              const int t = 4 * (t0 / 4 + trj) + ROW, f = 4 * tfj + (le & 3);
              float* dst = t < T ? opix(t, f, n, T, F) : tr_lane;
              if constexpr (SEDX_W43_ABL & 16) dst = tr_lane;   // timing: fully coalesced stores
              *reinterpret_cast<w43_f32x4*>(dst) = ost2[j];
            }
          }
        } else {   // POOL2 / FMEAN: the channel tile's 4 registers done: one 4-channel group
          if (E2 || (q & 1)) {
            float* dst;
            if constexpr (EPI == EPI_POOL2) {
              const int to = 2 * trg + (ROW >> 1), fo = 2 * tf + (ROW & 1);
              dst = to < T / 2 ? opix(to, fo, n, T / 2, F / 2) : tr_lane;
              if constexpr (SEDX_W43_ABL & 32) dst = tr_lane;   // timing: coalesced pool stores
            } else {
              const int t = 4 * trg + ROW;
              dst = (t < T && !(tf & 1)) ? out + (int64_t)(b * T + t) * Cout + n : tr_lane;
            }
            *reinterpret_cast<w43_f32x4*>(dst) = ost[nt];
          }
        }
      }
    }
    W43_MARK(2)
#ifdef SEDX_W43_STAMPS
    w43_st[4] += 1;
#endif
    if (!has_next) break;
    item = nitem;
    b = nb_;
    t0 = nt0;
    grp = ng;
    hof = nhof;
  }
  claim_done();
#ifdef SEDX_W43_STAMPS
  if (lane == 0 && (blockIdx.x & 15) == 0) {
    w43_st[3] = __builtin_amdgcn_s_memtime() - w43_t0;
    for (int i = 0; i < 5; ++i) atomicAdd(&g_w43_stamps[i], w43_st[i]);
    atomicAdd(&g_w43_stamps[5], 1ull);
  }
#endif
}

#define SEDX_W43_ROWS(F_, EPI_, C4_, NT_, TG_, ...)                         \
  switch (TG_ == 2 ? wv >> 1 : wv) {                                       \
    case 0: w43_body<F_, EPI_, 0, C4_, NT_, TG_>(__VA_ARGS__); break;      \
    case 1: w43_body<F_, EPI_, 1, C4_, NT_, TG_>(__VA_ARGS__); break;      \
    case 2: w43_body<F_, EPI_, 2, C4_, NT_, TG_>(__VA_ARGS__); break;      \
    case 3: w43_body<F_, EPI_, 3, C4_, NT_, TG_>(__VA_ARGS__); break;      \
    case 4: w43_body<F_, EPI_, 4, C4_, NT_, TG_>(__VA_ARGS__); break;      \
    default: w43_body<F_, EPI_, 5, C4_, NT_, TG_>(__VA_ARGS__); break;     \
  }

template <int F, int EPI, bool C4, int NT = 4, int TG = 2>
__global__ __launch_bounds__(384 * TG, 1) void conv3x3_wino43_kernel(const float* __restrict__ in, int B, int T, int Cin,
                                                                int Cout, const float* __restrict__ U, int u_bytes,
                                                                const float* __restrict__ bias, float* __restrict__ out,
                                                                float* __restrict__ trash, int tb_per_clip,
                                                                int ngroups, int order2d, int* __restrict__ sched) {
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
#if SEDX_W43_PRIO == 1
  if (wv >= 8) __builtin_amdgcn_s_setprio(1);   // the youngest wave of each SIMD
#elif SEDX_W43_PRIO == 2
  if (wv >= 8) __builtin_amdgcn_s_setprio(2);
  else if (wv >= 4) __builtin_amdgcn_s_setprio(1);
#elif SEDX_W43_PRIO == 3
  if (wv < 4) __builtin_amdgcn_s_setprio(2);
  else if (wv < 8) __builtin_amdgcn_s_setprio(1);
#endif
#ifdef SEDX_W43_DELAY
  // diagnostic builds only (tools/wino43_bench.cpp): the odd workgroups of
  // the first resident round start SEDX_W43_DELAY cycles late, so half the
  // CUs run their epilogues (and its output store bursts) out of phase
  // with the other half
  if ((blockIdx.x & 1) && blockIdx.x < 256) {
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0_ < (unsigned long long)SEDX_W43_DELAY) __builtin_amdgcn_s_sleep(8);
  }
#endif
  SEDX_W43_ROWS(F, EPI, C4, NT, TG, in, B, T, Cin, Cout, U, u_bytes, bias, out, trash, tb_per_clip, ngroups, order2d,
                sched, wv)
}
#undef SEDX_W43_ROWS

// items per workgroup.  Alone on the chip 16 (one persistent workgroup per
// CU: one exposed prologue per CU) is fastest — blocks 1-4 2.41 -> 2.35 ms
// (tools/gpu_r05n.sh, profiles/r05n_w43_items.log; 3 and 6 are slower:
// their grids break the L2 round order) — but in the two-stream headline
// long-lived workgroups hold the CUs the other batch's frontend / GRU /
// head need: 11,362-11,424 clips/s at 16, 11,546-11,585 at 4,
// 11,708-11,724 at 2 (profiles/r05p_items_ab.log).  2 stays.
#ifndef SEDX_W43_ITEMS
#define SEDX_W43_ITEMS 2
#endif

// one launch of the F(4x4,3x3) kernel with TG tile groups per item and
// 16- (nt1) or 64-channel items
template <int F, int TG>
static void launch_w43_g(const float* in, int B, int T, int Cin, int Cout, const float* U, const float* bias,
                         float* out, int epi, float* trash, int order, bool c4, bool nt1, int ncu, int* sched,
                         hipStream_t s) {
  using G = W43Geom<F, TG>;
  // output rows the epilogue covers: POOL2 drops an odd last row
  const int rows = epi == EPI_POOL2 ? 2 * (T / 2) : T;
  const int trows = (rows + 3) / 4;
  const int tb_per_clip = (trows + G::TRW - 1) / G::TRW;
  const int64_t tblocks = (int64_t)B * tb_per_clip;
  const int ngroups = Cout / (nt1 ? 16 : G::NCH);
  // NT 1: 8 XCD lanes x ceil(groups / 8) channel tiles x every tile block
  const int64_t nitems = nt1 ? 8 * ((ngroups + 7) / 8) * tblocks : (tblocks + 7) / 8 * 8 * ngroups;
  const int64_t u_bytes = 2 * (int64_t)Cin * Cout * 36 * 4;   // the NT 4 pack, then the NT 1 pack
  if (nitems > INT32_MAX || tblocks <= 0 || (int64_t)B * T * F * Cin * 4 >= INT32_MAX || u_bytes >= INT32_MAX)
    return note_launch_error(hipErrorInvalidValue);
  const int64_t resident = (int64_t)ncu / 8 * 8;
  const int64_t per = (nitems + SEDX_W43_ITEMS - 1) / SEDX_W43_ITEMS;
  int64_t nwg = std::min<int64_t>(nitems, std::max<int64_t>(std::max<int64_t>(8, resident), (per + 7) / 8 * 8));
  // item claims where there are more than two items per CU: one persistent
  // workgroup per CU (nwg a multiple of 8: every XCD lane has workgroups).
  // Below that the first claim's latency is not amortised (B = 4 block 1:
  // 0.0645 vs 0.0627 ms static, profiles/r06zb_*) and the static order runs.
  const bool claim = SEDX_W43_CLAIM && sched != nullptr && nitems > 2 * resident && resident >= 8;
  if (claim) nwg = resident;
  int* const sched_k = claim ? sched : nullptr;
  // rounds of 32 / G tile blocks x G channel groups (conv_wino.hip): the G
  // whose round streams the fewest bytes through an XCD's L2
  int order2d = F == 64 && order == 2 && !nt1 ? -1 : 0;
  if (order && !nt1 && F != 64 && nwg % 256 == 0 && (nitems / 8) % 32 == 0) {
    const int64_t slab = (int64_t)36 * Cin * G::NCH * 4, halo = (int64_t)G::RT * G::CS * Cin * 4;
    int64_t best = (int64_t)ngroups * slab + (32 / std::min(ngroups, 32)) * halo;
    for (int gr = 1; gr <= 8 && gr < ngroups; gr *= 2) {
      const int64_t bytes = gr * slab + (32 / gr) * halo;
      if (ngroups % gr == 0 && tblocks % (8 * (32 / gr)) == 0 && bytes < best) {
        best = bytes;
        order2d = gr;
      }
    }
  }
  // Counted vmcnt waits and spills: the chunk-of-4 builds (the product
  // path) are refused if the compiler ever makes them spill (launch_info
  // no_scratch; 0 bytes in this build, -Rpass-analysis / the ISA's
  // ScratchSize).  The NHWC builds (opt-in: SEDX_TUNE_WINO_BLOCK1 0 or 1, the
  // NHWC A/B of the C4 layout) spill 12-192 bytes in their epilogue index
  // math: a scratch op the compiler inserts only ever ADDS vector-memory ops
  // to a wave's in-order count, so a counted wait then retires more of the
  // older DMAs than it names, never fewer — stricter, not looser.
#define SEDX_W43_GO(k_)                                                                                     \
  {                                                                                                         \
    if (!launch_info(reinterpret_cast<const void*>(k_), G::THREADS, G::LDS_BYTES, c4).ok) return;           \
    hipLaunchKernelGGL(k_, dim3((unsigned)nwg), dim3(G::THREADS), G::LDS_BYTES, s, in, B, T, Cin, Cout, U,  \
                       (int)u_bytes, bias, out, trash, tb_per_clip, ngroups, order2d, sched_k);             \
    return;                                                                                                 \
  }
#define SEDX_W43_LAUNCH(E)                                                                                  \
  {                                                                                                         \
    if constexpr (TG == 1) {   /* 16-tile items: 16-channel, chunk-of-4 only */                             \
      if (!nt1 || !c4) return note_launch_error(hipErrorInvalidValue);                                     \
      SEDX_W43_GO((conv3x3_wino43_kernel<F, E, true, 1, 1>));                                              \
    } else {                                                                                                \
      auto* k_ = nt1 ? (c4 ? conv3x3_wino43_kernel<F, E, true, 1> : conv3x3_wino43_kernel<F, E, false, 1>)  \
                     : (c4 ? conv3x3_wino43_kernel<F, E, true, 4> : conv3x3_wino43_kernel<F, E, false, 4>); \
      SEDX_W43_GO(k_);                                                                                      \
    }                                                                                                       \
  }
  if constexpr (F == 64) {   // block 1's conv2 (conv1's output in, 2 x 2 pool)
    if (epi == EPI_POOL2) SEDX_W43_LAUNCH(EPI_POOL2);
  } else if constexpr (F == 8) {
    if (epi == EPI_STORE) SEDX_W43_LAUNCH(EPI_STORE);
    if (epi == EPI_FMEAN) SEDX_W43_LAUNCH(EPI_FMEAN);
  } else {
    if (epi == EPI_STORE) SEDX_W43_LAUNCH(EPI_STORE);
    if (epi == EPI_POOL2) SEDX_W43_LAUNCH(EPI_POOL2);
  }
#undef SEDX_W43_LAUNCH
#undef SEDX_W43_GO
  note_launch_error(hipErrorInvalidValue);
}

// nt_force: 0 = choose; 4 = 64-channel items; 1 = 16-channel items of 32
// tiles; 2 = 16-channel items of 16 tiles (F = 16 / 8, chunk-of-4)
template <int F>
static void launch_w43_f(const float* in, int B, int T, int Cin, int Cout, const float* U, const float* bias,
                         float* out, int epi, float* trash, int order, bool c4, int nt_force, int* sched,
                         hipStream_t s) {
  using G = W43Geom<F>;
  const int rows = epi == EPI_POOL2 ? 2 * (T / 2) : T;
  const int64_t tblocks = (int64_t)B * (((rows + 3) / 4 + G::TRW - 1) / G::TRW);
  int ncu = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  // 16-channel items (NT 1, bit-identical) when 64-channel ones would give
  // at most a quarter of the CUs one (measured, profiles/r05q_small_batch.log:
  // at 128 items — b3c2 at B = 4, b4 at B = 8 — NT 1's four times the items
  // at a quarter the work each were slower; at <= 64 faster)
  const bool nt1 = nt_force ? nt_force != 4 : (tblocks + 7) / 8 * 8 * (Cout / G::NCH) <= ncu / 4;
  // 16-channel items of one tile group (16 tiles, 6 waves) where those of
  // two would leave CUs idle (one clip: the 256- and 512-channel layers, 128
  // and 64 items of 32 tiles; bit-identical — the same chains per output)
  constexpr bool tg1_ok = F == 16 || F == 8;
  const bool tg1 = tg1_ok && c4 && nt1 &&
                   (nt_force ? nt_force == 2 : 8 * ((Cout / 16 + 7) / 8) * tblocks < ncu);
  if (nt_force == 2 && !tg1) return note_launch_error(hipErrorInvalidValue);
  if constexpr (tg1_ok) {
    if (tg1) return launch_w43_g<F, 1>(in, B, T, Cin, Cout, U, bias, out, epi, trash, order, c4, true, ncu, sched, s);
  }
  launch_w43_g<F, 2>(in, B, T, Cin, Cout, U, bias, out, epi, trash, order, c4, nt1, ncu, sched, s);
}

void launch_conv3x3_wino43(const float* in, int B, int T, int F, int Cin, int Cout, const float* U43,
                           const float* bias, float* out, int epi, float* trash, hipStream_t s, int order, bool c4,
                           int nt_force, int* sched) {
  if (Cin % 8 != 0 || Cin < 16 || Cout % 64 != 0 || Cout > 512 || B <= 0 || T <= 0)
    return note_launch_error(hipErrorInvalidValue);
  // byte offsets are 32-bit (buffer DMA): batches whose input passes 2^31
  // bytes run as several launches over whole clips (same per-clip work)
  const int64_t in_clip = (int64_t)T * F * Cin;
  const int64_t out_clip = epi == EPI_STORE ? (int64_t)T * F * Cout
                           : epi == EPI_POOL2 ? (int64_t)(T / 2) * (F / 2) * Cout : (int64_t)T * Cout;
  const int64_t bmax = (INT32_MAX / 4 - 1) / in_clip;
  if (bmax < 1) return note_launch_error(hipErrorInvalidValue);
  for (int64_t b0 = 0; b0 < B; b0 += bmax) {
    const int bs = (int)std::min<int64_t>(bmax, B - b0);
    const float* in_s = in + b0 * in_clip;
    float* out_s = out + b0 * out_clip;
    switch (F) {
      case 64: launch_w43_f<64>(in_s, bs, T, Cin, Cout, U43, bias, out_s, epi, trash, order, c4, nt_force, sched, s); break;
      case 32: launch_w43_f<32>(in_s, bs, T, Cin, Cout, U43, bias, out_s, epi, trash, order, c4, nt_force, sched, s); break;
      case 16: launch_w43_f<16>(in_s, bs, T, Cin, Cout, U43, bias, out_s, epi, trash, order, c4, nt_force, sched, s); break;
      case 8: launch_w43_f<8>(in_s, bs, T, Cin, Cout, U43, bias, out_s, epi, trash, order, c4, nt_force, sched, s); break;
      default: return note_launch_error(hipErrorInvalidValue);
    }
  }
}

#ifdef SEDX_W43_STAMPS
void w43_stamps_rw(unsigned long long* h, bool reset) {
  if (reset) {
    static const unsigned long long z[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_w43_stamps), z, sizeof(z));
  } else {
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_w43_stamps), 8 * sizeof(unsigned long long));
  }
}
#endif

// [B][C/4][T][F][4] -> [B][T][F][C]: one thread per 16-byte group
__global__ __launch_bounds__(256) void c4_to_nhwc_kernel(const float4* __restrict__ src, int T, int F, int C4,
                                                         int64_t n, float4* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;   // source group: ((b C4 + c) T + t) F + f
  if (i >= n) return;
  int64_t r = i;
  const int f = (int)(r % F);
  r /= F;
  const int t = (int)(r % T);
  r /= T;
  const int c = (int)(r % C4);
  const int64_t b = r / C4;
  dst[((b * T + t) * F + f) * C4 + c] = src[i];
}

void launch_c4_to_nhwc(const float* src, int B, int T, int F, int C, float* dst, hipStream_t s) {
  const int64_t n = (int64_t)B * T * F * (C / 4);
  if (n <= 0 || C % 4 != 0) return note_launch_error(hipErrorInvalidValue);
  hipLaunchKernelGGL(c4_to_nhwc_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const float4*>(src), T, F, C / 4, n, reinterpret_cast<float4*>(dst));
}

// U = G g G^T per (input channel, output channel) in float64 from the
// BN-folded weights wf [Cout][Cin][9], rounded once to fp32, packed twice:
// [Cout/64][Cin/4][36 p][4 k][16 m][4 nt] with output channel 64 group +
// 16 nt + m and input channel 4 chunk + k (a chunk's slab is the LDS image;
// lane l = 16 k + m reads its 4 channel tiles as one 16-byte word), then the
// same values as [Cout/16][Cin/4][36 p][4 k][16 m] (16-channel items: a
// chunk's 9 KiB slab of one channel tile).  Up: 2 Cin Cout 36 floats.
void pack_conv_wino43(const double* wf, int Cin, int Cout, float* Up) {
  static const double Gm[6][3] = {{1.0 / 4, 0, 0},
                                  {-1.0 / 6, -1.0 / 6, -1.0 / 6},
                                  {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                  {1.0 / 24, 1.0 / 12, 1.0 / 6},
                                  {1.0 / 24, -1.0 / 12, 1.0 / 6},
                                  {0, 0, 1}};
  const int nch = Cin / 4;
  for (int o = 0; o < Cout; ++o)
    for (int i = 0; i < Cin; ++i) {
      const double* g = wf + ((size_t)o * Cin + i) * 9;
      double tmp[6][3];
      for (int a = 0; a < 6; ++a)
        for (int y = 0; y < 3; ++y) tmp[a][y] = Gm[a][0] * g[0 * 3 + y] + Gm[a][1] * g[1 * 3 + y] + Gm[a][2] * g[2 * 3 + y];
      const int grp = o / 64, nt = (o % 64) / 16, m = o % 16, chunk = i / 4, k = i % 4;
      for (int a = 0; a < 6; ++a)
        for (int c = 0; c < 6; ++c) {
          const double u = tmp[a][0] * Gm[c][0] + tmp[a][1] * Gm[c][1] + tmp[a][2] * Gm[c][2];
          const int p = 6 * a + c;
          Up[(((((size_t)grp * nch + chunk) * 36 + p) * 4 + k) * 16 + m) * 4 + nt] = (float)u;
          Up[(size_t)Cin * Cout * 36 + ((((size_t)(o / 16) * nch + chunk) * 36 + p) * 4 + k) * 16 + m] = (float)u;
        }
    }
}

}  // namespace sedx
