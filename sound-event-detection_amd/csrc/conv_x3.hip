// 3x3 conv + folded BN + ReLU (+ pool / freq-mean) on bf16 MFMA with a
// 3-term split: every fp32 operand x = hi + lo (hi = bf16(x), lo = bf16(x - hi)),
// and each 32x32x16 tile accumulates hi*hi + hi*lo + lo*hi in fp32
// (v_mfma_f32_32x32x16_bf16 x3).  Operand representation error <= 2^-17 |x|,
// product error ~2^-16: fp32-class results (parity tests: |d| ~1e-6) at
// 16/3 the fp32-MFMA rate.  Same data layout and epilogues as conv.hip
// (ConvBlock, pytorch/models.py:98-141).
//
// Block = 512 threads (8 waves, wave tile 64 x 64), output tile BM pixels x
// BN channels (256 x 128, or 512 x 64 for the 64-channel layer).  K loop =
// 16-channel chunks x 9 taps.  Per chunk the (TT+2) x (F+2) halo of the fp32
// input is split to bf16 hi/lo and written once to LDS as 80-B pixel records
// [hi k0-7 | hi k8-15 | lo k0-7 | lo k8-15 | pad]; all 9 taps read it with
// shifted positions (row stride CSP chosen per shape so every A-fragment
// ds_read_b128 is bank-conflict-free and every tap offset is an immediate).
// Weights are pre-split + pre-swizzled on the host in the exact LDS image,
// [ntile][chunk][tap][BN][64 B].
//
// Pipeline (persistent workgroups, one per resident slot):
//   * A halo images are double-buffered per chunk;
//   * weights stream in stages of one kernel row (3 taps) through a 2-slot
//     LDS ring;
//   * one barrier per stage; after it each thread writes the stage-after-next
//     weights and (once per chunk) the next chunk's halo from registers, then
//     issues the global loads that refill those registers, while the MFMAs of
//     the current stage keep the matrix pipes busy;
//   * A/B fragments of tap t+1 are read from LDS (two register sets) while
//     tap t's 12 MFMAs issue, across stage, chunk and tile boundaries.
//   * all layers but the fused block 1 stream the weights by LDS-DMA
//     instead (global_load_lds_dwordx4 straight into the slot freed by the
//     barrier, one stage ahead; counted vmcnt + raw s_barrier): no weight
//     VGPRs or ds_writes, ~40 fewer VGPRs, 1-2 % faster per layer.
// The MFMA row -> pixel map is chosen per epilogue so that 2x2 pooling (and
// the 8-bin freq mean) is an in-lane register sum.
#include <algorithm>

#include "sedx_internal.h"

namespace sedx {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// hi = bf16_rne(x), lo = bf16_rne(x - hi): v_cvt_pk_bf16_f32 (RNE) per pair
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& hi, uint32_t& lo) {
  const bf16x2 h = {(__bf16)x0, (__bf16)x1};
  hi = __builtin_bit_cast(uint32_t, h);
  const float r0 = x0 - __uint_as_float(hi << 16);
  const float r1 = x1 - __uint_as_float(hi & 0xFFFF0000u);
  const bf16x2 l = {(__bf16)r0, (__bf16)r1};
  lo = __builtin_bit_cast(uint32_t, l);
}

__device__ __forceinline__ void split8(const float4 a, const float4 b, uint4& hi, uint4& lo) {
  split2(a.x, a.y, hi.x, lo.x);
  split2(a.z, a.w, hi.y, lo.y);
  split2(b.x, b.y, hi.z, lo.z);
  split2(b.z, b.w, hi.w, lo.w);
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// 4x4 transpose across the 4 lanes of a quad (j = lane & 3): on entry lane j
// holds column j of a 4x4 block in v[0..3] (v[k] = row k), on exit row j
// (v[k] = column k).  Two butterfly stages (lane bit 0, lane bit 1), each a
// DPP quad permute + select per register.
template <int CTRL>
__device__ __forceinline__ float quad_perm(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ void quad_transpose4(float* v, int j) {
  const bool odd = j & 1, upper = j & 2;
  const float t0 = quad_perm<0xB1>(v[1]), t1 = quad_perm<0xB1>(v[0]);   // lanes (1,0,3,2)
  const float t2 = quad_perm<0xB1>(v[3]), t3 = quad_perm<0xB1>(v[2]);
  const float a0 = odd ? t0 : v[0], a1 = odd ? v[1] : t1;
  const float a2 = odd ? t2 : v[2], a3 = odd ? v[3] : t3;
  const float u0 = quad_perm<0x4E>(a2), u1 = quad_perm<0x4E>(a3);      // lanes (2,3,0,1)
  const float u2 = quad_perm<0x4E>(a0), u3 = quad_perm<0x4E>(a1);
  v[0] = upper ? u0 : a0;
  v[1] = upper ? u1 : a1;
  v[2] = upper ? a2 : u2;
  v[3] = upper ? a3 : u3;
}

// MFMA row R (0..BM-1 of the block tile) -> (t_local, f)
template <int F, int EPI>
__device__ __forceinline__ void rowmap(int R, int& tl, int& f) {
  if (EPI == EPI_POOL2) {            // R = 4q + e: a 2x2 pool group in one lane's regs 4g..4g+3
    const int q = R >> 2, e = R & 3;
    const int tp = q / (F / 2), fp = q % (F / 2);
    tl = 2 * tp + (e >> 1);
    f = 2 * fp + (e & 1);
  } else if (F == 8) {
    // 32 rows = 4 t x 8 f.  ds_read_b128 lane groups {0-3,12-15,20-27} and
    // {4-11,16-19,28-31} each get two whole t rows ({t0,t2} / {t1,t3}), so at
    // row stride 12 their 16 positions are distinct mod 16 (conflict-free);
    // in the C layout a lane's regs {0-3,12-15} and {4-11} are each one t
    // (t0/t1 for lanes 0-31, t3/t2 for lanes 32-63): the freq mean stays
    // in-lane.
    const int r = R & 31, half = r >> 4, q = (r >> 2) & 3;
    const int tq = half ? ((0x3021 >> (4 * q)) & 0xF) : ((0x2130 >> (4 * q)) & 0xF);
    tl = 4 * (R >> 5) + tq;
    f = (r & 3) + 4 * half;
  } else {
    tl = R / F;
    f = R % F;
  }
}

// Tiles (b, t-tile, n-tile), n-tile fastest so tiles sharing an input halo
// run side by side, are cut into 8 contiguous ranges, one per XCD, so
// neighbouring t-tiles share one L2.  Workgroups claim tiles dynamically: a
// workgroup takes the next tile of its own XCD's range (HW_REG_XCC_ID, one
// atomic counter per range) and, once that range is empty, steals from the
// others.  So a workgroup that starts late — its CU was busy with a kernel of
// another stream, e.g. the GRU recurrence of the previous batch — finds the
// work already shared out instead of holding the layer back.  A tile's claim
// is issued one tile ahead and lands in a 4-entry LDS ring read by decode().
// A workgroup's units (tile, chunk) form one stream: the pipeline runs
// straight through tile boundaries, where only the epilogue (stores from the
// accumulators) is inserted.
#ifdef SEDX_CONV_STAMPS
// diagnostic build (tools/conv_bench.cpp): per-wave s_memtime sums
__device__ unsigned long long g_conv_stamps[8];
#define SEDX_ST_DECL                                                                    \
  unsigned long long st_bar = 0, st_vm = 0, st_epi = 0, st_x = 0;                       \
  const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();                        \
  const unsigned long long st_r0 = __builtin_amdgcn_s_memrealtime();
#define SEDX_ST_BEGIN() st_x = __builtin_amdgcn_s_memtime()
#define SEDX_ST_END(a) a += __builtin_amdgcn_s_memtime() - st_x
#define SEDX_ST_VMWAIT()                                                                \
  {                                                                                     \
    SEDX_ST_BEGIN();                                                                    \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                    \
    SEDX_ST_END(st_vm);                                                                 \
  }
#define SEDX_ST_FLUSH()                                                                 \
  if (lane == 0) {                                                                      \
    atomicAdd(&g_conv_stamps[0], __builtin_amdgcn_s_memtime() - st_t0);                 \
    atomicAdd(&g_conv_stamps[1], st_bar);                                               \
    atomicAdd(&g_conv_stamps[2], st_vm);                                                \
    atomicAdd(&g_conv_stamps[3], st_epi);                                               \
    atomicAdd(&g_conv_stamps[4], 1ull);                                                 \
    atomicAdd(&g_conv_stamps[5], __builtin_amdgcn_s_memrealtime() - st_r0);             \
  }
#else
#define SEDX_ST_DECL
#define SEDX_ST_BEGIN()
#define SEDX_ST_END(a)
#define SEDX_ST_VMWAIT()
#define SEDX_ST_FLUSH()
#endif

struct ConvCursor {
  int k, chunk, b, t0, nb;
  bool valid;
};

template <int F, int BN>
struct ConvGeom {
  static constexpr int BM = (BN == 64) ? 512 : 256;
  static constexpr int TT = BM / F;
};

// FUSE (block 1 only): `in` is the bn0 output padded by one zero row/column
// on each side, [B][T+2][F+2], and the kernel's input channels (Cin = 64) are
// block 1's conv1 (Cin 1 -> 64, BN folded into w1/b1, ReLU) computed while
// the halo is staged: the 525 MB conv1 activation never touches HBM.  The
// conv1 arithmetic is the fma chain of conv_c1_kernel (same order, same bits).
template <int F, int BN, int EPI, bool FUSE>
__global__ __launch_bounds__(512) void conv3x3_x3_kernel(const float* __restrict__ in, int B, int T,
                                                         int Cin, int Cout,
                                                         const uint4* __restrict__ wsp,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out,
                                                         const float* __restrict__ w1,
                                                         const float* __restrict__ b1,
                                                         int* __restrict__ sched) {
  constexpr int BM = ConvGeom<F, BN>::BM, TT = ConvGeom<F, BN>::TT;
  constexpr int RT = TT + 2, CS = F + 2;
  constexpr int CSP = (EPI == EPI_POOL2) ? (F == 64 ? 72 : F == 32 ? 40 : 24)
                                         : (F == 64 ? 66 : F == 32 ? 34 : F == 16 ? 32 : 12);
  constexpr int NPOS = RT * CSP;
  constexpr int WAVES_N = BN / 64, WAVES_M = 8 / WAVES_N, WM = BM / WAVES_M;
  constexpr int MT = WM / 32, NT = 2;
  static_assert(MT == 2, "64 x 64 wave tiles");
  constexpr int A_U4 = NPOS * 5;          // one halo image
  constexpr int W_U4 = BN * 4;            // one tap
  constexpr int WS_U4 = 3 * W_U4;         // one stage (kernel row)
  // staging items: (halo position, 4-channel quarter): the 4 lanes of a
  // position read its chunk's 64 contiguous bytes, so one load instruction
  // covers 16 positions (16 cache-line segments) instead of 32 positions at
  // 16 B each; FUSE: one item per halo position (all 16 channels: the
  // chunk's conv1 weights are wave-uniform)
  constexpr int A_ITEMS = FUSE ? RT * CS : 4 * RT * CS;
  constexpr int NA = (A_ITEMS + 511) / 512;
  constexpr int NW = (WS_U4 + 511) / 512;
  // store instructions one epilogue issues per wave (all of them issue)
  constexpr int EPI_NST = (EPI == EPI_FMEAN) ? 2 * MT * 2 : 4 * MT * 2;
  // weight stages go global -> LDS by LDS-DMA (global_load_lds_dwordx4): the
  // host-prepared image is copied lane-linearly, no VGPR round trip, no
  // ds_write pass.  A DMA issued after a stage barrier must land before the
  // next one (2-slot ring), so each barrier waits on a counted vmcnt.
  // (not FUSE: block 1 measured 2 % slower with it — its conv1 VALU work
  // and conditional halo loads force vmcnt(0) at every barrier)
  constexpr bool GW = !FUSE;

  // one LDS object per W slot and one for the halo images: every fragment
  // read is (lane base VGPR) + immediate, and the compiler's alias scopes
  // tell a DMA into one W slot apart from reads of the other slot / halo
  __shared__ uint4 lds_w0[WS_U4], lds_w1[WS_U4], lds_a[2 * A_U4];
  __shared__ int s_tiles[4];              // claimed tile of the workgroup's k-th tile, at k & 3
  uint4* const Abuf = lds_a;
#define SEDX_WSLOT(slot) ((slot) ? lds_w1 : lds_w0)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int h = lane >> 5;
  const int tiles_t = (T + TT - 1) / TT;
  const int nN = Cout / BN;
  const int ntiles = B * tiles_t * nN;
  const int per_xcd = (ntiles + 7) >> 3;
  const int nchunks = Cin >> 4;           // even for every layer (host checks)

  // ---- dynamic tile claims (thread 0) ----
  unsigned xid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xid));
  const int xcd = (int)(xid & 7u);
  auto range_len = [&](int x) { return min(per_xcd, ntiles - x * per_xcd); };
  // claim from ranges xcd+r, r >= r0; returns a tile or -1
  auto steal = [&](int r0) -> int {
    for (int r = r0; r < 8; ++r) {
      const int x = (xcd + r) & 7;
      if (range_len(x) <= 0) continue;
      const int v = atomicAdd(&sched[32 * x], 1);
      if (v < range_len(x)) return x * per_xcd + v;
    }
    return -1;
  };
  int g_pend = 0, g_k = 0;                // thread 0: own-range claim in flight for tile g_k
  bool g_have = false, g_done = false;
  auto claim_issue = [&](int k) {         // at decode of tile k - 1 (thread 0)
    if (g_done) return;
    g_k = k;
    g_have = true;
    g_pend = range_len(xcd) > 0 ? atomicAdd(&sched[32 * xcd], 1) : 0x7fffffff;
  };
  auto claim_land = [&]() {               // >= 1 barrier before decode of tile g_k (thread 0)
    if (!g_have) return;
    g_have = false;
    int t = g_pend < range_len(xcd) ? xcd * per_xcd + g_pend : steal(1);
    if (t < 0) g_done = true;
    s_tiles[g_k & 3] = t;
  };

  auto decode = [&](ConvCursor& c) {
    const int tile = s_tiles[c.k & 3];
    c.valid = tile >= 0;
    const int m = c.valid ? tile / nN : 0;   // past the end: loads stay in bounds
    c.nb = c.valid ? tile - m * nN : 0;
    c.b = m / tiles_t;
    c.t0 = (m - c.b * tiles_t) * TT;
    if (tid == 0 && c.valid) claim_issue(c.k + 1);
  };
  auto advance = [&](ConvCursor& c) {
    if (++c.chunk == nchunks) {
      c.chunk = 0;
      ++c.k;
      decode(c);
    }
  };

  // per-lane LDS bases (uint4 units), kept opaque so the compiler folds only
  // the tap / buffer / slot constants into the ds_read immediates
  int abase[2][MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int tl, f;
    rowmap<F, EPI>(wm * WM + mt * 32 + (lane & 31), tl, f);
    const int p = (tl * CSP + f) * 5 + h;
    abase[0][mt] = p;
    abase[1][mt] = p + A_U4;
    asm volatile("" : "+v"(abase[0][mt]));
    asm volatile("" : "+v"(abase[1][mt]));
  }
  int wbase[NT][2];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = wn * 64 + nt * 32 + (lane & 31);
    const int s = (n >> 2) & 3;
    wbase[nt][0] = n * 4 + (h ^ s);
    wbase[nt][1] = n * 4 + ((2 + h) ^ s);
    asm volatile("" : "+v"(wbase[nt][0]));
    asm volatile("" : "+v"(wbase[nt][1]));
  }

  f32x16 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.0f;

  float4 ra0[NA];                         // staged halo items (16 B each)
  bool rok[NA];                           // ... inside the image (else zero)
  float xr[FUSE ? NA : 1][9];             // FUSE: conv1 input neighbourhoods
  uint4 rw0[NW], rw1[NW];                 // W stage x lives in rw(x & 1)

  // Staging loads and stores are branch-free (indices clamped, halo zeroes by
  // select) so the compiler's vmcnt bookkeeping stays exact and each wait
  // covers only the loads it needs.  Per-item halo geometry is loop-invariant.
  int a_r[NA], a_f[NA], a_off[NA], a_rec[NA];
  bool a_fok[NA], a_live[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    // FUSE: the last item round is ragged (660 halo positions over 512
    // threads): whole waves past the end skip its conv1 work and LDS writes
    // (their clamped loads stay, keeping the vmcnt bookkeeping branch-free)
    a_live[i] = !FUSE || __builtin_amdgcn_readfirstlane(i * 512 + (tid & ~63)) < A_ITEMS;
    const int idx = min(tid + i * 512, A_ITEMS - 1);
    const int pos = FUSE ? idx : idx >> 2, qq = FUSE ? 0 : idx & 3;
    const int r = pos / CS, c = pos - r * CS;
    a_r[i] = r;
    a_f[i] = c - 1;
    a_fok[i] = c >= 1 && c <= F;
    a_off[i] = FUSE ? min(max(c - 1, 0), F - 1) : min(max(c - 1, 0), F - 1) * Cin + 4 * qq;
    // FUSE: record index in uint4; else the quarter's hi slot in uint2 units
    // (record = 10 x 8 B: hi quarters 0-3, lo quarters 4-7, pad)
    a_rec[i] = FUSE ? (r * CSP + c) * 5 : (r * CSP + c) * 10 + qq;
  }
#define SEDX_LOAD_A(c_)                                                                 \
  if constexpr (FUSE) {                                                                 \
    /* 3x3 neighbourhood of every staged pixel in the padded bn0 output */              \
    const float* in_b_ = in + (int64_t)(c_).b * (T + 2) * (F + 2);                      \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                    \
      const int t = (c_).t0 - 1 + a_r[i];                                               \
      rok[i] = a_fok[i] && t >= 0 && t < T;                                             \
      const float* x_ = in_b_ + (min(max(t, 0), T - 1) * (F + 2) + a_off[i]);           \
      _Pragma("unroll") for (int k = 0; k < 9; ++k) xr[i][k] = x_[(k / 3) * (F + 2) + k % 3]; \
    }                                                                                   \
    asm volatile("" ::: "memory");                                                      \
  } else {                                                                              \
    const float* in_b_ = in + (int64_t)(c_).b * T * F * Cin + (c_).chunk * 16;          \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                    \
      const int t = (c_).t0 - 1 + a_r[i];                                               \
      const bool ok = a_fok[i] && t >= 0 && t < T;                                      \
      const int tc = min(max(t, 0), T - 1);                                             \
      ra0[i] = *reinterpret_cast<const float4*>(in_b_ + (tc * F * Cin + a_off[i]));     \
      rok[i] = ok;     /* halo zeroes applied at the LDS write, not here */             \
    }                                                                                   \
    asm volatile("" ::: "memory"); /* issue here: not sunk to the use */                \
  }
#define SEDX_STORE_A(buf, c_) SEDX_STORE_A_ITEMS(buf, c_, 0, NA)
#define SEDX_STORE_A_ITEMS(buf, c_, i0, i1)                                             \
  {                                                                                     \
    uint4* dst_ = Abuf + (buf) * A_U4;                                                  \
    _Pragma("unroll") for (int i = (i0); i < (i1); ++i) {                               \
      if (!a_live[i]) continue;  /* wave-uniform: no lane of this wave has item i */    \
      uint4 hi, lo;                                                                     \
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);                                 \
      if constexpr (FUSE) {                                                             \
        /* the chunk's 16 conv1 channels (w1 is [tap][64]: wave-uniform scalars); */    \
        /* per channel the fma chain of conv1, scalar v_fma_f32: no packed f32   */      \
        /* VALU beside MFMAs (see sedx_internal.h "packed FP32")                  */      \
        const int ch0 = (c_).chunk * 16;                                                \
        _Pragma("unroll") for (int hh = 0; hh < 2; ++hh) {                              \
          float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};                       \
          _Pragma("unroll") for (int k = 0; k < 9; ++k)                                 \
            _Pragma("unroll") for (int j = 0; j < 8; ++j)                               \
              a8[j] = fmaf(w1[k * 64 + ch0 + 8 * hh + j], xr[i][k], a8[j]);             \
          float o[8];                                                                   \
          _Pragma("unroll") for (int j = 0; j < 8; ++j)                                 \
            o[j] = rok[i] ? fmaxf(a8[j] + b1[ch0 + 8 * hh + j], 0.0f) : 0.0f;           \
          split8(make_float4(o[0], o[1], o[2], o[3]), make_float4(o[4], o[5], o[6], o[7]), hi, lo); \
          dst_[a_rec[i] + hh] = hi;                                                     \
          dst_[a_rec[i] + 2 + hh] = lo;                                                 \
        }                                                                               \
      } else {                                                                          \
        const float4 v_ = rok[i] ? ra0[i] : z;                                          \
        uint2 h2, l2;                                                                   \
        split2(v_.x, v_.y, h2.x, l2.x);                                                 \
        split2(v_.z, v_.w, h2.y, l2.y);                                                 \
        uint2* d2_ = reinterpret_cast<uint2*>(dst_);                                    \
        d2_[a_rec[i]] = h2;                                                             \
        d2_[a_rec[i] + 4] = l2;                                                         \
        (void)hi;                                                                       \
        (void)lo;                                                                       \
      }                                                                                 \
    }                                                                                   \
    asm volatile("" ::: "memory");                                                      \
  }
#define SEDX_LOAD_W(rs, c_, ky_)                                                        \
  {                                                                                     \
    const uint4* src_ = wsp + (((int64_t)(c_).nb * nchunks + (c_).chunk) * 3 + (ky_)) * WS_U4; \
    _Pragma("unroll") for (int i = 0; i < NW; ++i) {                                    \
      const uint4 v_ = src_[min(tid + i * 512, WS_U4 - 1)];                             \
      if ((rs) == 0) rw0[i] = v_; else rw1[i] = v_;                                     \
    }                                                                                   \
    asm volatile("" ::: "memory");                                                      \
  }
#define SEDX_STORE_W(rs, slot)                                                          \
  {                                                                                     \
    uint4* dst_ = SEDX_WSLOT(slot);                                                \
    _Pragma("unroll") for (int i = 0; i < NW; ++i)                                      \
      dst_[min(tid + i * 512, WS_U4 - 1)] = ((rs) == 0) ? rw0[i] : rw1[i];              \
    asm volatile("" ::: "memory"); /* before the refill loads are issued */             \
  }

  // GW: W stage ky_ of unit c_ -> LDS slot `slot` (wave-uniform LDS base, lane x 16 B)
  const int wv_ = __builtin_amdgcn_readfirstlane(wave);
#define SEDX_DMA_W(c_, ky_, slot)                                                       \
  {                                                                                     \
    const uint4* src_ = wsp + (((int64_t)(c_).nb * nchunks + (c_).chunk) * 3 + (ky_)) * WS_U4 + tid; \
    _Pragma("unroll") for (int i = 0; i < NW; ++i) {                                    \
      if (WS_U4 % 512 == 0 || i * 512 + (wv_ << 6) < WS_U4) {                           \
        const uint32_t m0_ = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(        \
            (__attribute__((address_space(3))) uint4*)(SEDX_WSLOT(slot) + i * 512 + (wv_ << 6)))); \
        sedx_glds16(src_ + i * 512, m0_);                                               \
      }                                                                                 \
    }                                                                                   \
    asm volatile("" ::: "memory");                                                      \
  }
  // stage barrier under GW: this wave's DMAs older than its n_ youngest VMEM
  // ops have landed, its LDS writes are done, then the workgroup barrier
#define SEDX_BAR_VM(n_)                                                                 \
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(n_) : "memory")

  bf16x8 fa[2][2 * MT], fb[2][2 * NT];
  // fragments of tap a (0..8) of a unit whose halo is in A buffer `abuf`
  // and whose stage a/3 sits in W slot `wslot`
#define SEDX_READ_FRAGS(set, abuf, wslot, tap_)                                         \
  {                                                                                     \
    constexpr int aoff_ = (((tap_) / 3) * CSP + ((tap_) % 3)) * 5;                      \
    constexpr int woff_ = ((tap_) % 3) * W_U4;                        \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                 \
      fa[set][2 * mt] = as_bf16x8(lds_a[abase[abuf][mt] + aoff_]);                        \
      fa[set][2 * mt + 1] = as_bf16x8(lds_a[abase[abuf][mt] + aoff_ + 2]);                \
    }                                                                                   \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                 \
      fb[set][2 * nt] = as_bf16x8(SEDX_WSLOT(wslot)[wbase[nt][0] + woff_]);                           \
      fb[set][2 * nt + 1] = as_bf16x8(SEDX_WSLOT(wslot)[wbase[nt][1] + woff_]);                       \
    }                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  }
// epilogue stores: default cache policy (nt measured neutral in the model)
constexpr int EPI_AUX = 0;
#ifdef SEDX_SETPRIO
#define SEDX_PRIO(p) __builtin_amdgcn_s_setprio(p)
#else
#define SEDX_PRIO(p)
#endif
#define SEDX_MFMAS(set)                                                                 \
  {                                                                                     \
    SEDX_PRIO(1);                                                                       \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                   \
    _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) {                                 \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * mt], fb[set][2 * nt], acc[mt][nt], 0, 0, 0);     \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * mt], fb[set][2 * nt + 1], acc[mt][nt], 0, 0, 0); \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * mt + 1], fb[set][2 * nt], acc[mt][nt], 0, 0, 0); \
    }                                                                                   \
    SEDX_PRIO(0);                                                                       \
  }

  // bias of the current tile's columns, loaded when the tile starts (a load
  // issued in the epilogue would make its wait drain every prefetch in flight)
  float bcur[NT];
  auto load_bias = [&](const ConvCursor& c) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bcur[nt] = bias[c.nb * BN + wn * 64 + nt * 32 + (lane & 31)];
    asm volatile("" ::: "memory");
  };

  auto epilogue = [&](const ConvCursor& c) {
    int lane_ = lane;                    // opaque: keep the address math here
    asm volatile("" : "+v"(lane_));
    const int h = lane_ >> 5;
    const int n0 = c.nb * BN;
    // stores go through a buffer resource over the clip's output from the
    // tile's first row on: every store instruction issues (rows past the
    // clip's end get an out-of-range offset, which the range check drops), so
    // their count is static and the next stage barrier can leave them in
    // flight (EPI_NST).  Offsets stay below one tile's rows (< 1 MB) and the
    // record count is clamped to 2^31 - 1, so any clip length is safe.
    constexpr int ROW = (EPI == EPI_POOL2) ? (F / 2) * 1 : (EPI == EPI_FMEAN) ? 1 : F;
    const int T_out = (EPI == EPI_POOL2) ? T / 2 : T;
    const int row0 = (EPI == EPI_POOL2) ? c.t0 / 2 : c.t0;
    const int64_t clip_floats = (int64_t)T_out * ROW * Cout;
    const int64_t rest_bytes = ((int64_t)(T_out - row0) * ROW * Cout) * 4;
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
        out + (int64_t)c.b * clip_floats + (int64_t)row0 * ROW * Cout, (short)0,
        (int)(rest_bytes < 0x7fffffff ? rest_bytes : 0x7fffffff), 0x00020000);
    constexpr uint32_t OOB = 0x80000000u;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + wn * 64 + nt * 32 + (lane_ & 31);
      const float bv = bcur[nt];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int Rbase = wm * WM + mt * 32;
        float r[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) r[i] = fmaxf(acc[mt][nt][i] + bv, 0.0f);
        if (EPI == EPI_STORE) {
          // regs 4g..4g+3 are 4 consecutive pixels of this lane's channel; a
          // 4x4 transpose inside each lane quad gives every lane 4 consecutive
          // channels of one pixel: 4 dwordx4 stores instead of 16 dword stores,
          // same bytes, the same 128-B lines per group of stores
          const int j = lane_ & 3;
          const int tlim = T - c.t0;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float* v = r + 4 * g;
            quad_transpose4(v, j);
            int tl, f;
            rowmap<F, EPI>(Rbase + 8 * g + 4 * h + j, tl, f);
            const uint32_t off = (tl < tlim) ? (uint32_t)(((tl * F + f) * Cout + n - j) * 4) : OOB;
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 w = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
            __builtin_amdgcn_raw_buffer_store_b128(w, ors, off, 0, EPI_AUX);
            __builtin_amdgcn_sched_barrier(0);
          }
        } else if (EPI == EPI_POOL2) {
          constexpr int FO = F / 2;
          const int To = T / 2;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int q = (Rbase + 8 * g + 4 * h) >> 2;
            const int tp = q / FO, fp = q % FO;
            const int to = c.t0 / 2 + tp;
            const float v = (((r[4 * g] + r[4 * g + 1]) + r[4 * g + 2]) + r[4 * g + 3]) * 0.25f;
            const uint32_t off = (to < To) ? (uint32_t)(((tp * FO + fp) * Cout + n) * 4) : OOB;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ors, off, 0, EPI_AUX);
          }
        } else {  // EPI_FMEAN, F == 8: regs {0-3,12-15} and {4-11} are one t each (rowmap)
          const float sa = (((r[0] + r[1]) + (r[2] + r[3])) + ((r[12] + r[13]) + (r[14] + r[15])));
          const float sb = (((r[4] + r[5]) + (r[6] + r[7])) + ((r[8] + r[9]) + (r[10] + r[11])));
          const int tb = c.t0 + 4 * (Rbase >> 5);
          const int ta = tb + (h ? 3 : 0), tb2 = tb + (h ? 2 : 1);
          const uint32_t offa = (ta < T) ? (uint32_t)(((ta - c.t0) * Cout + n) * 4) : OOB;
          const uint32_t offb = (tb2 < T) ? (uint32_t)(((tb2 - c.t0) * Cout + n) * 4) : OOB;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sa * 0.125f), ors, offa, 0, EPI_AUX);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sb * 0.125f), ors, offb, 0, EPI_AUX);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[mt][nt][i] = 0.0f;
      }
    }
  };

  SEDX_ST_DECL
  if (tid == 0) {
    const int t = steal(0);
    if (t < 0) g_done = true;
    s_tiles[0] = t;
  }
  __syncthreads();
  // cur = unit being computed, n1 / n2 = the next two units of the stream
  ConvCursor cur{0, 0, 0, 0, 0, false};
  decode(cur);
  if (!cur.valid) return;
  ConvCursor n1 = cur;
  advance(n1);
  ConvCursor n2 = n1;
  advance(n2);

  // prologue: halo(cur) -> A0, W(cur, row 0/1) -> slots 0/1; registers hold
  // W(cur, row 2), W(n1, row 0) and halo(n1)
  load_bias(cur);
  SEDX_LOAD_A(cur);
  if constexpr (GW) {
    SEDX_DMA_W(cur, 0, 0);
    SEDX_DMA_W(cur, 1, 1);
    SEDX_STORE_A(0, cur);
    SEDX_LOAD_A(n1);
    SEDX_BAR_VM(NA);
  } else {
  SEDX_LOAD_W(0, cur, 0);
  SEDX_LOAD_W(1, cur, 1);
  SEDX_STORE_A(0, cur);
  SEDX_STORE_W(0, 0);
  SEDX_STORE_W(1, 1);
  // pending loads enter the loop in the order the loop's back edge leaves
  // them, so the waitcnt bookkeeping at the loop header stays exact
  if constexpr (FUSE) {
    SEDX_LOAD_W(0, cur, 2);
    SEDX_LOAD_A(n1);
    SEDX_LOAD_W(1, n1, 0);
  } else {
    SEDX_LOAD_A(n1);
    SEDX_LOAD_W(0, cur, 2);
    SEDX_LOAD_W(1, n1, 0);
  }
  __syncthreads();
  }
  SEDX_READ_FRAGS(0, 0, 0, 0);

  // One stage = taps 3KY..3KY+2 of the current unit (parity U: halo in A
  // buffer U, stage KY in W slot (U + KY) & 1, fragment set of tap a =
  // (U + a) & 1).  After the barrier the slot of stage KY is free:
  //   KY 0: W(cur, 2) -> slot U;      halo(n1) -> A buffer U^1; load halo(n2)
  //   KY 1: W(n1, 0)  -> slot U^1
  //   KY 2: W(n1, 1)  -> slot U
  // each followed by the load of the weights two stages further on into the
  // register set just drained (W(n1, 1), W(n1, 2), W(n2, 0)).
// After the stage barrier the wave interleaves the stage's LDS writes and
// global refill loads with the 4 MFMA groups of the stage's last tap (whose
// fragments were read before the barrier), so the matrix pipe is not idle
// while both waves of a SIMD stage data:
//   group (0,0) | W store | group (0,1) | W load | group (1,0) | halo work | group (1,1)
// then the fragments of the next tap are read.
#define SEDX_MFMA_G(set, mt, nt)                                                        \
  {                                                                                     \
    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * (mt)], fb[set][2 * (nt)], acc[mt][nt], 0, 0, 0);     \
    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * (mt)], fb[set][2 * (nt) + 1], acc[mt][nt], 0, 0, 0); \
    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[set][2 * (mt) + 1], fb[set][2 * (nt)], acc[mt][nt], 0, 0, 0); \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  }
#define SEDX_MFMA_PIECE(set, mt, nt) SEDX_MFMA_G(set, mt, nt)
#define SEDX_MFMA_REST(set) SEDX_MFMA_G(set, 1, 1)
// FUSE: the conv1 work of n1's halo items (VALU-heavy) is issued between the
// MFMAs of the stage's first tap, BEFORE the stage barrier.  Legal: A buffer
// U^1 was last read by unit U-1 before its stage-2 barrier, and n1's inputs
// were loaded two stages earlier.
#define SEDX_STAGE_POST(U, KY, set)                                                     \
  if constexpr (GW) {                                                                   \
    /* halo(n1) first (its loads are older than this stage's DMA), then the */          \
    /* DMA of the stage after next into the slot just freed, then halo(n2)   */          \
    SEDX_MFMA_PIECE(set, 0, 0);                                                         \
    if ((KY) == 0) {                                                                    \
      SEDX_STORE_A((U) ^ 1, n1);                                                    \
    }                                                                                   \
    SEDX_MFMA_PIECE(set, 0, 1);                                                         \
    if ((KY) == 0) {                                                                    \
      SEDX_DMA_W(cur, 2, U);                                                            \
    } else if ((KY) == 1) {                                                             \
      SEDX_DMA_W(n1, 0, ((U) + 1) & 1);                                                 \
    } else {                                                                            \
      if (tid == 0) claim_land();                                                       \
      SEDX_DMA_W(n1, 1, U);                                                             \
    }                                                                                   \
    SEDX_MFMA_PIECE(set, 1, 0);                                                         \
    if ((KY) == 0) {                                                                    \
      SEDX_LOAD_A(n2);                                                              \
    }                                                                                   \
    SEDX_MFMA_REST(set);                                                                \
  } else {                                                                              \
    SEDX_MFMA_PIECE(set, 0, 0);                                                         \
    if ((KY) == 0) {                                                                    \
      SEDX_STORE_W((U) & 1, U);                                                     \
    } else if ((KY) == 1) {                                                             \
      SEDX_STORE_W(((U) + 1) & 1, ((U) + 1) & 1);                                   \
    } else {                                                                            \
      SEDX_STORE_W((U) & 1, (U) & 1);                                               \
    }                                                                                   \
    SEDX_MFMA_PIECE(set, 0, 1);                                                         \
    if ((KY) == 0) {                                                                    \
      SEDX_LOAD_W((U) & 1, n1, 1);                                                  \
    } else if ((KY) == 1) {                                                             \
      SEDX_LOAD_W(((U) + 1) & 1, n1, 2);                                            \
    } else {                                                                            \
      if (tid == 0) claim_land();                                                       \
      SEDX_LOAD_W((U) & 1, n2, 0);                                                  \
    }                                                                                   \
    SEDX_MFMA_PIECE(set, 1, 0);                                                         \
    if constexpr (FUSE) {                                                               \
      /* conv1's input (one channel) is the same for every chunk of a tile: */          \
      /* the neighbourhoods in xr are reloaded only when n2 starts a new tile */        \
      if ((KY) == 1 && n2.chunk == 0) {                                                 \
        SEDX_LOAD_A(n2);                                                                \
      }                                                                                 \
    } else if ((KY) == 0) {                                                             \
      SEDX_STORE_A((U) ^ 1, n1);                                                    \
      SEDX_LOAD_A(n2);                                                              \
    }                                                                                   \
    SEDX_MFMA_REST(set);                                                                \
  }
#define SEDX_STAGE(U, KY)                                                               \
  {                                                                                     \
    SEDX_READ_FRAGS(((U) + 3 * (KY) + 1) & 1, U, ((U) + (KY)) & 1, 3 * (KY) + 1);       \
    if constexpr (FUSE) {                                                               \
      if ((KY) == 0) {                                                                  \
        SEDX_STORE_A_ITEMS((U) ^ 1, n1, 0, 1);                                          \
      } else if ((KY) == 1) {                                                           \
        SEDX_STORE_A_ITEMS((U) ^ 1, n1, 1, NA);                                         \
      }                                                                                 \
    }                                                                                   \
    SEDX_MFMAS(((U) + 3 * (KY)) & 1);                                                   \
    SEDX_READ_FRAGS(((U) + 3 * (KY) + 2) & 1, U, ((U) + (KY)) & 1, 3 * (KY) + 2);       \
    SEDX_MFMAS(((U) + 3 * (KY) + 1) & 1);                                               \
    SEDX_ST_BEGIN();                                                                    \
    if constexpr (GW) {                                                                 \
      /* KY 1: the halo loads of n2, issued after KY 0's DMA, stay in flight */          \
      /* KY 0 after a tile's epilogue: its stores, issued after KY 2's DMA, too */ \
      if ((KY) == 1) SEDX_BAR_VM(NA);                                                   \
      else if ((KY) == 0 && epi_prev) SEDX_BAR_VM(EPI_NST);                            \
      else SEDX_BAR_VM(0);                              \
    } else {                                                                            \
      __syncthreads();                                                                  \
    }                                                                                   \
    SEDX_ST_END(st_bar);                                                                \
    SEDX_ST_VMWAIT();                                                                   \
    SEDX_STAGE_POST(U, KY, ((U) + 3 * (KY) + 2) & 1);                                   \
    if ((KY) < 2) {                                                                     \
      SEDX_READ_FRAGS(((U) + 3 * (KY) + 3) & 1, U, ((U) + (KY) + 1) & 1, 3 * (KY) + 3); \
    } else {                                                                            \
      SEDX_READ_FRAGS(((U) + 1) & 1, (U) ^ 1, ((U) + 1) & 1, 0);                        \
    }                                                                                   \
  }

#define SEDX_UNIT(U)                                                                    \
  {                                                                                     \
    SEDX_STAGE(U, 0);                                                                   \
    SEDX_STAGE(U, 1);                                                                   \
    SEDX_STAGE(U, 2);                                                                   \
    if (cur.chunk == nchunks - 1) {                                                     \
      SEDX_ST_BEGIN();                                                                  \
      epilogue(cur);                                                                    \
      SEDX_ST_END(st_epi);                                                              \
    }                                                                                   \
    epi_prev = cur.chunk == nchunks - 1;                                                \
    cur = n1;                                                                           \
    n1 = n2;                                                                            \
    advance(n2);                                                                        \
    if (!cur.valid) break;                                                              \
    if (cur.chunk == 0) load_bias(cur);                                                 \
  }

  bool epi_prev = false;
  while (true) {
    SEDX_UNIT(0);
    SEDX_UNIT(1);
  }
  SEDX_ST_FLUSH();
#undef SEDX_UNIT
#undef SEDX_STAGE
#undef SEDX_STAGE_POST
#undef SEDX_MFMA_G
#undef SEDX_MFMA_PIECE
#undef SEDX_MFMA_REST
#undef SEDX_READ_FRAGS
#undef SEDX_MFMAS
#undef SEDX_LOAD_W
#undef SEDX_DMA_W
#undef SEDX_WSLOT
#undef SEDX_BAR_VM
#undef SEDX_STORE_W
#undef SEDX_LOAD_A
#undef SEDX_STORE_A
#undef SEDX_STORE_A_ITEMS
}

template <int F, int BN, int EPI, bool FUSE = false>
static void launch_x3_epi(const float* in, int B, int T, int Cin, int Cout, const uint4* wp,
                          const float* bias, float* out, int* sched, hipStream_t s,
                          const float* w1 = nullptr, const float* b1 = nullptr) {
  constexpr int TT = ConvGeom<F, BN>::TT;
  // workgroups resident on the whole device (per device)
  const LaunchInfo li =
      launch_info(reinterpret_cast<const void*>(conv3x3_x3_kernel<F, BN, EPI, FUSE>), 512, 0);
  if (!li.ok) return;
  const int resident = li.ncu * li.per_cu;
  const size_t pad = li.dyn;
  const int ntiles = B * ((T + TT - 1) / TT) * (Cout / BN);
  const int per_xcd = (ntiles + 7) / 8;
  int grid = resident & ~7;
  if (grid < 8) grid = 8;
  if (grid > 8 * per_xcd) grid = 8 * per_xcd;
  hipLaunchKernelGGL((conv3x3_x3_kernel<F, BN, EPI, FUSE>), dim3(grid), dim3(512), pad, s, in, B, T, Cin,
                     Cout, wp, bias, out, w1, b1, sched);
}

template <int F, int BN>
static void launch_x3(const float* in, int B, int T, int Cin, int Cout, const uint4* wp,
                      const float* bias, float* out, int epi, int* sched, hipStream_t s) {
  // only the (F, epilogue) pairs of the model are instantiated
  if constexpr (F == 8) {
    if (epi == EPI_STORE)
      launch_x3_epi<8, BN, EPI_STORE>(in, B, T, Cin, Cout, wp, bias, out, sched, s);
    else if (epi == EPI_FMEAN)
      launch_x3_epi<8, BN, EPI_FMEAN>(in, B, T, Cin, Cout, wp, bias, out, sched, s);
  } else if constexpr (F == 64) {
    if (epi == EPI_POOL2)
      launch_x3_epi<F, BN, EPI_POOL2>(in, B, T, Cin, Cout, wp, bias, out, sched, s);
  } else {
    if (epi == EPI_STORE)
      launch_x3_epi<F, BN, EPI_STORE>(in, B, T, Cin, Cout, wp, bias, out, sched, s);
    else if (epi == EPI_POOL2)
      launch_x3_epi<F, BN, EPI_POOL2>(in, B, T, Cin, Cout, wp, bias, out, sched, s);
  }
}

// Shapes: Cin a multiple of 32 (the unit stream pairs chunks), Cout a
// multiple of the n-tile; api.cpp routes only such layers here.
void launch_conv3x3_x3(const float* in, int B, int T, int F, int Cin, int Cout, const void* wp,
                       const float* bias, float* out, int epi, int* sched, hipStream_t s) {
  const uint4* w = static_cast<const uint4*>(wp);
  if (Cin % 32 != 0 || Cin < 64) return;   // the claim of tile k+1 lands >= 1 unit before its decode
  switch (F) {
    case 64:   // block 1 conv2 (Cout 64)
      if (Cout % 64 == 0) launch_x3<64, 64>(in, B, T, Cin, Cout, w, bias, out, epi, sched, s);
      break;
    case 32:
      if (Cout % 128 == 0) launch_x3<32, 128>(in, B, T, Cin, Cout, w, bias, out, epi, sched, s);
      break;
    case 16:
      if (Cout % 128 == 0) launch_x3<16, 128>(in, B, T, Cin, Cout, w, bias, out, epi, sched, s);
      break;
    case 8:
      if (Cout % 128 == 0) launch_x3<8, 128>(in, B, T, Cin, Cout, w, bias, out, epi, sched, s);
      break;
    default: break;
  }
}

// bn0 output [B][T][64] -> [B][T+2][66] with a zero border (the fused block-1
// kernel's conv1 then needs no bounds tests)
__global__ __launch_bounds__(256) void pad_x0_kernel(const float* __restrict__ x0, int B, int T,
                                                     float* __restrict__ xp) {
  const int64_t n = (int64_t)B * (T + 2) * 66;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int f = (int)(i % 66) - 1;
    const int64_t bt = i / 66;
    const int t = (int)(bt % (T + 2)) - 1;
    const int64_t b = bt / (T + 2);
    xp[i] = (t >= 0 && t < T && f >= 0 && f < 64) ? x0[(b * T + t) * 64 + f] : 0.0f;
  }
}

void launch_pad_x0(const float* x0, int B, int T, float* xpad, hipStream_t s) {
  const int64_t n = (int64_t)B * (T + 2) * 66;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(pad_x0_kernel, dim3(blocks), dim3(256), 0, s, x0, B, T, xpad);
}

void launch_block1_fused_x3(const float* x0, int B, int T, float* xpad, const float* w1, const float* b1,
                            const void* wp, const float* bias, float* out, int* sched, hipStream_t s) {
  if (x0) launch_pad_x0(x0, B, T, xpad, s);
  if (out)
    launch_x3_epi<64, 64, EPI_POOL2, true>(xpad, B, T, 64, 64, static_cast<const uint4*>(wp), bias, out,
                                           sched, s, w1, b1);
}

size_t block1_pad_floats(int B, int T) { return (size_t)B * (T + 2) * 66; }

#ifdef SEDX_CONV_STAMPS
void conv_stamps_rw(unsigned long long* out8, bool reset) {
  (void)hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_conv_stamps), 8 * sizeof(unsigned long long));
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_conv_stamps), z, sizeof(z));
  }
}
#endif

}  // namespace sedx
