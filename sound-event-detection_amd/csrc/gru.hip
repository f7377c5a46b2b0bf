// Cooperative bi-GRU recurrence for gfx950 (nn.GRU(512, 256, bidirectional,
// batch_first) of Cnn_9layers_Gru_FrameAtt, pytorch/models.py:614-615, :670;
// ATen gate order r, z, n and h' = n + z (h - n)).
//
// Per (clip group of 32, direction) eight workgroups ("slices") each own 32
// hidden units = 96 gate rows of W_hh, kept for the whole kernel in VGPRs as
// bf16 hi/lo MFMA B-fragments (12 waves = 3 gates x 4 K-quarters, 32 VGPRs
// each).  Per step: wait until all 8 slices published h_{s-1} -> gather
// h_{s-1} [32 x 256] with sc1 loads -> split to a bf16 hi/lo A image in LDS ->
// 12 MFMAs per wave (x3 split, fp32 acc) -> K-quarter partials summed in LDS
// -> gates -> publish the h_s slice.
//
// Two hand-off protocols, chosen once per launch:
//  * XCD-local (fast): the grid puts the 8 slices of a (slot, dir) pair on
//    blocks b = r + 8k (one residue r), which the dispatcher deals to one XCD.
//    At start every slice reads HW_REG_XCC_ID and the 8 ids are exchanged
//    with the global protocol; only if all 8 agree does the pair use plain
//    stores (they stay in the XCD's shared L2) + s_waitcnt vmcnt(0) + a plain
//    per-slice flag, with sc1 (L1-bypassing, L2-served) polls and loads.
//  * global (fallback, any placement): MI355X_MICROARCH.md "Valid forms"
//    row 1: sc1 (write-through) payload stores, s_waitcnt vmcnt(0) in every
//    storing wave, barrier, one agent-scope atomic add per slice; sc1 poll of
//    the counter, barrier, sc1 loads of the payload.
// Results are identical in both modes (same arithmetic; only the transport
// differs).
//
// Arithmetic (template EXACT): false = the bf16 hi/lo x3 split above;
// true = fp32 operands on v_mfma_f32_32x32x2_f32 (the reference's fp32
// nn.GRU): each wave keeps its 32 gate rows x 64-K quarter of W_hh as 32 fp32
// B-fragments (lane: row lane&31, k = 2 st + (lane>>5)) and reads h_{s-1}
// from an fp32 [k][clip] LDS image whose rows are XOR-swizzled by (k>>3)&31
// (conflict-free for both the gather's writes and the fragment reads).  The exchange buffer is double-buffered by step parity (a slice
// publishes step gs only after it has gathered step gs-1 from every slice,
// i.e. after all slices finished reading step gs-2's buffer; at group
// boundaries the wait still runs although h is reset).  Flags, counters and
// the id table are zeroed by hipMemsetAsync before every launch; every spin is
// bounded: a timeout sets sync->err and turns every later H value of that
// workgroup into NaN, so it surfaces in framewise / clipwise output.
#include "sedx_internal.h"

namespace sedx {

typedef float f32x16_g __attribute__((ext_vector_type(16)));
typedef float f32x4_g __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_g __attribute__((ext_vector_type(8)));

typedef __bf16 bf16x2_g __attribute__((ext_vector_type(2)));
// x = hi + lo, hi = bf16_rne(x), lo = bf16_rne(x - hi) (v_cvt_pk_bf16_f32)
__device__ __forceinline__ void g_split8(const float* v, uint4& hi, uint4& lo) {
  uint32_t hh[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16x2_g h2 = {(__bf16)v[2 * i], (__bf16)v[2 * i + 1]};
    hh[i] = __builtin_bit_cast(uint32_t, h2);
    const bf16x2_g l2 = {(__bf16)(v[2 * i] - __uint_as_float(hh[i] << 16)),
                         (__bf16)(v[2 * i + 1] - __uint_as_float(hh[i] & 0xFFFF0000u))};
    ll[i] = __builtin_bit_cast(uint32_t, l2);
  }
  hi = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  lo = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}
// gates on v_exp_f32 (__expf): |error| ~1e-7 against the libm forms, well
// inside the 1e-3 framewise bar; tanh(x) = 2 / (1 + e^(-2x)) - 1 saturates
// correctly at both ends
__device__ __forceinline__ float g_sigmoid(float x) { return __frcp_rn(1.0f + __expf(-x)); }
__device__ __forceinline__ float g_tanh(float x) { return 2.0f * __frcp_rn(1.0f + __expf(-2.0f * x)) - 1.0f; }
// one GRU cell (ATen gate order r, z, n; h' = n + z (h - n)); gh* = the
// recurrent pre-activations with b_hh added, gi* = x W_ih^T + b_ih.  Every
// recurrence kernel calls this one function, so their gate arithmetic (and
// its fma contraction) is the same instruction sequence
__device__ __forceinline__ float gru_cell(float gir, float giz, float gin, float ghr, float ghz, float ghn, float hp) {
  const float r = g_sigmoid(gir + ghr);
  const float z = g_sigmoid(giz + ghz);
  const float n = g_tanh(gin + r * ghn);
  return n + z * (hp - n);
}
__device__ __forceinline__ unsigned g_ld(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1
}

constexpr int GRU_MAX_SLOTS = 4;      // 2 * slots (slot, dir) pairs on 8 XCD residues
constexpr int GRU_VALU_CLIPS = 8;     // exact launches this small run the VALU product
constexpr int GRU_HV_LD = 260;        // Hv row stride (floats): 8 rows fit the A-image space
static_assert(GRU_VALU_CLIPS * GRU_HV_LD <= 16 * 32 * 4 * 4, "Hv inside Aimg");
// VALU granules [2 pairs][2 parities][clips][256] u64 at the start of the exchange space
static_assert(2 * 2 * GRU_VALU_CLIPS * 256 * 8 <= 8 * 2 * 32 * 256 * 4, "granules inside X");
// bound of every hand-off spin, in polls: the handle's SEDX_TUNE_GRU_SPIN
// (2^24 by default; tests force a timeout with 0 — fail at the first poll
// that finds the data not there yet)

struct GruSync {                      // zeroed every launch
  unsigned err;
  unsigned pad0[63];
  unsigned ready[8][16];              // per pair: id-exchange arrivals
  unsigned xcc[8][16];                // per pair: slice XCC ids (+1)
  unsigned cnt[8][16];                // per pair: global-protocol step counter
  unsigned flag[8][16][16];           // per pair, per slice: fast-protocol step flag
  unsigned long long stamps[8];       // SEDX_GRU_STAMPS diagnostic builds only
  unsigned mode;                      // 1 = XCD-local protocol was used by pair 0
};
// a bounded spin timed out: the launch's own flag word and the handle's
// host-mapped word (sedx_forward* returns SEDX_EHIP on the next call)
// (a plain system-scope store of the code with bit 31 set: any nonzero word
// reports the failure, and a store needs no PCIe / xGMI atomics on host memory)
__device__ __forceinline__ void gru_fail(GruSync* sync, unsigned* host_err, unsigned code) {
  atomicOr(&sync->err, code);
  if (host_err) __hip_atomic_store(host_err, code | 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// spin bound 0 (tests): every step that would wait fails at once, whether
// or not its data has already arrived (a bound of 0 polls is otherwise a
// race against the producers' timing)
__device__ __forceinline__ void gru_forced_fail(unsigned spin_limit, int gs, GruSync* sync, unsigned* host_err,
                                                int* s_err) {
  if (spin_limit == 0 && gs > 0) {
    gru_fail(sync, host_err, 8u);
    *s_err = 1;
  }
}
// the workgroup's timeout word (a __shared__ int): read as an LDS access
// (a generic volatile pointer would become a flat load, which the compiler
// orders with vmcnt(0) — a drain of every store in flight)
__device__ __forceinline__ bool gru_dead(const int* s_err) {
  return *(const volatile __attribute__((address_space(3))) int*)(s_err) != 0;
}

#ifdef SEDX_GRU_STAMPS
#define GRU_STAMP(i)                                                                    \
  if (tid == 0 && pair == 0 && p == 0) {                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
    st_acc[i] += now_ - st_last;                                                        \
    st_last = now_;                                                                     \
  }
#else
#define GRU_STAMP(i)
#endif

// NS slices per (group, direction): 8 (32 hidden units each), or 16 (exact
// MFMA product only: 16 units each, 16x16x4 MFMAs, half the serial product
// per step; the same fma chains, so bit-identical to NS 8)
template <bool EXACT, bool VALU, int NS = 8>
__global__ __launch_bounds__(768) void gru_coop_kernel(const float* __restrict__ G, int B, int T,
                                                       const float* __restrict__ whh,
                                                       const float* __restrict__ bhh,
                                                       float* __restrict__ H, float* X,
                                                       GruSync* sync, int nslots, int allow_fast,
                                                       unsigned* host_err, unsigned spin_limit, int spread) {
  __shared__ uint4 Aimg[16 * 32 * 4];          // h_{s-1} hi/lo, [kstep][clip][4 slots]
  // partial gate pre-activations: K quarters (x3) / eighths (exact: two
  // independent chains per wave, summed in order in the gate phase)
  constexpr int KP = EXACT ? 8 : 4;
  __shared__ float part[KP][3][32][33];
  __shared__ float hprev[32][33];              // own-slice h_{s-1}
  __shared__ int s_fast;
  __shared__ int s_err;                        // a bounded spin timed out: outputs become NaN
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  static_assert(NS == 8 || (NS == 16 && EXACT && !VALU), "16 slices: the exact MFMA product");
  constexpr int US = 256 / NS;                 // hidden units per slice
  constexpr int NPAIR = 32 * US;               // (clip, unit) pairs of a slice's gate phase
  // default: the slices of a pair on blocks b = pair + 8 k — one dispatch
  // residue, one XCD (observed) — for the XCD-local hand-off; spread: slice
  // p on block NS pair + p, so a pair's slices cover every XCD (beside a
  // concurrent conv stack whose items are dealt to XCDs evenly, no XCD loses
  // a quarter of its CUs to the recurrence)
  const int pair = spread ? (int)blockIdx.x / NS : (int)(blockIdx.x & 7);
  const int p = spread ? (int)blockIdx.x % NS : (int)(blockIdx.x >> 3);   // slice 0 .. NS - 1
  const int slot = pair >> 1, dir = pair & 1;
  if (slot >= nslots) return;                  // whole workgroup exits (uniform)
  const int nt = wave % 3, kq = wave / 3, h = lane >> 5;
  const int ngroups = (B + 31) / 32;

  // ---- placement check (global protocol) ----
  if (tid == 0) {
    s_err = 0;
    unsigned xid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xid));
    __hip_atomic_store(&sync->xcc[pair][p], (xid & 0xffu) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(&sync->ready[pair][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (g_ld(&sync->ready[pair][0]) < (unsigned)NS) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > spin_limit) {
        gru_fail(sync, host_err, 1u);
        s_err = 1;
        break;
      }
    }
    int fast = allow_fast;
    const unsigned x0 = g_ld(&sync->xcc[pair][0]);
    for (int i = 1; i < NS; ++i) fast &= (g_ld(&sync->xcc[pair][i]) == x0);
    s_fast = fast;
  }
  __syncthreads();
  const bool fast = s_fast != 0;
  if (tid == 0 && pair == 0 && p == 0) sync->mode = fast ? 1u : 0u;
#ifdef SEDX_GRU_STAMPS
  unsigned long long st_acc[4] = {0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif

  // W_hh slice -> B fragments: B[k][n] = W_hh[gate row n][k]
  bf16x8_g Bhi[4], Blo[4];
  static_assert(EXACT || !VALU, "the VALU product is the exact arithmetic");
  float Bf[EXACT && !VALU ? (NS == 16 ? 16 : 32) : 1];
  float4 Wv[VALU ? 16 : 1];   // VALU: the lane's gate row over its whole K quarter
  if constexpr (NS == 16) {
    // 16x16x4: lane (k = lane >> 4, unit lane & 15) of steps s of eighths
    // 2 kq + e: Bf[8 e + s] = W_hh[row][64 kq + 32 e + 4 s + (lane >> 4)]
    const float* wrow = whh + ((int64_t)dir * 768 + nt * 256 + US * p + (lane & 15)) * 256;
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int st = 0; st < 8; ++st) Bf[8 * e + st] = wrow[64 * kq + 32 * e + 4 * st + (lane >> 4)];
  } else {
    const float* wrow = whh + ((int64_t)dir * 768 + nt * 256 + 32 * p + (lane & 31)) * 256;
    if constexpr (VALU) {
#pragma unroll
      for (int q = 0; q < 16; ++q) Wv[q] = reinterpret_cast<const float4*>(wrow + 64 * kq)[q];
    } else if constexpr (EXACT) {
#pragma unroll
      for (int st = 0; st < 32; ++st) Bf[st] = wrow[64 * kq + 2 * st + h];
    } else {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const float4* q = reinterpret_cast<const float4*>(wrow + 16 * (4 * kq + ks) + 8 * h);
        const float4 a = q[0], b = q[1];
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint4 hi, lo;
        g_split8(v, hi, lo);
        Bhi[ks] = __builtin_bit_cast(bf16x8_g, hi);
        Blo[ks] = __builtin_bit_cast(bf16x8_g, lo);
      }
    }
  }
  float* Af = reinterpret_cast<float*>(Aimg);  // EXACT: h_{s-1} [256 k][32 clips], swizzled
  const int u = tid % US;                      // gate-phase unit (768 % US == 0)
  const float br = bhh[dir * 768 + US * p + u];
  const float bz = bhh[dir * 768 + 256 + US * p + u];
  const float bn = bhh[dir * 768 + 512 + US * p + u];
  float* Xs = X + (int64_t)pair * 2 * 32 * 256;
  unsigned* C = &sync->cnt[pair][0];
  unsigned* Fl = &sync->flag[pair][0][0];

  int j = 0;
  for (int g = slot; g < ngroups; g += nslots, ++j) {
    const int c0 = g * 32;
    const int nc = min(32, B - c0);
    // VALU (exact, launches of at most GRU_VALU_CLIPS clips): the recurrent
    // product as VALU fma chains instead of MFMAs padded to 32 clips.
    // v_mfma_f32_32x32x2_f32 is bit for bit acc = fma(a1, b1, fma(a0, b0,
    // acc)) (measured over 16.7 M random elements incl. cancellation,
    // tools/mfma_f32_semantics.cpp), so the chain over k ascending gives the
    // MFMA kernel's bits: results do not depend on the batch size.  h_{s-1}
    // then lives as Hv[clip][k] (row stride GRU_HV_LD) in the A-image space.
    // Its hand-off is data-tagged (cdna_hip_programming.md Guideline 16 R2):
    // each h value travels as one 8-byte {tag = step + 1, value} granule
    // written by ONE sc1 store and swept with sc1 loads until the tag
    // matches, so the data is the flag: no drain, no flag store, no
    // separate poll, and placement-independent (granules zeroed every launch).
    unsigned long long* Gx =
        reinterpret_cast<unsigned long long*>(X) + (int64_t)pair * 2 * GRU_VALU_CLIPS * 256;
    float hreg[2] = {0.f, 0.f};   // VALU: this thread's h_{s-1} for its (clip, unit) pairs
    for (int s = 0; s < T; ++s) {
      const int gs = j * T + s;                // step of this pair; flags/counts are gs-based
      const int t = dir ? T - 1 - s : s;
      float gi[2][3];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int pr = tid + 768 * i;
        const int c = pr / US;
        if (pr < NPAIR && c < nc) {
          const float* gp = G + ((int64_t)(c0 + c) * T + t) * 1536 + dir * 768 + US * p + u;
          gi[i][0] = gp[0];
          gi[i][1] = gp[256];
          gi[i][2] = gp[512];
        } else {
          gi[i][0] = gi[i][1] = gi[i][2] = 0.f;
        }
      }
      // after a timed-out spin (s_err) no later wait is attempted: the
      // workgroup runs its remaining steps on NaN instead of timing out again
      // at every step
      if (tid == 0) gru_forced_fail(spin_limit, gs, sync, host_err, &s_err);
      if (!VALU && gs > 0) {
        if (fast) {
          if (tid < NS) {
            unsigned spins = 0;
            while (!gru_dead(&s_err) && g_ld(Fl + tid * 16) < (unsigned)gs) {
              if (++spins > spin_limit) {
                gru_fail(sync, host_err, 2u);
                s_err = 1;
                break;
              }
            }
          }
        } else if (tid == 0) {
          const unsigned target = (unsigned)NS * (unsigned)gs;
          unsigned spins = 0;
          while (!gru_dead(&s_err) && g_ld(C) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > spin_limit) {
              gru_fail(sync, host_err, 1u);
              s_err = 1;
              break;
            }
          }
        }
        __syncthreads();
      }
      GRU_STAMP(0);
      if (s == 0) {
        for (int i = tid; i < 16 * 32 * 4; i += 768) Aimg[i] = make_uint4(0, 0, 0, 0);
        for (int i = tid; i < 32 * 32; i += 768) hprev[i >> 5][i & 31] = 0.f;
      } else if constexpr (VALU) {
        // sweep: every granule loaded once, then re-polled until its tag == gs
        const unsigned long long* src = Gx + ((gs - 1) & 1) * GRU_VALU_CLIPS * 256;
        constexpr int NGR = (GRU_VALU_CLIPS * 256 + 767) / 768;
        unsigned long long w[NGR];
#pragma unroll
        for (int k = 0; k < NGR; ++k) {
          const int it = tid + 768 * k;
          w[k] = it < nc * 256 ? __hip_atomic_load(src + it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        }
#pragma unroll
        for (int k = 0; k < NGR; ++k) {
          const int it = tid + 768 * k;
          if (it < nc * 256) {
            unsigned spins = 0;
            while (!gru_dead(&s_err) && (unsigned)(w[k] >> 32) != (unsigned)gs) {
              if (++spins > spin_limit) {
                gru_fail(sync, host_err, 4u);
                s_err = 1;
                break;
              }
              w[k] = __hip_atomic_load(src + it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const int c = it >> 8, kk = it & 255;
            const float v = __uint_as_float((unsigned)w[k]);
            Af[c * GRU_HV_LD + kk] = v;
          }
        }
      } else {
        const float* src = Xs + ((gs - 1) & 1) * 32 * 256;
        // all of a thread's loads are issued before any is consumed (one L2
        // round trip per step, not one per item)
        float vv[2][8];
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          const int it = min(tid + 768 * k2, 32 * 32 - 1);
          // a partial group moves only its nc clips (nc/32 of the 32 KB; rows
          // of absent clips are zero and never read back); a full group keeps
          // the straight-line loads (nc is uniform: no divergence)
          if (nc == 32 || (it >> 5) < nc) {
            const unsigned long long* q =
                reinterpret_cast<const unsigned long long*>(src + (it >> 5) * 256 + 8 * (it & 31));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const unsigned long long w = __hip_atomic_load(q + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              vv[k2][2 * e] = __uint_as_float((uint32_t)w);
              vv[k2][2 * e + 1] = __uint_as_float((uint32_t)(w >> 32));
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) vv[k2][e] = 0.f;
          }
        }
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) {
          const int it = tid + 768 * k2;
          if (it >= 32 * 32) break;
          const int c = it >> 5, oct = it & 31;
          const float* v = vv[k2];
          if constexpr (VALU) {
            float4* hv = reinterpret_cast<float4*>(Af + c * GRU_HV_LD + 8 * oct);
            if (c < nc) {
              hv[0] = make_float4(v[0], v[1], v[2], v[3]);
              hv[1] = make_float4(v[4], v[5], v[6], v[7]);
            }
          } else if constexpr (EXACT) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const int k = 8 * oct + e;
              Af[k * 32 + (c ^ ((k >> 3) & 31))] = v[e];
            }
          } else {
            uint4 hi, lo;
            g_split8(v, hi, lo);
            const int ks = oct >> 1, hh = oct & 1, sw = (c >> 2) & 3;
            Aimg[(ks * 32 + c) * 4 + (hh ^ sw)] = hi;
            Aimg[(ks * 32 + c) * 4 + ((2 + hh) ^ sw)] = lo;
          }
          if (oct / (US / 8) == p) {   // the slice's own units: h_{s-1} for the gate phase
#pragma unroll
            for (int e = 0; e < 8; ++e) hprev[c][8 * (oct % (US / 8)) + e] = v[e];
          }
        }
      }
      __syncthreads();
      GRU_STAMP(1);
      f32x16_g acc, acc1;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      if constexpr (VALU) {
        // lane: gate row u = lane & 31 of gate nt, clips h, h + 2, ...
        for (int c = h; c < nc; c += 2) {
          const float4* hv = reinterpret_cast<const float4*>(Af + c * GRU_HV_LD + 64 * kq);
          float a0 = 0.f, a1 = 0.f;   // K eighths 2 kq and 2 kq + 1
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float4 x = hv[q], w = Wv[q], y = hv[q + 8], v = Wv[q + 8];
            a0 = fmaf(x.x, w.x, a0);
            a1 = fmaf(y.x, v.x, a1);
            a0 = fmaf(x.y, w.y, a0);
            a1 = fmaf(y.y, v.y, a1);
            a0 = fmaf(x.z, w.z, a0);
            a1 = fmaf(y.z, v.z, a1);
            a0 = fmaf(x.w, w.w, a0);
            a1 = fmaf(y.w, v.w, a1);
          }
          part[2 * kq][nt][c][lane & 31] = a0;
          part[2 * kq + 1][nt][c][lane & 31] = a1;
        }
      } else if constexpr (EXACT && NS == 16) {
        // four chains per wave — (eighth 2 kq + e, clip tile mt) — each over
        // its 32 k in ascending order, 4 k per v_mfma_f32_16x16x4_f32: the
        // fma chains of the 32x32x2 form, so the same bits
        const int cl = lane & 15, kk = lane >> 4;
        f32x4_g a4[2][2];
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) a4[e][mt][r] = 0.f;
#pragma unroll
        for (int st = 0; st < 8; ++st)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int k = 64 * kq + 32 * e + 4 * st + kk;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
              const float a = Af[k * 32 + ((16 * mt + cl) ^ ((k >> 3) & 31))];
              a4[e][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bf[8 * e + st], a4[e][mt], 0, 0, 0);
            }
          }
        // D row 4 (lane >> 4) + r = clip 16 mt + 4 kk + r, column = unit cl
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[2 * kq + e][nt][16 * mt + 4 * kk + r][cl] = a4[e][mt][r];
      } else if constexpr (EXACT) {
        const int c = lane & 31;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc1[r] = 0.f;
#pragma unroll
        for (int st = 0; st < 16; ++st) {   // two chains: K eighths 2 kq (acc), 2 kq + 1 (acc1)
          const int k = 64 * kq + 2 * st + h, k1 = k + 32;
          const float a = Af[k * 32 + (c ^ ((k >> 3) & 31))];
          const float a1 = Af[k1 * 32 + (c ^ ((k1 >> 3) & 31))];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Bf[st], acc, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, Bf[st + 16], acc1, 0, 0, 0);
        }
      } else {
        const int c = lane & 31, sw = (c >> 2) & 3;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int kk = 4 * kq + ks;
          const bf16x8_g ahi = __builtin_bit_cast(bf16x8_g, Aimg[(kk * 32 + c) * 4 + (h ^ sw)]);
          const bf16x8_g alo = __builtin_bit_cast(bf16x8_g, Aimg[(kk * 32 + c) * 4 + ((2 + h) ^ sw)]);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, Bhi[ks], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, Blo[ks], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo, Bhi[ks], acc, 0, 0, 0);
        }
      }
      if constexpr (EXACT && !VALU && NS == 8) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          part[2 * kq][nt][(r & 3) + 8 * (r >> 2) + 4 * h][lane & 31] = acc[r];
          part[2 * kq + 1][nt][(r & 3) + 8 * (r >> 2) + 4 * h][lane & 31] = acc1[r];
        }
      } else if constexpr (!EXACT) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          part[kq][nt][(r & 3) + 8 * (r >> 2) + 4 * h][lane & 31] = acc[r];
      }
      __syncthreads();
      GRU_STAMP(2);
      float* dst = Xs + (gs & 1) * 32 * 256;
      float hvs[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int pr = tid + 768 * i;
        hvs[i] = 0.f;
        if (pr < NPAIR) {
          const int c = pr / US;
          if (c < nc) {
            float ghr = part[0][0][c][u], ghz = part[0][1][c][u], ghn = part[0][2][c][u];
#pragma unroll
            for (int q = 1; q < KP; ++q) {   // partials in K order
              ghr += part[q][0][c][u];
              ghz += part[q][1][c][u];
              ghn += part[q][2][c][u];
            }
            ghr += br;
            ghz += bz;
            ghn += bn;
            const float hp = VALU ? hreg[i] : hprev[c][u];
            const float hn = gru_cell(gi[i][0], gi[i][1], gi[i][2], ghr, ghz, ghn, hp);
            hvs[i] = s_err ? __builtin_nanf("") : hn;   // NaN propagates to every slice
          }
          float* xp = dst + c * 256 + US * p + u;
          if (c >= nc) {
            // absent clip: nothing to publish
          } else if (VALU) {
            __hip_atomic_store(Gx + (gs & 1) * GRU_VALU_CLIPS * 256 + c * 256 + US * p + u,
                               ((unsigned long long)(gs + 1) << 32) | __float_as_uint(hvs[i]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
          } else if (fast) {
            *xp = hvs[i];
          } else {
            __hip_atomic_store(reinterpret_cast<unsigned*>(xp), __float_as_uint(hvs[i]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
      if constexpr (VALU) {
        // h_prev stays in this thread's registers (same (clip, unit) every
        // step), Hv and part are next written behind the post-sweep barrier:
        // no barrier and no drain here
        hreg[0] = hvs[0];
        hreg[1] = hvs[1];
      } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (fast)
          *reinterpret_cast<volatile unsigned*>(Fl + p * 16) = (unsigned)(gs + 1);
        else
          __hip_atomic_fetch_add(C, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      }
      GRU_STAMP(3);
      // the H output is not part of the hand-off: store it after the publish
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int pr = tid + 768 * i;
        const int c = pr / US;
        if (pr < NPAIR && c < nc)
          H[((int64_t)(c0 + c) * T + t) * 512 + dir * 256 + US * p + u] = hvs[i];
      }
    }
  }
#ifdef SEDX_GRU_STAMPS
  if (tid == 0 && pair == 0 && p == 0)
    for (int i = 0; i < 4; ++i) sync->stamps[i] = st_acc[i];
#endif
}

// ---------------------------------------------------------------------------
// Batched exact recurrence on 16-clip groups (launches of more than
// GRU_VALU_CLIPS clips), data-tagged hand-off straight into MFMA operands.
// Per (16-clip group, direction) NS workgroups ("slices") own U = 256 / NS
// hidden units = 3 U gate rows each.  Two roles per workgroup:
//   8 product waves, wave e = K eighth e (k = 32 e .. 32 e + 31), holding
//     W_hh[the slice's 3 U rows][its 32 k] as v_mfma_f32_16x16x4_f32 A
//     fragments.  Lane (q, n) needs h_{t-1}[clip n][k = 32 e + 4 s + q],
//     s = 0..7: exactly its B operands.  Every h value travels as one 8-byte
//     granule {tag = step + 1, value} written by ONE sc1 store; the lane polls
//     one of its granules with back-off until the tag matches, reads the
//     other seven and re-polls stragglers (cdna_hip_programming.md Guideline
//     16 R2: the data is the flag: no flag, fence or LDS image), then 3 RT
//     independent chains of 8 MFMAs -> LDS partials (double-buffered by step
//     parity);
//     The first U / 4 product waves also load the gate inputs x W_ih^T + b_ih
//     one step ahead and stage them in LDS next to the partials;
//   U / 4 gate waves, thread = (unit, clip): after the step's barrier the
//     eight partials summed in K order + b_hh, gru_cell, the new h published
//     as a granule (double-buffered by step parity) and stored to H.
// The roles matter because vmcnt counts stores and loads in one in-order
// queue: a wave that stored a granule (write-through) would wait for that
// store's completion before it could consume its next loads.  The product
// waves never store to global memory, the gate waves never load from it, and
// the step barrier is LDS-only (a __syncthreads() would drain the stores).
// Hazards: part[parity] of step s + 2 is written after the step s + 1
// barrier, which every gate wave reaches after its step-s reads; a slice
// publishes step gs only after each of its product waves saw gs - 1 from
// every slice of its K eighth, and every slice's gs - 1 granules only after
// all of gs - 2 was seen, so a parity buffer is never overwritten while
// read.  Group boundaries keep the sweep (values discarded) for the same
// reason.
// Arithmetic contract shared by every exact kernel of this file: per (gate
// row, clip) eight partials, each the in-order fma chain over its 32 k from
// 0 (v_mfma_f32_16x16x4_f32 is the in-order fma chain over its four k, and
// v_mfma_f32_32x32x2_f32 over its two: tools/mfma16_f32_semantics.cpp,
// tools/mfma_f32_semantics.cpp), summed p0 + p1 + ... + p7, then gru_cell:
// the outputs are bit-identical to the 32-clip MFMA and the small-batch VALU
// kernels.
constexpr int GRU_PLD = 17;        // partial rows (16 clips + pad)
template <int NS>
constexpr size_t gru_tag_lds() {   // partials [2][8][3][U][GRU_PLD], gate inputs [2][3][U][16]
  return (size_t)2 * 8 * 3 * (256 / NS) * GRU_PLD * 4 + (size_t)2 * 3 * (256 / NS) * 16 * 4;
}
template <int NS>
constexpr int gru_tag_threads() {
  return 64 * (8 + (256 / NS) / 4);
}
// LDS-only workgroup barrier (no vmcnt wait: global stores stay in flight)
__device__ __forceinline__ void gru_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NS>
__global__ __launch_bounds__(gru_tag_threads<NS>()) void gru_tag_kernel(
    const float* __restrict__ G, int B, int T, const float* __restrict__ whh, const float* __restrict__ bhh,
    float* __restrict__ H, unsigned long long* X, GruSync* sync, int nslots, unsigned* host_err,
    unsigned spin_limit) {
  constexpr int U = 256 / NS;          // hidden units per slice
  constexpr int RT = U / 16;           // 16-row tiles per gate
  constexpr int PB = 8 * 3 * U * GRU_PLD;   // floats per partial buffer
  static_assert(U % 16 == 0, "slice rows");
  extern __shared__ __attribute__((aligned(16))) float smem[];   // part[2][8 eighths][3 gates][U][GRU_PLD], gin[2][3][U][16]
  float* const gin = smem + 2 * PB;
  __shared__ int s_err;                          // a bounded spin timed out: outputs become NaN
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pair = blockIdx.x & 7;               // dispatch residue -> one XCD (observed; speed only)
  const int p = blockIdx.x >> 3;                 // slice 0..NS-1
  const int slot = pair >> 1, dir = pair & 1;
  if (slot >= nslots) return;                    // whole workgroup exits (uniform)
  const int ngroups = (B + 15) / 16;
  if (tid == 0) s_err = 0;
  unsigned long long* Xp = X + (int64_t)pair * 2 * 16 * 256;
  __syncthreads();

  if (wave < 8) {
    // ================= product wave: K eighth e =================
    const int e = wave, q = lane >> 4, n16 = lane & 15;
    // W_hh -> A fragments: A[m][kk] = W_hh[g 256 + U p + 16 rt + m][32 e + 4 s + kk], lane = (kk, m)
    float Wf[3][RT][8];
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const float* wrow = whh + ((int64_t)dir * 768 + g * 256 + U * p + 16 * rt + n16) * 256 + 32 * e + q;
#pragma unroll
        for (int st = 0; st < 8; ++st) Wf[g][rt][st] = wrow[4 * st];
      }
    // gate-input loader lanes: waves 0 .. U/4 - 1, lane = (unit, clip) as in the gate waves
    const bool gl = wave < U / 4;
    const int lu = (tid >> 4), lc = tid & 15;
    int j = 0;
    for (int grp = slot; grp < ngroups; grp += nslots, ++j) {
      const int c0 = grp * 16;
      const int nc = min(16, B - c0);
      auto load_gi = [&](int s_, float (&v)[3]) {
        const int t_ = dir ? T - 1 - s_ : s_;
        if (gl && lc < nc) {
          const float* gp = G + ((int64_t)(c0 + lc) * T + t_) * 1536 + dir * 768 + U * p + lu;
          v[0] = gp[0];
          v[1] = gp[256];
          v[2] = gp[512];
        } else {
          v[0] = v[1] = v[2] = 0.f;
        }
      };
      float gcur[3];
      load_gi(0, gcur);
      for (int s = 0; s < T; ++s) {
        const int gs = j * T + s;                // step of this pair; tags / parities are gs-based
        float gnext[3] = {0.f, 0.f, 0.f};
        if (s + 1 < T) load_gi(s + 1, gnext);    // in flight across this step's sweep and product
        float hb[8];
        if (tid == 0) gru_forced_fail(spin_limit, gs, sync, host_err, &s_err);
        if (gs > 0 && n16 < nc) {
          const unsigned long long* src = Xp + ((gs - 1) & 1) * 16 * 256 + n16 * 256 + 32 * e + q;
          unsigned long long w[8];
          // poll ONE granule with back-off, then read the other seven (a
          // slice writes all its granules within a few cycles) and re-poll
          // stragglers only: 8x fewer polling loads than sweeping them all
          unsigned spins = 0;
          w[0] = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          while ((unsigned)(w[0] >> 32) != (unsigned)gs && !gru_dead(&s_err)) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > spin_limit) {
              gru_fail(sync, host_err, 4u);
              s_err = 1;
              break;
            }
            w[0] = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
#pragma unroll
          for (int st = 1; st < 8; ++st)
            w[st] = __hip_atomic_load(src + 4 * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          for (;;) {
            bool ok = true;
#pragma unroll
            for (int st = 0; st < 8; ++st) ok &= (unsigned)(w[st] >> 32) == (unsigned)gs;
            if (ok || gru_dead(&s_err)) break;
            __builtin_amdgcn_s_sleep(1);
            if (++spins > spin_limit) {
              gru_fail(sync, host_err, 4u);
              s_err = 1;
              break;
            }
#pragma unroll
            for (int st = 0; st < 8; ++st)
              if ((unsigned)(w[st] >> 32) != (unsigned)gs)
                w[st] = __hip_atomic_load(src + 4 * st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
#pragma unroll
          for (int st = 0; st < 8; ++st) hb[st] = s > 0 ? __uint_as_float((unsigned)w[st]) : 0.f;
        } else {
#pragma unroll
          for (int st = 0; st < 8; ++st) hb[st] = 0.f;
        }
        f32x4_g acc[3][RT];
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) acc[g][rt] = f32x4_g{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 8; ++st)
#pragma unroll
          for (int g = 0; g < 3; ++g)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
              acc[g][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Wf[g][rt][st], hb[st], acc[g][rt], 0, 0, 0);
        // D[m][n]: lane (q, n) register i holds row 4 q + i
        float* pw = smem + (s & 1) * PB + e * 3 * U * GRU_PLD + (4 * q) * GRU_PLD + n16;
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 4; ++i) pw[(g * U + 16 * rt + i) * GRU_PLD] = acc[g][rt][i];
        if (gl) {
#pragma unroll
          for (int g = 0; g < 3; ++g) gin[(((s & 1) * 3 + g) * U + lu) * 16 + lc] = gcur[g];
        }
#pragma unroll
        for (int g = 0; g < 3; ++g) gcur[g] = gnext[g];
        gru_lds_barrier();
      }
    }
  } else {
    // ================= gate wave: thread = (unit gu, clip gc) =================
    const int gt = tid - 8 * 64;
    const int gu = gt >> 4, gc = gt & 15;
    const float br = bhh[dir * 768 + U * p + gu];
    const float bz = bhh[dir * 768 + 256 + U * p + gu];
    const float bn = bhh[dir * 768 + 512 + U * p + gu];
    int j = 0;
    for (int grp = slot; grp < ngroups; grp += nslots, ++j) {
      const int c0 = grp * 16;
      const int nc = min(16, B - c0);
      float hreg = 0.f;                          // h_{t-1} of this (clip, unit): own slice, same thread every step
      for (int s = 0; s < T; ++s) {
        const int gs = j * T + s;
        const int t = dir ? T - 1 - s : s;
        gru_lds_barrier();                       // the product waves' partials and gate inputs of step s
        float hv = 0.f;
        if (gc < nc) {
          const float* gq = gin + ((s & 1) * 3 * U + gu) * 16 + gc;
          const float gi0 = gq[0], gi1 = gq[U * 16], gi2 = gq[2 * U * 16];
          const float* pp = smem + (s & 1) * PB + gu * GRU_PLD + gc;
          constexpr int GS = U * GRU_PLD;        // gate stride; eighth stride 3 GS
          float ghr = pp[0], ghz = pp[GS], ghn = pp[2 * GS];
#pragma unroll
          for (int k8 = 1; k8 < 8; ++k8) {       // partials in K order
            ghr += pp[3 * GS * k8];
            ghz += pp[3 * GS * k8 + GS];
            ghn += pp[3 * GS * k8 + 2 * GS];
          }
          ghr += br;
          ghz += bz;
          ghn += bn;
          const float hn = gru_cell(gi0, gi1, gi2, ghr, ghz, ghn, hreg);
          hv = gru_dead(&s_err) ? __builtin_nanf("") : hn;   // NaN propagates to every slice
          __hip_atomic_store(Xp + (gs & 1) * 16 * 256 + gc * 256 + U * p + gu,
                             ((unsigned long long)(gs + 1) << 32) | __float_as_uint(hv), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          H[((int64_t)(c0 + gc) * T + t) * 512 + dir * 256 + U * p + gu] = hv;
        }
        hreg = hv;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K-split hand-off (round 4, launch variant 4): per (32-clip group,
// direction) 16 slices of 16 hidden units (48 gate rows); 8 waves, wave e =
// K eighth e = the hidden units of slices 2e and 2e + 1.  A wave waits for
// ITS two slices' flags only and loads their h(t-1) straight into its MFMA A
// fragments (v_mfma_f32_16x16x4_f32: lane (clip m, k-quarter kk) needs
// h[m][32 e + 4 st + kk], st = 0..7 — 8 consecutive floats in the K-permuted
// exchange layout below, two 16-byte sc1 loads per clip tile), so a wave
// whose slices published early starts its product while the others still
// wait: no LDS image of h, no gather barrier (variant 3 waits for all 16
// flags, gathers 32 KB into LDS, then multiplies).  Then the 8 eighth
// partials -> LDS, one barrier, the gate phase on (clip, unit) threads, sc1
// payload stores, vmcnt(0), barrier, the slice's flag (placement-independent:
// agent-scope stores and polls).  Exchange layout per (pair, parity):
// [clip 32][256] with unit u at 32 (u >> 5) + 8 (u & 3) + ((u >> 2) & 7).
// Arithmetic: each eighth the in-order fma chain over its 32 k (16x16x4 =
// the in-order chain over its 4 k), the 8 partials summed in K order, then
// gru_cell — the contract of every exact kernel here: bit-identical.
constexpr int GRU_KS_LD = 20;         // partial rows: 4 rows = 80 floats (16 mod 64 banks)
__device__ __forceinline__ int gru_kperm(int u) { return 32 * (u >> 5) + 8 * (u & 3) + ((u >> 2) & 7); }

__global__ __launch_bounds__(512) void gru_ksplit_kernel(const float* __restrict__ G, int B, int T,
                                                         const float* __restrict__ whh,
                                                         const float* __restrict__ bhh, float* __restrict__ H,
                                                         float* X, GruSync* sync, int nslots, unsigned* host_err,
                                                         unsigned spin_limit) {
  __shared__ float part[8][3][32][GRU_KS_LD];  // [eighth][gate][clip][unit]
  __shared__ int s_err;
  const int tid = threadIdx.x, lane = tid & 63;
  const int e = __builtin_amdgcn_readfirstlane(tid >> 6);   // K eighth of this wave
  const int pair = blockIdx.x & 7;             // dispatch residue -> one XCD (speed only)
  const int p = blockIdx.x >> 3;               // slice 0..15
  const int slot = pair >> 1, dir = pair & 1;
  if (slot >= nslots) return;                  // whole workgroup exits (uniform)
  if (tid == 0) s_err = 0;
  __syncthreads();
  const int ngroups = (B + 31) / 32;
  const int n16 = lane & 15, kk = lane >> 4;
  // W_hh B fragments: B[k][n] = W_hh[gate g row 16 p + n][32 e + 4 st + kk]
  float Wf[3][8];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int st = 0; st < 8; ++st)
      Wf[g][st] = whh[((int64_t)dir * 768 + g * 256 + 16 * p + n16) * 256 + 32 * e + 4 * st + kk];
  // gate-phase thread: (clip gc, unit gu of the slice)
  const int gc = tid >> 4, gu = tid & 15;
  const int uo = 16 * p + gu;
  const float br = bhh[dir * 768 + uo], bz = bhh[dir * 768 + 256 + uo], bn = bhh[dir * 768 + 512 + uo];
  const int upos = gru_kperm(uo);
  float* const Xs = X + (int64_t)pair * 2 * 32 * 256;
  unsigned* const Fl = &sync->flag[pair][0][0];
#ifdef SEDX_GRU_STAMPS
  unsigned long long st_acc[4] = {0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
#define GRU_KSTAMP(i)                                                                   \
  if (tid == 0 && pair == 0 && p == 0) {                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
    st_acc[i] += now_ - st_last;                                                        \
    st_last = now_;                                                                     \
  }
#else
#define GRU_KSTAMP(i)
#endif
  int j = 0;
  for (int grp = slot; grp < ngroups; grp += nslots, ++j) {
    const int c0 = grp * 32;
    const int nc = min(32, B - c0);
    auto load_gi = [&](int s_, float (&v)[3]) {
      const int t_ = dir ? T - 1 - s_ : s_;
      if (gc < nc) {
        const float* gp = G + ((int64_t)(c0 + gc) * T + t_) * 1536 + dir * 768 + uo;
        v[0] = gp[0];
        v[1] = gp[256];
        v[2] = gp[512];
      } else {
        v[0] = v[1] = v[2] = 0.f;
      }
    };
    float gcur[3];
    load_gi(0, gcur);
    float hreg = 0.f;                          // this thread's h(t-1): same (clip, unit) every step
    for (int s = 0; s < T; ++s) {
      const int gs = j * T + s;                // step of this pair; flags / parities are gs-based
      const int t = dir ? T - 1 - s : s;
      float gnext[3] = {0.f, 0.f, 0.f};
      if (s + 1 < T) load_gi(s + 1, gnext);    // in flight across the wait and the product
      // ---- product wave e: wait for slices 2e, 2e + 1 (step gs - 1).  At a
      // group boundary the wait still runs (values discarded): a slice
      // publishes step gs only after every slice finished reading gs - 2 ----
      if (tid == 0) gru_forced_fail(spin_limit, gs, sync, host_err, &s_err);
      if (gs > 0 && lane < 2) {
        unsigned spins = 0;
        while (!gru_dead(&s_err) && g_ld(Fl + (2 * e + lane) * 16) < (unsigned)gs) {
          if (++spins > spin_limit) {
            gru_fail(sync, host_err, 2u);
            s_err = 1;
            break;
          }
        }
      }
      GRU_KSTAMP(0);
      float a[2][8];
      if (s > 0) {
        const float* src = Xs + ((gs - 1) & 1) * 32 * 256 + 32 * e + 8 * kk;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int c = 16 * mt + n16;
          if (c < nc) {
            const unsigned long long* q = reinterpret_cast<const unsigned long long*>(src + c * 256);
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              const unsigned long long v = __hip_atomic_load(q + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              a[mt][2 * w] = __uint_as_float((uint32_t)v);
              a[mt][2 * w + 1] = __uint_as_float((uint32_t)(v >> 32));
            }
          } else {
#pragma unroll
            for (int st = 0; st < 8; ++st) a[mt][st] = 0.f;
          }
        }
      } else {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int st = 0; st < 8; ++st) a[mt][st] = 0.f;
      }
      GRU_KSTAMP(1);
      f32x4_g acc[3][2];
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[g][mt] = f32x4_g{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 8; ++st)
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
            acc[g][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt][st], Wf[g][st], acc[g][mt], 0, 0, 0);
      // D[clip][unit]: lane (unit n16, kk) register i = clip 16 mt + 4 kk + i
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int i = 0; i < 4; ++i) part[e][g][16 * mt + 4 * kk + i][n16] = acc[g][mt][i];
      __syncthreads();
      GRU_KSTAMP(2);
      // ---- gate phase: thread (gc, gu) ----
      float hv = 0.f;
      if (gc < nc) {
        float ghr = part[0][0][gc][gu], ghz = part[0][1][gc][gu], ghn = part[0][2][gc][gu];
#pragma unroll
        for (int q = 1; q < 8; ++q) {          // partials in K order
          ghr += part[q][0][gc][gu];
          ghz += part[q][1][gc][gu];
          ghn += part[q][2][gc][gu];
        }
        ghr += br;
        ghz += bz;
        ghn += bn;
        const float hn = gru_cell(gcur[0], gcur[1], gcur[2], ghr, ghz, ghn, hreg);
        hv = gru_dead(&s_err) ? __builtin_nanf("") : hn;   // NaN propagates to every slice
        __hip_atomic_store(reinterpret_cast<unsigned*>(Xs + (gs & 1) * 32 * 256 + gc * 256 + upos),
                           __float_as_uint(hv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      hreg = hv;
      // every storing wave drains its payload stores, then one flag per slice;
      // the barrier also orders this step's partial reads before the next
      // step's partial writes
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(Fl + p * 16, (unsigned)(gs + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      GRU_KSTAMP(3);
      // the H output is not part of the hand-off: stored after the flag
      if (gc < nc) H[((int64_t)(c0 + gc) * T + t) * 512 + dir * 256 + uo] = hv;
#pragma unroll
      for (int g = 0; g < 3; ++g) gcur[g] = gnext[g];
    }
  }
#ifdef SEDX_GRU_STAMPS
  if (tid == 0 && pair == 0 && p == 0)
    for (int i = 0; i < 4; ++i) sync->stamps[i] = st_acc[i];
#endif
#undef GRU_KSTAMP
}

// ---------------------------------------------------------------------------
// Two interleaved 16-clip recurrences per workgroup (round 5, launch variant
// 5): the K-split structure above (16 slices of 16 hidden units per 32-clip
// group and direction; 8 waves = the 8 K eighths, each waiting only for the
// flags of its two slices and loading their h(t-1) straight into its
// v_mfma_f32_16x16x4_f32 A fragments) with the group's two halves (clips
// 0-15, 16-31) as two recurrences stepped alternately: phase (half X, step s)
// multiplies X's h(s-1) (loaded during the previous phase), then — while its
// partials are summed and its gates run — polls the flags of the other half
// Y's step that just finished and issues Y's loads, so Y's hand-off (flag
// propagation and the L2 round trip) hides behind X's product and gates
// instead of stalling the workgroup.  Per phase: 24 MFMAs per wave, one
// LDS barrier for the partials, the gate phase on (clip, unit) threads,
// payload stores, vmcnt(0), barrier, the slice's per-half flag.
// Exchange: the K-split layout, half h in rows 16 h .. 16 h + 15 of each
// parity's [32][256]; flags Fl[slice * 16 + 8 h].  Hazards as in the K-split
// kernel, per half: a slice publishes X(s + 2) only after its waves saw
// X(s + 1) from every slice, each of which read X(s) before publishing
// X(s + 1).  Arithmetic: the same per-eighth fma chains, partials summed in K
// order, gru_cell — bit-identical to every exact kernel here.
__global__ __launch_bounds__(512) void gru_pair_kernel(const float* __restrict__ G, int B, int T,
                                                       const float* __restrict__ whh, const float* __restrict__ bhh,
                                                       float* __restrict__ H, float* X, GruSync* sync, int nslots,
                                                       unsigned* host_err, unsigned spin_limit, int spread) {
  __shared__ float part[8][3][16][GRU_KS_LD];  // [eighth][gate][clip][unit]
  __shared__ int s_err;
  const int tid = threadIdx.x, lane = tid & 63;
  const int e = __builtin_amdgcn_readfirstlane(tid >> 6);   // K eighth of this wave
  const int pair = spread ? (int)blockIdx.x / 16 : (int)(blockIdx.x & 7);
  const int p = spread ? (int)blockIdx.x % 16 : (int)(blockIdx.x >> 3);   // slice 0..15
  const int slot = pair >> 1, dir = pair & 1;
  if (slot >= nslots) return;                  // whole workgroup exits (uniform)
  if (tid == 0) s_err = 0;
  __syncthreads();
  const int ngroups = (B + 31) / 32;
  const int n16 = lane & 15, kk = lane >> 4;
  float Wf[3][8];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int st = 0; st < 8; ++st)
      Wf[g][st] = whh[((int64_t)dir * 768 + g * 256 + 16 * p + n16) * 256 + 32 * e + 4 * st + kk];
  // gate-phase thread (threads 0..255): (clip gc of the half, unit gu of the slice)
  const bool gt = tid < 256;
  const int gc = (tid >> 4) & 15, gu = tid & 15;
  const int uo = 16 * p + gu;
  const float br = bhh[dir * 768 + uo], bz = bhh[dir * 768 + 256 + uo], bn = bhh[dir * 768 + 512 + uo];
  const int upos = gru_kperm(uo);
  float* const Xs = X + (int64_t)pair * 2 * 32 * 256;
  unsigned* const Fl = &sync->flag[pair][0][0];
#ifdef SEDX_GRU_STAMPS
  // [0] product  [1] next phase's flag wait + load issue  [2] gates  [3] drain + flag
  unsigned long long st_acc[4] = {0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
#define GRU_PSTAMP(i)                                                                   \
  if (tid == 0 && pair == 0 && p == 0) {                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                       \
    st_acc[i] += now_ - st_last;                                                        \
    st_last = now_;                                                                     \
  }
#else
#define GRU_PSTAMP(i)
#endif
  int j = 0;
  for (int grp = slot; grp < ngroups; grp += nslots, ++j) {
    const int c0 = grp * 32;
    const int nc = min(32, B - c0);
    // gate inputs of (half h, step s_) for this thread
    auto load_gi = [&](int h, int s_, float (&v)[3]) {
      const int t_ = dir ? T - 1 - s_ : s_;
      const int c = 16 * h + gc;
      if (gt && c < nc) {
        const float* gp = G + ((int64_t)(c0 + c) * T + t_) * 1536 + dir * 768 + uo;
        v[0] = gp[0];
        v[1] = gp[256];
        v[2] = gp[512];
      } else {
        v[0] = v[1] = v[2] = 0.f;
      }
    };
    // wait for half h's step gs_ - 1 from this wave's two slices, then load
    // its 8 k of h(gs_ - 1) for every clip of the half (zeros at gs_ == j T)
    auto fetch = [&](int h, int gs_, bool first, float (&a)[8]) {
      if (!first && lane < 2) {
        unsigned spins = 0;
        while (!gru_dead(&s_err) && g_ld(Fl + (2 * e + lane) * 16 + 8 * h) < (unsigned)gs_) {
          if (++spins > spin_limit) {
            gru_fail(sync, host_err, 2u);
            s_err = 1;
            break;
          }
        }
      }
      const int c = 16 * h + n16;
      if (!first && c < nc) {
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(
            Xs + ((gs_ - 1) & 1) * 32 * 256 + c * 256 + 32 * e + 8 * kk);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const unsigned long long v = __hip_atomic_load(q + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          a[2 * w] = __uint_as_float((uint32_t)v);
          a[2 * w + 1] = __uint_as_float((uint32_t)(v >> 32));
        }
      } else {
#pragma unroll
        for (int st = 0; st < 8; ++st) a[st] = 0.f;
      }
    };
    float hreg0 = 0.f, hreg1 = 0.f;           // this thread's h(t-1), halves 0 / 1
    float acur[8], anext[8], gcur[3], gnext[3];
    const int gs0 = j * T;
    fetch(0, gs0, true, acur);
    load_gi(0, 0, gcur);
    // phase (half H, step s); order (0, 0), (1, 0), (0, 1), (1, 1), ...
    auto phase = [&](auto h_tag, int s) {
      constexpr int h = decltype(h_tag)::value;
      const int gs = gs0 + s;
      const int t = dir ? T - 1 - s : s;
      if (tid == 0) gru_forced_fail(spin_limit, gs, sync, host_err, &s_err);
      f32x4_g acc[3];
#pragma unroll
      for (int g = 0; g < 3; ++g) acc[g] = f32x4_g{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 8; ++st)
#pragma unroll
        for (int g = 0; g < 3; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(acur[st], Wf[g][st], acc[g], 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) part[e][g][4 * kk + i][n16] = acc[g][i];
      GRU_PSTAMP(0);
      // the next phase's operands: half h ^ 1 at step s + h (its flags were
      // set a phase ago), and its gate inputs
      constexpr int nh = h ^ 1;
      const int ns = s + h;
      const bool more = ns < T;
      if (more) {
        fetch(nh, gs0 + ns, ns == 0, anext);
        load_gi(nh, ns, gnext);
      }
      GRU_PSTAMP(1);
      gru_lds_barrier();                       // partials written (payload stores stay in flight)
      float hv = 0.f;
      const int c = 16 * h + gc;
      if (gt && c < nc) {
        float ghr = part[0][0][gc][gu], ghz = part[0][1][gc][gu], ghn = part[0][2][gc][gu];
#pragma unroll
        for (int q = 1; q < 8; ++q) {          // partials in K order
          ghr += part[q][0][gc][gu];
          ghz += part[q][1][gc][gu];
          ghn += part[q][2][gc][gu];
        }
        ghr += br;
        ghz += bz;
        ghn += bn;
        const float hn = gru_cell(gcur[0], gcur[1], gcur[2], ghr, ghz, ghn, h ? hreg1 : hreg0);
        hv = gru_dead(&s_err) ? __builtin_nanf("") : hn;   // NaN propagates to every slice
        __hip_atomic_store(reinterpret_cast<unsigned*>(Xs + (gs & 1) * 32 * 256 + c * 256 + upos),
                           __float_as_uint(hv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (h) hreg1 = hv;
      else hreg0 = hv;
      GRU_PSTAMP(2);
      // payload stores (and the next phase's loads) drained, partial reads
      // done, then the slice's flag for half h
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(Fl + p * 16 + 8 * h, (unsigned)(gs + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      GRU_PSTAMP(3);
      if (gt && c < nc) H[((int64_t)(c0 + c) * T + t) * 512 + dir * 256 + uo] = hv;
      if (more) {
#pragma unroll
        for (int st = 0; st < 8; ++st) acur[st] = anext[st];
#pragma unroll
        for (int g = 0; g < 3; ++g) gcur[g] = gnext[g];
      }
    };
    for (int s = 0; s < T; ++s) {
      phase(std::integral_constant<int, 0>{}, s);
      phase(std::integral_constant<int, 1>{}, s);
    }
  }
#ifdef SEDX_GRU_STAMPS
  if (tid == 0 && pair == 0 && p == 0)
    for (int i = 0; i < 4; ++i) sync->stamps[i] = st_acc[i];
#endif
#undef GRU_PSTAMP
}

size_t gru_coop_workspace_bytes(int B) {
  (void)B;
  // sync block, then the exchange space: 32-clip kernel 8 pairs x 2 parities
  // x 32 x 256 floats; tagged kernel 8 pairs x 2 parities x 16 x 256 granules
  // (the same 512 KB)
  static_assert((size_t)8 * 2 * 16 * 256 * 8 == (size_t)8 * 2 * 32 * 256 * 4, "exchange space");
  return ((sizeof(GruSync) + 255) & ~size_t(255)) + (size_t)8 * 2 * 32 * 256 * 4;
}

template <int NS>
static void launch_gru_tag(const float* G, int B, int T, const float* whh, const float* bhh, float* H, GruSync* sync,
                           unsigned long long* X, size_t sync_bytes, unsigned* host_err, unsigned spin,
                           hipStream_t s) {
  const int ngroups = (B + 15) / 16;
  const int nslots = ngroups < GRU_MAX_SLOTS ? ngroups : GRU_MAX_SLOTS;
  const LaunchInfo li =
      launch_info(reinterpret_cast<const void*>(gru_tag_kernel<NS>), gru_tag_threads<NS>(), gru_tag_lds<NS>());
  if (!li.ok) return;
  // sync block + the granules of the pairs in use (every tag 0)
  (void)hipMemsetAsync(sync, 0, sync_bytes + (size_t)2 * nslots * 2 * 16 * 256 * 8, s);
  hipLaunchKernelGGL(gru_tag_kernel<NS>, dim3(8 * NS), dim3(gru_tag_threads<NS>()), li.dyn, s, G, B, T, whh, bhh, H, X, sync, nslots,
                     host_err, spin);
}

void launch_gru_coop(const float* G, int B, int T, const float* whh, const float* bhh, float* H,
                     void* ws, bool exact, bool allow_fast, int variant, unsigned* host_err, unsigned spin,
                     hipStream_t s, bool spread) {
  const int sp = spread ? 1 : 0;
  if (spread) allow_fast = false;
  GruSync* sync = static_cast<GruSync*>(ws);
  const size_t sync_bytes = (sizeof(GruSync) + 255) & ~size_t(255);
  float* X = reinterpret_cast<float*>(static_cast<char*>(ws) + sync_bytes);
  const bool valu = exact && B <= GRU_VALU_CLIPS;
  if (exact && !valu && variant == 4) {   // K-split hand-off, 16 slices
    const int ngroups = (B + 31) / 32;
    const int nslots = ngroups < GRU_MAX_SLOTS ? ngroups : GRU_MAX_SLOTS;
    (void)hipMemsetAsync(sync, 0, sync_bytes, s);
    launch_kernel(gru_ksplit_kernel, dim3(128), 512, s, G, B, T, whh, bhh, H, X, sync, nslots, host_err, spin);
    return;
  }
  if (exact && !valu && variant == 5) {   // two interleaved 16-clip recurrences, 16 slices
    const int ngroups = (B + 31) / 32;
    const int nslots = ngroups < GRU_MAX_SLOTS ? ngroups : GRU_MAX_SLOTS;
    (void)hipMemsetAsync(sync, 0, sync_bytes, s);
    launch_kernel(gru_pair_kernel, dim3(128), 512, s, G, B, T, whh, bhh, H, X, sync, nslots, host_err, spin, sp);
    return;
  }
  if (exact && !valu && variant != 2 && variant != 3) {
    auto* Xg = reinterpret_cast<unsigned long long*>(X);
    if (variant == 1)
      launch_gru_tag<8>(G, B, T, whh, bhh, H, sync, Xg, sync_bytes, host_err, spin, s);
    else
      launch_gru_tag<16>(G, B, T, whh, bhh, H, sync, Xg, sync_bytes, host_err, spin, s);
    return;
  }
  const int ngroups = (B + 31) / 32;
  const int nslots = ngroups < GRU_MAX_SLOTS ? ngroups : GRU_MAX_SLOTS;
  // one fill launch: the sync block rounded to 256 B (the exchange buffers
  // start there) and, for the tagged hand-off, its granules (every tag 0)
  (void)hipMemsetAsync(sync, 0, sync_bytes + (valu ? (size_t)2 * 2 * GRU_VALU_CLIPS * 256 * 8 : 0), s);
  if (valu)
    launch_kernel(gru_coop_kernel<true, true>, dim3(64), 768, s, G, B, T, whh, bhh, H, X, sync, nslots,
                  allow_fast ? 1 : 0, host_err, spin, sp);
  else if (exact && variant == 3)   // 16 slices per (group, direction)
    launch_kernel(gru_coop_kernel<true, false, 16>, dim3(128), 768, s, G, B, T, whh, bhh, H, X, sync, nslots,
                  allow_fast ? 1 : 0, host_err, spin, sp);
  else if (exact)
    launch_kernel(gru_coop_kernel<true, false>, dim3(64), 768, s, G, B, T, whh, bhh, H, X, sync, nslots,
                  allow_fast ? 1 : 0, host_err, spin, sp);
  else
    launch_kernel(gru_coop_kernel<false, false>, dim3(64), 768, s, G, B, T, whh, bhh, H, X, sync, nslots,
                  allow_fast ? 1 : 0, host_err, spin, sp);
}

}  // namespace sedx
