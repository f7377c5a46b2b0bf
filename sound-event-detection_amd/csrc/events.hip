// On-GPU thresholding into events.
//
//  mode 0  activity_detection (utils/vad.py:11-45) per (clip, class) series,
//          as driven by frame_prediction_to_event_prediction_v2
//          (pytorch/predict.py:57-121 == utils/utilities.py:155-214);
//  mode 1  activity_detection_binary (utils/vad.py:47-106) on merged window
//          votes, as driven by frame_binary_prediction_to_event_prediction
//          (utils/utilities.py:216-276) in inference_prob_vote
//          (pytorch/main_strong.py:885-1122).
//
// The reference builds python lists stage by stage: locts -> find_bgn_fin_pairs
// -> (second threshold -> smooth(1)) -> smooth(n_smooth) -> remove_salt_noise.
// Every stage is an in-order streaming transform of a pair sequence, so one
// thread per series runs the whole chain in a single pass over its frames with
// O(1) state per stage (a pending run for the find_bgn_fin_pairs quirk, a
// (mem_bgn, pre_fin) pair per smoother).  Quirks kept bit-for-bit:
//   * every non-first run begins at locts+1, every non-last run ends at
//     last+1, the last run ends at locts[-1] (vad.py:115-121);
//   * the second threshold walks x[bgn] / x[fin] from those quirky indices;
//     a non-first run whose bgn is T (a run starting at the last frame) is the
//     reference's IndexError -> reported in info[1];
//   * smooth() keeps the FIRST bgn of a merged group and the LAST pair's fin;
//   * mode 0 compares in float32 (numpy compares a float32 row with a python
//     float threshold in float32); mode 1's x are float64 vote counts in the
//     reference (exact small integers here) compared in float64;
//   * mode 1 locts come from 100*overlap-frame blocks i in
//     range(0, T - step, step) (the last block is never scanned) with
//     x >= num_overlaps(i), the avg_merge schedule (vad.py:62-85).
// Output order = (clip, class, time), the reference's event_list order:
// per-series slots, then one exclusive scan + copy (2 launches).
//
// One wavefront per series.  Pass 1 turns the series into two bitmaps, 64
// frames per ballot: on(t) (the locts test) and below(t) (x < low, the stop
// test of the second-threshold walks), kept in LDS.  Pass 2 is wave-uniform
// scalar code over runs of the on-bitmap (ctz over words) — the cost scales
// with the number of runs, not frames — and the walks are bit scans over the
// below-bitmap.  The streaming state machine of the reference's list stages
// is unchanged.
#include <algorithm>

#include "sedx_internal.h"

namespace sedx {

namespace {

// Streaming state of one series: the find_bgn_fin_pairs run tracker and the
// two smoothers (utils/vad.py:158-183).  Resumable across frame chunks.
struct SeriesState {
  bool ok, in_run, pending, first, s1_any, s2_any;
  int64_t rs, re, pb, pe, s1_mem, s1_pre, s2_mem, s2_pre;
};

__device__ __forceinline__ void series_init(SeriesState& st) {
  st.ok = true;
  st.in_run = st.pending = st.s1_any = st.s2_any = false;
  st.first = true;
  st.rs = st.re = st.pb = st.pe = st.s1_mem = st.s1_pre = st.s2_mem = st.s2_pre = 0;
}

template <typename Emit>
__device__ __forceinline__ void final_out(int64_t b, int64_t f, int64_t n_salt, Emit& emit) {
  if (f - b <= n_salt) return;                     // remove_salt_noise vad.py:186-199
  emit(b, f);
}

template <typename Emit>                           // smooth(n_smooth)
__device__ __forceinline__ void push2(SeriesState& st, int64_t b, int64_t f, int64_t n_smooth,
                                      int64_t n_salt, Emit& emit) {
  if (!st.s2_any) {
    st.s2_any = true;
    st.s2_mem = b;
  } else if (!(b - st.s2_pre <= n_smooth)) {
    final_out(st.s2_mem, st.s2_pre, n_salt, emit);
    st.s2_mem = b;
  }
  st.s2_pre = f;
}

template <typename Emit>                           // smooth(n_smooth=1) of the 2nd threshold
__device__ __forceinline__ void push1(SeriesState& st, int64_t b, int64_t f, int64_t n_smooth,
                                      int64_t n_salt, Emit& emit) {
  if (!st.s1_any) {
    st.s1_any = true;
    st.s1_mem = b;
  } else if (!(b - st.s1_pre <= 1)) {
    push2(st, st.s1_mem, st.s1_pre, n_smooth, n_salt, emit);
    st.s1_mem = b;
  }
  st.s1_pre = f;
}

constexpr int EV_WAVES = 4;                 // wavefronts per workgroup (at most)
constexpr int64_t EV_LDS_BYTES = 160 * 1024;
constexpr int64_t EV_MAX_WORDS = EV_LDS_BYTES / 16;   // bitmap words per series (T <= 655,360)

__device__ __forceinline__ uint64_t ev_uniform(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// below-bitmap scans: last set bit <= b (or -1), first set bit >= f (or T)
struct BelowMask {
  const uint64_t* m;
  int64_t W, T;
  __device__ int64_t prev_set(int64_t b) const {
    int64_t w = b >> 6;
    uint64_t bits = ev_uniform(m[w]) & (~0ull >> (63 - (b & 63)));
    while (true) {
      if (bits) return w * 64 + 63 - __builtin_clzll(bits);
      if (--w < 0) return -1;
      bits = ev_uniform(m[w]);
    }
  }
  __device__ int64_t next_set(int64_t f) const {
    int64_t w = f >> 6;
    if (w >= W) return T;
    uint64_t bits = ev_uniform(m[w]) & (~0ull << (f & 63));
    while (true) {
      if (bits) return w * 64 + __builtin_ctzll(bits);
      if (++w >= W) return T;
      bits = ev_uniform(m[w]);
    }
  }
};

template <typename Emit>
__device__ __forceinline__ void push_pair_m(SeriesState& st, const BelowMask& bm, int64_t T, int64_t b,
                                            int64_t f, bool use_lo, int64_t n_smooth, int64_t n_salt,
                                            Emit& emit) {
  if (!use_lo) {
    push2(st, b, f, n_smooth, n_salt, emit);
    return;
  }
  // activity_detection_with_second_thres vad.py:139-151: walk left from b
  // while x >= low (x[b] read first: b == T is the reference's IndexError),
  // right from f until x < low or T
  if (b >= T || f > T) {
    st.ok = false;
    return;
  }
  b = bm.prev_set(b);
  if (f < T) f = bm.next_set(f);
  push1(st, b + 1, f, n_smooth, n_salt, emit);
}

// dynamic LDS: [wpb][2][W] words (on, below); wpb series per workgroup
template <int MODE>
__global__ __launch_bounds__(64 * EV_WAVES) void events_series_kernel(EventArgs a, int64_t W, int wpb) {
  extern __shared__ uint64_t ev_lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t C = a.C, T = a.T;
  const int64_t sid = (int64_t)blockIdx.x * wpb + wave;
  if (wave >= wpb || sid >= a.N * C) return;        // wave-uniform
  const int64_t n = sid / C, k = sid - n * C;
  uint64_t* om = ev_lds + (int64_t)wave * 2 * W;
  uint64_t* lm = om + W;
  const float* xs = a.x + n * T * C + k;
  const float hi = a.hi[k];
  const double lo = a.lo[k];
  const float lo_f = (float)lo;
  const bool use_lo = a.use_lo != 0;
  // mode 1: scan limit and per-block vote requirement (vad.py:62-78)
  const int64_t step = a.step, sd = a.sd, interval = sd * 100 - step;
  // (step < 0: range(0, T - step, step) is empty, no candidate frame)
  const int64_t lim = MODE == 0 ? T : ((step > 0 && T - step > 0) ? ((T - step + step - 1) / step) * step : 0);

  // pass 1: bitmaps, 8 words (512 frames) of loads in flight per lane
  for (int64_t w0 = 0; w0 < W; w0 += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t t = (w0 + j) * 64 + lane;
      v[j] = t < T ? xs[t * C] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (w0 + j >= W) break;
      const int64_t t = (w0 + j) * 64 + lane;
      bool on;
      if (MODE == 0) {
        on = t < T && v[j] > hi;                    // float32 compare (numpy f32 row vs python float)
      } else {
        const int64_t st = step > 0 ? step : 1;
        const int64_t i = (t / st) * st;
        const int64_t nov = i < interval ? i / st + 1 : (i >= T - interval ? (T - i) / st + 1 : sd);
        on = t < lim && (double)v[j] >= (double)nov;
      }
      const bool below = t < T && (MODE == 0 ? (v[j] < lo_f) : ((double)v[j] < lo));
      const uint64_t bon = __ballot(on), bbe = __ballot(below);
      if (lane == 0) {
        om[w0 + j] = bon;
        lm[w0 + j] = bbe;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // pass 2: runs of the on-bitmap through the reference's list stages
  const int64_t ns = a.n_smooth[k], nsalt = a.n_salt[k];
  int2* slot = reinterpret_cast<int2*>(a.slots) + sid * a.slot_cap;
  int64_t cnt = 0;
  auto emit = [&](int64_t b, int64_t f) {
    if (lane == 0 && cnt < a.slot_cap) slot[cnt] = make_int2((int)b, (int)f);
    ++cnt;
  };
  const BelowMask bm{lm, W, T};
  SeriesState st;
  series_init(st);
  int64_t w = 0;
  uint64_t cur = W > 0 ? ev_uniform(om[0]) : 0;     // on-bits of word w not yet consumed
  while (st.ok) {
    while (!cur && ++w < W) cur = ev_uniform(om[w]);
    if (!cur) break;
    const int64_t rs = w * 64 + __builtin_ctzll(cur);
    // run end: first off bit after rs
    uint64_t off = ~ev_uniform(om[w]) & (~0ull << (rs & 63));
    int64_t we = w;
    while (!off && ++we < W) off = ~ev_uniform(om[we]);
    const int64_t re1 = off ? we * 64 + __builtin_ctzll(off) : W * 64;   // one past the run
    const int64_t re = (re1 < T ? re1 : T) - 1;
    // find_bgn_fin_pairs vad.py:115-121: a completed run is held until the
    // next one shows it was not the last
    if (st.pending) push_pair_m(st, bm, T, st.pb, st.pe + 1, use_lo, ns, nsalt, emit);
    st.pb = st.first ? rs : rs + 1;
    st.pe = re;
    st.pending = true;
    st.first = false;
    if (re1 >= W * 64) break;
    w = re1 >> 6;
    cur = ev_uniform(om[w]) & (~0ull << (re1 & 63));
  }
  if (st.ok && st.pending) push_pair_m(st, bm, T, st.pb, st.pe, use_lo, ns, nsalt, emit);  // fin = locts[-1]
  if (st.ok && use_lo && st.s1_any) push2(st, st.s1_mem, st.s1_pre, ns, nsalt, emit);
  if (st.ok && st.s2_any) final_out(st.s2_mem, st.s2_pre, nsalt, emit);
  if (lane == 0) {
    a.counts[sid] = st.ok ? cnt : 0;
    if (!st.ok) atomicOr(reinterpret_cast<unsigned long long*>(a.info + 1), 1ull);
  }
}

// exclusive scan of the per-series counts + copy of the slots into the
// (clip, class, time)-ordered output (one workgroup; clips x classes is small)
__global__ __launch_bounds__(1024) void events_compact_kernel(EventArgs a) {
  __shared__ int64_t part[1024];
  __shared__ int64_t carry;
  const int tid = threadIdx.x;
  const int64_t n = a.N * a.C;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 1024) {
    const int64_t i = base + tid;
    const int64_t v = i < n ? a.counts[i] : 0;
    part[tid] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {      // Hillis-Steele inclusive scan
      const int64_t add = tid >= off ? part[tid - off] : 0;
      __syncthreads();
      part[tid] += add;
      __syncthreads();
    }
    if (i < n) {
      const int64_t o = carry + part[tid] - v;
      const int2* slot = reinterpret_cast<const int2*>(a.slots) + i * a.slot_cap;
      const int cls = (int)(i % a.C), clip = (int)(i / a.C);
      for (int64_t e = 0; e < v && o + e < a.capacity; ++e) {
        const int2 bf = slot[e];
        *reinterpret_cast<int4*>(a.events + 4 * (o + e)) = make_int4(clip, cls, bf.x, bf.y);
      }
    }
    __syncthreads();
    if (tid == 1023) carry += part[1023];
    __syncthreads();
  }
  if (tid == 0) a.info[0] = carry;
}

}  // namespace

int64_t events_slot_cap(int64_t T) { return T / 2 + 2; }

size_t events_workspace_bytes(int64_t n_series, int64_t T, int64_t C) {
  // counts [n_series] i64 + slots [n_series][T/2+2] int2 + hi f32 [C] + lo f64 [C]
  // + n_smooth [C] + n_salt [C], 256-B aligned pieces
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  return al(n_series * 8) + al(n_series * events_slot_cap(T) * 8) + al(C * 4) + 3 * al(C * 8);
}

int64_t events_max_frames() { return EV_MAX_WORDS * 64; }

void launch_events(const EventArgs& a, int mode, hipStream_t s) {
  (void)hipMemsetAsync(a.info, 0, 2 * sizeof(int64_t), s);
  const int64_t n = a.N * a.C;
  if (n == 0) return;
  const int64_t W = (a.T + 63) / 64;              // <= EV_MAX_WORDS (api.cpp checks)
  int wpb = (int)std::min<int64_t>(EV_WAVES, std::max<int64_t>(1, EV_LDS_BYTES / (16 * std::max<int64_t>(W, 1))));
  const unsigned blocks = (unsigned)((n + wpb - 1) / wpb);
  const size_t lds = (size_t)wpb * 2 * W * 8;
  // > 64 KB of dynamic LDS must be opted into (per device: launch_info)
  if (!launch_info(reinterpret_cast<const void*>(events_series_kernel<0>), 64, EV_LDS_BYTES).ok ||
      !launch_info(reinterpret_cast<const void*>(events_series_kernel<1>), 64, EV_LDS_BYTES).ok)
    return;
  if (mode == 0)
    hipLaunchKernelGGL(events_series_kernel<0>, dim3(blocks), dim3(64 * wpb), lds, s, a, W, wpb);
  else
    hipLaunchKernelGGL(events_series_kernel<1>, dim3(blocks), dim3(64 * wpb), lds, s, a, W, wpb);
  hipLaunchKernelGGL(events_compact_kernel, dim3(1), dim3(1024), 0, s, a);
}

}  // namespace sedx
