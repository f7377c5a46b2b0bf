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
// Memory: each clip's [T][C] block is read once, coalesced, into LDS; the
// per-frame work of a series is then LDS-latency bound (800 series x 1000
// frames at B=32).
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

template <int MODE, typename XF, typename Emit>
__device__ __forceinline__ void push_pair(SeriesState& st, XF& X, int64_t T, int64_t b, int64_t f,
                                          double lo, bool use_lo, int64_t n_smooth, int64_t n_salt,
                                          Emit& emit) {
  if (!use_lo) {
    push2(st, b, f, n_smooth, n_salt, emit);
    return;
  }
  const float lo_f = (float)lo;
  auto below = [&](int64_t i) { return MODE == 0 ? (X(i) < lo_f) : ((double)X(i) < lo); };
  // activity_detection_with_second_thres vad.py:139-151
  while (b != -1) {
    if (b < 0 || b >= T) {                         // the reference's IndexError
      st.ok = false;
      return;
    }
    if (below(b)) break;
    --b;
  }
  while (f != T) {
    if (f < 0 || f > T) {
      st.ok = false;
      return;
    }
    if (below(f)) break;
    ++f;
  }
  push1(st, b + 1, f, n_smooth, n_salt, emit);
}

// frames [c0, c1) of the series (find_bgn_fin_pairs over locts, streamed: a
// completed run is held until the next one shows it was not the last)
template <int MODE, typename XF, typename Emit>
__device__ void series_frames(SeriesState& st, XF& X, int64_t T, int64_t c0, int64_t c1, float hi,
                              double lo, bool use_lo, int64_t n_smooth, int64_t n_salt, int64_t step,
                              int64_t sd, Emit& emit) {
  // mode 1: scan limit and per-block vote requirement (vad.py:62-78)
  const int64_t interval = sd * 100 - step;
  int64_t lim = T;
  if (MODE == 1) lim = (T - step > 0) ? ((T - step + step - 1) / step) * step : 0;
  const int64_t e = c1 < lim ? c1 : lim;
  for (int64_t t = c0; t < e && st.ok; ++t) {
    bool on;
    if (MODE == 0) {
      on = X(t) > hi;
    } else {
      const int64_t i = (t / step) * step;
      int64_t nov;
      if (i < interval) nov = i / step + 1;
      else if (i >= T - interval) nov = (T - i) / step + 1;
      else nov = sd;
      on = (double)X(t) >= (double)nov;
    }
    if (on) {
      if (!st.in_run) {
        st.in_run = true;
        st.rs = t;
      }
      st.re = t;
    } else if (st.in_run) {
      st.in_run = false;
      if (st.pending) push_pair<MODE>(st, X, T, st.pb, st.pe + 1, lo, use_lo, n_smooth, n_salt, emit);
      st.pb = st.first ? st.rs : st.rs + 1;       // non-first run: bgn = first + 1
      st.pe = st.re;
      st.pending = true;
      st.first = false;
    }
  }
}

template <int MODE, typename XF, typename Emit>
__device__ void series_finish(SeriesState& st, XF& X, int64_t T, double lo, bool use_lo,
                              int64_t n_smooth, int64_t n_salt, Emit& emit) {
  if (!st.ok) return;
  if (st.in_run) {
    if (st.pending) push_pair<MODE>(st, X, T, st.pb, st.pe + 1, lo, use_lo, n_smooth, n_salt, emit);
    if (!st.ok) return;
    st.pb = st.first ? st.rs : st.rs + 1;
    st.pe = st.re;
    st.pending = true;
  }
  if (st.pending) push_pair<MODE>(st, X, T, st.pb, st.pe, lo, use_lo, n_smooth, n_salt, emit);  // last: fin = locts[-1]
  if (!st.ok) return;
  if (use_lo && st.s1_any) push2(st, st.s1_mem, st.s1_pre, n_smooth, n_salt, emit);
  if (st.s2_any) final_out(st.s2_mem, st.s2_pre, n_salt, emit);
}

// One workgroup per clip: the clip's [T][C] block is staged through LDS in
// chunks of TC frames (one coalesced contiguous copy per chunk; C <= 256), and
// thread k < C runs series (clip, k) over the chunk from LDS.  The streaming
// state machine carries across chunks; the second-threshold walks read LDS
// inside the chunk and global memory (L2-resident) outside it.  Events go to
// per-series slots (a series has at most T/2 + 2 events: consecutive events
// are separated by at least one frame), compacted by events_compact_kernel.
constexpr int EV_LDS_FLOATS = 16384;   // 64 KB chunk

template <int MODE>
__global__ __launch_bounds__(256) void events_clip_kernel(EventArgs a) {
  __shared__ float s_x[EV_LDS_FLOATS];
  const int64_t n = blockIdx.x;
  const int k = threadIdx.x;
  const int64_t C = a.C, T = a.T;
  const int64_t TC = EV_LDS_FLOATS / C;
  const float* xg = a.x + n * T * C;
  const bool active = k < C;
  const int64_t sid = n * C + k;
  int2* slot = reinterpret_cast<int2*>(a.slots) + (active ? sid : 0) * a.slot_cap;
  int64_t cnt = 0;
  int64_t t0 = 0, t1 = 0;              // frames [t0, t1) in LDS
  auto X = [&](int64_t i) -> float {
    return (i >= t0 && i < t1) ? s_x[(i - t0) * C + k] : xg[i * C + k];
  };
  SeriesState st;
  series_init(st);
  const float hi = active ? a.hi[k] : 0.f;
  const double lo = active ? a.lo[k] : 0.0;
  const int64_t ns = active ? a.n_smooth[k] : 0, nsalt = active ? a.n_salt[k] : 0;
  auto emit = [&](int64_t b, int64_t f) {
    if (cnt < a.slot_cap) slot[cnt] = make_int2((int)b, (int)f);
    ++cnt;
  };
  for (int64_t c0 = 0; c0 < T; c0 += TC) {
    const int64_t c1 = min(T, c0 + TC);
    __syncthreads();
    const float* src = xg + c0 * C;
    for (int64_t i = threadIdx.x; i < (c1 - c0) * C; i += 256) s_x[i] = src[i];
    __syncthreads();
    t0 = c0;
    t1 = c1;
    if (active && st.ok)
      series_frames<MODE>(st, X, T, c0, c1, hi, lo, a.use_lo != 0, ns, nsalt, a.step, a.sd, emit);
  }
  if (!active) return;
  if (st.ok) series_finish<MODE>(st, X, T, lo, a.use_lo != 0, ns, nsalt, emit);
  a.counts[sid] = st.ok ? cnt : 0;
  if (!st.ok) atomicOr(reinterpret_cast<unsigned long long*>(a.info + 1), 1ull);
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

void launch_events(const EventArgs& a, int mode, hipStream_t s) {
  (void)hipMemsetAsync(a.info, 0, 2 * sizeof(int64_t), s);
  if (a.N * a.C == 0) return;
  if (mode == 0)
    hipLaunchKernelGGL(events_clip_kernel<0>, dim3((unsigned)a.N), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(events_clip_kernel<1>, dim3((unsigned)a.N), dim3(256), 0, s, a);
  hipLaunchKernelGGL(events_compact_kernel, dim3(1), dim3(1024), 0, s, a);
}

}  // namespace sedx
