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
// Output order = (clip, class, time), the reference's event_list order, made
// deterministic by a count pass + exclusive scan + write pass (3 launches).
// Memory: one row read per frame per series (x[t*C + k]; a clip's classes
// are adjacent threads, so a 100-B row per clip and frame); the
// second-threshold walks re-read frames already in L1/L2.  Tiny next to the
// model (800 series x 1000 frames at B=32).
#include "sedx_internal.h"

namespace sedx {

namespace {

struct Smoother {          // utils/vad.py:158-183, streamed
  bool any;
  int64_t mem, pre;
};

// Runs the chain for one series; emit(bgn, fin) for every surviving event,
// in order.  Returns false where the reference raises IndexError.
template <int MODE, typename Emit>
__device__ bool series_events(const float* __restrict__ x, int64_t C, int64_t T, float hi,
                              double lo, bool use_lo, int64_t n_smooth, int64_t n_salt, int64_t step,
                              int64_t sd, Emit&& emit) {
  Smoother s1{false, 0, 0}, s2{false, 0, 0};
  bool ok = true;
  auto final_out = [&](int64_t b, int64_t f) {
    if (f - b <= n_salt) return;                   // remove_salt_noise vad.py:186-199
    emit(b, f);
  };
  auto push2 = [&](int64_t b, int64_t f) {         // smooth(n_smooth)
    if (!s2.any) {
      s2.any = true;
      s2.mem = b;
    } else if (!(b - s2.pre <= n_smooth)) {
      final_out(s2.mem, s2.pre);
      s2.mem = b;
    }
    s2.pre = f;
  };
  auto push1 = [&](int64_t b, int64_t f) {         // smooth(n_smooth=1) of the 2nd threshold
    if (!s1.any) {
      s1.any = true;
      s1.mem = b;
    } else if (!(b - s1.pre <= 1)) {
      push2(s1.mem, s1.pre);
      s1.mem = b;
    }
    s1.pre = f;
  };
  const float lo_f = (float)lo;
  auto below_lo = [&](int64_t i) {
    return MODE == 0 ? (x[i * C] < lo_f) : ((double)x[i * C] < lo);
  };
  auto push_pair = [&](int64_t b, int64_t f) {
    if (!use_lo) {
      push2(b, f);
      return;
    }
    // activity_detection_with_second_thres vad.py:139-151
    while (b != -1) {
      if (b < 0 || b >= T) {
        ok = false;
        return;
      }
      if (below_lo(b)) break;
      --b;
    }
    while (f != T) {
      if (f < 0 || f > T) {
        ok = false;
        return;
      }
      if (below_lo(f)) break;
      ++f;
    }
    push1(b + 1, f);
  };

  // mode 1: scan limit and per-block vote requirement (vad.py:62-78)
  const int64_t interval = sd * 100 - step;
  int64_t lim = T;
  if (MODE == 1) lim = (T - step > 0) ? ((T - step + step - 1) / step) * step : 0;
  // find_bgn_fin_pairs over locts, streamed: a completed run is held until
  // the next one shows it was not the last
  bool in_run = false, pending = false, first = true;
  int64_t rs = 0, re = 0, pb = 0, pe = 0;
  for (int64_t t = 0; t < lim && ok; ++t) {
    bool on;
    if (MODE == 0) {
      on = x[t * C] > hi;
    } else {
      const int64_t i = (t / step) * step;
      int64_t nov;
      if (i < interval) nov = i / step + 1;
      else if (i >= T - interval) nov = (T - i) / step + 1;
      else nov = sd;
      on = (double)x[t * C] >= (double)nov;
    }
    if (on) {
      if (!in_run) {
        in_run = true;
        rs = t;
      }
      re = t;
    } else if (in_run) {
      in_run = false;
      if (pending) push_pair(pb, pe + 1);         // non-last run: fin = last + 1
      pb = first ? rs : rs + 1;                   // non-first run: bgn = first + 1
      pe = re;
      pending = true;
      first = false;
    }
  }
  if (!ok) return false;
  if (in_run) {
    if (pending) push_pair(pb, pe + 1);
    pb = first ? rs : rs + 1;
    pe = re;
    pending = true;
  }
  if (pending) push_pair(pb, pe);                 // last run: fin = locts[-1]
  if (!ok) return false;
  if (use_lo && s1.any) push2(s1.mem, s1.pre);
  if (s2.any) final_out(s2.mem, s2.pre);
  return true;
}

template <int MODE, bool WRITE>
__global__ __launch_bounds__(256) void events_kernel(EventArgs a) {
  const int64_t sid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (sid >= a.N * a.C) return;
  const int64_t n = sid / a.C, k = sid - n * a.C;
  const float* x = a.x + n * a.T * a.C + k;
  int64_t cnt = 0;
  const int64_t base = WRITE ? a.counts[sid] : 0;
  const bool ok = series_events<MODE>(x, a.C, a.T, a.hi[k], a.lo[k], a.use_lo != 0, a.n_smooth[k],
                                      a.n_salt[k], a.step, a.sd, [&](int64_t b, int64_t f) {
                                        if (WRITE) {
                                          const int64_t i = base + cnt;
                                          if (i < a.capacity)
                                            *reinterpret_cast<int4*>(a.events + 4 * i) =
                                                make_int4((int)n, (int)k, (int)b, (int)f);
                                        }
                                        ++cnt;
                                      });
  if (!WRITE) {
    a.counts[sid] = cnt;
    if (!ok) atomicOr(reinterpret_cast<unsigned long long*>(a.info + 1), 1ull);
  }
}

// exclusive scan of the per-series counts (one workgroup; clips x classes is small)
__global__ __launch_bounds__(1024) void events_scan_kernel(int64_t* counts, int64_t n, int64_t* info) {
  __shared__ int64_t part[1024];
  __shared__ int64_t carry;
  const int tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 1024) {
    const int64_t i = base + tid;
    const int64_t v = i < n ? counts[i] : 0;
    part[tid] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {      // Hillis-Steele inclusive scan
      const int64_t add = tid >= off ? part[tid - off] : 0;
      __syncthreads();
      part[tid] += add;
      __syncthreads();
    }
    if (i < n) counts[i] = carry + part[tid] - v;
    __syncthreads();
    if (tid == 1023) carry += part[1023];
    __syncthreads();
  }
  if (tid == 0) info[0] = carry;
}

}  // namespace

size_t events_workspace_bytes(int64_t n_series, int64_t C) {
  // counts [n_series] + hi f32 [C] + lo f64 [C] + n_smooth [C] + n_salt [C], 256-B aligned pieces
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  return al(n_series * 8) + al(C * 4) + 3 * al(C * 8);
}

void launch_events(const EventArgs& a, int mode, hipStream_t s) {
  const int64_t nser = a.N * a.C;
  (void)hipMemsetAsync(a.info, 0, 2 * sizeof(int64_t), s);
  if (nser == 0) return;
  const int blocks = (int)((nser + 255) / 256);
  if (mode == 0) {
    hipLaunchKernelGGL((events_kernel<0, false>), dim3(blocks), dim3(256), 0, s, a);
    hipLaunchKernelGGL(events_scan_kernel, dim3(1), dim3(1024), 0, s, a.counts, nser, a.info);
    hipLaunchKernelGGL((events_kernel<0, true>), dim3(blocks), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((events_kernel<1, false>), dim3(blocks), dim3(256), 0, s, a);
    hipLaunchKernelGGL(events_scan_kernel, dim3(1), dim3(1024), 0, s, a.counts, nser, a.info);
    hipLaunchKernelGGL((events_kernel<1, true>), dim3(blocks), dim3(256), 0, s, a);
  }
}

}  // namespace sedx
