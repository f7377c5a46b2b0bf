// Host-side loop control and merge plan of the reference's windowed drivers:
//   pytorch/predict.py:297-349            (predict: stride 1 s with --overlap,
//                                          else sample_duration s)
//   pytorch/main_strong.py:786-835, :1052-1100
//                                         (inference_prob_overlap / _vote:
//                                          clip padded to 10 s, stride
//                                          overlap_value s)
//   utils/utilities.py:405-446            (merge / avg_merge)
//
// The merge is not a plain overlap-add: utilities.merge places window k at
// frame (k-1) * int(100 * overlap_value) of the running array WHATEVER the
// stride, with numpy's slice clamping and broadcasting.  build_merge_plan
// replays those numpy operations on index lists (each merged frame = the
// ordered list of (window, frame) values numpy added into it), so the GPU
// merge (seq.hip merge_plan_kernel) and sedx_merge_host reproduce every case
// the reference accepts, including degenerate ones, and fail exactly where
// numpy raises.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/sedx.h"
#include "sedx_internal.h"

namespace sedx {

const char* window_loop(int sample_rate, int64_t L_clip, const sedx_window_spec& sp, WindowLoop* out) {
  out->start.clear();
  out->len.clear();
  if (sample_rate <= 0 || L_clip <= 0) return "empty clip or bad sample rate";
  if (sp.vote != 0 && sp.vote != 1) return "sedx_window_spec.vote must be 0 (averaged merge) or 1 (vote merge)";
  if (sp.driver != SEDX_DRIVER_PREDICT && sp.driver != SEDX_DRIVER_MAIN_STRONG) return "unknown window driver";
  if (sp.sample_duration <= 0) return "sample_duration must be a positive number of seconds";
  const double sd = sp.sample_duration;
  // predict.py:334-337: the stride is an int (start stays an int); main_strong
  // :829 accumulates overlap_value in float64
  const double stride = sp.driver == SEDX_DRIVER_PREDICT ? (sp.overlap ? 1.0 : sd) : sp.overlap_value;
  if (!(stride > 0)) return "stride <= 0: the reference's window loop never ends";
  const double duration = sp.audio_duration > 0 ? sp.audio_duration : (double)L_clip / sample_rate;
  const int64_t full = (int64_t)sp.sample_duration * sample_rate;   // int((sd * sr) + start_index) - start_index
  // main_strong.py:790 pad_truncate's the clip to 10 s and slices the windows
  // from it without padding them (:795-797)
  const int64_t padded = (int64_t)sample_rate * 10;
  double start = 0.0, end = 0.0;
  while (end <= duration) {                                    // predict.py:297, main_strong.py:791
    if (out->start.size() >= ((size_t)1 << 24)) return "too many windows per clip";
    const int64_t s = (int64_t)(start * (double)sample_rate);  // int(start * sample_rate)
    int64_t n = full;
    if (sp.driver == SEDX_DRIVER_MAIN_STRONG) n = std::max<int64_t>(0, std::min<int64_t>(s + full, padded) - s);
    out->start.push_back(s);
    out->len.push_back(n);
    start += stride;
    end = start + sd;
  }
  return nullptr;
}

namespace {
// numpy basic slicing bounds for a[lo:] / a[:hi] with one index i on length n
int64_t py_index(int64_t i, int64_t n) {
  if (i < 0) return std::max<int64_t>(0, n + i);
  return std::min(i, n);
}
}  // namespace

const char* build_merge_plan(const std::vector<int64_t>& frames, int64_t step, int sample_duration, bool avg,
                             MergePlan* plan) {
  const size_t n = frames.size();
  if (n == 0) return "no windows";
  std::vector<std::vector<int32_t>> m;   // merged frame -> ordered (window, frame) entries, packed
  std::vector<int32_t> wbase(n + 1, 0);  // first packed id of window w (ids = wbase[w] + t)
  for (size_t w = 0; w < n; ++w) {
    if (frames[w] < 0 || (int64_t)wbase[w] + frames[w] > INT32_MAX) return "merge plan too large";
    wbase[w + 1] = wbase[w] + (int32_t)frames[w];
  }
  // the merged length never exceeds the frames of all windows (a window adds
  // at most its own frames), however large the step
  m.reserve((size_t)std::min<int64_t>(wbase[n], frames[0] + (int64_t)(n - 1) * std::max<int64_t>(step, 1)));
  for (int64_t t = 0; t < frames[0]; ++t) m.push_back({wbase[0] + (int32_t)t});     // merged = curr_preds
  for (size_t w = 1; w < n; ++w) {
    // merge(prev, curr, sample_duration, num_segment = w + 1, overlap_value)
    const int64_t P = (int64_t)m.size(), Tw = frames[w];
    const int64_t front = (int64_t)w * step;            // (num_segment - 1) * overlap_interval
    const int64_t back = P - front;                     // prev.shape[1] - front_cutoff
    const int64_t a = py_index(front, P);               // prev[:, front:] / prev[:, :front]
    const int64_t e = py_index(back, Tw);               // curr[:, :back] / curr[:, back:]
    const int64_t lp = P - a, lc = e;
    int64_t lm;                                          // prev_overlap + curr_overlap (broadcast)
    if (lp == lc) lm = lp;
    else if (lp == 1) lm = lc;
    else if (lc == 1) lm = lp;
    else return "merge: operands could not be broadcast together (numpy raises ValueError)";
    std::vector<std::vector<int32_t>> mid((size_t)lm);
    for (int64_t i = 0; i < lm; ++i) {
      mid[i] = m[(size_t)(a + (lp == 1 ? 0 : i))];
      mid[i].push_back(wbase[w] + (int32_t)(lc == 1 ? 0 : i));
    }
    m.resize((size_t)a);                                 // prev[:, :front]
    for (auto& v : mid) m.push_back(std::move(v));
    for (int64_t t = e; t < Tw; ++t) m.push_back({wbase[w] + (int32_t)t});   // curr[:, back:]
  }
  const int64_t N = (int64_t)m.size();
  plan->N = N;
  plan->win_base = wbase;
  plan->off.assign((size_t)N + 1, 0);
  plan->src.clear();
  for (int64_t f = 0; f < N; ++f) {
    plan->off[f] = (int32_t)plan->src.size();
    for (int32_t id : m[f]) plan->src.push_back(id);
    if (plan->src.size() > (size_t)INT32_MAX) return "merge plan too large";
  }
  plan->off[N] = (int32_t)plan->src.size();
  plan->div.assign((size_t)N, 1);
  if (avg) {
    // avg_merge (utilities.py:425-446): for i in range(step, N - step, step)
    if (step == 0) return "avg_merge: range() step is zero (int(100 * overlap_value) == 0; numpy raises)";
    const int64_t interval = (int64_t)sample_duration * 100 - step;
    if (step > 0) {
      for (int64_t i = step; i < N - step; i += step) {
        int64_t d;
        if (i < interval) d = i / step + 1;
        else if (i >= N - interval) d = (N - i) / step + 1;
        else d = sample_duration;
        for (int64_t f = i; f < std::min(i + step, N); ++f) plan->div[f] = (int32_t)d;
      }
    }
    // step < 0: range(step, N - step, step) is empty (no division)
  }
  return nullptr;
}

}  // namespace sedx

using namespace sedx;

extern "C" {

// (host vectors: a failed allocation returns SEDX_ENOMEM, never throws
// across the C ABI)
sedx_status sedx_window_starts(int32_t sample_rate, int64_t L_clip, const sedx_window_spec* spec,
                               int64_t* h_start, int64_t* h_len, int64_t capacity, int64_t* n_windows) {
  if (!spec || !n_windows || capacity < 0) return SEDX_EINVAL;
  try {
    WindowLoop wl;
    if (window_loop(sample_rate, L_clip, *spec, &wl)) return SEDX_EINVAL;
    *n_windows = (int64_t)wl.start.size();
    const int64_t k = std::min<int64_t>(capacity, *n_windows);
    if (h_start) std::copy(wl.start.begin(), wl.start.begin() + k, h_start);
    if (h_len) std::copy(wl.len.begin(), wl.len.begin() + k, h_len);
    return SEDX_OK;
  } catch (const std::bad_alloc&) {
    return SEDX_ENOMEM;
  } catch (...) {
    return SEDX_EINVAL;
  }
}

sedx_status sedx_merge_host(const float* h_win, const int64_t* frames, int64_t n_win, int64_t C,
                            int32_t sample_duration, double overlap_value, int32_t avg, float* h_out,
                            int64_t capacity_frames, int64_t* merged_frames) {
  if (!frames || n_win <= 0 || C <= 0 || !merged_frames || (h_out && !h_win)) return SEDX_EINVAL;
  // int(100 * overlap_value) in float64; the same range as the handle API
  // (a NaN / inf / huge value would be undefined in the cast)
  const double stepd = 100.0 * overlap_value;
  if (!std::isfinite(stepd) || !(std::fabs(stepd) < 1e9)) return SEDX_EINVAL;
  const int64_t step = (int64_t)stepd;
  try {
  MergePlan plan;
  if (build_merge_plan(std::vector<int64_t>(frames, frames + n_win), step, sample_duration, avg != 0, &plan))
    return SEDX_EINVAL;
  *merged_frames = plan.N;
  if (!h_out) return SEDX_OK;
  if (capacity_frames < plan.N) return SEDX_EINVAL;
  for (int64_t f = 0; f < plan.N; ++f)
    for (int64_t k = 0; k < C; ++k) {
      float s = 0.f;
      for (int32_t j = plan.off[f]; j < plan.off[f + 1]; ++j) {
        const float v = h_win[(int64_t)plan.src[j] * C + k];
        s = j == plan.off[f] ? v : s + v;              // numpy's prev + curr, in window order
      }
      const int32_t d = plan.div[f];
      h_out[f * C + k] = d > 1 ? s / (float)d : s;      // float32 /= int (utilities.py:435)
    }
  return SEDX_OK;
  } catch (const std::bad_alloc&) {
    return SEDX_ENOMEM;
  } catch (...) {
    return SEDX_EINVAL;
  }
}

}  // extern "C"
