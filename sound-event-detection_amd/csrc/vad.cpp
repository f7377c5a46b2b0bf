// Host-side thresholding into events, quirk-exact restatement of
// utils/vad.py:11-199 as driven by frame_prediction_to_event_prediction_v2
// (pytorch/predict.py:57-121).  Comparisons are float32 (numpy compares a
// float32 array with a Python-float threshold in float32).
#include <cstdint>
#include <vector>

#include "../../include/sedx.h"

namespace {

typedef std::vector<std::pair<int64_t, int64_t>> Pairs;

// utils/vad.py:108-130: every non-first run starts at locts+1 and the final
// fin is locts[-1] (not +1).
Pairs find_bgn_fin_pairs(const std::vector<int64_t>& locts) {
  Pairs out;
  if (locts.empty()) return out;
  std::vector<int64_t> bgns{locts[0]}, fins;
  for (size_t i = 1; i < locts.size(); ++i)
    if (locts[i] - locts[i - 1] > 1) {
      fins.push_back(locts[i - 1] + 1);
      bgns.push_back(locts[i] + 1);
    }
  fins.push_back(locts.back());
  for (size_t i = 0; i < bgns.size(); ++i) out.push_back({bgns[i], fins[i]});
  return out;
}

// utils/vad.py:158-183
Pairs smooth(const Pairs& p, int64_t n_smooth) {
  Pairs out;
  if (p.empty()) return out;
  int64_t mem_bgn = p[0].first, fin = p[0].second;
  for (size_t n = 1; n < p.size(); ++n) {
    const int64_t pre_fin = p[n - 1].second;
    const int64_t bgn = p[n].first;
    fin = p[n].second;
    if (!(bgn - pre_fin <= n_smooth)) {
      out.push_back({mem_bgn, pre_fin});
      mem_bgn = bgn;
    }
  }
  out.push_back({mem_bgn, fin});
  return out;
}

// utils/vad.py:133-155; returns false where the reference raises IndexError
// (a run's bgn == len(x) after the find_bgn_fin_pairs quirk).
bool second_threshold(const float* x, int64_t T, int64_t stride, const Pairs& p, float thres,
                      Pairs* out) {
  Pairs r;
  for (auto pr : p) {
    int64_t bgn = pr.first, fin = pr.second;
    while (bgn != -1) {
      if (bgn < 0 || bgn >= T) return false;
      if (x[bgn * stride] < thres) break;
      bgn -= 1;
    }
    while (fin != T) {
      if (fin < 0 || fin > T) return false;
      if (x[fin * stride] < thres) break;
      fin += 1;
    }
    r.push_back({bgn + 1, fin});
  }
  *out = smooth(r, 1);
  return true;
}

}  // namespace

extern "C" sedx_status sedx_events(const float* h_framewise, int64_t n_clips, int64_t T,
                                   int64_t C, const double* high_thres, const double* low_thres,
                                   int32_t use_low_thres, const int64_t* n_smooth,
                                   const int64_t* n_salt, int32_t* h_events, int64_t capacity,
                                   int64_t* n_events) {
  if (!h_framewise || !high_thres || !n_smooth || !n_salt || !n_events || n_clips < 0 || T < 0 ||
      C <= 0 || (use_low_thres && !low_thres))
    return SEDX_EINVAL;
  int64_t count = 0;
  for (int64_t n = 0; n < n_clips; ++n)
    for (int64_t k = 0; k < C; ++k) {
      const float* x = h_framewise + n * T * C + k;
      const float hi = (float)high_thres[k];
      std::vector<int64_t> locts;
      for (int64_t t = 0; t < T; ++t)
        if (x[t * C] > hi) locts.push_back(t);
      Pairs pairs = find_bgn_fin_pairs(locts);
      if (use_low_thres) {
        Pairs r;
        if (!second_threshold(x, T, C, pairs, (float)low_thres[k], &r)) return SEDX_EINVAL;
        pairs = r;
      }
      pairs = smooth(pairs, n_smooth[k]);
      for (auto& pr : pairs) {
        if (pr.second - pr.first <= n_salt[k]) continue;   // remove_salt_noise vad.py:186-199
        if (count < capacity && h_events) {
          int32_t* e = h_events + 4 * count;
          e[0] = (int32_t)n;
          e[1] = (int32_t)k;
          e[2] = (int32_t)pr.first;
          e[3] = (int32_t)pr.second;
        }
        ++count;
      }
    }
  *n_events = count;
  return count > capacity ? SEDX_EINVAL : SEDX_OK;
}
