// Input side of the path: what librosa.core.load(path,
// sr=sample_rate, mono=True) does before pytorch/predict.py:295 /
// pytorch/main_strong.py:787 slice the windows.
//
//   * WAV parsing on the host (RIFF/WAVE: PCM 8/16/24/32-bit, IEEE float
//     32/64, WAVE_FORMAT_EXTENSIBLE), the data chunk copied to the device as
//     it is;
//   * decode + downmix on the GPU with libsndfile's float conversion
//     (int16 * 2^-15, int24 * 2^-23, (float)int32 * 2^-31, (u8 - 128) * 2^-7,
//     float as is) and librosa's to_mono (np.mean over channels of the
//     float32 [C, N] array: float32 running sum over channels, then / C);
//   * resampling on the GPU with resampy's band-limited interpolation
//     (librosa 0.8 res_type 'kaiser_best' / 'kaiser_fast' -> resampy.resample,
//     then librosa.util.fix_length to ceil(n * sr_new / sr_orig)).  resampy is
//     not part of the reference nor installed here: its filter (sinc_window
//     with a Kaiser taper) and resample_f loop are restated from the published
//     algorithm (parity unpinned).  One thread per output
//     sample runs resample_f's two wings in its order with its float64
//     weights, rounding the float32 accumulator after every tap as numba
//     does for a float32 output array; the time register (a running float64
//     sum in resample_f) is precomputed on the host in the same order.
//   This file is built with -ffp-contract=off so a*b+c is not fused.
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/sedx.h"
#include "sedx_internal.h"

namespace sedx {

namespace {

__global__ __launch_bounds__(256) void wav_decode_mono_kernel(const unsigned char* __restrict__ data,
                                                              int64_t frames, int channels, int kind,
                                                              int bytes_per_sample, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= frames) return;
  const unsigned char* f = data + i * (int64_t)channels * bytes_per_sample;
  float acc = 0.f;
  for (int c = 0; c < channels; ++c) {
    const unsigned char* q = f + (int64_t)c * bytes_per_sample;
    float v;
    switch (kind) {
      case 0:  // PCM unsigned 8-bit
        v = (float)((int)q[0] - 128) * 0.0078125f;
        break;
      case 1: {  // PCM int16 little endian
        const int16_t s = (int16_t)((uint16_t)q[0] | ((uint16_t)q[1] << 8));
        v = (float)s * 3.0517578125e-05f;
        break;
      }
      case 2: {  // PCM int24
        const int32_t s = (int32_t)(((uint32_t)q[0] << 8) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 24));
        v = (float)s * 4.656612873077393e-10f;
        break;
      }
      case 3: {  // PCM int32
        const int32_t s = (int32_t)((uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) |
                                    ((uint32_t)q[3] << 24));
        v = (float)s * 4.656612873077393e-10f;
        break;
      }
      case 4: {  // IEEE float32
        uint32_t u = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        v = __uint_as_float(u);
        break;
      }
      default: {  // IEEE float64
        uint64_t u = 0;
        for (int b = 7; b >= 0; --b) u = (u << 8) | q[b];
        v = (float)__longlong_as_double((long long)u);
        break;
      }
    }
    acc = c == 0 ? v : acc + v;
  }
  out[i] = channels > 1 ? acc / (float)channels : acc;
}

// resampy.interp.resample_f for one output sample per thread
__global__ __launch_bounds__(256) void resample_kernel(const float* __restrict__ x, int64_t n_orig,
                                                       const double* __restrict__ treg, int64_t n_res,
                                                       int64_t n_fix, const double* __restrict__ win,
                                                       const double* __restrict__ delta, int64_t nwin,
                                                       double scale, int64_t num_table, int64_t index_step,
                                                       float* __restrict__ y) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_fix) return;
  if (t >= n_res) {           // librosa.util.fix_length zero padding
    y[t] = 0.f;
    return;
  }
  const double time_register = treg[t];
  const int64_t n = (int64_t)time_register;
  double frac = scale * (time_register - (double)n);
  double index_frac = frac * (double)num_table;
  int64_t offset = (int64_t)index_frac;
  double eta = index_frac - (double)offset;
  float acc = 0.f;
  int64_t i_max = (nwin - offset) / index_step;
  if (n + 1 < i_max) i_max = n + 1;
  for (int64_t i = 0; i < i_max; ++i) {
    const int64_t o = offset + i * index_step;
    const double w = win[o] + eta * delta[o];
    acc = (float)((double)acc + w * (double)x[n - i]);
  }
  frac = scale - frac;
  index_frac = frac * (double)num_table;
  offset = (int64_t)index_frac;
  eta = index_frac - (double)offset;
  int64_t k_max = (nwin - offset) / index_step;
  if (n_orig - n - 1 < k_max) k_max = n_orig - n - 1;
  for (int64_t k = 0; k < k_max; ++k) {
    const int64_t o = offset + k * index_step;
    const double w = win[o] + eta * delta[o];
    acc = (float)((double)acc + w * (double)x[n + k + 1]);
  }
  y[t] = acc;
}

struct ResampleFilter {
  int num_zeros, precision;
  double rolloff, beta;
};

bool filter_params(int quality, ResampleFilter* f) {
  if (quality == SEDX_RESAMPLE_KAISER_BEST) {
    *f = {64, 9, 0.9475937167399596, 14.769656459379492};
    return true;
  }
  if (quality == SEDX_RESAMPLE_KAISER_FAST) {
    *f = {16, 9, 0.85, 8.555504641634386};
    return true;
  }
  return false;
}

// resampy.filters.sinc_window with a symmetric Kaiser taper (np.kaiser):
// the right half of the windowed sinc, num_zeros * 2^precision + 1 taps
std::vector<double> sinc_window(const ResampleFilter& f) {
  const int64_t num_bits = (int64_t)1 << f.precision;
  const int64_t n = num_bits * f.num_zeros;
  std::vector<double> w(n + 1);
  const double i0b = std::cyl_bessel_i(0.0, f.beta);
  for (int64_t k = 0; k <= n; ++k) {
    // np.linspace(0, num_zeros, n + 1)[k]
    const double xk = (double)f.num_zeros * (double)k / (double)n;
    const double a = f.rolloff * xk;
    const double sinc = a == 0.0 ? 1.0 : std::sin(M_PI * a) / (M_PI * a);
    const double r = (double)k / (double)n;               // kaiser(2n+1)[n + k]
    const double taper = std::cyl_bessel_i(0.0, f.beta * std::sqrt(std::max(0.0, 1.0 - r * r))) / i0b;
    w[k] = taper * (f.rolloff * sinc);
  }
  return w;
}

size_t al256(size_t b) { return (b + 255) & ~size_t(255); }

}  // namespace

}  // namespace sedx

using namespace sedx;

extern "C" {

sedx_status sedx_wav_decode_mono(const void* d_data, const sedx_wav_info* info, float* d_out,
                                 void* stream) {
  if (!info || (info->frames > 0 && (!d_data || !d_out)) || info->channels <= 0) return SEDX_EINVAL;
  int kind;
  const int bps = info->bits_per_sample;
  if (info->format == SEDX_WAV_PCM)
    kind = bps == 8 ? 0 : bps == 16 ? 1 : bps == 24 ? 2 : bps == 32 ? 3 : -1;
  else if (info->format == SEDX_WAV_FLOAT)
    kind = bps == 32 ? 4 : bps == 64 ? 5 : -1;
  else
    kind = -1;
  if (kind < 0) return SEDX_EINVAL;
  if (info->frames == 0) return SEDX_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t blocks = (info->frames + 255) / 256;
  hipLaunchKernelGGL(wav_decode_mono_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     static_cast<const unsigned char*>(d_data), info->frames, info->channels, kind, bps / 8,
                     d_out);
  return hipGetLastError() == hipSuccess ? SEDX_OK : SEDX_EHIP;
}

sedx_status sedx_resample_size(int64_t n_in, int32_t sr_in, int32_t sr_out, int64_t* n_out) {
  if (n_in < 0 || sr_in <= 0 || sr_out <= 0 || !n_out) return SEDX_EINVAL;
  const double ratio = (double)sr_out / (double)sr_in;
  *n_out = sr_in == sr_out ? n_in : (int64_t)std::ceil((double)n_in * ratio);   // librosa fix_length
  return SEDX_OK;
}

sedx_status sedx_resample_workspace_size(int64_t n_in, int32_t sr_in, int32_t sr_out, int32_t quality,
                                         size_t* bytes) {
  ResampleFilter f;
  if (n_in < 0 || sr_in <= 0 || sr_out <= 0 || !bytes || !filter_params(quality, &f)) return SEDX_EINVAL;
  const int64_t nwin = ((int64_t)1 << f.precision) * f.num_zeros + 1;
  const int64_t n_res = (int64_t)((double)n_in * ((double)sr_out / (double)sr_in));
  *bytes = 2 * al256(nwin * 8) + al256((size_t)std::max<int64_t>(n_res, 1) * 8);
  return SEDX_OK;
}

sedx_status sedx_resample(const float* d_in, int64_t n_in, int32_t sr_in, int32_t sr_out, int32_t quality,
                          float* d_out, void* d_workspace, size_t workspace_bytes, void* stream) {
  ResampleFilter f;
  if (n_in < 0 || sr_in <= 0 || sr_out <= 0 || !filter_params(quality, &f)) return SEDX_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int64_t n_fix = 0;
  sedx_resample_size(n_in, sr_in, sr_out, &n_fix);
  if (n_fix == 0) return SEDX_OK;
  if (!d_in || !d_out) return SEDX_EINVAL;
  if (sr_in == sr_out)                      // librosa: no resampling at the native rate
    return hipMemcpyAsync(d_out, d_in, n_in * sizeof(float), hipMemcpyDeviceToDevice, s) == hipSuccess
               ? SEDX_OK : SEDX_EHIP;
  size_t need = 0;
  sedx_resample_workspace_size(n_in, sr_in, sr_out, quality, &need);
  if (!d_workspace || workspace_bytes < need) return SEDX_EINVAL;
  // resampy.resample: filter, scaled for downsampling; delta = diff(win)
  const double sample_ratio = (double)sr_out / (double)sr_in;
  std::vector<double> win = sinc_window(f);
  if (sample_ratio < 1.0)
    for (double& v : win) v *= sample_ratio;
  const int64_t nwin = (int64_t)win.size();
  std::vector<double> delta(nwin, 0.0);
  for (int64_t i = 0; i + 1 < nwin; ++i) delta[i] = win[i + 1] - win[i];
  const int64_t n_res = (int64_t)((double)n_in * sample_ratio);
  // resample_f's time register: a running float64 sum of 1 / sample_ratio
  std::vector<double> treg((size_t)std::max<int64_t>(n_res, 1));
  const double time_increment = 1.0 / sample_ratio;
  double tr = 0.0;
  for (int64_t t = 0; t < n_res; ++t) {
    treg[t] = tr;
    tr += time_increment;
  }
  const int64_t num_table = (int64_t)1 << f.precision;
  const double scale = std::min(1.0, sample_ratio);
  const int64_t index_step = (int64_t)(scale * (double)num_table);
  char* ws = static_cast<char*>(d_workspace);
  double* d_win = reinterpret_cast<double*>(ws);
  double* d_delta = reinterpret_cast<double*>(ws + al256(nwin * 8));
  double* d_treg = reinterpret_cast<double*>(ws + 2 * al256(nwin * 8));
  // one pinned-free upload of the three tables (the host vectors outlive the
  // copies: hipMemcpyAsync from pageable memory returns after staging them)
  if (hipMemcpyAsync(d_win, win.data(), nwin * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(d_delta, delta.data(), nwin * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      (n_res > 0 && hipMemcpyAsync(d_treg, treg.data(), n_res * 8, hipMemcpyHostToDevice, s) != hipSuccess))
    return SEDX_EHIP;
  const int64_t blocks = (n_fix + 255) / 256;
  hipLaunchKernelGGL(resample_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_in, n_in, d_treg, n_res,
                     n_fix, d_win, d_delta, nwin, scale, num_table, index_step, d_out);
  return hipGetLastError() == hipSuccess ? SEDX_OK : SEDX_EHIP;
}

}  // extern "C"
