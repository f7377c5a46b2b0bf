// Frontend kernels for gfx950.
//
//  logmel_kernel: reflect-padded framing -> periodic-Hann window -> real FFT
//  (N/2-point complex Stockham radix-4/2 FFT in LDS, one wavefront per frame)
//  -> |X|^2 -> sparse mel-band reduction (lane m owns mel band m) ->
//  10*log10(max(.,1e-10)) -> bn0 affine -> X0[item][t][m].
//  Replaces Spectrogram + LogmelFilterBank + bn0 of the reference
//  (pytorch/stft.py:223-247 conv1d-DFT, :660-663 power, :709 matmul melW,
//  :721-726 power_to_db with top_db=None; pytorch/models.py:642-644 bn0).
//
//  gamma kernels: un-centred framing, centred-Hann(nwin) in nfft, |FFT|,
//  dense ERB weight reduction / nfft, power_to_db(top_db=80), per-clip
//  max-abs normalisation and int16 quantisation (utils/gammatone/fftweight.py:
//  15-60,126-168; utils/features.py:361-370; utils/utilities.py:73-79).
#include "sedx_internal.h"

namespace sedx {

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// LDS hand-off inside one wavefront: a wave's LDS operations complete in
// issue order, so waiting for its own (lgkmcnt) and fencing the compiler is
// enough — no workgroup barrier, and global loads in flight are not drained.
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
struct BlockSync {
  __device__ void operator()() const { __syncthreads(); }
};
struct WaveSync {
  __device__ void operator()() const { wave_lds_sync(); }
};

// In-LDS Stockham FFT of N2 complex points (forward, e^{-2 pi i}); one wave.
// tw = exp(-2 pi i m / NFFT) with NFFT = 2*N2.  Radix 4 while N2/Ns allows,
// then radix 2; every stage's geometry is a compile-time constant.
// BlockSync: every lane of the block calls it (block barriers inside).
template <int N2, int Ns, typename Sync>
__device__ __forceinline__ float2* stockham_stages(float2* X, float2* Y, const float2* tw, int lane) {
  if constexpr (Ns >= N2) {
    return X;
  } else {
    constexpr int NFFT = 2 * N2;
    constexpr int R = ((N2 / Ns) % 4 == 0) ? 4 : 2;
    constexpr int nb = N2 / R;
    constexpr int step = NFFT / (Ns * R);
#pragma unroll
    for (int j0 = 0; j0 < nb; j0 += 64) {
      const int j = j0 + lane;
      if (j >= nb) break;
      const int k = j & (Ns - 1);
      const int base = (j - k) * R + k;
      if constexpr (R == 4) {
        float2 v0 = X[j], v1 = X[j + nb], v2 = X[j + 2 * nb], v3 = X[j + 3 * nb];
        if constexpr (Ns > 1) {
          v1 = cmul(v1, tw[k * step]);
          v2 = cmul(v2, tw[2 * k * step]);
          v3 = cmul(v3, tw[3 * k * step]);
        }
        const float2 a0 = cadd(v0, v2), a1 = csub(v0, v2);
        const float2 b0 = cadd(v1, v3), b1 = csub(v1, v3);
        const float2 mib1 = make_float2(b1.y, -b1.x);   // -i * b1
        Y[base] = cadd(a0, b0);
        Y[base + Ns] = cadd(a1, mib1);
        Y[base + 2 * Ns] = csub(a0, b0);
        Y[base + 3 * Ns] = csub(a1, mib1);
      } else {
        float2 v0 = X[j], v1 = X[j + nb];
        if constexpr (Ns > 1) v1 = cmul(v1, tw[k * step]);
        Y[base] = cadd(v0, v1);
        Y[base + Ns] = csub(v0, v1);
      }
    }
    Sync()();
    return stockham_stages<N2, Ns * R, Sync>(Y, X, tw, lane);
  }
}

template <int N2, typename Sync = BlockSync>
__device__ __forceinline__ void stockham_fft(float2* X, float2* Y, const float2* tw, int lane,
                                             float2** res) {
  *res = stockham_stages<N2, 1, Sync>(X, Y, tw, lane);
}

// Real-input spectrum bin k (0..N2) from the N2-point complex FFT Z of
// z[m] = x[2m] + i x[2m+1].
template <int N2>
__device__ __forceinline__ float2 real_bin(const float2* Z, const float2* tw, int k) {
  const float2 A = Z[k & (N2 - 1)];
  const float2 Bz = Z[(N2 - k) & (N2 - 1)];
  const float2 Bc = make_float2(Bz.x, -Bz.y);
  const float2 E = make_float2(0.5f * (A.x + Bc.x), 0.5f * (A.y + Bc.y));
  const float2 O = make_float2(0.5f * (A.y - Bc.y), -0.5f * (A.x - Bc.x));  // -i (A - Bc) / 2
  return cadd(E, cmul(tw[k], O));
}

// One wavefront per frame, the waves of a workgroup independent (no
// workgroup barrier after the table staging).  Twiddles, window and the
// packed mel weights sit in LDS; a lane's mel band geometry and bn0 constants
// sit in registers; the next frame's samples are loaded into registers while
// the current frame is transformed.
//
// One 1024-thread workgroup per CU, and the workgroup claims the CU's whole
// LDS (the dynamic part beyond the mel weights is padding): no workgroup of
// another kernel can share its CU.  Measured on MI355X (tools/fe_race.cpp):
// this FFT, sharing a CU with MFMA (or other heavy) waves of a kernel on
// another stream, intermittently produced wrong spectra (11 of 32 launches);
// CU-exclusive, 0 of 64.  MFMA kernels are padded the same way
// (mfma_cu_exclusive_lds).
constexpr int FE_WAVES = 16;
constexpr int LDS_PER_CU = 160 * 1024;

template <int NFFT, bool I16>
__global__ __launch_bounds__(64 * FE_WAVES) void logmel_kernel(FrontendParams p) {
  constexpr int N2 = NFFT / 2;
  constexpr int NS = NFFT / 64;          // samples per lane per frame
  __shared__ float2 s_tw[NFFT];
  __shared__ float s_win[NFFT];
  __shared__ float2 s_buf[FE_WAVES][2][N2];
  extern __shared__ float s_melw[];      // [p.mel_lds_floats]: packed mel weights, then padding
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nnz = p.mel_off[64];
  const bool mel_in_lds = nnz <= p.mel_lds_floats;
  for (int i = threadIdx.x; i < NFFT; i += 64 * FE_WAVES) {
    s_tw[i] = p.twiddle[i];
    s_win[i] = p.window[i];
  }
  if (mel_in_lds)
    for (int i = threadIdx.x; i < nnz; i += 64 * FE_WAVES) s_melw[i] = p.mel_w[i];
  const int m = lane;                    // mel band of this lane
  const int mlo = p.mel_lo[m], o0 = p.mel_off[m], o1 = p.mel_off[m + 1];
  const float bmu = p.bn_mean[m], bsc = p.bn_scale[m], bbi = p.bn_bias[m];
  __syncthreads();

  const int64_t total = (int64_t)p.n_clips * p.n_win * p.T;
  const int64_t L = p.sig_len;
  float2* X = s_buf[wave][0];
  float2* Y = s_buf[wave][1];
  // samples of frame fr: lane holds j = pos0 + 2 (lane + 64 i) + e
  auto load = [&](int64_t fr, float* v) {
    const int64_t item = fr / p.T;
    const int t = (int)(fr - item * p.T);
    const int64_t clip = item / p.n_win;
    const int w = (int)(item - clip * p.n_win);
    const int64_t wstart = p.win_start[w];
    const int64_t src_off = clip * p.clip_stride + wstart;
    const int64_t avail = p.clip_len - wstart;      // samples of this item backed by audio
    const int64_t pos0 = (int64_t)t * p.hop - N2;   // start in un-padded coordinates
#pragma unroll
    for (int i = 0; i < NS / 2; ++i)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        int64_t j = pos0 + 2 * (lane + 64 * i) + e;
        if (j < 0) j = -j;                           // reflect (F.pad mode='reflect')
        if (j >= L) j = 2 * (L - 1) - j;
        const bool ok = j < avail;                   // pad_truncate zeros
        const int64_t jc = ok ? j : 0;
        if (I16)   // int16_to_float32: float64 x / 32767, rounded to float32
          v[2 * i + e] = ok ? (float)((double)p.audio_i16[src_off + jc] / 32767.0) : 0.0f;
        else
          v[2 * i + e] = ok ? p.audio[src_off + jc] : 0.0f;
      }
  };
  int64_t fr = (int64_t)blockIdx.x * FE_WAVES + wave;
  const int64_t fstride = (int64_t)gridDim.x * FE_WAVES;
  float v[NS];
  if (fr < total) load(fr, v);
  for (; fr < total; fr += fstride) {
#pragma unroll
    for (int i = 0; i < NS / 2; ++i) {
      const int mm = lane + 64 * i;
      X[mm] = make_float2(v[2 * i] * s_win[2 * mm], v[2 * i + 1] * s_win[2 * mm + 1]);
    }
    if (fr + fstride < total) load(fr + fstride, v);   // next frame, in flight during the FFT
    wave_lds_sync();
    float2* Z;
    stockham_fft<N2, WaveSync>(X, Y, s_tw, lane, &Z);
    float* P = reinterpret_cast<float*>(Z == X ? Y : X);   // the other buffer
#pragma unroll
    for (int i = 0; i < N2 / 64; ++i) {
      const int k = lane + 64 * i;
      const float2 Xk = real_bin<N2>(Z, s_tw, k);
      P[k] = Xk.x * Xk.x + Xk.y * Xk.y;
    }
    if (lane == 0) {                      // Nyquist bin
      const float2 Xk = real_bin<N2>(Z, s_tw, N2);
      P[N2] = Xk.x * Xk.x + Xk.y * Xk.y;
    }
    wave_lds_sync();
    // band sum in bin order (the fma chain of the sparse dot product), four
    // bins' loads issued together
    float acc = 0.0f;
    if (mel_in_lds) {
      for (int i = o0; i < o1; i += 4) {
        float pw[4], ww[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = i + e < o1;
          pw[e] = ok ? P[mlo + (i + e - o0)] : 0.f;
          ww[e] = ok ? s_melw[i + e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (i + e < o1) acc = fmaf(pw[e], ww[e], acc);
      }
    } else {
      for (int i = o0; i < o1; ++i) acc = fmaf(P[mlo + (i - o0)], p.mel_w[i], acc);
    }
    float db = 10.0f * log10f(fmaxf(acc, 1e-10f));
    db = (db - bmu) * bsc + bbi;
    p.out[fr * 64 + m] = db;
    wave_lds_sync();                      // P / Z reads done before the next frame's writes
  }
}

// one CU-exclusive workgroup per CU; every wave walks several frames, so the
// register prefetch of the next frame overlaps the current FFT
template <int NFFT, bool I16>
static void launch_logmel_t(const FrontendParams& p0, int64_t total, hipStream_t s) {
  static size_t dyn = 0;
  static int ncu = 0;
  if (!ncu) {
    hipFuncAttributes fa{};
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(logmel_kernel<NFFT, I16>));
    dyn = (LDS_PER_CU - fa.sharedSizeBytes) & ~size_t(511);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(logmel_kernel<NFFT, I16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  FrontendParams p = p0;
  p.mel_lds_floats = (int32_t)(dyn / 4);
  int64_t blocks = (total + FE_WAVES - 1) / FE_WAVES;
  if (blocks > ncu) blocks = ncu;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((logmel_kernel<NFFT, I16>), dim3((unsigned)blocks), dim3(64 * FE_WAVES), dyn, s, p);
}

void launch_logmel(const FrontendParams& p, int n_fft, hipStream_t s) {
  const int64_t total = (int64_t)p.n_clips * p.n_win * p.T;
  const bool i16 = p.audio_i16 != nullptr;
  switch (n_fft) {
    case 256:
      if (i16) launch_logmel_t<256, true>(p, total, s);
      else launch_logmel_t<256, false>(p, total, s);
      break;
    case 512:
      if (i16) launch_logmel_t<512, true>(p, total, s);
      else launch_logmel_t<512, false>(p, total, s);
      break;
    case 1024:
      if (i16) launch_logmel_t<1024, true>(p, total, s);
      else launch_logmel_t<1024, false>(p, total, s);
      break;
    default: break;
  }
}

// feat [B][64][T] -> out [B][T][64] with bn0 (models.py:636-644, gamma branch).
__global__ __launch_bounds__(256) void features_bn0_kernel(const float* __restrict__ feat, int B,
                                                           int T, const float* sc, const float* mu,
                                                           const float* bi, float* out) {
  __shared__ float tile[64][65];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int m = i >> 6, tt = i & 63;
    const int t = t0 + tt;
    tile[m][tt] = (t < T) ? feat[((int64_t)b * 64 + m) * T + t] : 0.0f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int tt = i >> 6, m = i & 63;
    const int t = t0 + tt;
    if (t < T) out[((int64_t)b * T + t) * 64 + m] = (tile[m][tt] - mu[m]) * sc[m] + bi[m];
  }
}

void launch_features_bn0(const float* feat, int B, int T, const float* bn_scale,
                         const float* bn_mean, const float* bn_bias, float* out,
                         hipStream_t s) {
  hipLaunchKernelGGL(features_bn0_kernel, dim3((T + 63) / 64, B), dim3(256), 0, s, feat, B, T,
                     bn_scale, bn_mean, bn_bias, out);
}

// ---------------------------------------------------------------------------
// Gammatone frontend (nfft = 2048 at 32 kHz, 1024 at 16 kHz)
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned int f2ord(float f) {
  const unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(unsigned int u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

template <int NFFT>
__global__ __launch_bounds__(256) void gamma_frames_kernel(GammaParams p, unsigned int* mm) {
  constexpr int N2 = NFFT / 2;
  constexpr int NB = N2 + 1;
  __shared__ float2 s_tw[NFFT];
  __shared__ float2 s_buf[2][2][N2];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;   // 0..3 ; waves 0,1 do FFTs, all 4 help in the ERB sum
  for (int i = threadIdx.x; i < NFFT; i += 256) s_tw[i] = p.twiddle[i];
  __syncthreads();
  const int64_t total = (int64_t)p.B * p.T;
  for (int64_t f0 = (int64_t)blockIdx.x * 2; f0 < total; f0 += (int64_t)gridDim.x * 2) {
    const int sub = wave & 1;
    const int64_t fr = f0 + sub;
    const bool valid = fr < total;
    float2* X = s_buf[sub][0];
    float2* Y = s_buf[sub][1];
    int64_t b = 0;
    int t = 0;
    if (valid) {
      b = fr / p.T;
      t = (int)(fr - b * p.T);
    }
    if (valid && wave < 2) {
      const float* src = p.audio + b * p.L + (int64_t)t * p.hop;
      for (int m = lane; m < N2; m += 64)
        X[m] = make_float2(src[2 * m] * p.window[2 * m], src[2 * m + 1] * p.window[2 * m + 1]);
    }
    __syncthreads();
    // both FFT waves run the transform; waves 2,3 follow the barriers only
    float2* Z;
    {
      float2* XX = X;
      float2* YY = Y;
      if (wave >= 2) { XX = s_buf[sub][0]; YY = s_buf[sub][1]; }
      // waves 2/3 must not write: give them an empty loop by lane >= 64 trick
      const int l = (wave < 2) ? lane : 1 << 20;
      stockham_fft<N2>(XX, YY, s_tw, l, &Z);
    }
    float* Mg = reinterpret_cast<float*>(Z == X ? Y : X);
    if (valid && wave < 2) {
      for (int k = lane; k < NB; k += 64) {
        const float2 Xk = real_bin<N2>(Z, s_tw, k);
        Mg[k] = sqrtf(Xk.x * Xk.x + Xk.y * Xk.y);
      }
    }
    __syncthreads();
    // ERB reduction: 64 channels x 2 frames = 128 outputs; 4 waves -> each
    // (wave&1) frame, half of the bins per wave pair, combined via LDS.
    __shared__ float s_part[2][2][64];
    if (valid) {
      const int half = wave >> 1;
      const int kb = half ? NB / 2 : 0, ke = half ? NB : NB / 2;
      const float* w = p.weights;  // transposed: [NB][64]
      float acc = 0.0f;
      for (int k = kb; k < ke; ++k) acc = fmaf(w[(int64_t)k * 64 + lane], Mg[k], acc);
      s_part[sub][half][lane] = acc;
    }
    __syncthreads();
    if (valid && wave < 2) {
      const float g = (t < p.T_fill) ? s_part[sub][0][lane] + s_part[sub][1][lane] : 0.0f;
      const float db = 10.0f * log10f(fmaxf(g, 1e-10f));
      p.gt[(b * 64 + lane) * p.T + t] = db;
      // per-clip max / min of dB (ordered-int atomics)
      atomicMax(&mm[2 * b], f2ord(db));
      atomicMin(&mm[2 * b + 1], f2ord(db));
    }
    __syncthreads();
  }
}

__global__ void gamma_init_kernel(unsigned int* mm, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) {
    mm[2 * i] = 0u;
    mm[2 * i + 1] = 0xffffffffu;
  }
}

__global__ __launch_bounds__(256) void gamma_quant_kernel(GammaParams p, const unsigned int* mm) {
  const int64_t n = (int64_t)p.B * 64 * p.T;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / (64 * (int64_t)p.T);
    const double mx = (double)ord2f(mm[2 * b]);
    const double mn = (double)ord2f(mm[2 * b + 1]);
    const double floor_db = mx - 80.0;                 // power_to_db top_db
    const double lo = mn > floor_db ? mn : floor_db;
    const double maxabs = fmax(fabs(mx), fabs(lo));
    double x = (double)p.gt[i];
    if (x < floor_db) x = floor_db;
    if (maxabs > 1.0) x /= maxabs;                     // float32_to_int16
    const double q = trunc(x * 32767.0);               // astype(int16): toward zero
    p.out[i] = (float)(q / 32767.0);                   // int16_to_float32
  }
}

void launch_gamma(const GammaParams& p, hipStream_t s) {
  unsigned int* mm = reinterpret_cast<unsigned int*>(p.maxbuf);
  hipLaunchKernelGGL(gamma_init_kernel, dim3((p.B + 255) / 256), dim3(256), 0, s, mm, p.B);
  const int64_t total = (int64_t)p.B * p.T;
  int64_t blocks = (total + 1) / 2;
  if (blocks > 4096) blocks = 4096;
  // the same in-LDS FFT as the logmel frontend: CU-exclusive LDS footprint
  // (mfma_cu_exclusive_lds keeps the kernel's own workgroups per CU)
  auto go = [&](const void* k, auto kern) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), mfma_cu_exclusive_lds(k, 256), s, p, mm);
  };
  if (p.nfft == 2048)
    go(reinterpret_cast<const void*>(gamma_frames_kernel<2048>), gamma_frames_kernel<2048>);
  else if (p.nfft == 1024)
    go(reinterpret_cast<const void*>(gamma_frames_kernel<1024>), gamma_frames_kernel<1024>);
  else if (p.nfft == 512)
    go(reinterpret_cast<const void*>(gamma_frames_kernel<512>), gamma_frames_kernel<512>);
  hipLaunchKernelGGL(gamma_quant_kernel, dim3(2048), dim3(256), 0, s, p, mm);
}

}  // namespace sedx
