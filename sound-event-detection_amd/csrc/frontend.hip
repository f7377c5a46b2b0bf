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
#include <type_traits>

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

// FFT buffers hold one pad element per 32 (pidx): the radix-4 stages write
// with strides 4 Ns, which unpadded put 8 lanes of a write on one bank
__device__ __forceinline__ int pidx(int i) { return i + (i >> 5); }
template <int N2>
constexpr int fe_buf_len() { return N2 + N2 / 32; }

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
        float2 v0 = X[pidx(j)], v1 = X[pidx(j + nb)], v2 = X[pidx(j + 2 * nb)], v3 = X[pidx(j + 3 * nb)];
        if constexpr (Ns > 1) {
          v1 = cmul(v1, tw[k * step]);
          v2 = cmul(v2, tw[2 * k * step]);
          v3 = cmul(v3, tw[3 * k * step]);
        }
        const float2 a0 = cadd(v0, v2), a1 = csub(v0, v2);
        const float2 b0 = cadd(v1, v3), b1 = csub(v1, v3);
        const float2 mib1 = make_float2(b1.y, -b1.x);   // -i * b1
        Y[pidx(base)] = cadd(a0, b0);
        Y[pidx(base + Ns)] = cadd(a1, mib1);
        Y[pidx(base + 2 * Ns)] = csub(a0, b0);
        Y[pidx(base + 3 * Ns)] = csub(a1, mib1);
      } else {
        float2 v0 = X[pidx(j)], v1 = X[pidx(j + nb)];
        if constexpr (Ns > 1) v1 = cmul(v1, tw[k * step]);
        Y[pidx(base)] = cadd(v0, v1);
        Y[pidx(base + Ns)] = csub(v0, v1);
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
  const float2 A = Z[pidx(k & (N2 - 1))];
  const float2 Bz = Z[pidx((N2 - k) & (N2 - 1))];
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
// 1024-thread workgroups (16 waves), as many per CU as the LDS allows.
// Built without packed FP32 VALU (Makefile): with v_pk_* arithmetic this FFT
// returned wrong spectra while MFMA waves shared its CU (sedx_internal.h
// "packed FP32").
constexpr int FE_WAVES = 16;

template <int NFFT, bool I16>
__global__ __launch_bounds__(64 * FE_WAVES) void logmel_kernel(FrontendParams p) {
  constexpr int N2 = NFFT / 2;
  constexpr int NS = NFFT / 64;          // samples per lane per frame
  __shared__ float2 s_tw[NFFT];
  __shared__ float s_win[NFFT];
  __shared__ float2 s_buf[FE_WAVES][2][fe_buf_len<N2>()];
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

  // frame bookkeeping in 32-bit (the host checks items * T < 2^31 and
  // sig_len < 2^31): 64-bit division costs hundreds of instructions
  const int total = p.n_clips * p.n_win * p.T;
  const int L = (int)p.sig_len;
  float2* X = s_buf[wave][0];
  float2* Y = s_buf[wave][1];
  // samples of frame fr: lane holds j = pos0 + 2 (lane + 64 i) + e
  auto load = [&](int fr, float* v) {
    const unsigned item = (unsigned)fr / (unsigned)p.T;
    const int t = fr - (int)item * p.T;
    const unsigned clip = item / (unsigned)p.n_win;
    const int w = (int)(item - clip * (unsigned)p.n_win);
    const int64_t wstart = p.win_start ? p.win_start[w] : 0;
    const int64_t src_off = (int64_t)clip * p.clip_stride + wstart;
    const int64_t av64 = p.clip_len - wstart;        // samples of this item backed by audio
    const int avail = av64 > L ? L : (int)av64;       // (j < L always)
    const int pos0 = t * p.hop - N2;                  // start in un-padded coordinates
    if (!I16 && pos0 >= 0 && pos0 + NFFT <= avail && ((src_off + pos0) & 1) == 0) {
      // interior frame (no reflection, no pad_truncate): 8-byte loads
      const float2* src = reinterpret_cast<const float2*>(p.audio + src_off + pos0);
#pragma unroll
      for (int i = 0; i < NS / 2; ++i) {
        const float2 q = src[lane + 64 * i];
        v[2 * i] = q.x;
        v[2 * i + 1] = q.y;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NS / 2; ++i)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        int j = pos0 + 2 * (lane + 64 * i) + e;
        if (j < 0) j = -j;                           // reflect (F.pad mode='reflect')
        if (j >= L) j = 2 * (L - 1) - j;
        const bool ok = j < avail;                   // pad_truncate zeros
        const int jc = ok ? j : 0;
        if (I16)   // int16_to_float32: float64 x / 32767, rounded to float32
          v[2 * i + e] = ok ? (float)((double)p.audio_i16[src_off + jc] / 32767.0) : 0.0f;
        else
          v[2 * i + e] = ok ? p.audio[src_off + jc] : 0.0f;
      }
  };
  int fr = (int)blockIdx.x * FE_WAVES + wave;
  const int fstride = (int)gridDim.x * FE_WAVES;
  float v[NS];
  if (fr < total) load(fr, v);
  for (; fr < total; fr += fstride) {
#pragma unroll
    for (int i = 0; i < NS / 2; ++i) {
      const int mm = lane + 64 * i;
      X[pidx(mm)] = make_float2(v[2 * i] * s_win[2 * mm], v[2 * i + 1] * s_win[2 * mm + 1]);
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
    p.out[(int64_t)fr * 64 + m] = db;
    wave_lds_sync();                      // P / Z reads done before the next frame's writes
  }
}

// ---------------------------------------------------------------------------
// 16 kHz preset (n_fft 512): register FFT, four frames per wavefront.
//
// A 16-lane row of the wave owns one frame; the 256-point complex FFT of
// z[m] = w x[2m] + i w x[2m+1] is a four-step 16 x 16 FFT with m = 16 a + b:
//   1. lane b: 16-point DFT over a of z[16 a + b] (in registers; its 16
//      samples are 16 float2 loads, the row's 16 lanes reading 128 contiguous
//      bytes per a);
//   2. times W256^(b k1) (per-lane constants, loaded once);
//   3. one transpose through LDS (8 ds_write_b128 + 16 ds_read_b64 per lane),
//      then lane k1: 16-point DFT over b -> Z[k1 + 16 k2], k2 = 0..15;
//   4. real-input unpack in pairs (k, N2 - k): lane c takes k2 = 0..7 and
//      gets the partner lane's (16 - c) values by 8 cross-lane permutes; both
//      bins of a pair come from one E / W^k O (|X[N2 - k]| = |E - W^k O|).
// The power spectrum (bit-identical to the Stockham kernel's formula given
// the same Z) goes to LDS; lane b then sums mel bands b, 31 - b, 32 + b,
// 63 - b (balanced widths) in bin order, dB, bn0, store.
// Two LDS round trips per four frames instead of four per frame, and every
// FFT stage has 16 independent complex values per lane.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  const float2 s02 = cadd(a0, a2), d02 = csub(a0, a2);
  const float2 s13 = cadd(a1, a3), d13 = csub(a1, a3);
  a0 = cadd(s02, s13);
  a2 = csub(s02, s13);
  a1 = make_float2(d02.x + d13.y, d02.y - d13.x);   // d02 - i d13
  a3 = make_float2(d02.x - d13.y, d02.y + d13.x);   // d02 + i d13
}

// X[k] = sum_n x[n] W16^(n k), natural order in and out (4 x 4)
__device__ __forceinline__ void dft16(float2 (&x)[16]) {
  constexpr float C1 = 0.92387953251128674f, S1 = 0.38268343236508978f, R2 = 0.70710678118654757f;
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) dft4(x[n2], x[4 + n2], x[8 + n2], x[12 + n2]);
  // x[4 k1 + n2] now holds y[n2][k1]; twiddle by W16^(n2 k1)
  auto w1 = [](float2 a) { return make_float2(C1 * a.x + S1 * a.y, C1 * a.y - S1 * a.x); };   // W^1
  auto w2 = [](float2 a) { return make_float2(R2 * (a.x + a.y), R2 * (a.y - a.x)); };         // W^2
  auto w3 = [](float2 a) { return make_float2(S1 * a.x + C1 * a.y, S1 * a.y - C1 * a.x); };   // W^3
  auto w4 = [](float2 a) { return make_float2(a.y, -a.x); };                                  // W^4 = -i
  auto w6 = [](float2 a) { return make_float2(R2 * (a.y - a.x), -R2 * (a.x + a.y)); };        // W^6
  auto w9 = [](float2 a) { return make_float2(-C1 * a.x - S1 * a.y, S1 * a.x - C1 * a.y); };  // W^9
  x[5] = w1(x[5]);
  x[9] = w2(x[9]);
  x[13] = w3(x[13]);
  x[6] = w2(x[6]);
  x[10] = w4(x[10]);
  x[14] = w6(x[14]);
  x[7] = w3(x[7]);
  x[11] = w6(x[11]);
  x[15] = w9(x[15]);
  // DFT4 over n2 for each k1: inputs x[4 k1 + n2], outputs X[k1 + 4 k2]
  float2 y[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) y[i] = x[i];
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    float2 a0 = y[4 * k1], a1 = y[4 * k1 + 1], a2 = y[4 * k1 + 2], a3 = y[4 * k1 + 3];
    dft4(a0, a1, a2, a3);
    x[k1] = a0;
    x[k1 + 4] = a1;
    x[k1 + 8] = a2;
    x[k1 + 12] = a3;
  }
}

constexpr int FE16_WAVES = 4;
constexpr int FE16_ROW = 36;                       // floats per transpose row (16 float2 + pad)
// floats per frame (transpose, then power).  592 = 16 mod 64: the four frames
// of a wave start 16 banks apart (band-sum path); 596 = 20 mod 64: the 16
// frames of a workgroup start 20 banks apart, so the MFMA mel path's A
// fragment reads (lane: frame l & 15, bin + (l >> 4)) hit 64 distinct banks
template <bool MT>
constexpr int fe16_frame() { return MT ? 16 * FE16_ROW + 20 : 16 * FE16_ROW + 16; }
constexpr int FE16_MW = FE16_MEL_MW;               // widest mel band of the table path (bins, multiple of 4)
__device__ __forceinline__ int fe16_band(int b, int q) { return q == 0 ? b : q == 1 ? 31 - b : q == 2 ? 32 + b : 63 - b; }
typedef float fe_f32x4 __attribute__((ext_vector_type(4)));

// MT (mel on the matrix pipe): the workgroup's 16 frames (4 waves x 4) meet
// in LDS after their FFTs; wave w then computes mel bands 16 w .. 16 w + 15
// of all 16 frames as v_mfma_f32_16x16x4_f32 over the bin range those bands
// cover (host table: per band tile the first bin and the 4-bin steps,
// weights [step][4 bins][16 bands], zero outside each band).  A band's value
// is the in-order fma chain over its bins from 0 (the MFMA is the in-order
// fma chain over its four k; zero weights leave the chain unchanged for the
// finite, non-negative powers), i.e. the band-sum path's bits, with ~1/4 of
// its instructions per frame.
template <bool I16, bool MT>
__global__ __launch_bounds__(64 * FE16_WAVES) void logmel512_kernel(FrontendParams p) {
  constexpr int NFFT = 512, N2 = 256;
  constexpr int FE16_FRAME = fe16_frame<MT>();
  __shared__ __attribute__((aligned(16))) float s_fr[FE16_WAVES][4 * FE16_FRAME];
  extern __shared__ float s_melw[];   // [p.mel_lds_floats]: per-band weights, or the MT table
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane >> 4, b = lane & 15;
  const int nnz = p.mel_off[64];
  const bool mel_in_lds = nnz <= p.mel_lds_floats;
  if constexpr (MT) {
    for (int i = threadIdx.x; i < p.mt_floats; i += 64 * FE16_WAVES) s_melw[i] = p.mel_mt[i];
  } else {
    if (mel_in_lds && p.mel_wmax > FE16_MW)
      for (int i = threadIdx.x; i < nnz; i += 64 * FE16_WAVES) s_melw[i] = p.mel_w[i];
  }

  // per-lane constants: window of its 32 samples, step-2 twiddles W256^(b k1),
  // unpack twiddles W512^(b + 16 k2), its four mel bands.  The twiddle and
  // window tables are staged through the (not yet used) frame buffers with
  // coalesced loads, so each lane reads its constants from LDS
  float* stage = &s_fr[0][0];
  for (int i = threadIdx.x; i < NFFT; i += 64 * FE16_WAVES) {
    reinterpret_cast<float2*>(stage)[i] = p.twiddle[i];
    stage[2 * NFFT + i] = p.window[i];
  }
  __syncthreads();
  float win[32];
#pragma unroll
  for (int a = 0; a < 16; ++a) {
    const float2 wv = *reinterpret_cast<const float2*>(stage + 2 * NFFT + 32 * a + 2 * b);
    win[2 * a] = wv.x;
    win[2 * a + 1] = wv.y;
  }
  float2 tw1[16], tw2[9];
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) tw1[k1] = reinterpret_cast<const float2*>(stage)[(2 * b * k1) & (NFFT - 1)];
#pragma unroll
  for (int k2 = 0; k2 < 9; ++k2) tw2[k2] = reinterpret_cast<const float2*>(stage)[b + 16 * k2];
  // mel constants: band-sum path, lane b of frame row g sums bands
  // fe16_band(b, q); MT path, lane l owns band 16 wave + (l & 15)
  constexpr int NQ = MT ? 1 : 4;
  int mlo[NQ], o0[NQ], o1[NQ];
  float bmu[NQ], bsc[NQ], bbi[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int m = MT ? 16 * wave + b : fe16_band(b, q);
    mlo[q] = p.mel_lo[m];
    o0[q] = p.mel_off[m];
    o1[q] = p.mel_off[m + 1];
    bmu[q] = p.bn_mean[m];
    bsc[q] = p.bn_scale[m];
    bbi[q] = p.bn_bias[m];
  }
  // band weights per (slot q, lane b), zero-padded to the widest band rounded
  // to 4 (host table; fma(P, 0, acc) == acc exactly for finite P, so the
  // padded chain gives the band's own bits)
  __shared__ __attribute__((aligned(16))) float s_wt[MT ? 4 : 4 * 16 * FE16_MW];
  const int wmax = p.mel_wmax;
  const bool mel_table = wmax <= FE16_MW;
  if constexpr (!MT) {
    static_assert((4 * 16 * FE16_MW) % (64 * FE16_WAVES) == 0, "table fill");
#pragma unroll
    for (int k = 0; k < 4 * 16 * FE16_MW / (64 * FE16_WAVES); ++k)
      s_wt[threadIdx.x + 64 * FE16_WAVES * k] = p.mel_tab[threadIdx.x + 64 * FE16_WAVES * k];
  }
  __syncthreads();

  const int total = p.n_clips * p.n_win * p.T;
  const int L = (int)p.sig_len;
  float* fb = s_fr[wave] + g * FE16_FRAME;   // this frame's LDS (transpose rows, then power)
  // samples of frame fr: v[2 a + e] = x[pos0 + 32 a + 2 b + e]
  auto load = [&](int fr, float* v) {
    if (fr >= total) {
#pragma unroll
      for (int i = 0; i < 32; ++i) v[i] = 0.0f;
      return;
    }
    const unsigned item = (unsigned)fr / (unsigned)p.T;
    const int t = fr - (int)item * p.T;
    const unsigned clip = item / (unsigned)p.n_win;
    const int w = (int)(item - clip * (unsigned)p.n_win);
    const int64_t wstart = p.win_start ? p.win_start[w] : 0;   // window table (any length), L2-resident
    const int64_t src_off = (int64_t)clip * p.clip_stride + wstart;
    const int64_t av64 = p.clip_len - wstart;
    const int avail = av64 > L ? L : (int)av64;
    const int pos0 = t * p.hop - N2;
    if (!I16 && pos0 >= 0 && pos0 + NFFT <= avail && ((src_off + pos0) & 1) == 0) {
      const float2* src = reinterpret_cast<const float2*>(p.audio + src_off + pos0) + b;
#pragma unroll
      for (int a = 0; a < 16; ++a) {
        const float2 q = src[16 * a];
        v[2 * a] = q.x;
        v[2 * a + 1] = q.y;
      }
      return;
    }
#pragma unroll
    for (int a = 0; a < 16; ++a)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        int j = pos0 + 32 * a + 2 * b + e;
        if (j < 0) j = -j;                           // reflect (F.pad mode='reflect')
        if (j >= L) j = 2 * (L - 1) - j;
        const bool ok = j < avail;                   // pad_truncate zeros
        const int jc = ok ? j : 0;
        if (I16)
          v[2 * a + e] = ok ? (float)((double)p.audio_i16[src_off + jc] / 32767.0) : 0.0f;
        else
          v[2 * a + e] = ok ? p.audio[src_off + jc] : 0.0f;
      }
  };

  // workgroup groups of 16 frames (4 per wave): every wave runs every group
  // of its workgroup (the MT path's barriers); frames past the end compute
  // on zeros and are not stored
  const int ngroups = (total + 3) >> 2;
  const int nwg = (ngroups + FE16_WAVES - 1) / FE16_WAVES;
  int G = (int)blockIdx.x;
  float v[32];
  if (G < nwg) load(4 * (FE16_WAVES * G + wave) + g, v);
  for (; G < nwg; G += (int)gridDim.x) {
    const int gi = FE16_WAVES * G + wave;
    const int fr = 4 * gi + g;
    if (!MT && gi >= ngroups) break;             // band-sum path: waves are independent
    float2 x[16];
#pragma unroll
    for (int a = 0; a < 16; ++a) x[a] = make_float2(v[2 * a] * win[2 * a], v[2 * a + 1] * win[2 * a + 1]);
    if (G + (int)gridDim.x < nwg) load(4 * (FE16_WAVES * (G + (int)gridDim.x) + wave) + g, v);   // next group, in flight
    // 1-2: DFT over a, twiddle W256^(b k1)
    dft16(x);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) x[k1] = cmul(x[k1], tw1[k1]);
    // 3: transpose (row b = lane, column k1) -> lane k1 reads column b
#pragma unroll
    for (int k1 = 0; k1 < 16; k1 += 2)
      *reinterpret_cast<float4*>(fb + b * FE16_ROW + 2 * k1) = make_float4(x[k1].x, x[k1].y, x[k1 + 1].x, x[k1 + 1].y);
    wave_lds_sync();
#pragma unroll
    for (int bb = 0; bb < 16; ++bb) x[bb] = *reinterpret_cast<const float2*>(fb + bb * FE16_ROW + 2 * b);
    dft16(x);   // x[k2] = Z[b + 16 k2]
    // 4: unpack pairs (k = b + 16 k2, N2 - k), k2 = 0..7 (+ k2 = 8 on lane 0:
    // bin 128).  Partner lane (16 - b) & 15 holds Z[N2 - k] at its 15 - k2;
    // lane 0 pairs with itself at (16 - k2) & 15.
    const int partner = (g << 4) | ((16 - b) & 15);
    wave_lds_sync();   // every lane's column reads done before power overwrites the rows
    float2 bzs[8];   // all 16 permutes issued before any use (one latency)
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      bzs[k2].x = __shfl(x[15 - k2].x, partner);
      bzs[k2].y = __shfl(x[15 - k2].y, partner);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k2 = 0; k2 < 9; ++k2) {
      float2 bz;
      if (k2 < 8) {
        bz = b == 0 ? x[(16 - k2) & 15] : bzs[k2];
      } else {
        bz = x[8];
      }
      const float2 A = x[k2];
      const float2 E2 = make_float2(A.x + bz.x, A.y - bz.y);   // 2 E
      const float2 D = make_float2(A.x - bz.x, A.y + bz.y);    // A - conj(Z[N2 - k])
      const float2 O2 = make_float2(D.y, -D.x);                // 2 O = -i D
      const float2 WO = cmul(tw2[k2], O2);
      const float2 Xa = cadd(E2, WO), Xb = csub(E2, WO);       // 2 X[k], 2 conj(X[N2 - k])
      const int k = b + 16 * k2;
      if (k2 < 8) {
        fb[k] = (Xa.x * Xa.x + Xa.y * Xa.y) * 0.25f;
        fb[N2 - k] = (Xb.x * Xb.x + Xb.y * Xb.y) * 0.25f;
      } else if (b == 0) {
        fb[N2 / 2] = (Xa.x * Xa.x + Xa.y * Xa.y) * 0.25f;
      }
    }
    if constexpr (MT) {
      // 5 (MT): the workgroup's 16 power spectra -> mel tile of this wave
      __syncthreads();
      const int fl = lane & 15, kq = lane >> 4;
      const int kl = p.mt_klo[wave], ns = p.mt_ns[wave];
      const float* Pf = &s_fr[0][0] + fl * FE16_FRAME + kl + kq;   // frame fl: wave fl >> 2, row fl & 3
      const float* Wt = s_melw + p.mt_off[wave] + lane;
      const int kmax = N2 - kl - kq;              // bins past N2 read bin N2 (finite; its weight is 0)
      fe_f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int st = 0; st < ns; ++st)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Pf[min(4 * st, kmax)], Wt[64 * st], acc, 0, 0, 0);
      // D[frame][band]: lane l register i holds frame 4 (l >> 4) + i, band 16 wave + (l & 15)
      const int band = 16 * wave + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float db = 10.0f * log10f(fmaxf(acc[i], 1e-10f));
        db = (db - bmu[0]) * bsc[0] + bbi[0];
        const int f = 16 * G + 4 * (lane >> 4) + i;
        if (f < total) p.out[(int64_t)f * 64 + band] = db;
      }
      __syncthreads();   // mel reads done before the next group's transpose writes
    } else {
    wave_lds_sync();
    // 5: mel bands (bin order fma chains, the four bands interleaved so
    // each step has 16 LDS reads in flight), dB, bn0
    float accq[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (mel_table) {
      for (int e = 0; e < wmax; e += 4) {
        float pw[4][4];
        float4 ww[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ww[q] = *reinterpret_cast<const float4*>(s_wt + (q * 16 + b) * FE16_MW + e);
#pragma unroll
          for (int j = 0; j < 4; ++j) pw[q][j] = fb[mlo[q] + e + j];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          accq[q] = fmaf(pw[q][0], ww[q].x, accq[q]);
          accq[q] = fmaf(pw[q][1], ww[q].y, accq[q]);
          accq[q] = fmaf(pw[q][2], ww[q].z, accq[q]);
          accq[q] = fmaf(pw[q][3], ww[q].w, accq[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float acc = accq[q];
      if (mel_table) {
      } else if (mel_in_lds) {
        for (int i = o0[q]; i < o1[q]; i += 4) {
          float pw[4], ww[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool ok = i + e < o1[q];
            pw[e] = ok ? fb[mlo[q] + (i + e - o0[q])] : 0.f;
            ww[e] = ok ? s_melw[i + e] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (i + e < o1[q]) acc = fmaf(pw[e], ww[e], acc);
        }
      } else {
        for (int i = o0[q]; i < o1[q]; ++i) acc = fmaf(fb[mlo[q] + (i - o0[q])], p.mel_w[i], acc);
      }
      float db = 10.0f * log10f(fmaxf(acc, 1e-10f));
      db = (db - bmu[q]) * bsc[q] + bbi[q];
      if (fr < total) p.out[(int64_t)fr * 64 + fe16_band(b, q)] = db;
    }
    wave_lds_sync();   // power reads done before the next group's transpose writes
    }
  }
}

// at most the resident workgroups of the chip; every wave walks several
// frames, so the register prefetch of the next frame overlaps the current FFT
// (launch facts per device: launch_info)
// room for the packed mel weights: at most 2 (n_fft/2 + 1) floats (each bin
// in at most two triangular bands), rounded to 256 B
template <int NFFT>
constexpr size_t fe_mel_lds() { return ((size_t)2 * (NFFT / 2 + 1) * 4 + 255) / 256 * 256; }
// the kernel's static LDS: twiddles, window, two FFT buffers per wave
template <int NFFT>
constexpr size_t fe_static_lds() {
  return (size_t)NFFT * 8 + NFFT * 4 + (size_t)FE_WAVES * 2 * fe_buf_len<NFFT / 2>() * 8;
}

template <int NFFT, bool I16>
static void launch_logmel_t(const FrontendParams& p0, int64_t total, hipStream_t s) {
  const LaunchInfo li =
      launch_info(reinterpret_cast<const void*>(logmel_kernel<NFFT, I16>), 64 * FE_WAVES, fe_mel_lds<NFFT>());
  if (!li.ok) return;
  FrontendParams p = p0;
  p.mel_lds_floats = (int32_t)(li.dyn / 4);
  // the frame loop is LDS-latency bound (PMC: VALU busy ~27 %), so fill the
  // CU: as many 16-wave workgroups as its 160 KB LDS holds, up to 32 waves
  // (the occupancy query assumes 64 KB of LDS per CU on this part)
  constexpr int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(2, (int64_t)(160 * 1024) /
                                                                       (int64_t)(fe_static_lds<NFFT>() +
                                                                                 fe_mel_lds<NFFT>())));
  int64_t blocks = (total + FE_WAVES - 1) / FE_WAVES;
  blocks = std::min<int64_t>(blocks, (int64_t)li.ncu * per_cu);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((logmel_kernel<NFFT, I16>), dim3((unsigned)blocks), dim3(64 * FE_WAVES), li.dyn, s, p);
}

// one wave per four frames; every wave walks several groups so the register
// prefetch of the next group overlaps the current one
template <bool I16, bool MT>
static void launch_logmel512(const FrontendParams& p0, int64_t total, hipStream_t s) {
  const size_t dyn = MT ? ((size_t)p0.mt_floats * 4 + 255) / 256 * 256 : fe_mel_lds<512>();
  const LaunchInfo li = launch_info(reinterpret_cast<const void*>(logmel512_kernel<I16, MT>), 64 * FE16_WAVES,
                                    MT ? FE_MT_MAX_FLOATS * 4 : fe_mel_lds<512>());
  if (!li.ok) return;
  FrontendParams p = p0;
  p.mel_lds_floats = (int32_t)((MT ? dyn : li.dyn) / 4);
  const int64_t groups = (total + 3) / 4;
  int64_t blocks = (groups + FE16_WAVES - 1) / FE16_WAVES;
  // register-limited to 2 waves per SIMD (~215 VGPRs): two 4-wave workgroups
  // per CU (82 KB of the 160 KB LDS; the occupancy query assumes 64 KB per CU
  // and would say one)
  blocks = std::min<int64_t>(blocks, (int64_t)li.ncu * 2);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((logmel512_kernel<I16, MT>), dim3((unsigned)blocks), dim3(64 * FE16_WAVES), MT ? dyn : li.dyn,
                     s, p);
}

void launch_logmel(const FrontendParams& p, int n_fft, hipStream_t s) {
  const int64_t total = (int64_t)p.n_clips * p.n_win * p.T;
  if (total >= ((int64_t)1 << 31) - 4 ||p.sig_len >= (int64_t)1 << 31) return note_launch_error(hipErrorInvalidValue);
  const bool i16 = p.audio_i16 != nullptr;
  switch (n_fft) {
    case 256:
      if (i16) launch_logmel_t<256, true>(p, total, s);
      else launch_logmel_t<256, false>(p, total, s);
      break;
    case 512:
      // the MFMA mel path when the host built its table (melW bands fit)
      if (p.mel_mt && p.mt_floats <= FE_MT_MAX_FLOATS) {
        if (i16) launch_logmel512<true, true>(p, total, s);
        else launch_logmel512<false, true>(p, total, s);
      } else {
        if (i16) launch_logmel512<true, false>(p, total, s);
        else launch_logmel512<false, false>(p, total, s);
      }
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
// Gammatone frontend (nfft = 2048 at 32 kHz, 1024 at 16 kHz, 512 at 8 kHz),
// float64 throughout like the reference's numpy path:
//   specgram (fftweight.py:33-60): frames b in range(0, s - n, h), un-centred,
//     u = win * x[b:b+n] (float64 window x float32 samples), t = fft(u)[:n/2+1]
//   fft_gtgram (:126-168): W . |specgram| / nfft
//   power_to_db (features.py:363, ref 1.0, amin 1e-10, top_db 80)
//   float32_to_int16 / int16_to_float32 (utilities.py:73-79)
// Three launches: gamma_spec_kernel (one 256-thread workgroup per frame:
// Stockham FFT in LDS, |X| rows to HBM), gamma_erb_kernel (the dense
// 64 x (nfft/2+1) ERB product as a float64 GEMM over 64-frame tiles, dB and
// the per-clip max / min in its epilogue), gamma_quant_kernel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double2 zmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 zadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 zsub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

// Stockham FFT of N2 complex points by P threads of the block (block
// barriers).  The twiddles a thread multiplies by depend only on its thread
// index and the stage, so they live in registers (ZTw slots, loaded once per
// launch from the host table): the LDS holds just the two FFT buffers.
template <int N2, int Ns>
constexpr int zradix() { return ((N2 / Ns) % 4 == 0) ? 4 : 2; }
// register slots of the stages from Ns on (butterflies per thread x (R - 1))
template <int N2, int Ns, int P>
constexpr int zslots() {
  if constexpr (Ns >= N2) {
    return 0;
  } else {
    constexpr int R = zradix<N2, Ns>();
    constexpr int nb = N2 / R;
    constexpr int bpt = (nb + P - 1) / P;
    return (Ns > 1 ? bpt * (R - 1) : 0) + zslots<N2, Ns * R, P>();
  }
}
template <int N2, int Ns, int P, int OFF, int NT>
__device__ __forceinline__ void zload_tw(const double2* __restrict__ g_tw, double2 (&tw)[NT], int tid) {
  if constexpr (Ns < N2) {
    constexpr int NFFT = 2 * N2;
    constexpr int R = zradix<N2, Ns>();
    constexpr int nb = N2 / R;
    constexpr int bpt = (nb + P - 1) / P;
    constexpr int step = NFFT / (Ns * R);
    if constexpr (Ns > 1) {
#pragma unroll
      for (int bb = 0; bb < bpt; ++bb) {
        const int j = bb * P + tid;
        const int k = j & (Ns - 1);
#pragma unroll
        for (int r = 1; r < R; ++r) tw[OFF + bb * (R - 1) + r - 1] = j < nb ? g_tw[r * k * step] : make_double2(0.0, 0.0);
      }
    }
    zload_tw<N2, Ns * R, P, OFF + (Ns > 1 ? bpt * (R - 1) : 0)>(g_tw, tw, tid);
  }
}
template <int N2, int Ns, int P, int OFF, int NT>
__device__ __forceinline__ double2* zstockham(double2* X, double2* Y, const double2 (&tw)[NT], int tid) {
  if constexpr (Ns >= N2) {
    return X;
  } else {
    constexpr int R = zradix<N2, Ns>();
    constexpr int nb = N2 / R;
    constexpr int bpt = (nb + P - 1) / P;
#pragma unroll
    for (int bb = 0; bb < bpt; ++bb) {
      const int j = bb * P + tid;
      if (j >= nb) break;
      const int k = j & (Ns - 1);
      const int base = (j - k) * R + k;
      if constexpr (R == 4) {
        double2 v0 = X[j], v1 = X[j + nb], v2 = X[j + 2 * nb], v3 = X[j + 3 * nb];
        if constexpr (Ns > 1) {
          v1 = zmul(v1, tw[OFF + bb * 3]);
          v2 = zmul(v2, tw[OFF + bb * 3 + 1]);
          v3 = zmul(v3, tw[OFF + bb * 3 + 2]);
        }
        const double2 a0 = zadd(v0, v2), a1 = zsub(v0, v2);
        const double2 b0 = zadd(v1, v3), b1 = zsub(v1, v3);
        const double2 mib1 = make_double2(b1.y, -b1.x);
        Y[base] = zadd(a0, b0);
        Y[base + Ns] = zadd(a1, mib1);
        Y[base + 2 * Ns] = zsub(a0, b0);
        Y[base + 3 * Ns] = zsub(a1, mib1);
      } else {
        double2 v0 = X[j], v1 = X[j + nb];
        if constexpr (Ns > 1) v1 = zmul(v1, tw[OFF + bb]);
        Y[base] = zadd(v0, v1);
        Y[base + Ns] = zsub(v0, v1);
      }
    }
    __syncthreads();
    return zstockham<N2, Ns * R, P, OFF + (Ns > 1 ? bpt * (R - 1) : 0)>(Y, X, tw, tid);
  }
}

// Real-input spectrum bin k (0..N2) from the N2-point complex FFT Z of the
// packed sequence z[m] = x[2m] + i x[2m+1].
template <int N2>
__device__ __forceinline__ double2 zreal_bin(const double2* Z, double2 twk, int k) {
  const double2 A = Z[k & (N2 - 1)];
  const double2 Bz = Z[(N2 - k) & (N2 - 1)];
  const double2 E = make_double2(0.5 * (A.x + Bz.x), 0.5 * (A.y - Bz.y));
  const double2 O = make_double2(0.5 * (A.y + Bz.y), -0.5 * (A.x - Bz.x));
  return zadd(E, zmul(twk, O));
}

constexpr int GAMMA_SPEC_THREADS = 256;

template <int NFFT>
constexpr size_t gamma_spec_lds() {   // the two FFT buffers
  return (size_t)NFFT * sizeof(double2);
}

// One workgroup per frame at a time, walking frames.  Thread tid owns the
// packed complex samples m = tid + 256 i: their window values, every
// twiddle of its butterflies and of its unpack bins stay in registers for
// the whole launch (LDS holds only the FFT buffers: several workgroups per
// CU), and the next frame's samples are loaded while the current frame is
// transformed.
template <int NFFT>
__global__ __launch_bounds__(GAMMA_SPEC_THREADS) void gamma_spec_kernel(GammaParams p) {
  constexpr int N2 = NFFT / 2;
  constexpr int NB = N2 + 1;
  constexpr int P = GAMMA_SPEC_THREADS;
  constexpr int PER = N2 / P;                                  // packed samples per thread
  constexpr int NT = zslots<N2, 1, P>();
  constexpr int UB = (NB + P - 1) / P;                         // unpack bins per thread
  static_assert(N2 % P == 0, "whole packed samples per thread");
  extern __shared__ double2 s_gdyn[];
  double2* X = s_gdyn;                                         // [N2]
  double2* Y = X + N2;                                         // [N2]
  const int tid = threadIdx.x;
  double2 tw[NT > 0 ? NT : 1];
  if constexpr (NT > 0) zload_tw<N2, 1, P, 0>(p.twiddle, tw, tid);
  double2 twu[UB];
#pragma unroll
  for (int i = 0; i < UB; ++i) {
    const int k = tid + P * i;
    twu[i] = k < NB ? p.twiddle[k] : make_double2(0.0, 0.0);
  }
  double2 wv[PER];                                             // window of this thread's samples
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int m = tid + P * i;
    wv[i] = make_double2(p.window[2 * m], p.window[2 * m + 1]);
  }
  const int64_t total = (int64_t)p.B * p.T;
  // samples of frame fr (zeros past the filled frames: the row is zeroed)
  auto load = [&](int64_t fr, float2 (&v)[PER]) {
    const int64_t b = fr / p.T;
    const int t = (int)(fr - b * p.T);
    if (fr >= total || t >= p.T_fill) {
#pragma unroll
      for (int i = 0; i < PER; ++i) v[i] = make_float2(0.f, 0.f);
      return;
    }
    const float* src = p.audio + b * p.L + (int64_t)t * p.hop;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int m = tid + P * i;
      v[i] = make_float2(src[2 * m], src[2 * m + 1]);
    }
  };
  float2 v[PER];
  int64_t fr = blockIdx.x;
  load(fr, v);
  for (; fr < total; fr += gridDim.x) {
    const int64_t b = fr / p.T;
    const int t = (int)(fr - b * p.T);
    double* row = p.mag + fr * p.kp;
    if (t >= p.T_fill) {        // column never written by specgram's loop: zeros
      for (int k = tid; k < p.kp; k += P) row[k] = 0.0;
      load(fr + gridDim.x, v);
      continue;
    }
    const double2* Z;
    if constexpr (PER == 4 && zradix<N2, 1>() == 4 && N2 / 4 == P) {
      // (nfft 2048) the first radix-4 stage's butterfly of thread tid reads
      // exactly the samples it owns (m = tid + 256 i): computed from its
      // registers, so the windowed frame never goes through LDS (one LDS
      // write + read pass and one barrier fewer per frame)
      double2 u[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) u[i] = make_double2(wv[i].x * (double)v[i].x, wv[i].y * (double)v[i].y);
      load(fr + gridDim.x, v);  // next frame's samples, in flight during this FFT
      const double2 a0 = zadd(u[0], u[2]), a1 = zsub(u[0], u[2]);
      const double2 b0 = zadd(u[1], u[3]), b1 = zsub(u[1], u[3]);
      const double2 mib1 = make_double2(b1.y, -b1.x);
      Y[4 * tid] = zadd(a0, b0);
      Y[4 * tid + 1] = zadd(a1, mib1);
      Y[4 * tid + 2] = zsub(a0, b0);
      Y[4 * tid + 3] = zsub(a1, mib1);
      __syncthreads();
      Z = zstockham<N2, 4, P, 0>(Y, X, tw, tid);
    } else {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int m = tid + P * i;
        X[m] = make_double2(wv[i].x * (double)v[i].x, wv[i].y * (double)v[i].y);
      }
      load(fr + gridDim.x, v);  // next frame's samples, in flight during this FFT
      __syncthreads();
      Z = zstockham<N2, 1, P, 0>(X, Y, tw, tid);
    }
#pragma unroll
    for (int i = 0; i < UB; ++i) {
      const int k = tid + P * i;
      if (k < NB) {
        const double2 Xk = zreal_bin<N2>(Z, twu[i], k);
        // numpy abs(complex) is hypot; sqrt(x^2 + y^2) with one fma is within an
        // ulp of it (the int16 codes are ~3e-5 relative apart: identical)
        row[k] = sqrt(fma(Xk.x, Xk.x, Xk.y * Xk.y));
      }
    }
    for (int k = NB + tid; k < p.kp; k += P) row[k] = 0.0;   // row padding
    __syncthreads();            // Z read before the next frame's writes
  }
}

// ---------------------------------------------------------------------------
// nfft 2048, one WAVE per frame (round 4, SEDX_TUNE_GAMMA_SPEC 1): the
// 1024-point complex FFT of the packed frame as a 16 x 16 x 4 four-step in
// registers (each lane 16 complex values), with wave-local LDS transposes
// between the passes — no workgroup barrier, 16 values of independent work
// per lane.  m = l + 64 j (lane l holds j = 0..15), k = p + 16 q:
//   pass 1 (lane l):       Y[l][p]  = DFT16_j z[l + 64 j]  x  W1024^(l p)
//   pass 2 (lane 4 p + s): R[p][s][u] = DFT16_r Y[s + 4 r][p]  x  W64^(s u)
//   pass 3 (lane 4 p + w): Z[p + 16 u + 256 v] = DFT4_s R[p][s][u], u = 4 w + c
// then the real-spectrum unpack of bins l + 64 i (+ 1024) from Z[k] and
// Z[1024 - k] (a third transpose) and sqrt(fma) magnitudes, coalesced row
// stores.  The window and every twiddle a lane uses stay in its registers
// for the whole launch (one wave per SIMD).
__device__ __forceinline__ void zdft4(double2& x0, double2& x1, double2& x2, double2& x3) {
  const double2 a0 = zadd(x0, x2), a1 = zsub(x0, x2);
  const double2 b0 = zadd(x1, x3), b1 = zsub(x1, x3);
  const double2 mib1 = make_double2(b1.y, -b1.x);   // -i (x1 - x3)
  x0 = zadd(a0, b0);
  x1 = zadd(a1, mib1);
  x2 = zsub(a0, b0);
  x3 = zsub(a1, mib1);
}
// v[j] -> V[p] = sum_j v[j] W16^(j p), in place (natural order out);
// w16[k] = W16^k for k = 0..9 (only 1, 2, 3, 4, 6, 9 used)
__device__ __forceinline__ void zdft16(double2 (&v)[16], const double2 (&w16)[10]) {
  // j = j1 + 4 j2: DFT4 over j2 for each j1 -> a[j1][p2] (stored back in v[j1 + 4 p2])
#pragma unroll
  for (int j1 = 0; j1 < 4; ++j1) zdft4(v[j1], v[j1 + 4], v[j1 + 8], v[j1 + 12]);
  // twiddle a[j1][p2] by W16^(j1 p2)
#pragma unroll
  for (int j1 = 1; j1 < 4; ++j1)
#pragma unroll
    for (int p2 = 1; p2 < 4; ++p2) v[j1 + 4 * p2] = zmul(v[j1 + 4 * p2], w16[j1 * p2]);
  // DFT4 over j1 for each p2: V[p2 + 4 p1]
  double2 o[16];
#pragma unroll
  for (int p2 = 0; p2 < 4; ++p2) {
    double2 x0 = v[4 * p2], x1 = v[4 * p2 + 1], x2 = v[4 * p2 + 2], x3 = v[4 * p2 + 3];
    zdft4(x0, x1, x2, x3);
    o[p2] = x0;
    o[p2 + 4] = x1;
    o[p2 + 8] = x2;
    o[p2 + 12] = x3;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = o[i];
}

constexpr int GSW_WAVES = 4;                 // waves (frames in flight) per workgroup
constexpr int GSW_LD = 1024 + 64 + 16;       // complex per wave buffer (padded layouts below)
__global__ __launch_bounds__(64 * GSW_WAVES, 1) void gamma_spec_wave_kernel(GammaParams p) {
  extern __shared__ double2 s_gsw[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double2* buf = s_gsw + wave * GSW_LD;
  const int pp = lane >> 2, qs = lane & 3;   // pass 2 / 3 roles: (p, s) and (p, w)
  // registers for the whole launch: window of the lane's samples, twiddles
  double2 win[16], tw1[16], tw2[16], tw3[16], w16[10];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int m = lane + 64 * j;
    win[j] = make_double2(p.window[2 * m], p.window[2 * m + 1]);
    tw1[j] = p.twiddle[2 * ((lane * j) & 1023)];          // W1024^(l p), p = j
    tw2[j] = p.twiddle[32 * qs * j];                       // W64^(s u), u = j
    tw3[j] = p.twiddle[lane + 64 * j];                     // W2048^k, k = l + 64 i
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) w16[k] = p.twiddle[128 * k];
  const double2 twn = p.twiddle[1024 & (p.nfft - 1)];     // bin 1024 (W2048^1024 = -1)
  const int64_t total = (int64_t)p.B * p.T;
  const int64_t step = (int64_t)gridDim.x * GSW_WAVES;
  auto load = [&](int64_t fr, float2 (&v)[16]) {
    const int64_t b = fr / p.T;
    const int t = (int)(fr - b * p.T);
    if (fr >= total || t >= p.T_fill) {
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = make_float2(0.f, 0.f);
      return;
    }
    const float2* src = reinterpret_cast<const float2*>(p.audio + b * p.L + (int64_t)t * p.hop);
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = src[lane + 64 * j];
  };
  float2 xs[16];
  int64_t fr = (int64_t)blockIdx.x * GSW_WAVES + wave;
  load(fr, xs);
  for (; fr < total; fr += step) {
    const int64_t b = fr / p.T;
    const int t = (int)(fr - b * p.T);
    double* row = p.mag + fr * p.kp;
    if (t >= p.T_fill) {        // column never written by specgram's loop: zeros
      for (int k = lane; k < p.kp; k += 64) row[k] = 0.0;
      load(fr + step, xs);
      continue;
    }
    double2 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = make_double2(win[j].x * (double)xs[j].x, win[j].y * (double)xs[j].y);
    load(fr + step, xs);        // next frame's samples, in flight during this FFT
    // ---- pass 1: DFT16 over j, twiddle, transpose: buf[p * 65 + l] ----
    zdft16(v, w16);
#pragma unroll
    for (int q = 1; q < 16; ++q) v[q] = zmul(v[q], tw1[q]);
#pragma unroll
    for (int q = 0; q < 16; ++q) buf[q * 65 + lane] = v[q];
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- pass 2: lane (p, s) reads Y[s + 4 r][p] = buf[p * 65 + s + 4 r] ----
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = buf[pp * 65 + qs + 4 * r];
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    zdft16(v, w16);
#pragma unroll
    for (int u = 1; u < 16; ++u) v[u] = zmul(v[u], tw2[u]);
    // R[p][s][u = 4 w + c] -> buf[(4 p + w) * 17 + 4 s + c]
#pragma unroll
    for (int u = 0; u < 16; ++u) buf[(4 * pp + (u >> 2)) * 17 + 4 * qs + (u & 3)] = v[u];
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- pass 3: lane (p, w) reads R[p][s][4 w + c] for s, c ----
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = buf[lane * 17 + i];   // v[4 s + c]
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // DFT4 over s for each c: Z[p + 16 (4 w + c) + 256 v] -> buf[k + (k >> 4)]
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double2 x0 = v[c], x1 = v[4 + c], x2 = v[8 + c], x3 = v[12 + c];
      zdft4(x0, x1, x2, x3);
      const int k0 = pp + 16 * (4 * qs + c);
      buf[k0 + (k0 >> 4)] = x0;
      buf[k0 + 256 + ((k0 + 256) >> 4)] = x1;
      buf[k0 + 512 + ((k0 + 512) >> 4)] = x2;
      buf[k0 + 768 + ((k0 + 768) >> 4)] = x3;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- unpack bins l + 64 i (and 1024 on lane 0), magnitudes ----
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = lane + 64 * i;
      const int kn = (1024 - k) & 1023;
      const double2 A = buf[k + (k >> 4)];
      const double2 Bz = buf[kn + (kn >> 4)];
      const double2 E = make_double2(0.5 * (A.x + Bz.x), 0.5 * (A.y - Bz.y));
      const double2 O = make_double2(0.5 * (A.y + Bz.y), -0.5 * (A.x - Bz.x));
      const double2 Xk = zadd(E, zmul(tw3[i], O));
      row[k] = sqrt(fma(Xk.x, Xk.x, Xk.y * Xk.y));
    }
    if (lane == 0) {            // bin 1024: A = Bz = Z[0]
      const double2 A = buf[0];
      const double2 E = make_double2(A.x, 0.0);
      const double2 O = make_double2(A.y, 0.0);
      const double2 Xk = zadd(E, zmul(twn, O));
      row[1024] = sqrt(fma(Xk.x, Xk.x, Xk.y * Xk.y));
    }
    for (int k = 1025 + lane; k < p.kp; k += 64) row[k] = 0.0;   // row padding
    __builtin_amdgcn_wave_barrier();   // this frame's reads before the next frame's writes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

__device__ __forceinline__ unsigned long long d2ord(double d) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double ord2d(unsigned long long u) {
  return __longlong_as_double((long long)((u & 0x8000000000000000ull) ? (u & 0x7fffffffffffffffull) : ~u));
}

// db[b][ch][t] = 10 log10(max(1e-10, sum_k W[ch][k] |X_t[k]| / nfft)) over a
// tile of 64 frames of one clip x 64 channels on the f64 matrix pipe:
// v_mfma_f64_16x16x4f64, wave w = frames 16 w .. 16 w + 15 x the 4
// 16-channel tiles, K in 4-bin steps (one A and four B ds_read_b64 per 4
// MFMAs; the VALU form of this product was LDS-bandwidth bound at 4 B per
// FMA).  K staged in blocks of 32 bins: LDS double buffer, loads issued two
// blocks ahead into registers (the magnitudes stream from HBM: one block's
// MFMAs are shorter than a load's latency), one barrier per block.  Two
// workgroups per CU.  The int16 codes are
// checked against the reference's (test_gamma*): f64 sums in a different
// order move a value by ~1e-16 relative, a code step is ~3e-5 relative.
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int ERB_TF = 64, ERB_KB = 32;
__global__ __launch_bounds__(256) void gamma_erb_kernel(GammaParams p) {
  __shared__ __attribute__((aligned(16))) double As[2][ERB_KB][ERB_TF];   // [k][frame]
  __shared__ __attribute__((aligned(16))) double Ws[2][ERB_KB][64];       // [k][channel]
  __shared__ double s_red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t b = blockIdx.y;
  const int t0 = blockIdx.x * ERB_TF;
  const double* M = p.mag + b * (int64_t)p.T * p.kp;
  // staging roles: A: frame lf, bins lk .. lk + 7 of the block; W: 8
  // contiguous doubles of the [k][64] block
  const int lf = tid >> 2, lk = (tid & 3) * 8;
  const bool frame_ok = t0 + lf < p.T;
  const double* arow = M + (int64_t)(frame_ok ? t0 + lf : 0) * p.kp + lk;
  // register stages: blocks kb + 1, kb + 2 (native vectors: HIP's double2
  // struct copies kept these in scratch)
  typedef double d2v __attribute__((ext_vector_type(2)));
  d2v ra[2][4], rw[2][4];
  auto gload = [&](int k0, int r) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      ra[r][j] = frame_ok ? *reinterpret_cast<const d2v*>(arow + k0 + 2 * j) : d2v{0.0, 0.0};
    const d2v* wsrc = reinterpret_cast<const d2v*>(p.weightsT + (int64_t)k0 * 64) + 4 * tid;
#pragma unroll
    for (int j = 0; j < 4; ++j) rw[r][j] = wsrc[j];
  };
  auto swrite = [&](int buf, int r) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      As[buf][lk + 2 * j][lf] = ra[r][j][0];
      As[buf][lk + 2 * j + 1][lf] = ra[r][j][1];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) reinterpret_cast<d2v*>(&Ws[buf][0][0])[4 * tid + j] = rw[r][j];
  };
  f64x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int kq = lane >> 4, c16 = lane & 15;
  const int nkb = p.kp / ERB_KB;                 // kp is a multiple of 32
  gload(0, 0);
  if (nkb > 1) gload(ERB_KB, 1);
  swrite(0, 0);
  __syncthreads();
  // block kb: LDS buffer kb & 1; register stage (kb + 1) & 1 holds block kb + 1.
  // Blocks in pairs so every register-stage index is a compile-time constant
  // (a runtime index would put the stages in scratch memory)
  auto block = [&](int kb, auto par) __attribute__((always_inline)) {   // inlined: ra / rw stay in VGPRs
    constexpr int PAR = decltype(par)::value;    // kb & 1
    if (kb >= nkb) return;
    if (kb + 2 < nkb) gload((kb + 2) * ERB_KB, PAR);   // two blocks ahead (stage PAR was written out)
#pragma unroll
    for (int st = 0; st < ERB_KB / 4; ++st) {
      // A[m = frame][k]: lane (kq, m = c16); B[k][n = channel]: lane (kq, n = c16)
      const double a = As[PAR][4 * st + kq][16 * w + c16];
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Ws[PAR][4 * st + kq][16 * n + c16], acc[n], 0, 0, 0);
    }
    if (kb + 1 < nkb) swrite(PAR ^ 1, PAR ^ 1);  // the other buffer: last read in block kb - 1
    __syncthreads();
  };
  for (int kb = 0; kb < nkb; kb += 2) {
    block(kb, std::integral_constant<int, 0>{});
    block(kb + 1, std::integral_constant<int, 1>{});
  }
  // D[frame][channel] (f64 16x16 layout, cdna_hip_programming.md): lane
  // (q = lane >> 4, c16) register i holds frame 16 w + q + 4 i, channel 16 n + c16
  double mx = -INFINITY, mn = INFINITY;
  const double nfft = (double)p.nfft;
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = t0 + 16 * w + kq + 4 * i;
      if (t >= p.T) continue;
      const double g = acc[n][i] / nfft;
      const double db = 10.0 * log10(fmax(1e-10, g));   // - 10 log10(max(amin, ref=1)) == 0
      p.db[(b * 64 + 16 * n + c16) * p.T + t] = db;
      mx = fmax(mx, db);
      mn = fmin(mn, db);
    }
  // block max / min -> one atomic each per tile (every tile lies in one clip)
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmax(mx, __shfl_xor(mx, o));
    mn = fmin(mn, __shfl_xor(mn, o));
  }
  if (lane == 0) {
    s_red[0][w] = mx;
    s_red[1][w] = mn;
  }
  __syncthreads();
  if (tid == 0) {
    mx = fmax(fmax(s_red[0][0], s_red[0][1]), fmax(s_red[0][2], s_red[0][3]));
    mn = fmin(fmin(s_red[1][0], s_red[1][1]), fmin(s_red[1][2], s_red[1][3]));
    atomicMax(&p.mm[2 * b], d2ord(mx));
    atomicMin(&p.mm[2 * b + 1], d2ord(mn));
  }
}

__global__ void gamma_init_kernel(unsigned long long* mm, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) {
    mm[2 * i] = 0ull;
    mm[2 * i + 1] = ~0ull;
  }
}

// power_to_db's top_db clamp, float32_to_int16 (per-clip max |x| scaling,
// x 32767, truncation toward zero by astype(int16)), int16_to_float32 —
// all on the float64 dB values.
__global__ __launch_bounds__(256) void gamma_quant_kernel(GammaParams p) {
  const int64_t n = (int64_t)p.B * 64 * p.T;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / (64 * (int64_t)p.T);
    const double mx = ord2d(p.mm[2 * b]);
    const double mn = ord2d(p.mm[2 * b + 1]);
    const double floor_db = mx - 80.0;                 // log_spec.max() - top_db
    const double lo = fmax(mn, floor_db);
    const double maxabs = fmax(fabs(mx), fabs(lo));    // np.max(np.abs(x)) after the clamp
    double x = fmax(p.db[i], floor_db);
    if (maxabs > 1.0) x = x / maxabs;
    const double q = trunc(x * 32767.0);
    p.out[i] = (float)(q / 32767.0);
  }
}

int gamma_kp(int nfft) { return ((nfft / 2 + 1) + 31) / 32 * 32; }

size_t gamma_workspace_bytes(int64_t B, int64_t T, int nfft) {
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  return al((size_t)B * T * gamma_kp(nfft) * sizeof(double)) + al((size_t)B * 64 * T * sizeof(double)) +
         al((size_t)B * 2 * sizeof(unsigned long long));
}

template <int NFFT>
static void launch_gamma_spec(const GammaParams& p, hipStream_t s) {
  const void* k = reinterpret_cast<const void*>(gamma_spec_kernel<NFFT>);
  const LaunchInfo li = launch_info(k, GAMMA_SPEC_THREADS, gamma_spec_lds<NFFT>());
  if (!li.ok) return;
  const int64_t total = (int64_t)p.B * p.T;
  int64_t blocks = std::min<int64_t>(total, (int64_t)li.ncu * li.per_cu * 4);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(gamma_spec_kernel<NFFT>, dim3((unsigned)blocks), dim3(GAMMA_SPEC_THREADS), li.dyn, s, p);
}

void launch_gamma(const GammaParams& p, hipStream_t s, int spec_variant) {
  hipLaunchKernelGGL(gamma_init_kernel, dim3((p.B + 255) / 256), dim3(256), 0, s, p.mm, p.B);
  if (p.nfft == 2048 && spec_variant == 1 && p.L % 2 == 0 && p.hop % 2 == 0) {   // float2 sample loads
    const void* k = reinterpret_cast<const void*>(gamma_spec_wave_kernel);
    const size_t lds = (size_t)GSW_WAVES * GSW_LD * sizeof(double2);
    const LaunchInfo li = launch_info(k, 64 * GSW_WAVES, lds);
    if (!li.ok) return;
    const int64_t frames = (int64_t)p.B * p.T;
    int64_t blocks = std::min<int64_t>((frames + GSW_WAVES - 1) / GSW_WAVES, (int64_t)li.ncu * li.per_cu);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(gamma_spec_wave_kernel, dim3((unsigned)blocks), dim3(64 * GSW_WAVES), li.dyn, s, p);
  } else if (p.nfft == 2048)
    launch_gamma_spec<2048>(p, s);
  else if (p.nfft == 1024)
    launch_gamma_spec<1024>(p, s);
  else if (p.nfft == 512)
    launch_gamma_spec<512>(p, s);
  else
    return note_launch_error(hipErrorInvalidValue);
  hipLaunchKernelGGL(gamma_erb_kernel, dim3((p.T + ERB_TF - 1) / ERB_TF, p.B), dim3(256), 0, s, p);
  hipLaunchKernelGGL(gamma_quant_kernel, dim3(2048), dim3(256), 0, s, p);
}

}  // namespace sedx
