// Internal declarations shared by the HIP translation units of libsedx.
// Layout conventions (all fp32, row-major, device memory):
//   wave      [items][L]                       (or per-item descriptors, window mode)
//   X0        [items][T][64]                   log-mel after bn0 (conv input, Cin=1, F=64)
//   act NHWC  [items][T][F][C]                 conv activations, channels innermost
//   seq       [items][T4][512]                 CNN output after freq-mean (GRU/MHA input)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdint.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "../../include/sedx.h"

namespace sedx {

// ---- frontend -------------------------------------------------------------
// logmel512_kernel: lane b of a frame's 16-lane row sums mel bands b, 31 - b,
// 32 + b, 63 - b (slots q = 0..3, balanced widths) from a zero-padded table
constexpr int FE16_MEL_MW = 36;
constexpr int FE_MT_MAX_FLOATS = 8192;    // MFMA mel table limit (32 KB of LDS)
inline int fe16_band_host(int b, int q) { return q == 0 ? b : q == 1 ? 31 - b : q == 2 ? 32 + b : 63 - b; }
struct FrontendParams {
  const float* audio;       // base pointer (fp32 samples)
  const int16_t* audio_i16; // or int16 samples, dequantised x / 32767 on load (utilities.py:78-79)
  int64_t clip_stride;      // samples between clips
  int32_t n_clips;          // items = n_clips * n_win
  int32_t n_win;            // windows per clip (1 in clip mode)
  const int64_t* win_start; // [n_win] device table of window sample offsets
                            // (the windowed driver's host table); nullptr: every item starts at 0
  int64_t clip_len;         // valid samples per clip (beyond => zeros; pad_truncate)
  int64_t sig_len;          // samples per item fed to the STFT (L or window length)
  int32_t T;                // frames per item = sig_len / hop + 1
  int32_t hop;
  const float2* twiddle;    // [n_fft] exp(-2 pi i m / n_fft)
  const float* window;      // [n_fft]
  const float* mel_w;       // packed band weights
  const int32_t* mel_off;   // [65] offsets into mel_w
  const int32_t* mel_lo;    // [64] first fft bin of each band
  int32_t mel_lds_floats;   // set by launch_logmel: LDS room for the packed mel weights
  const float* mel_tab;     // [4][16][FE16_MEL_MW] band weights of slot q, lane b (n_fft 512 kernel)
  int32_t mel_wmax;         // widest band rounded up to 4 (> FE16_MEL_MW: the per-band loop)
  // MFMA mel (n_fft 512): per 16-band tile j the first bin, the number of
  // 4-bin steps and the table offset; table [step][4 bins][16 bands] per tile
  const float* mel_mt;      // nullptr: the band-sum path
  int32_t mt_klo[4], mt_ns[4], mt_off[4];
  int32_t mt_floats;
  const float* bn_scale;    // [64] bn0 folded
  const float* bn_mean;     // [64]
  const float* bn_bias;     // [64]
  float* out;               // X0 [items][T][64]
};
void launch_logmel(const FrontendParams& p, int n_fft, hipStream_t s);

// gamma features [B][64][T] -> X0 [B][T][64] with bn0
void launch_features_bn0(const float* feat, int B, int T, const float* bn_scale,
                         const float* bn_mean, const float* bn_bias, float* out,
                         hipStream_t s);

// Gammatone frontend, float64 end to end like the reference's numpy
// (utils/gammatone/fftweight.py:126-168 computes in float64; power_to_db and
// float32_to_int16 run on that float64 array, utils/features.py:361-370).
struct GammaParams {
  const float* audio;      // [B][L] (float32 samples, as librosa.load returns)
  int64_t L;
  int32_t B, T, hop, nfft;
  int32_t T_fill;          // frames actually filled by specgram's range(0, s-n, h)
  int32_t kp;              // padded bin count (row stride of mag / rows of weightsT)
  const double2* twiddle;  // [nfft] exp(-2 pi i m / nfft)
  const double* window;    // [nfft] centred hann (specgram_window)
  const double* weightsT;  // [kp][64] ERB weights (fft_weights), zero rows past nfft/2
  double* mag;             // [B][T][kp] workspace: |FFT| (zero for unfilled frames)
  double* db;              // [B][64][T] workspace: 10 log10(max(1e-10, W.|X| / nfft))
  unsigned long long* mm;  // [B][2] workspace: ordered max / min of db per clip
  float* out;              // [B][64][T] dequantised features
};
int gamma_kp(int nfft);
// host: ERB weights [kp][nfilts] (zero rows past nfft/2), twiddles [2 nfft], window [nfft]
void gamma_tables(double fs, int nfft, int nwin, int nfilts, double fmin, std::vector<double>& weightsT,
                  int kp, std::vector<double>& twiddle, std::vector<double>& window);
size_t gamma_workspace_bytes(int64_t B, int64_t T, int nfft);
// spec_variant (nfft 2048): 0 the workgroup Stockham spectrum, 1 one wave per frame
void launch_gamma(const GammaParams& p, hipStream_t s, int spec_variant = 0);

// ---- conv stack -----------------------------------------------------------
// bn0 output X0 [B][T][64] -> zero-bordered [B][T+2][66] (block1_pad_floats)
void launch_pad_x0(const float* x0, int B, int T, float* xpad, hipStream_t s);
// exact block 1 in one launch: conv1 (w1 [64][9], b1 [64], BN folded) computed
// while conv2's halo is staged, conv2 + BN + ReLU + 2x2 avg-pool -> out
// [B][T/2][32][64]
void launch_block1_exact(const float* xpad, int B, int T, const float* w1, const float* b1, const float* wp,
                         const float* bias, float* out, const float* zero16, hipStream_t s);

enum ConvEpi { EPI_STORE = 0, EPI_POOL2 = 1, EPI_FMEAN = 2 };
// floats in the handle's device zero block (the halo DMA's source for pixels
// outside the clip; the Winograd DMA walks it by up to Cin + 4 floats)
constexpr int ZERO_BLOCK_FLOATS = 1024;
constexpr int CONV_SCHED_INTS = 256;   // per conv launch: 8 tile-claim counters, 128 B apart
// 3x3 conv (pad 1) + folded BN + ReLU (+ epilogue), implicit GEMM on fp32 MFMA.
//  in [B][T][F][Cin] -> EPI_STORE: [B][T][F][Cout], EPI_POOL2: [B][T/2][F/2][Cout],
//  EPI_FMEAN: [B][T][Cout].  wp = packed [Cin/4][9][2][Cout][2] (channel 2 ks + khalf), bias [Cout].
//  F in {32, 16, 8}, Cout % 128 == 0 (block 1 runs launch_block1_exact).
// zero16: >= 16 bytes of zeros in device memory (the halo DMA's source for
// pixels outside the clip).
void launch_conv3x3(const float* in, int B, int T, int F, int Cin, int Cout,
                    const float* wp, const float* bias, float* out, int epi,
                    const float* zero16, hipStream_t s);

// Same contract as fp32 Winograd F(2x2, 3x3) (conv_wino.hip): U from
// pack_conv_wino (wf = BN-folded weights [Cout][Cin][9] in float64);
// F in {64, 32, 16, 8}, Cout % 32 == 0 (F = 64: block 1's conv2, fed by
// launch_conv1_nhwc).
// zero16 here: >= Cin + 4 floats of zeros; trash: >= 64 x 128 floats of device scratch; out-of-range epilogue stores land
// there (every store is issued, so the persistent kernel's counted waits are exact).
// order: 1 = the 4 tile blocks x 8 channel groups round order on the
// 512-channel layers where it applies (SEDX_TUNE_WINO_ORDER), 0 = tile block
// major.  Same per-item work either way: bit-identical outputs.
void launch_conv3x3_wino(const float* in, int B, int T, int F, int Cin, int Cout,
                         const float* U, const float* bias, float* out, int epi,
                         const float* zero16, float* trash, hipStream_t s, int order = 0);
void pack_conv_wino(const double* wf, int Cin, int Cout, float* U);   // U: Cin * Cout * 16 floats
// Same contract as fp32 Winograd F(4x4,3x3) (conv_wino43.hip), blocks 2-4:
// F in {32, 16, 8}, Cin % 8 == 0 and >= 16, Cout % 64 == 0 and <= 512; U43
// from pack_conv_wino43 (2 Cin Cout 36 floats: the 64- and the 16-channel
// item packs); nt_force: 0 = the launcher's choice of item shape, 4 =
// 64-channel items, 1 = 16-channel items of 32 tiles, 2 = 16-channel items of
// 16 tiles (F = 16 / 8, c4 only) — A/B and tests, all bit-identical; pixels outside the clip are
// zero-filled by the buffer DMA's range check (no zero block); trash >= 64 x
// 128 floats of device scratch for the out-of-range epilogue stores.
// c4: input and output in the chunk-of-4 layout [B][C/4][T][F][4] (the
// freq-mean output stays [B][T][C]); else NHWC.  Batches are split over whole
// clips, so B-major offsets hold in both layouts.  sched: CONV_SCHED_INTS
// zeroed ints (item-claim counters; left zero by the launch) or nullptr =
// the static item order — the same outputs either way.
void launch_conv3x3_wino43(const float* in, int B, int T, int F, int Cin, int Cout, const float* U43,
                           const float* bias, float* out, int epi, float* trash, hipStream_t s, int order = 0,
                           bool c4 = false, int nt_force = 0, int* sched = nullptr);
// [B][C/4][T][F][4] -> [B][T][F][C] (stage captures of the C4 layers)
void launch_c4_to_nhwc(const float* src, int B, int T, int F, int C, float* dst, hipStream_t s);
void pack_conv_wino43(const double* wf, int Cin, int Cout, float* U);   // U: 2 * Cin * Cout * 36 floats
// block 1 as one Winograd launch: conv1 (w1 [64][9] folded, b1 [64], ReLU)
// computed into conv2's halo images in LDS, conv2 (U of block 1's conv2) +
// bias + ReLU + 2x2 pool: X0 [B][T][64] -> [B][T/2][32][64]; bit-identical to
// launch_conv1_nhwc followed by launch_conv3x3_wino
// c4: the pooled output in the chunk-of-4 layout [B][16][T/2][32][4] (the
// F(4x4,3x3) layers' input), else NHWC
void launch_block1_wino(const float* x0, int B, int T, const float* w1, const float* b1, const float* U,
                        const float* bias, float* out, const float* zero16, float* trash, hipStream_t s,
                        bool c4 = false);
// block 1's conv1 + BN + ReLU: X0 [B][T][64] -> [B][T][64][64] (w1 [64][9] folded, b1 [64])
void launch_conv1_nhwc(const float* x0, int B, int T, const float* w1, const float* b1, float* out,
                       hipStream_t s);
// the same conv1 into the chunk-of-4 layout [B][16][T][64][4] (conv_wino.hip)
void launch_conv1_c4(const float* x0, int B, int T, const float* w1, const float* b1, float* out, hipStream_t s);

// Same contract on bf16 MFMA with a 3-term hi/lo split (fp32-class accuracy).
// wp = host-packed split weights [Cout/BN][Cin/16][9][BN][4 x 16 B] (BN = 64 if
// Cout == 64 else 128), slots XOR-swizzled by ((n >> 2) & 3).
//
// packed FP32: no kernel of this library contains packed FP32 VALU
// instructions (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32); the Makefile
// compiles with -fno-slp-vectorize -fno-vectorize and `make isa-check`
// (tests/test_host_cpu.py) verifies every kernel's ISA.  Measured on MI355X
// (tools/fe_race.cpp, round 2): an FFT kernel whose float2 arithmetic the
// compiler had packed into v_pk_* produced wrong values in 16-27 of 64
// launches while an MFMA loop ran on the same CU from another stream (the
// round-1 "co-residency corruption"); the identical kernel compiled without
// packed FP32, 0 of 192.  The corruption needs only the two instruction kinds
// on one SIMD — any kernel with MFMAs whose own VALU code was packed (the x3
// fused block 1's conv1 chain, epilogues) was exposed to it through its own
// partner waves — so the fix is the instruction ban, not CU-exclusive LDS
// footprints (round 1's workaround, removed).
//
// Launch failures that happen while preparing a launch (attribute queries /
// hipFuncSetAttribute) are recorded per host thread and turned into
// SEDX_EHIP by the C ABI entry point that issued the work
// (take_launch_error); the launch is then skipped, never run with a
// different LDS footprint.
inline thread_local hipError_t t_launch_err = hipSuccess;
inline void note_launch_error(hipError_t e) {
  if (e != hipSuccess && t_launch_err == hipSuccess) t_launch_err = e;
}
inline hipError_t take_launch_error() {
  const hipError_t e = t_launch_err;
  t_launch_err = hipSuccess;
  return e;
}


// Per (device, kernel) launch facts, computed once under a mutex: the CU
// count, the kernel's workgroups per CU at its own LDS footprint, and the
// dynamic LDS to launch with.  ok == false: the attribute calls failed (the
// error was noted; callers skip the launch).
struct LaunchInfo {
  bool ok = false;
  int ncu = 0;
  int per_cu = 0;
  size_t dyn = 0;
};
// dyn_need: dynamic LDS the kernel uses (set as its maximum once).
// no_scratch: the kernel's counted vmcnt waits assume it issues no scratch
// (register spill) loads / stores, which would count in vmcnt too and make
// the waits too loose (LDS read before its DMA landed: silently wrong
// outputs).  A build that spills is refused here, loudly, instead.
inline LaunchInfo launch_info(const void* kernel, int block_threads, size_t dyn_need, bool no_scratch = false) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, LaunchInfo> cache;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    note_launch_error(e);
    return LaunchInfo{};
  }
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(dev, kernel);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  LaunchInfo li;
  if ((e = hipDeviceGetAttribute(&li.ncu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) {
    note_launch_error(e);
    return LaunchInfo{};
  }
  if (dyn_need && (e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)dyn_need)) != hipSuccess) {
    note_launch_error(e);
    return LaunchInfo{};
  }
  if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&li.per_cu, kernel, block_threads, dyn_need)) !=
      hipSuccess) {
    note_launch_error(e);
    return LaunchInfo{};
  }
  if (no_scratch) {
    hipFuncAttributes fa{};
    if ((e = hipFuncGetAttributes(&fa, kernel)) != hipSuccess) {
      note_launch_error(e);
      return LaunchInfo{};
    }
    if (fa.localSizeBytes != 0) {
      note_launch_error(hipErrorInvalidDeviceFunction);
      return LaunchInfo{};
    }
  }
  if (li.per_cu < 1) li.per_cu = 1;
  if (li.ncu < 1) li.ncu = 256;
  li.dyn = dyn_need;
  li.ok = true;
  cache[key] = li;
  return li;
}

// LDS-DMA of 16 B per lane: LDS[m0 + lane * 16] = *src.  Inline asm, so the
// compiler neither counts it nor guards LDS reads against it: the caller
// orders it with counted vmcnt waits before its barriers (its own waits for
// ordinary loads only get more conservative, never less).
__device__ __forceinline__ void sedx_glds16(const void* src, uint32_t m0) {
  // m0 is reserved to the compiler, which uses it nowhere else in the kernels
  // that call this (checked in their ISA); the clobber keeps it from caching
  // a value there
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
#pragma clang diagnostic pop
}

// hipLaunchKernelGGL after the per-device launch facts were established;
// skipped (error noted) if they could not be
template <typename... P, typename... A>
inline void launch_kernel(void (*kern)(P...), dim3 grid, int threads, hipStream_t s, A... args) {
  if (!launch_info(reinterpret_cast<const void*>(kern), threads, 0).ok) return;
  hipLaunchKernelGGL(kern, grid, dim3(threads), 0, s, args...);
}

// sched: CONV_SCHED_INTS zeroed ints per launch (the 8 per-XCD tile-claim counters)
void launch_conv3x3_x3(const float* in, int B, int T, int F, int Cin, int Cout, const void* wp,
                       const float* bias, float* out, int epi, int* sched, hipStream_t s);
// block 1 of the CNN in one conv launch (x3): with x0, pads the bn0 output
// into xpad (block1_pad_floats(B, T) floats); with out, runs conv2 with conv1
// computed while its halo is staged (conv_x3.hip)
void launch_block1_fused_x3(const float* x0, int B, int T, float* xpad, const float* w1, const float* b1,
                            const void* wp, const float* bias, float* out, int* sched, hipStream_t s);
size_t block1_pad_floats(int B, int T);

// ---- sequence / head ------------------------------------------------------
// C[M][N] = act(A[M][K] . W[N][K]^T + bias[N]);  act: 0 none, 1 relu
void launch_linear(const float* A, int M, int K, const float* W, int N, const float* bias,
                   float* C, int act, hipStream_t s);
// x3 (split-bf16 MFMA) GEMM, W pre-packed by the host (linear_x3.hip);
// K % 32 == 0, N % BN == 0, BN in {64, 128}
void launch_linear_x3(const float* A, int M, int K, const void* Wp, int N, int BN, const float* bias,
                      float* C, int act, hipStream_t s);

// bi-GRU recurrence.  G [B][T][1536] = x W_ih^T + b_ih (both dirs);
// whhT [2][256][768]; bhh [2][768]; H [B][T][512]
void launch_gru(const float* G, int B, int T, const float* whhT, const float* bhh, float* H,
                hipStream_t s);

// Cooperative bi-GRU recurrence (8 workgroups per (32-clip group, direction)
// exchanging h slices each step).  whh = W_hh [2][768][256] (natural layout);
// ws >= gru_coop_workspace_bytes(B) bytes of device scratch (counters + exchange).
size_t gru_coop_workspace_bytes(int B);
// exact: fp32 MFMA (else the x3 bf16 split); allow_fast: XCD-local hand-off
// when the placement allows it (else always the global protocol).
// host_err (nullable): host-mapped word OR-ed with the failure code when a
// bounded hand-off spin times out (outputs of that launch are then NaN).
// variant (exact, B > 8): 2 the 32-clip flag hand-off kernel (default; x3
// always), 0 the 16-clip data-tagged kernel with 16 slices, 1 with 8 slices,
// 3 the flag kernel on 16 slices, 4 the K-split hand-off on 16 slices.
// spin: bound of every hand-off spin in polls (the handle's SEDX_TUNE_GRU_SPIN, 2^24 by default).
// spread (flag kernels): a (group, direction)'s slices on every XCD instead of
// one (global protocol; bit-identical).
void launch_gru_coop(const float* G, int B, int T, const float* whh, const float* bhh, float* H,
                     void* ws, bool exact, bool allow_fast, int variant, unsigned* host_err, unsigned spin,
                     hipStream_t s, bool spread = false);

// MHA core: QKV [B][T][1536] (q|k|v, head h = cols 64h..64h+63) -> O [B][T][512]
void launch_mha(const float* QKV, int B, int T, float* O, hipStream_t s);

// AttBlock finish + framewise expansion.  logits [B][T][ldl] (0..C-1 att, C..2C-1 cla)
void launch_att_head(const float* logits, int B, int T, int C, int ldl, int out_frames,
                     float* framewise, float* clipwise, float* emb_cla, hipStream_t s);
// embedding for the Transformer model: E [B][T][D] -> emb [B][D][T]
void launch_transpose_btd(const float* E, int B, int T, int D, float* out, hipStream_t s);

// ---- windowed drivers (windows.cpp) ---------------------------------------
// loop control of predict.py:297-338 / main_strong.py:786-832: the sample
// offset of every window and the samples fed to the model for it
struct WindowLoop {
  std::vector<int64_t> start, len;
};
// nullptr on success, else why the reference's loop raises / never ends
const char* window_loop(int sample_rate, int64_t L_clip, const sedx_window_spec& sp, WindowLoop* out);
// utilities.merge replayed window by window on index lists, then avg_merge's
// divisors: merged frame f = left fold, in order, of the values with packed
// ids src[off[f] .. off[f+1]) (window w, frame t -> win_base[w] + t), divided
// by div[f] when div[f] > 1.
struct MergePlan {
  int64_t N = 0;
  std::vector<int32_t> win_base;   // [n_win + 1]
  std::vector<int32_t> off;        // [N + 1]
  std::vector<int32_t> src;
  std::vector<int32_t> div;        // [N]
};
const char* build_merge_plan(const std::vector<int64_t>& frames, int64_t step, int sample_duration, bool avg,
                             MergePlan* plan);
// GPU merge of every clip by one plan.  Window w of clip c has its framewise
// output at fw + wb[w] + c * wcs[w] (floats, frames of C classes); the plan's
// tables (off, src as (window, frame) int2, div) live in device memory.
// vote_thr != nullptr (device, [C] f64): every value binarised first (x >
// thr[k] in float64, pytorch/main_strong.py:870-883); the plan then carries
// no divisors (main_strong.py:1097 skips avg_merge).
struct MergeArgs {
  const float* fw;
  const int64_t* wb;      // [n_win] float offset of window w's clip-0 output
  const int64_t* wcs;     // [n_win] floats between clips for window w
  const int32_t* off;     // [N + 1]
  const int2* src;        // (window, frame)
  const int32_t* div;     // [N]
  const double* vote_thr;
  int32_t n_clips, N, C;
  float* merged;          // [n_clips][N][C]
};
void launch_merge_plan(const MergeArgs& a, hipStream_t s);

// ---- events (events.hip) --------------------------------------------------
struct EventArgs {
  const float* x;            // [N][T][C] framewise probabilities (mode 0) / vote counts (mode 1)
  int64_t N, T, C;
  const float* hi;           // [C] high threshold (mode 0)
  const double* lo;          // [C] low threshold
  const int64_t* n_smooth;   // [C]
  const int64_t* n_salt;     // [C]
  int32_t use_lo;
  int64_t step, sd;          // mode 1: int(100*overlap), sample_duration
  int64_t* counts;           // [N*C] scratch
  int64_t* slots;            // [N*C][slot_cap] (bgn, fin) int32 pairs, scratch
  int64_t slot_cap;          // events_slot_cap(T)
  int64_t* info;             // [2]: number of events, IndexError flag
  int32_t* events;           // [capacity][4] (clip, class, bgn, fin)
  int64_t capacity;
};
int64_t events_slot_cap(int64_t T);
int64_t events_max_frames();
size_t events_workspace_bytes(int64_t n_series, int64_t T, int64_t C);
void launch_events(const EventArgs& a, int mode, hipStream_t s);

}  // namespace sedx
