/*
 * sedx.h — C ABI of the MI355X-native sound-event-detection inference path.
 *
 * Drop-in boundary for the reference's hot path (yazdayy/sound-event-detection,
 * read-only at /root/reference).  The reference is pure Python/PyTorch; its
 * "plugin API" for this path is the model classes instantiated by name
 * (`Model = eval(model_type)`, pytorch/predict.py:229, pytorch/main_strong.py:529)
 * with a fixed constructor, `forward()` and state_dict.  Each entry point below
 * names the reference interface it replaces.  The host-side mirror of those
 * classes (sound-event-detection_amd/sedx/models.py) binds these symbols with
 * ctypes; INTEGRATION.md shows the binding a reference maintainer would add.
 *
 * Conventions
 *  - Plain pointers and sizes; no torch / HIP types.  `stream` is a
 *    hipStream_t passed as void* (NULL = the null stream).
 *  - All `d_*` pointers are device pointers on the handle's device, fp32,
 *    row-major, caller-owned.  `h_*` pointers are host memory.
 *  - Every call returns sedx_status; on failure sedx_last_error(h) holds a
 *    message (the Python shim raises RuntimeError with it), replacing the
 *    reference's Python exceptions (e.g. pytorch/models.py:139).
 *  - A handle is bound to one device and owns packed weights + a cached
 *    workspace.  Host calls on one handle must be serialised by the caller
 *    (the reference's DataParallel uses one replica per device, one thread
 *    each); the device work they issue may run concurrently on different
 *    streams when every such call passes its own d_workspace (the weights
 *    are read-only after sedx_finalize_weights).  Handles share no mutable
 *    state: calls on different handles (e.g. one per device, each from its
 *    own thread) need no coordination.
 */
#ifndef SEDX_H
#define SEDX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  SEDX_OK = 0,
  SEDX_EINVAL = 1,    /* bad argument / shape                     */
  SEDX_ENOMEM = 2,    /* device allocation failed                  */
  SEDX_EHIP = 3,      /* HIP runtime error                         */
  SEDX_ESTATE = 4,    /* weights not finalised / wrong call order  */
  SEDX_EKEY = 5       /* unknown or mis-shaped state_dict key      */
} sedx_status;

typedef enum {
  SEDX_MODEL_GRU_FRAMEATT = 0,          /* Cnn_9layers_Gru_FrameAtt   pytorch/models.py:564 */
  SEDX_MODEL_TRANSFORMER_FRAMEATT = 1   /* Cnn_9layers_Transformer_FrameAtt  :981       */
} sedx_model;

typedef enum { SEDX_FEATURE_LOGMEL = 0, SEDX_FEATURE_GAMMA = 1 } sedx_feature;

/* Constructor arguments of the reference models (pytorch/models.py:565-566):
 * (sample_rate, window_size, hop_size, mel_bins, fmin, fmax, classes_num,
 * feature_type).  mel_bins must be 64 (bn0 is BatchNorm2d(64), models.py:607). */
typedef struct {
  int32_t model_type;     /* sedx_model   */
  int32_t feature_type;   /* sedx_feature */
  int32_t sample_rate;
  int32_t window_size;    /* n_fft: 256, 512 or 1024 */
  int32_t hop_size;
  int32_t mel_bins;
  float fmin;
  float fmax;
  int32_t classes_num;
} sedx_config;

typedef struct sedx_handle sedx_handle;

/* Model construction: replaces Model(...) (pytorch/models.py:565-623 / :982-1024). */
sedx_status sedx_create(const sedx_config* cfg, int device, sedx_handle** out);
void sedx_destroy(sedx_handle* h);
const char* sedx_last_error(const sedx_handle* h);
/* "sedx <major>.<minor> (abi N)".  SEDX_ABI_VERSION changes whenever an
 * entry point's signature or a struct layout changes incompatibly; a caller
 * built against this header checks sedx_abi_version() == SEDX_ABI_VERSION
 * at load time ("ABI history"). */
#define SEDX_ABI_VERSION 5
const char* sedx_version(void);
int32_t sedx_abi_version(void);

/* One state_dict entry (host fp32; int64 scalars such as num_batches_tracked
 * are skipped by the caller).  Keys/shapes exactly as the reference
 * state_dict; unused keys (att_block.bn_att.*,
 * multihead.layer_norm.*) are accepted and ignored.  Replaces
 * model.load_state_dict(checkpoint['model']) (pytorch/predict.py:232-233). */
sedx_status sedx_load_param(sedx_handle* h, const char* key, const float* h_data,
                            const int64_t* shape, int32_t ndim);
/* Folds BN into conv weights, pre-packs GEMM layouts, uploads to the device.
 * Must follow the last sedx_load_param and precede any forward. */
sedx_status sedx_finalize_weights(sedx_handle* h);

/* Output geometry for a batch of waveforms of L samples (logmel) or of
 * feature matrices with T frames (gamma): frames of framewise_output
 * (after x8 interpolation and, GRU only, padding to a multiple of 100:
 * models.py:62-95, :678-681) and the sequence length after the CNN. */
sedx_status sedx_output_geometry(const sedx_handle* h, int64_t L_or_T, int64_t* out_frames,
                                 int64_t* seq_len);
/* Bytes of device workspace sedx_forward* needs for (B, L). */
sedx_status sedx_workspace_size(const sedx_handle* h, int64_t B, int64_t L_or_T, size_t* bytes);

/* Model forward (eval mode): replaces Cnn_9layers_*_FrameAtt.forward(input)
 * (pytorch/models.py:625-688, :1029-1077).
 *   d_wave       [B, L]                         (logmel models)
 *   d_framewise  [B, out_frames, classes_num]
 *   d_clipwise   [B, classes_num]
 *   d_embedding  GRU: [B, classes_num, seq_len]; Transformer: [B, 512, seq_len]
 *                (may be NULL)
 *   d_workspace  NULL = handle-owned cache, else >= sedx_workspace_size bytes. */
sedx_status sedx_forward(sedx_handle* h, const float* d_wave, int64_t B, int64_t L,
                         float* d_framewise, float* d_clipwise, float* d_embedding,
                         void* d_workspace, size_t workspace_bytes, void* stream);

/* Same forward on int16 waveforms as packed in the reference's HDF5 files
 * (utils/features.py:313-317, :370): the loader's int16_to_float32
 * (utils/data_generator.py:39, utils/utilities.py:78-79: float64 x / 32767
 * rounded to float32) is fused into the frontend's loads, halving the input
 * bytes.  Bit-identical to sedx_forward on the dequantised waveform. */
sedx_status sedx_forward_i16(sedx_handle* h, const int16_t* d_wave, int64_t B, int64_t L,
                             float* d_framewise, float* d_clipwise, float* d_embedding,
                             void* d_workspace, size_t workspace_bytes, void* stream);

/* Gamma branch (models.py:636-640): input is the [B, 64, T] feature matrix
 * that the reference model receives (int16-dequantised gammatone dB). */
sedx_status sedx_forward_features(sedx_handle* h, const float* d_feat, int64_t B, int64_t T,
                                  float* d_framewise, float* d_clipwise, float* d_embedding,
                                  void* d_workspace, size_t workspace_bytes, void* stream);

/* Gammatone frontend (utils/gammatone/fftweight.py:126-168 + power_to_db
 * top_db=80 + float32_to_int16 / int16_to_float32, utils/features.py:361-370,
 * utils/utilities.py:73-79): d_audio [B, L] (already pad_truncated to 10 s)
 * -> d_feat [B, 64, T], T = 1 + floor((L - nfft) / hop).  Computed in float64
 * like the reference's numpy (FFT, |X|, the ERB product, dB, top_db clamp and
 * the int16 quantisation), so the int16 codes equal the reference's.
 * d_feat == NULL: geometry query (T_out only).  Workspace:
 * sedx_gamma_workspace_size (NULL d_workspace = handle-owned cache). */
sedx_status sedx_gamma_features(sedx_handle* h, const float* d_audio, int64_t B, int64_t L,
                                float* d_feat, int64_t* T_out, void* d_workspace,
                                size_t workspace_bytes, void* stream);
sedx_status sedx_gamma_workspace_size(const sedx_handle* h, int64_t B, int64_t L, size_t* bytes);

/* Windowed drivers: pytorch/predict.py:297-349 (`predict`) and
 * pytorch/main_strong.py:786-835 (`inference_prob_overlap`) / :1052-1100
 * (`inference_prob_vote`).  The reference's loops take three independent
 * numbers, kept apart here exactly as they are there:
 *   stride      how far `start` advances per window:
 *                 predict.py  `start += 1` with --overlap, else
 *                             `start += sample_duration` (predict.py:334-337);
 *                 main_strong `start += overlap_value` (main_strong.py:829, :1094)
 *               (start is an int in predict.py, a float64 running sum in
 *               main_strong; window w reads samples int(start_w * sr) ...)
 *   merge step  int(100 * overlap_value) frames, computed in float64
 *               (utilities.py:406, :426; vad.py:63): window w lands at frame
 *               w * step of the merged output WHATEVER the stride
 *   loop bound  `while end <= audio_duration`, end = start + sample_duration,
 *               audio_duration = librosa.get_duration of the file (predict.py:277,
 *               main_strong.py:778).
 * predict.py pad_truncate's every window to sample_duration s (:305);
 * main_strong pad_truncate's the whole clip to 10 s (:790) and feeds each
 * window as sliced, so a window that runs past 10 s is SHORTER (its own
 * forward, fewer frames; the merge then follows numpy's slicing and
 * broadcasting exactly, raising SEDX_EINVAL where numpy raises). */
typedef enum { SEDX_DRIVER_PREDICT = 0, SEDX_DRIVER_MAIN_STRONG = 1 } sedx_window_driver;
typedef struct {
  int32_t driver;           /* sedx_window_driver */
  int32_t overlap;          /* PREDICT: predict.py --overlap (stride 1 s, else sample_duration s); MAIN_STRONG: ignored */
  int32_t sample_duration;  /* seconds (an int in both drivers: predict.py:701, main_strong.py:746) */
  int32_t vote;             /* 0: the averaged merge (sedx_forward_windows, avg_merge after merge);
                               1: the vote merge (sedx_forward_windows_vote, merge only).  Picks the
                               plan sedx_window_geometry / sedx_window_workspace_size size, so they
                               reject exactly what the matching forward rejects (avg_merge raises on
                               a zero step, the vote merge does not).  Was `reserved` (0) before
                               ABI 5: old callers get the averaged path, as before. */
  double overlap_value;     /* merge step int(100 * overlap_value); MAIN_STRONG: also the stride */
  double audio_duration;    /* the loop bound in seconds; <= 0: L_clip / sample_rate */
} sedx_window_spec;

/* Handle-free loop control: the sample offset of every window and the
 * samples the model receives for it (h_len: sample_duration * sr, except
 * main_strong windows that run past the 10 s padded clip).  Fills at most
 * `capacity` entries (h_start / h_len may be NULL) and sets *n_windows.
 * SEDX_EINVAL for sample_duration <= 0 or a stride <= 0 (the reference's loop
 * never ends).  The model-dependent limits (a window of <= n_fft/2 samples
 * fails the STFT's reflect padding, pytorch/stft.py:237; fewer than 8 frames
 * fail the third 2x2 pooling, models.py:139) are checked by
 * sedx_window_geometry, which needs the handle. */
sedx_status sedx_window_starts(int32_t sample_rate, int64_t L_clip, const sedx_window_spec* spec,
                               int64_t* h_start, int64_t* h_len, int64_t capacity, int64_t* n_windows);
/* Handle-free host merge: utilities.merge applied window by window exactly
 * as the drivers call it (predict.py:323-329), then utilities.avg_merge when
 * `avg` (predict.py:349), on float32 host arrays.  h_win = the windows'
 * framewise outputs [frames[w]][C] concatenated in window order; h_out
 * [merged_frames][C] (NULL: size query).  Slicing with numpy's clamping and
 * broadcasting semantics; SEDX_EINVAL where numpy raises (broadcast of
 * mismatched lengths, avg_merge with a zero step). */
sedx_status sedx_merge_host(const float* h_win, const int64_t* frames, int64_t n_win, int64_t C,
                            int32_t sample_duration, double overlap_value, int32_t avg, float* h_out,
                            int64_t capacity_frames, int64_t* merged_frames);

/* Runs ALL windows of ALL clips as one batch (a main_strong window shorter
 * than sample_duration as its own small batch), overlap-adds on the GPU
 * (utilities.py:405-423) and applies the avg_merge divisor schedule
 * (utilities.py:425-446).
 *   d_audio       [n_clips, L_clip] (every clip the same length)
 *   d_merged      [n_clips, merged_frames, classes_num]
 * sedx_window_geometry returns n_windows per clip, samples per full window
 * and merged_frames. */
sedx_status sedx_window_geometry(const sedx_handle* h, int64_t L_clip, const sedx_window_spec* spec,
                                 int64_t* n_windows, int64_t* window_samples, int64_t* merged_frames);
sedx_status sedx_forward_windows(sedx_handle* h, const float* d_audio, int64_t n_clips, int64_t L_clip,
                                 const sedx_window_spec* spec, float* d_merged, void* d_workspace,
                                 size_t workspace_bytes, void* stream);
sedx_status sedx_window_workspace_size(const sedx_handle* h, int64_t n_clips, int64_t L_clip,
                                       const sedx_window_spec* spec, size_t* bytes);
/* Voting variant (inference_prob_vote, pytorch/main_strong.py:1052-1100):
 * every window's framewise output is binarised, x > bin_thres[k] (host f64
 * [classes_num]; the reference passes sed_low_threshold, main_strong.py:1082,
 * binarize_pred :870-883), and the 0/1 windows are overlap-added with
 * utilities.merge — no avg_merge.  d_votes [n_clips, merged_frames,
 * classes_num] holds the vote counts (exact small integers) for
 * sedx_events_device(mode = 1).  Workspace: sedx_window_workspace_size. */
sedx_status sedx_forward_windows_vote(sedx_handle* h, const float* d_audio, int64_t n_clips, int64_t L_clip,
                                      const sedx_window_spec* spec, const double* bin_thres, float* d_votes,
                                      void* d_workspace, size_t workspace_bytes, void* stream);

/* Arithmetic of the GEMM-shaped work: the 9-layer conv stack (96.8 % of the
 * FLOPs), the GRU input projection and recurrence, the MHA projections and
 * the AttBlock projection.
 *  SEDX_PRECISION_EXACT  fp32 operands, fp32 accumulation
 *                       (v_mfma_f32_32x32x2_f32 / fp32 FMA): the reference's
 *                       arithmetic (pytorch/models.py:614-615, :663-670),
 *                       direct 3x3 convolution.
 *  SEDX_PRECISION_WINOGRAD (default)  fp32 throughout as EXACT, with block 1's conv2
 *                       (SEDX_TUNE_WINO_BLOCK1) and the six conv layers
 *                       of blocks 2-4 computed by Winograd F(4x4,3x3)
 *                       (SEDX_TUNE_WINO_F43; 1: block 1 by F(2x2,3x3), 0:
 *                       every layer by F(2x2,3x3)):
 *                       input / weight / output transforms and the
 *                       element-wise GEMMs all in fp32 (weights transformed
 *                       in float64, rounded once), 2.25x / 4x fewer
 *                       multiplies than the direct conv; F(2x2,3x3)'s error
 *                       vs a float64 conv is at or below the direct conv's,
 *                       F(4x4,3x3)'s ~6x it (tools/wino_bench.cpp,
 *                       tools/wino43_bench.cpp).  Different rounding from
 *                       EXACT, so not bit-identical to it.
 *  SEDX_PRECISION_X3    opt-in: bf16 MFMA with a 3-term hi/lo operand split
 *                       (hi*hi + hi*lo + lo*hi, fp32 accumulate): operands
 *                       carry 16 significant bits, products err ~2^-16 rel.
 * The frontend (FFT, mel, dB), the gates, softmax and the head's
 * element-wise work are fp32 in every mode; the gammatone frontend float64. */
typedef enum { SEDX_PRECISION_EXACT = 0, SEDX_PRECISION_X3 = 1, SEDX_PRECISION_WINOGRAD = 2 } sedx_precision;
sedx_status sedx_set_precision(sedx_handle* h, int32_t mode);

/* Implementation choices that leave the arithmetic's meaning unchanged (A/B
 * measurement and tests; the defaults are the fastest measured):
 *  SEDX_TUNE_GRU_KERNEL   SEDX_GRU_KERNEL_AUTO (default): COOP16 (the shorter
 *                         recurrence), on a pipelined handle with its
 *                         workgroups dealt over every XCD (the recurrence
 *                         runs beside the next batch's conv stack);
 *                         SEDX_GRU_KERNEL_COOP: the cooperative
 *                         recurrence, 8 workgroups per (32-clip group,
 *                         direction) exchanging h slices every step (up to 8
 *                         clips: the small-batch VALU kernel with a data-tagged
 *                         hand-off); SEDX_GRU_KERNEL_TAG16 / _TAG8 (exact,
 *                         more than 8 clips): 16-clip groups on 16 / 8
 *                         workgroups exchanging data-tagged granules straight
 *                         into the MFMA operands (lower product latency, more
 *                         CUs held: slower beside a second batch's conv stack);
 *                         SEDX_GRU_KERNEL_SIMPLE: one workgroup per (clip,
 *                         direction), W_hh streamed from L2 (fp32 FMA);
 *                         SEDX_GRU_KERNEL_COOP16 (exact, more than 8 clips):
 *                         the cooperative kernel on 16 workgroups per
 *                         (32-clip group, direction) — half the serial
 *                         product per step, twice the CUs held;
 *                         bit-identical to COOP.
 *                         SEDX_GRU_KERNEL_KSPLIT (exact, more than 8 clips):
 *                         16 workgroups per (32-clip group, direction), each
 *                         K-eighth wave waiting only for the two slices it
 *                         multiplies and loading their h straight into its
 *                         MFMA operands (no LDS gather); bit-identical.
 *                         SEDX_GRU_KERNEL_PAIR (exact, more than 8 clips):
 *                         the K-split structure with each 32-clip group's
 *                         two 16-clip halves stepped alternately in one
 *                         workgroup (one half's hand-off behind the other's
 *                         product); bit-identical.
 *  SEDX_TUNE_GRU_HANDOFF  (COOP) SEDX_GRU_HANDOFF_AUTO (default): XCD-local hand-off
 *                         when all 8 slices share an XCD, else global; on a
 *                         pipelined handle (sedx_set_pipelined) SPREAD;
 *                         SEDX_GRU_HANDOFF_GLOBAL: always the global protocol
 *                         (same bytes, bit-identical results);
 *                         SEDX_GRU_HANDOFF_SPREAD: the global protocol with a
 *                         (group, direction)'s workgroups dealt over every XCD
 *                         (beside a concurrent conv stack no XCD loses a
 *                         quarter of its CUs; bit-identical).
 *                         SEDX_GRU_HANDOFF_LOCAL: a (group, direction)'s
 *                         workgroups on one XCD with the XCD-local hand-off
 *                         when they all landed there, also on a pipelined
 *                         handle (A/B of the placement; bit-identical).
 *  SEDX_TUNE_MEL_MFMA     (n_fft 512) 0 (default): the log-mel frontend's mel
 *                         projection as VALU band sums; 1: on
 *                         v_mfma_f32_16x16x4_f32, the workgroup's 16 frames x
 *                         one 16-band tile per wave over the tile's bin range
 *                         (the same in-order fma chain per band:
 *                         bit-identical; measured 1.4x slower at B = 32: the
 *                         tile's single MFMA chain and two workgroup barriers
 *                         per 16 frames cost more than the band sums' VALU).
 *  SEDX_TUNE_WINO_BLOCK1  (SEDX_PRECISION_WINOGRAD only) 2 (default): block 1
 *                         as ONE launch — conv1 computed into conv2's halo
 *                         images in LDS (the 64-channel activation never
 *                         exists), conv2 as Winograd F(2x2,3x3), pool;
 *                         1: the same conv2 fed by a separate conv1 launch
 *                         (the activation through HBM; bit-identical to 2);
 *                         0: block 1 as the direct fused fp32 kernel.
 *                         With SEDX_TUNE_WINO_F43 2 (its default) 1 and 2
 *                         both run conv1's own launch + the F(4x4,3x3) conv2
 *                         (2: conv1 in the chunk-of-4 layout, 1: NHWC;
 *                         bit-identical).
 *  SEDX_TUNE_GRU_SPIN     bound of every GRU hand-off spin, in polls (default
 *                         2^24 = 16777216).  A spin that runs out turns that
 *                         forward's outputs into NaN and is reported by
 *                         sedx_check_error (tests force it with 0: every
 *                         step that would wait fails, whether or not its data
 *                         has arrived).
 *  SEDX_TUNE_GAMMA_SPEC   (gammatone, nfft 2048) 0 (default): the spectrum
 *                         as a 256-thread Stockham FFT per frame; 1: one
 *                         wave per frame (16 x 16 x 4 four-step in registers,
 *                         wave-local transposes).  Same int16 codes in every
 *                         test (f64 sums in another order).
 *  SEDX_TUNE_WINO_ORDER   (winograd) 1 (default): layers whose channel groups'
 *                         weight slabs exceed ~8 MB together (the 512-channel
 *                         layers) run each XCD's rounds of 32 concurrent items
 *                         as 8 tile blocks x 4 channel groups of 64 (4 slabs
 *                         per round through the XCD's L2 instead of 8);
 *                         0: tile block major; 2: as 1, and block 1's F(4x4,3x3)
 *                         conv2 gives each XCD a contiguous range of tile
 *                         blocks (neighbouring items' shared halo rows read
 *                         once into that XCD's L2).  Bit-identical outputs.
 *  SEDX_TUNE_WINO_F43     (winograd) 2 (default): block 1's conv2 and the
 *                         six conv layers of blocks 2-4 as fp32 Winograd
 *                         F(4x4,3x3) (36 multiplies per 4x4 tile,
 *                         v_mfma_f32_16x16x4_f32, csrc/conv_wino43.hip),
 *                         block 1 as a conv1 launch + that conv2 (conv1's
 *                         activation in the workspace); 1: blocks 2-4 only
 *                         (block 1 per SEDX_TUNE_WINO_BLOCK1 on F(2x2,3x3));
 *                         0: every layer F(2x2,3x3).  Different
 *                         rounding (both fp32 throughout; F(4,3)'s error vs a
 *                         float64 conv is ~6x the direct conv's, still ~1e-5
 *                         of the 1e-3 bar), so not bit-identical to each other.
 *
 * Co-residency: the cooperative GRU kernels need all workgroups of a
 * (32-clip group, direction) resident at once — 8 CUs (COOP) or 16 (COOP16)
 * per pair, one workgroup per CU — and spin on each other.  AUTO picks
 * COOP16; forwards running concurrently on other streams leave fewer CUs free
 * for it: the spins are bounded (SEDX_TUNE_GRU_SPIN), so the worst case is a
 * NaN batch reported by sedx_check_error, never a hang. */
typedef enum {
  SEDX_TUNE_GRU_KERNEL = 0,
  SEDX_TUNE_GRU_HANDOFF = 1,
  SEDX_TUNE_WINO_BLOCK1 = 2,
  SEDX_TUNE_MEL_MFMA = 3,
  SEDX_TUNE_GRU_SPIN = 4,
  SEDX_TUNE_WINO_ORDER = 5,
  SEDX_TUNE_GAMMA_SPEC = 6,
  SEDX_TUNE_WINO_F43 = 7
} sedx_tuning_knob;
enum {
  SEDX_GRU_KERNEL_COOP = 0,
  SEDX_GRU_KERNEL_SIMPLE = 1,
  SEDX_GRU_KERNEL_TAG16 = 2,
  SEDX_GRU_KERNEL_TAG8 = 3,
  SEDX_GRU_KERNEL_COOP16 = 4,
  SEDX_GRU_KERNEL_AUTO = 5,
  SEDX_GRU_KERNEL_KSPLIT = 6,
  SEDX_GRU_KERNEL_PAIR = 7
};
enum { SEDX_GRU_HANDOFF_AUTO = 0, SEDX_GRU_HANDOFF_GLOBAL = 1, SEDX_GRU_HANDOFF_SPREAD = 2, SEDX_GRU_HANDOFF_LOCAL = 3 };
sedx_status sedx_set_tuning(sedx_handle* h, int32_t knob, int32_t value);

/* Asynchronous failures of forwards already issued: a GRU recurrence whose
 * bounded hand-off spin ran out wrote NaN outputs and set a host-mapped word.
 * Call after the work of the forwards in question has completed (a stream
 * sync, or a device-to-host copy of their outputs): SEDX_EHIP (and
 * sedx_last_error names it) when one of them failed, clearing the word;
 * SEDX_OK otherwise.  Every forward entry point also checks it on entry. */
sedx_status sedx_check_error(sedx_handle* h);

/* Serving with several batches in flight (one stream per request): when on,
 * the conv stack of every forward on this handle starts only after the conv
 * stack of the previously issued forward finished (a device-side event wait,
 * no host sync), so batch i's GRU / MHA + head overlap batch i+1's conv stack
 * instead of two conv stacks splitting the chip.  Results are unchanged;
 * order = host issue order.  Off by default.  on = 2: the same, with block
 * 1's first launch (conv1, HBM-bound) issued before the wait, so it may run
 * beside the previous forward's conv tail (its time then counts in stage 11,
 * pipeline wait). */
sedx_status sedx_set_pipelined(sedx_handle* h, int32_t on);

/* Per-stage device timing (the reference only wall-clocks whole loops,
 * pytorch/main_strong.py:565-574).  When on, every forward records HIP events
 * on its stream at the stage boundaries; sedx_stage_times waits for them and
 * returns milliseconds for: 0 frontend, 1 conv1 of block 1, 2..8 the seven
 * implicit-GEMM convs (b1c2, b2c1, b2c2, b3c1, b3c2, b4c1, b4c2), 9 GRU / MHA
 * incl. projections, 10 AttBlock head, 11 pipeline wait: with
 * sedx_set_pipelined on, the stream's wait for the previous forward's conv
 * stack (between the frontend and block 1; ~0 otherwise), so stage 0 times
 * the frontend's own work.  on = 1: the last forward's times;
 * on = 2 (accumulate): every forward records into its own event set (so
 * forwards in flight on several streams time independently) and
 * sedx_stage_times returns per-stage averages over all forwards since the
 * previous call (or since profiling was switched on), then resets them. */
#define SEDX_N_STAGES 12
/* Stage capture (per-stage parity tests): every later forward copies the
 * output of stage `stage` (numbering as above) into d_buf (at most `bytes`),
 * on its stream, in the library's channels-last layout:
 *   0  bn0 output X0                  [items][T][64]
 *   2,4,6  block 1..3 output (pooled) [items][T/2^k][64/2^k][C_k]
 *   3,5,7  conv1 of block 2..4        [items][T'][F'][C]
 *   8  block 4 + freq mean            [items][T/8][512]
 *   9  GRU / MHA output               [items][T/8][512]
 * stage < 0 or d_buf == NULL switches capture off. */
sedx_status sedx_set_capture(sedx_handle* h, int32_t stage, float* d_buf, size_t bytes);
sedx_status sedx_set_profiling(sedx_handle* h, int32_t on);
sedx_status sedx_stage_times(sedx_handle* h, float* ms, int32_t capacity, int32_t* n_stages);

/* Thresholding into events: activity_detection per (clip, class)
 * (utils/vad.py:11-199) as called by frame_prediction_to_event_prediction_v2
 * (pytorch/predict.py:57-121).  Host-side, quirk-exact.
 *   h_framewise [n_clips, T, C] (host), per-class parameter arrays of length C.
 *   use_low_thres = 0 reproduces activity_detection(low_thres=None).
 * Events are written as int32 quadruples (clip, class, bgn_frame, fin_frame)
 * in (clip, class, time) order; onset = bgn / frames_per_second.  When
 * *n_events > capacity the call returns SEDX_EINVAL with the required count. */
sedx_status sedx_events(const float* h_framewise, int64_t n_clips, int64_t T, int64_t C,
                        const double* high_thres, const double* low_thres,
                        int32_t use_low_thres, const int64_t* n_smooth,
                        const int64_t* n_salt, int32_t* h_events, int64_t capacity,
                        int64_t* n_events);

/* The same thresholding on the GPU, one wavefront per (clip, class) series, no
 * host round trip (asynchronous on `stream`; the device that owns d_x must be
 * current).
 *   mode 0: activity_detection (utils/vad.py:11-45) of framewise
 *           probabilities, exactly as sedx_events;
 *   mode 1: activity_detection_binary (utils/vad.py:47-106) of window vote
 *           counts from sedx_forward_windows_vote, as
 *           frame_binary_prediction_to_event_prediction
 *           (utils/utilities.py:216-276) calls it; high_thres is unused there
 *           (may be NULL), overlap_value (float64, int(100 * overlap_value)
 *           frames per block, vad.py:63) / sample_duration give its blocks.
 *   d_x       [n_clips, T, C] device
 *   d_events  int32 [capacity][4] (clip, class, bgn, fin) in (clip, class,
 *             time) order; events past capacity are dropped
 *   d_info    int64 [2]: total number of events (may exceed capacity), and 1
 *             where the reference raises IndexError (see sedx_events)
 *   d_workspace >= sedx_events_workspace_size(n_clips, T, C) bytes;
 *             T <= 655,360 frames (a series' bitmaps are held in LDS). */
sedx_status sedx_events_workspace_size(int64_t n_clips, int64_t T, int64_t C, size_t* bytes);
sedx_status sedx_events_device(const float* d_x, int64_t n_clips, int64_t T, int64_t C,
                               const double* high_thres, const double* low_thres,
                               int32_t use_low_thres, const int64_t* n_smooth, const int64_t* n_salt,
                               int32_t mode, double overlap_value, int32_t sample_duration,
                               int32_t* d_events, int64_t capacity, int64_t* d_info,
                               void* d_workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Input side: librosa.core.load(path, sr, mono=True) as
 * pytorch/predict.py:295 and pytorch/main_strong.py:787 call it
 * (librosa 0.8: soundfile read -> to_mono -> resample(res_type='kaiser_best')
 * -> fix_length).  Handle-free; asynchronous on `stream`.
 * ------------------------------------------------------------------------ */
typedef enum { SEDX_WAV_PCM = 1, SEDX_WAV_FLOAT = 3 } sedx_wav_format;
typedef struct {
  int32_t format;           /* sedx_wav_format */
  int32_t channels;
  int32_t sample_rate;
  int32_t bits_per_sample;  /* PCM 8/16/24/32, float 32/64 */
  int64_t frames;
  int64_t data_offset;      /* byte offset of the interleaved samples in the file */
  int64_t data_bytes;
} sedx_wav_info;
/* Parse a RIFF/WAVE file image in host memory (PCM or IEEE float, including
 * WAVE_FORMAT_EXTENSIBLE).  SEDX_EINVAL for anything else. */
sedx_status sedx_wav_parse(const void* h_bytes, size_t n_bytes, sedx_wav_info* info);
/* Interleaved samples (a device copy of the data chunk) -> mono float32
 * d_out [frames]: libsndfile's float scaling, then the mean over channels
 * (librosa.to_mono on the float32 array). */
sedx_status sedx_wav_decode_mono(const void* d_data, const sedx_wav_info* info, float* d_out, void* stream);
typedef enum { SEDX_RESAMPLE_KAISER_BEST = 0, SEDX_RESAMPLE_KAISER_FAST = 1 } sedx_resample_quality;
/* librosa.resample(y, sr_in, sr_out, res_type) length: ceil(n_in * sr_out / sr_in). */
sedx_status sedx_resample_size(int64_t n_in, int32_t sr_in, int32_t sr_out, int64_t* n_out);
sedx_status sedx_resample_workspace_size(int64_t n_in, int32_t sr_in, int32_t sr_out, int32_t quality,
                                         size_t* bytes);
/* resampy band-limited interpolation (restated; resampy is not in the
 * reference) + librosa fix_length; a device copy when sr_in == sr_out. */
sedx_status sedx_resample(const float* d_in, int64_t n_in, int32_t sr_in, int32_t sr_out, int32_t quality,
                          float* d_out, void* d_workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SEDX_H */
