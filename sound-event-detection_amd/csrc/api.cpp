// libsedx C ABI (include/sedx.h): handle, state_dict ingestion + packing,
// forward orchestration, windowed driver.  Host C++; kernels live in *.hip.
#include <new>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sedx.h"
#include "sedx_internal.h"

using namespace sedx;

namespace {

struct Tensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
};

struct DevWeights {
  float2* twiddle = nullptr;
  float* window = nullptr;
  float* mel_w = nullptr;
  float* mel_tab = nullptr;   // logmel512_kernel's per-(slot, lane) band weights
  float* mel_mt = nullptr;    // logmel512_kernel's MFMA mel table (FrontendParams::mel_mt)
  int32_t mt_klo[4] = {}, mt_ns[4] = {}, mt_off[4] = {}, mt_floats = 0;
  int32_t mel_wmax = 0;
  int32_t* mel_off = nullptr;
  int32_t* mel_lo = nullptr;
  float* bn0_scale = nullptr;
  float* bn0_mean = nullptr;
  float* bn0_bias = nullptr;
  float* c1_w = nullptr;
  float* c1_wt = nullptr;
  float* c1_b = nullptr;
  float* zero = nullptr;   // ZERO_BLOCK_FLOATS zeros (LDS-DMA source of out-of-clip halo pixels)
  float* trash = nullptr;  // 32 KB write-only scratch (the Winograd kernel's dummy / out-of-range stores)
  float* wp[8] = {};    // packed conv weights: block k conv j -> index 2(k-1)+(j-1); [0] unused
  float* cb[8] = {};    // folded biases
  void* wx3[8] = {};    // split bf16 hi/lo packs for conv3x3_x3 (same indices)
  float* wu[8] = {};    // Winograd U = G g G^T packs for conv3x3_wino (same indices)
  float* wu43[8] = {};  // F(4x4,3x3) U packs for conv3x3_wino43 (block 1's conv2: 1, blocks 2-4: 2..7)
  float* w_ih = nullptr;   // [1536][512]
  float* b_ih = nullptr;   // [1536]
  float* whhT = nullptr;   // [2][256][768]
  float* whh = nullptr;    // [2][768][256] (cooperative recurrence)
  float* bhh = nullptr;    // [2][768]
  float* wqkv = nullptr;   // [1536][512]
  float* bqkv = nullptr;
  float* wfc = nullptr;    // [512][512]
  float* bfc = nullptr;
  float* wac = nullptr;    // [nac][512]
  float* bac = nullptr;
  // x3 (split bf16) packs of the linear weights for linear_x3.hip
  void* w_ih_x3 = nullptr;
  void* wqkv_x3 = nullptr;
  void* wfc_x3 = nullptr;
  void* wac_x3 = nullptr;
  // gamma
  double2* g_twiddle = nullptr;
  double* g_window = nullptr;
  double* g_weightsT = nullptr;  // [gamma_kp(nfft)][64] ERB weights (fft_weights)
};

}  // namespace

struct sedx_handle {
  sedx_config cfg;
  int device = 0;
  std::string err;
  std::map<std::string, Tensor> params;
  std::map<std::string, std::vector<int64_t>> expected;
  bool finalized = false;
  void* blob = nullptr;      // single device allocation for all packed weights
  size_t blob_bytes = 0;
  DevWeights w;
  int nac = 64;              // rows of the att|cla projection (2C rounded up to 64)
  int g_nfft = 0, g_nwin = 0, g_hop = 0;
  void* ws = nullptr;        // cached workspace
  size_t ws_bytes = 0;
  // optional per-stage timing (sedx_set_profiling): events at stage boundaries
  int precision = SEDX_PRECISION_WINOGRAD;   // GEMM arithmetic (sedx_set_precision; the default is fp32 Winograd)
  int gru_kernel = SEDX_GRU_KERNEL_AUTO;   // sedx_set_tuning
  int gru_handoff = SEDX_GRU_HANDOFF_AUTO;
  int wino_block1 = 2;                     // SEDX_TUNE_WINO_BLOCK1 (2: conv1 inside the Winograd launch)
  int mel_mfma = 0;                        // SEDX_TUNE_MEL_MFMA (measured slower: opt-in)
  unsigned gru_spin = 1u << 24;            // SEDX_TUNE_GRU_SPIN: bound of every GRU hand-off spin (polls)
  int wino_order = 1;                      // SEDX_TUNE_WINO_ORDER (4 x 8 rounds on the 512-channel layers)
  int wino_f43 = 2;                        // SEDX_TUNE_WINO_F43 (2: blocks 1-4 as F(4x4,3x3), 1: blocks 2-4)
  int gamma_spec = 0;                      // SEDX_TUNE_GAMMA_SPEC
  // sedx_set_capture: copy one stage's output of every later forward
  int cap_stage = -1;
  float* cap_buf = nullptr;
  size_t cap_bytes = 0;
  int profiling = 0;          // 0 off, 1 last forward, 2 accumulate
  // sedx_set_pipelined: conv stacks of successive forwards run in issue order
  // (each waits for the previous one's conv-done event), whatever streams
  // they are issued on, so the sequence + head of batch i overlap the conv
  // stack of batch i+1 instead of two conv stacks sharing the chip
  bool pipelined = false;
  bool pipe_conv1_first = false;           // sedx_set_pipelined(h, 2): block 1's conv1 before the wait
  bool conv_done_recorded = false;
  hipEvent_t conv_done = nullptr;
  // host-mapped word the GRU kernel ORs a failure code into when a bounded
  // hand-off spin times out (that forward's outputs are NaN); the next
  // forward / sedx_stage_times turns it into SEDX_EHIP
  unsigned* gru_err_host = nullptr;
  unsigned* gru_err_dev = nullptr;
  // events 0..10 bound stages 0..10 (stage i = [i, i + 1]) except stage 0 =
  // [0, 12] (frontend) and stage 11 = [12, 1] (pipeline wait): event 12 is
  // recorded after the frontend, before the cross-stream wait
  hipEvent_t ev[SEDX_N_STAGES + 1] = {};
  bool ev_recorded[SEDX_N_STAGES + 1] = {};
  // profiling mode 2 (accumulate): every forward takes its own event set from
  // this pool, so forwards in flight on different streams time independently;
  // sedx_stage_times folds the used sets into per-stage sums and averages
  struct EvSet {
    hipEvent_t ev[SEDX_N_STAGES + 1] = {};
    bool rec[SEDX_N_STAGES + 1] = {};
  };
  std::vector<EvSet> ev_pool;
  size_t ev_used = 0;
  EvSet* ev_cur = nullptr;
  double acc_ms[SEDX_N_STAGES] = {};
  int64_t acc_n[SEDX_N_STAGES] = {};
};


namespace {
// mode 2: sums the elapsed times of every used event set, frees the pool
// the events bounding stage i (see sedx_handle::ev)
inline int stage_begin(int i) { return i == 11 ? 12 : i; }
inline int stage_end(int i) { return i == 0 ? 12 : i == 11 ? 1 : i + 1; }
static_assert(SEDX_N_STAGES == 12, "stage event map");

void fold_ev_pool(sedx_handle* h) {
  for (size_t k = 0; k < h->ev_used; ++k) {
    auto& e = h->ev_pool[k];
    for (int i = 0; i < SEDX_N_STAGES; ++i) {
      const int a = stage_begin(i), b = stage_end(i);
      if (!e.rec[a] || !e.rec[b]) continue;
      float v = 0.f;
      if (hipEventSynchronize(e.ev[b]) == hipSuccess && hipEventElapsedTime(&v, e.ev[a], e.ev[b]) == hipSuccess) {
        h->acc_ms[i] += v;
        ++h->acc_n[i];
      }
    }
  }
  h->ev_used = 0;
  h->ev_cur = nullptr;
}

inline void mark(sedx_handle* h, int i, hipStream_t s) {
  if (!h->profiling) return;
  if (h->profiling == 2) {
    if (i == 0) {                       // a forward starts: next event set
      if (h->ev_used == 4096) fold_ev_pool(h);
      if (h->ev_used == h->ev_pool.size()) {
        h->ev_pool.emplace_back();
        for (auto& e : h->ev_pool.back().ev)
          if (hipEventCreate(&e) != hipSuccess) e = nullptr;
      }
      h->ev_cur = &h->ev_pool[h->ev_used++];
      for (auto& r : h->ev_cur->rec) r = false;
    }
    if (h->ev_cur && h->ev_cur->ev[i]) {
      (void)hipEventRecord(h->ev_cur->ev[i], s);
      h->ev_cur->rec[i] = true;
    }
    return;
  }
  if (h->ev[i]) {
    (void)hipEventRecord(h->ev[i], s);
    h->ev_recorded[i] = true;
  }
}
}  // namespace

namespace {

sedx_status fail(sedx_handle* h, sedx_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (h) h->err = buf;
  return st;
}

#define HIP_TRY(h, expr)                                                                \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(h, SEDX_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));         \
  } while (0)

// sedx_set_capture: stage `stage` just wrote `n` floats at `src`
void capture(sedx_handle* h, int stage, const float* src, size_t n, hipStream_t s) {
  if (h->cap_stage != stage || !h->cap_buf) return;
  const size_t bytes = std::min(n * sizeof(float), h->cap_bytes);
  if (hipMemcpyAsync(h->cap_buf, src, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
    note_launch_error(hipErrorInvalidValue);
}
// a stage held in the chunk-of-4 layout [B][C/4][T][F][4] (the F(4x4,3x3)
// layers): captured in the documented channels-last layout (a buffer short
// of the whole stage gets the raw prefix)
void capture_c4(sedx_handle* h, int stage, const float* src, int64_t B, int T, int F, int C, hipStream_t s) {
  if (h->cap_stage != stage || !h->cap_buf) return;
  const size_t n = (size_t)B * T * F * C;
  if (h->cap_bytes < n * sizeof(float)) return capture(h, stage, src, n, s);
  launch_c4_to_nhwc(src, (int)B, T, F, C, h->cap_buf, s);
}

// errors of the launches just issued: preparation failures noted by
// launch_info (sedx_internal.h) first, then the runtime's launch error
sedx_status launch_status(sedx_handle* h) {
  const hipError_t pe = take_launch_error();
  if (pe != hipSuccess) return fail(h, SEDX_EHIP, "kernel launch preparation failed: %s", hipGetErrorString(pe));
  const hipError_t le = hipGetLastError();
  if (le != hipSuccess) return fail(h, SEDX_EHIP, "kernel launch failed: %s", hipGetErrorString(le));
  return SEDX_OK;
}

// a GRU hand-off of an earlier forward timed out (its outputs were NaN)
sedx_status check_async_error(sedx_handle* h) {
  if (!h->gru_err_host) return SEDX_OK;
  const unsigned code = __atomic_exchange_n(h->gru_err_host, 0u, __ATOMIC_ACQ_REL);
  if (code)
    return fail(h, SEDX_EHIP, "a GRU recurrence hand-off of an earlier forward timed out (code %u): its "
                              "outputs were NaN", code);
  return SEDX_OK;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

bool is_gru(const sedx_handle* h) { return h->cfg.model_type == SEDX_MODEL_GRU_FRAMEATT; }

void add_bn(std::map<std::string, std::vector<int64_t>>& e, const std::string& p, int64_t n) {
  for (const char* s : {".weight", ".bias", ".running_mean", ".running_var"}) e[p + s] = {n};
}

void build_expected(sedx_handle* h) {
  auto& e = h->expected;
  const int64_t K = h->cfg.window_size / 2 + 1;
  e["spectrogram_extractor.stft.conv_real.weight"] = {K, 1, h->cfg.window_size};
  e["spectrogram_extractor.stft.conv_imag.weight"] = {K, 1, h->cfg.window_size};
  e["logmel_extractor.melW"] = {K, h->cfg.mel_bins};
  add_bn(e, "bn0", 64);
  const int64_t ch[5] = {1, 64, 128, 256, 512};
  for (int k = 1; k <= 4; ++k) {
    const std::string p = "conv_block" + std::to_string(k);
    e[p + ".conv1.weight"] = {ch[k], ch[k - 1], 3, 3};
    e[p + ".conv2.weight"] = {ch[k], ch[k], 3, 3};
    add_bn(e, p + ".bn1", ch[k]);
    add_bn(e, p + ".bn2", ch[k]);
  }
  const int64_t C = h->cfg.classes_num;
  e["att_block.att.weight"] = {C, 512, 1};
  e["att_block.att.bias"] = {C};
  e["att_block.cla.weight"] = {C, 512, 1};
  e["att_block.cla.bias"] = {C};
  add_bn(e, "att_block.bn_att", C);   // unused in forward (models.py:161-169)
  if (is_gru(h)) {
    for (const char* s : {"", "_reverse"}) {
      e[std::string("gru.weight_ih_l0") + s] = {768, 512};
      e[std::string("gru.weight_hh_l0") + s] = {768, 256};
      e[std::string("gru.bias_ih_l0") + s] = {768};
      e[std::string("gru.bias_hh_l0") + s] = {768};
    }
  } else {
    for (const char* n : {"w_qs", "w_ks", "w_vs", "fc"}) {
      e[std::string("multihead.") + n + ".weight"] = {512, 512};
      e[std::string("multihead.") + n + ".bias"] = {512};
    }
    e["multihead.layer_norm.weight"] = {512};   // unused in forward (models.py:853-877)
    e["multihead.layer_norm.bias"] = {512};
  }
}

int64_t conv_T(const sedx_handle* h, int64_t L) { return L / h->cfg.hop_size + 1; }

struct Geometry {
  int64_t T, T1, T2, T3, fw_len, out_frames;
};

Geometry geometry_from_T(const sedx_handle* h, int64_t T) {
  Geometry g;
  g.T = T;
  g.T1 = T / 2;
  g.T2 = g.T1 / 2;
  g.T3 = g.T2 / 2;
  g.fw_len = 8 * g.T3;
  g.out_frames = g.fw_len;
  if (is_gru(h) && g.fw_len != 1000)   // pad_framewise_output(roundup) models.py:678-681
    g.out_frames = (g.fw_len % 100 == 0) ? g.fw_len : g.fw_len + 100 - g.fw_len % 100;
  return g;
}

// workspace layout (floats), 256-B aligned regions
struct WsLayout {
  size_t x0, bufA, bufB, sched, total_bytes;
};

size_t align_up(size_t x) { return (x + 63) & ~size_t(63); }

bool wino_block1_on(const sedx_handle* h) { return h->precision == SEDX_PRECISION_WINOGRAD && h->wino_block1; }

WsLayout ws_layout(const sedx_handle* h, int64_t B, const Geometry& g) {
  WsLayout l;
  size_t off = 0;
  l.x0 = off;
  off += align_up((size_t)B * g.T * 64);
  // A: the zero-bordered bn0 output (block 1 is one fused launch in both
  // modes: conv1's 64-channel activation never exists), then the conv1
  // outputs of blocks 2-4, then the head scratch
  size_t a = block1_pad_floats((int)B, (int)g.T);
  if (wino_block1_on(h) && (h->wino_block1 == 1 || h->wino_f43 == 2))
    a = std::max(a, (size_t)B * g.T * 64 * 64);   // conv1's activation
  a = std::max(a, (size_t)B * g.T1 * 32 * 128);
  a = std::max(a, (size_t)B * g.T2 * 16 * 256);
  a = std::max(a, (size_t)B * g.T3 * 8 * 512);
  // head scratch (after the conv stack): G/QKV + H + O + logits
  a = std::max(a, (size_t)B * g.T3 * (1536 + 512 + 512 + h->nac) + 4 * 64 +
                      gru_coop_workspace_bytes((int)B) / sizeof(float) + 64);
  l.bufA = off;
  off += align_up(a);
  size_t b = (size_t)B * g.T1 * 32 * 64;
  b = std::max(b, (size_t)B * g.T2 * 16 * 128);
  b = std::max(b, (size_t)B * g.T3 * 8 * 256);
  b = std::max(b, (size_t)B * g.T3 * 512);
  l.bufB = off;
  off += align_up(b);
  l.sched = off;                                  // 7 conv launches x CONV_SCHED_INTS claim counters
  off += align_up(7 * CONV_SCHED_INTS);
  l.total_bytes = off * sizeof(float);
  return l;
}

sedx_status get_ws(sedx_handle* h, size_t need, void* user, size_t user_bytes, float** out) {
  if (user) {
    if (user_bytes < need)
      return fail(h, SEDX_EINVAL, "workspace too small: %zu < %zu bytes", user_bytes, need);
    *out = static_cast<float*>(user);
    return SEDX_OK;
  }
  if (h->ws_bytes < need) {
    if (h->ws) (void)hipFree(h->ws);
    h->ws = nullptr;
    h->ws_bytes = 0;
    HIP_TRY(h, hipMalloc(&h->ws, need));
    h->ws_bytes = need;
  }
  *out = static_cast<float*>(h->ws);
  return SEDX_OK;
}

// CNN + head on X0 [B][T][64] already in workspace
sedx_status run_body(sedx_handle* h, int64_t B, const Geometry& g, float* ws, const WsLayout& l,
                     float* d_fw, float* d_clip, float* d_emb, hipStream_t s) {
  const DevWeights& w = h->w;
  float* X0 = ws + l.x0;
  float* A = ws + l.bufA;
  float* P = ws + l.bufB;
  const int iB = (int)B;
  // the cross-stream wait for the previous forward's conv stack comes before
  // the b1c1 stage event, so stage 1 times only this forward's work
  mark(h, 12, s);   // the frontend's end: the wait below is stage 11, not the frontend's
  const bool x3 = h->precision == SEDX_PRECISION_X3;
  int* sched = reinterpret_cast<int*>(ws + l.sched);
  const bool wb1 = wino_block1_on(h);
  // winograd with F(4x4,3x3): block 1 (one launch) and blocks 2-4 keep their
  // activations in the chunk-of-4 layout [B][C/4][T][F][4] (dense halo DMA)
  const bool c4 = h->precision == SEDX_PRECISION_WINOGRAD && h->wino_f43 && wb1 && h->wino_block1 == 2;
  // Winograd block 1: 1 = conv1's activation [B][T][64][64] into A by its
  // own launch; 2 = conv1 inside the Winograd launch (reads X0 itself).
  // F(4x4,3x3) block 1 (wino_f43 2): conv1 by its own launch in both (2: in
  // the chunk-of-4 layout), then the F(4x4,3x3) conv2
  const bool b1_43 = wb1 && h->wino_f43 == 2;
  // block 1's first launch (conv1 / the zero-bordered copy of X0): before
  // the pipelined wait with sedx_set_pipelined(h, 2) — an HBM-bound launch
  // that may then overlap the previous forward's compute-bound conv tail —
  // else after it (stage 1)
  auto block1_first = [&]() {
    if (b1_43 && c4)
      launch_conv1_c4(X0, iB, (int)g.T, w.c1_w, w.c1_b, A, s);
    else if (wb1 && (h->wino_block1 == 1 || b1_43))
      launch_conv1_nhwc(X0, iB, (int)g.T, w.c1_w, w.c1_b, A, s);
    else if (!wb1)
      launch_pad_x0(X0, iB, (int)g.T, A, s);
  };
  // claim counters of the x3 launches and of the F(4x4,3x3) launches (the
  // workspace comes from the caller: zeroed once per forward, ahead of the
  // pipelined wait — this forward's memory only).  Below 8 clips the
  // F(4x4,3x3) launches get no counters (the static item order, same
  // outputs) and the forward no memset: one fill launch less on the
  // one-clip latency path
  const bool w43 = h->precision == SEDX_PRECISION_WINOGRAD && h->wino_f43 && B >= 8;
  int* const w43_sched = w43 ? sched : nullptr;
  if (x3 || w43) HIP_TRY(h, hipMemsetAsync(sched, 0, 7 * CONV_SCHED_INTS * sizeof(int), s));
  const bool first_early = h->pipelined && h->pipe_conv1_first;
  if (first_early) block1_first();
  if (h->pipelined && h->conv_done_recorded) HIP_TRY(h, hipStreamWaitEvent(s, h->conv_done, 0));
  mark(h, 1, s);
  capture(h, 0, X0, (size_t)B * g.T * 64, s);
  // block 1 as one launch in both modes: conv1 computed inside conv2's halo
  // staging (the b1c1 stage is just the zero-bordered copy of the bn0 output)
  if (!first_early) block1_first();
  struct L {
    const float* in;
    int T, F, cin, cout, idx, epi;
    float* out;
  };
  const L layers[7] = {{A, (int)g.T, 64, 64, 64, 1, EPI_POOL2, P},
                       {P, (int)g.T1, 32, 64, 128, 2, EPI_STORE, A},
                       {A, (int)g.T1, 32, 128, 128, 3, EPI_POOL2, P},
                       {P, (int)g.T2, 16, 128, 256, 4, EPI_STORE, A},
                       {A, (int)g.T2, 16, 256, 256, 5, EPI_POOL2, P},
                       {P, (int)g.T3, 8, 256, 512, 6, EPI_STORE, A},
                       {A, (int)g.T3, 8, 512, 512, 7, EPI_FMEAN, P}};
  for (int i = 0; i < 7; ++i) {
    const L& c = layers[i];
    mark(h, 2 + i, s);
    if (x3 && i == 0)
      launch_block1_fused_x3(nullptr, iB, c.T, A, w.c1_wt, w.c1_b, w.wx3[c.idx], w.cb[c.idx], c.out,
                             sched, s);
    else if (i == 0 && b1_43)
      launch_conv3x3_wino43(A, iB, c.T, 64, 64, 64, w.wu43[c.idx], w.cb[c.idx], c.out, EPI_POOL2, w.trash, s,
                            h->wino_order, c4, 0, w43_sched);
    else if (i == 0 && wb1 && h->wino_block1 == 2)
      launch_block1_wino(X0, iB, c.T, w.c1_w, w.c1_b, w.wu[c.idx], w.cb[c.idx], c.out, w.zero, w.trash, s, c4);
    else if (i == 0 && wb1)
      launch_conv3x3_wino(A, iB, c.T, 64, 64, 64, w.wu[c.idx], w.cb[c.idx], c.out, EPI_POOL2, w.zero, w.trash, s);
    else if (i == 0)
      launch_block1_exact(A, iB, c.T, w.c1_w, w.c1_b, w.wp[c.idx], w.cb[c.idx], c.out, w.zero, s);
    else if (x3)
      launch_conv3x3_x3(c.in, iB, c.T, c.F, c.cin, c.cout, w.wx3[c.idx], w.cb[c.idx], c.out, c.epi,
                        sched + i * CONV_SCHED_INTS, s);
    else if (h->precision == SEDX_PRECISION_WINOGRAD && h->wino_f43)
      launch_conv3x3_wino43(c.in, iB, c.T, c.F, c.cin, c.cout, w.wu43[c.idx], w.cb[c.idx], c.out, c.epi, w.trash, s,
                            h->wino_order, c4, 0, w43 ? sched + i * CONV_SCHED_INTS : nullptr);
    else if (h->precision == SEDX_PRECISION_WINOGRAD)
      launch_conv3x3_wino(c.in, iB, c.T, c.F, c.cin, c.cout, w.wu[c.idx], w.cb[c.idx], c.out, c.epi, w.zero, w.trash,
                          s, h->wino_order);
    else
      launch_conv3x3(c.in, iB, c.T, c.F, c.cin, c.cout, w.wp[c.idx], w.cb[c.idx], c.out, c.epi, w.zero, s);
    const size_t px = c.epi == EPI_STORE ? (size_t)c.T * c.F : c.epi == EPI_POOL2 ? (size_t)(c.T / 2) * (c.F / 2)
                                                                                   : (size_t)c.T;
    if (c4 && c.epi != EPI_FMEAN) {
      const int To = c.epi == EPI_POOL2 ? c.T / 2 : c.T, Fo = c.epi == EPI_POOL2 ? c.F / 2 : c.F;
      capture_c4(h, 2 + i, c.out, B, To, Fo, c.cout, s);
    } else {
      capture(h, 2 + i, c.out, (size_t)B * px * c.cout, s);
    }
  }
  mark(h, 9, s);
  if (h->pipelined) {
    HIP_TRY(h, hipEventRecord(h->conv_done, s));
    h->conv_done_recorded = true;
  }
  float* S = P;                                   // [B][T3][512]
  const int M = (int)(B * g.T3);
  float* G = A;                                   // [M][1536]
  float* Hs = A + align_up((size_t)M * 1536);     // [M][512]
  float* O = Hs + align_up((size_t)M * 512);      // [M][512]
  float* LG = O + align_up((size_t)M * 512);      // [M][nac]
  // GEMMs: x3 split-bf16 MFMA in x3 mode, fp32 MFMA in exact mode
  auto linear = [&](const float* a, const float* wf, void* wx, int n, int bn, const float* bias, float* c,
                    int act) {
    if (x3)
      launch_linear_x3(a, M, 512, wx, n, bn, bias, c, act, s);
    else
      launch_linear(a, M, 512, wf, n, bias, c, act, s);
  };
  if (is_gru(h)) {
    linear(S, w.w_ih, w.w_ih_x3, 1536, 128, w.b_ih, G, 0);
    if (h->gru_kernel == SEDX_GRU_KERNEL_SIMPLE)
      launch_gru(G, iB, (int)g.T3, w.whhT, w.bhh, Hs, s);
    else
      launch_gru_coop(G, iB, (int)g.T3, w.whh, w.bhh, Hs, LG + align_up((size_t)M * h->nac), !x3,
                      h->gru_handoff == SEDX_GRU_HANDOFF_AUTO || h->gru_handoff == SEDX_GRU_HANDOFF_LOCAL,
                      h->gru_kernel == SEDX_GRU_KERNEL_TAG16 ? 0 : h->gru_kernel == SEDX_GRU_KERNEL_TAG8 ? 1
                      : h->gru_kernel == SEDX_GRU_KERNEL_COOP16 ? 3
                      : h->gru_kernel == SEDX_GRU_KERNEL_KSPLIT ? 4
                      : h->gru_kernel == SEDX_GRU_KERNEL_PAIR ? 5
                      // AUTO: 16 slices (half the recurrence's serial product); on a
                      // pipelined handle dealt over every XCD (SPREAD, below): beside
                      // the next batch's conv stack the shorter recurrence then costs
                      // it less than the 8-slice kernel's half-size footprint
                      // (12,238-12,303 vs 11,886-11,923 clips/s, profiles/r05za_*)
                      : h->gru_kernel == SEDX_GRU_KERNEL_AUTO ? 3 : 2,
                      h->gru_err_dev, h->gru_spin, s,
                      // AUTO on a pipelined handle: the recurrence runs beside the
                      // next batch's conv stack, whose items are dealt to the 8
                      // XCDs evenly — slices on one XCD cost that XCD a quarter
                      // of its CUs and the whole launch waits for it (b1c2 0.61
                      // vs 0.51 ms in the timed region, profiles/r05t_*)
                      h->gru_handoff == SEDX_GRU_HANDOFF_SPREAD ||
                          (h->gru_handoff == SEDX_GRU_HANDOFF_AUTO && h->pipelined));
  } else {
    linear(S, w.wqkv, w.wqkv_x3, 1536, 128, w.bqkv, G, 0);
    launch_mha(G, iB, (int)g.T3, O, s);
    linear(O, w.wfc, w.wfc_x3, 512, 128, w.bfc, Hs, 1);
  }
  capture(h, 9, Hs, (size_t)M * 512, s);
  mark(h, 10, s);
  linear(Hs, w.wac, w.wac_x3, h->nac, 64, w.bac, LG, 0);
  launch_att_head(LG, iB, (int)g.T3, h->cfg.classes_num, h->nac, (int)g.out_frames, d_fw, d_clip,
                  is_gru(h) ? d_emb : nullptr, s);
  if (!is_gru(h) && d_emb) launch_transpose_btd(Hs, iB, (int)g.T3, 512, d_emb, s);
  mark(h, 11, s);
  return launch_status(h);
}

// -------- windowed drivers (predict.py:297-349 / main_strong.py:786-835) --------
// windows fed to the model as one batch: consecutive windows of one length
// (every predict.py window; main_strong's full windows, then each window
// that runs past the 10 s padded clip on its own)
struct WinGroup {
  int w0 = 0, nw = 0;
  int64_t len = 0;
  Geometry g{};
};
struct WinGeom {
  WindowLoop loop;
  int n_win = 0;
  int64_t full_len = 0;     // samples of a full window (sample_duration * sr)
  int64_t clip_len = 0;     // samples backing each clip (beyond: pad_truncate zeros)
  int64_t step = 0;         // int(100 * overlap_value)
  int sd = 0;
  std::vector<WinGroup> groups;
  MergePlan plan;
};

sedx_status window_geometry(const sedx_handle* h, int64_t L_clip, const sedx_window_spec* spec, bool avg,
                            WinGeom* wg) {
  sedx_handle* hm = const_cast<sedx_handle*>(h);
  if (!spec) return fail(hm, SEDX_EINVAL, "null window spec");
  const int sr = h->cfg.sample_rate;
  if (const char* why = window_loop(sr, L_clip, *spec, &wg->loop)) return fail(hm, SEDX_EINVAL, "%s", why);
  // int(100 * overlap_value) in float64 (utilities.py:406, :426)
  const double stepd = 100.0 * spec->overlap_value;
  if (!(std::fabs(stepd) < 1e9)) return fail(hm, SEDX_EINVAL, "overlap_value out of range");
  wg->step = (int64_t)stepd;
  wg->sd = spec->sample_duration;
  wg->n_win = (int)wg->loop.start.size();
  wg->full_len = (int64_t)spec->sample_duration * sr;
  wg->clip_len = spec->driver == SEDX_DRIVER_MAIN_STRONG ? std::min<int64_t>(L_clip, (int64_t)sr * 10) : L_clip;
  wg->groups.clear();
  std::vector<int64_t> frames(wg->n_win);
  for (int w = 0; w < wg->n_win; ++w) {
    const int64_t len = wg->loop.len[w];
    // the model raises on these windows: STFT reflect padding needs more
    // than n_fft/2 samples (stft.py:237), the third 2x2 pool one frame
    // (models.py:139)
    if (len <= h->cfg.window_size / 2)
      return fail(hm, SEDX_EINVAL, "window %d has %lld samples: too short for the STFT's reflect padding", w,
                  (long long)len);
    if (wg->groups.empty() || wg->groups.back().len != len) {
      WinGroup g;
      g.w0 = w;
      g.len = len;
      g.g = geometry_from_T(h, conv_T(h, len));
      if (g.g.T3 < 1) return fail(hm, SEDX_EINVAL, "window %d too short for the CNN", w);
      wg->groups.push_back(g);
    }
    ++wg->groups.back().nw;
    frames[w] = wg->groups.back().g.out_frames;
  }
  if (const char* why = build_merge_plan(frames, wg->step, wg->sd, avg, &wg->plan))
    return fail(hm, SEDX_EINVAL, "%s", why);
  return SEDX_OK;
}

// per-call device area after the model workspace: per-window framewise and
// clipwise outputs, vote thresholds, then the tables (window starts, output
// bases, merge plan), all at 256-B aligned float offsets
struct WinLayout {
  size_t model_bytes = 0;             // max over the groups' ws_layout
  std::vector<size_t> fw_off, clip_off;   // per group, floats from the area start
  size_t vthr = 0, tables = 0, table_bytes = 0, total_bytes = 0;
  size_t t_start = 0, t_wb = 0, t_wcs = 0, t_off = 0, t_src = 0, t_div = 0;   // byte offsets in the tables
};

WinLayout win_layout(const sedx_handle* h, int64_t n_clips, const WinGeom& wg) {
  WinLayout l;
  const int64_t C = h->cfg.classes_num;
  for (const auto& g : wg.groups) l.model_bytes = std::max(l.model_bytes, ws_layout(h, n_clips * g.nw, g.g).total_bytes);
  size_t off = l.model_bytes / sizeof(float);
  for (const auto& g : wg.groups) {
    l.fw_off.push_back(off);
    off += align_up((size_t)n_clips * g.nw * g.g.out_frames * C);
  }
  for (const auto& g : wg.groups) {
    l.clip_off.push_back(off);
    off += align_up((size_t)n_clips * g.nw * C);
  }
  l.vthr = off;
  off += align_up(2 * (size_t)C);
  l.tables = off;
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  size_t b = 0;
  l.t_start = b; b += al(8 * (size_t)wg.n_win);
  l.t_wb = b;    b += al(8 * (size_t)wg.n_win);
  l.t_wcs = b;   b += al(8 * (size_t)wg.n_win);
  l.t_off = b;   b += al(4 * ((size_t)wg.plan.N + 1));
  l.t_src = b;   b += al(8 * wg.plan.src.size());
  l.t_div = b;   b += al(4 * (size_t)wg.plan.N);
  l.table_bytes = b;
  l.total_bytes = off * sizeof(float) + b;
  return l;
}

// the MFMA mel table (nullptr when the host did not build one)
void set_mel_mt(FrontendParams& p, const DevWeights& w, int on) {
  p.mel_mt = on ? w.mel_mt : nullptr;
  for (int j = 0; j < 4; ++j) {
    p.mt_klo[j] = w.mt_klo[j];
    p.mt_ns[j] = w.mt_ns[j];
    p.mt_off[j] = w.mt_off[j];
  }
  p.mt_floats = w.mt_floats;
}

template <typename T>
T* carve(char*& p, size_t n) {
  T* r = reinterpret_cast<T*>(p);
  p += (n * sizeof(T) + 255) & ~size_t(255);
  return r;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

const char* sedx_version(void) {
  return "sedx 0.5 (abi 5; gfx950: fp32 MFMA exact direct conv | fp32 Winograd F(4x4,3x3) + F(2x2,3x3) | "
         "3xbf16-split MFMA)";
}

int32_t sedx_abi_version(void) { return SEDX_ABI_VERSION; }

sedx_status sedx_set_precision(sedx_handle* h, int32_t mode) {
  if (!h) return SEDX_EINVAL;
  if (mode != SEDX_PRECISION_EXACT && mode != SEDX_PRECISION_X3 && mode != SEDX_PRECISION_WINOGRAD)
    return fail(h, SEDX_EINVAL, "unknown precision mode %d", mode);
  h->precision = mode;
  return SEDX_OK;
}

const char* sedx_last_error(const sedx_handle* h) { return h ? h->err.c_str() : "null handle"; }

sedx_status sedx_set_capture(sedx_handle* h, int32_t stage, float* d_buf, size_t bytes) {
  if (!h) return SEDX_EINVAL;
  if (stage < 0 || !d_buf) {
    h->cap_stage = -1;
    h->cap_buf = nullptr;
    h->cap_bytes = 0;
    return SEDX_OK;
  }
  if (stage == 1 || stage > 9) return fail(h, SEDX_EINVAL, "stage %d cannot be captured", (int)stage);
  h->cap_stage = stage;
  h->cap_buf = d_buf;
  h->cap_bytes = bytes;
  return SEDX_OK;
}

sedx_status sedx_set_tuning(sedx_handle* h, int32_t knob, int32_t value) {
  if (!h) return SEDX_EINVAL;
  switch (knob) {
    case SEDX_TUNE_GRU_KERNEL:
      if (value != SEDX_GRU_KERNEL_COOP && value != SEDX_GRU_KERNEL_SIMPLE && value != SEDX_GRU_KERNEL_TAG16 &&
          value != SEDX_GRU_KERNEL_TAG8 && value != SEDX_GRU_KERNEL_COOP16 && value != SEDX_GRU_KERNEL_AUTO &&
          value != SEDX_GRU_KERNEL_KSPLIT && value != SEDX_GRU_KERNEL_PAIR)
        break;
      h->gru_kernel = value;
      return SEDX_OK;
    case SEDX_TUNE_GRU_HANDOFF:
      if (value != SEDX_GRU_HANDOFF_AUTO && value != SEDX_GRU_HANDOFF_GLOBAL && value != SEDX_GRU_HANDOFF_SPREAD &&
          value != SEDX_GRU_HANDOFF_LOCAL)
        break;
      h->gru_handoff = value;
      return SEDX_OK;
    case SEDX_TUNE_WINO_BLOCK1:
      if (value != 0 && value != 1 && value != 2) break;
      h->wino_block1 = value;
      return SEDX_OK;
    case SEDX_TUNE_MEL_MFMA:
      if (value != 0 && value != 1) break;
      h->mel_mfma = value;
      return SEDX_OK;
    case SEDX_TUNE_GRU_SPIN:
      if (value < 0) break;
      h->gru_spin = (unsigned)value;
      return SEDX_OK;
    case SEDX_TUNE_WINO_ORDER:
      if (value < 0 || value > 2) break;
      h->wino_order = value;
      return SEDX_OK;
    case SEDX_TUNE_GAMMA_SPEC:
      if (value != 0 && value != 1) break;
      h->gamma_spec = value;
      return SEDX_OK;
    case SEDX_TUNE_WINO_F43:
      if (value < 0 || value > 2) break;
      h->wino_f43 = value;
      return SEDX_OK;
    default:
      return fail(h, SEDX_EINVAL, "unknown tuning knob %d", (int)knob);
  }
  return fail(h, SEDX_EINVAL, "bad value %d for tuning knob %d", (int)value, (int)knob);
}

sedx_status sedx_check_error(sedx_handle* h) {
  if (!h) return SEDX_EINVAL;
  return check_async_error(h);
}

sedx_status sedx_create(const sedx_config* cfg, int device, sedx_handle** out) {
  if (!cfg || !out) return SEDX_EINVAL;
  *out = nullptr;
  if (cfg->model_type != SEDX_MODEL_GRU_FRAMEATT && cfg->model_type != SEDX_MODEL_TRANSFORMER_FRAMEATT)
    return SEDX_EINVAL;
  if (cfg->mel_bins != 64) return SEDX_EINVAL;
  if (cfg->window_size != 256 && cfg->window_size != 512 && cfg->window_size != 1024) return SEDX_EINVAL;
  if (cfg->hop_size <= 0 || cfg->sample_rate <= 0 || cfg->classes_num <= 0 || cfg->classes_num > 256)
    return SEDX_EINVAL;
  if (cfg->feature_type == SEDX_FEATURE_GAMMA && cfg->model_type != SEDX_MODEL_GRU_FRAMEATT)
    return SEDX_EINVAL;
  sedx_handle* h = new sedx_handle();
  h->cfg = *cfg;
  h->device = device;
  h->nac = ((2 * cfg->classes_num + 63) / 64) * 64;
  build_expected(h);
  *out = h;
  return SEDX_OK;
}

void sedx_destroy(sedx_handle* h) {
  if (!h) return;
  {
    DeviceGuard g(h->device);
    for (auto& e : h->ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& set : h->ev_pool)
      for (auto& e : set.ev)
        if (e) (void)hipEventDestroy(e);
    if (h->conv_done) (void)hipEventDestroy(h->conv_done);
    if (h->blob) (void)hipFree(h->blob);
    if (h->ws) (void)hipFree(h->ws);
    if (h->gru_err_host) (void)hipHostFree(h->gru_err_host);
  }
  delete h;
}

sedx_status sedx_load_param(sedx_handle* h, const char* key, const float* h_data,
                            const int64_t* shape, int32_t ndim) {
  if (!h || !key || !h_data || (ndim > 0 && !shape) || ndim < 0 || ndim > 8) return SEDX_EINVAL;
  auto it = h->expected.find(key);
  if (it == h->expected.end()) return fail(h, SEDX_EKEY, "unexpected key in state_dict: %s", key);
  std::vector<int64_t> sh(shape, shape + ndim);
  if (sh != it->second) return fail(h, SEDX_EKEY, "size mismatch for %s", key);
  int64_t n = 1;
  for (auto d : sh) n *= d;
  Tensor t;
  t.shape = sh;
  t.data.assign(h_data, h_data + n);
  h->params[key] = std::move(t);
  h->finalized = false;
  return SEDX_OK;
}

sedx_status sedx_finalize_weights(sedx_handle* h) {
  if (!h) return SEDX_EINVAL;
  for (auto& kv : h->expected)
    if (!h->params.count(kv.first))
      return fail(h, SEDX_EKEY, "missing key in state_dict: %s", kv.first.c_str());
  DeviceGuard dg(h->device);
  const auto& P = h->params;
  auto get = [&](const std::string& k) -> const std::vector<float>& { return P.at(k).data; };
  const int nfft = h->cfg.window_size, K = nfft / 2 + 1;
  const int C = h->cfg.classes_num;

  // ---- STFT weights -> window (row k=0 of conv_real is the window since DFT[n,0]=1) ----
  const auto& wr = get("spectrogram_extractor.stft.conv_real.weight");
  const auto& wi = get("spectrogram_extractor.stft.conv_imag.weight");
  std::vector<float> window(wr.begin(), wr.begin() + nfft);
  {
    // the FFT frontend requires conv_real/imag = Re/Im(DFT) * window (stft.py:209-217)
    double maxerr = 0;
    const int rows[6] = {1, 2, K / 3, K / 2, K - 2, K - 1};
    for (int r : rows)
      for (int n = 0; n < nfft; ++n) {
        const double ang = -2.0 * M_PI * (double)((int64_t)n * r % nfft) / nfft;
        maxerr = std::max(maxerr, std::fabs(wr[(size_t)r * nfft + n] - std::cos(ang) * window[n]));
        maxerr = std::max(maxerr, std::fabs(wi[(size_t)r * nfft + n] - std::sin(ang) * window[n]));
      }
    if (maxerr > 1e-5)
      return fail(h, SEDX_EINVAL, "STFT conv weights are not a windowed DFT (max err %.3g); "
                                  "the FFT frontend cannot reproduce them", maxerr);
  }
  std::vector<float> tw(2 * nfft);
  for (int m = 0; m < nfft; ++m) {
    tw[2 * m] = (float)std::cos(-2.0 * M_PI * m / nfft);
    tw[2 * m + 1] = (float)std::sin(-2.0 * M_PI * m / nfft);
  }
  // ---- mel bands ----
  const auto& melW = get("logmel_extractor.melW");  // [K][64]
  std::vector<float> mel_w;
  std::vector<int32_t> mel_off(65), mel_lo(64);
  for (int m = 0; m < 64; ++m) {
    int lo = -1, hi = -1;
    for (int k = 0; k < K; ++k)
      if (melW[(size_t)k * 64 + m] != 0.0f) {
        if (lo < 0) lo = k;
        hi = k;
      }
    mel_off[m] = (int32_t)mel_w.size();
    mel_lo[m] = lo < 0 ? 0 : lo;
    if (lo >= 0)
      for (int k = lo; k <= hi; ++k) mel_w.push_back(melW[(size_t)k * 64 + m]);
  }
  mel_off[64] = (int32_t)mel_w.size();
  // the n_fft 512 kernel's band table: slot q of lane b is band
  // fe16_band_host(b, q), zero-padded to FE16_MEL_MW bins
  std::vector<float> mel_tab((size_t)4 * 16 * FE16_MEL_MW, 0.f);
  int32_t mel_wmax = 0;
  for (int m = 0; m < 64; ++m) mel_wmax = std::max(mel_wmax, mel_off[m + 1] - mel_off[m]);
  mel_wmax = (mel_wmax + 3) & ~3;
  for (int q = 0; q < 4; ++q)
    for (int b = 0; b < 16; ++b) {
      const int m = fe16_band_host(b, q), wd = mel_off[m + 1] - mel_off[m];
      for (int e = 0; e < std::min(wd, FE16_MEL_MW); ++e)
        mel_tab[((size_t)q * 16 + b) * FE16_MEL_MW + e] = mel_w[mel_off[m] + e];
    }
  if (mel_w.empty()) mel_w.push_back(0.f);
  // the MFMA mel path's table (n_fft 512): per 16-band tile j the bin range
  // its bands cover, in 4-bin steps: [step][4 bins][16 bands] of melW (zero
  // outside a band, and past the last bin)
  std::vector<float> mel_mt;
  int32_t mt_klo[4] = {}, mt_ns[4] = {}, mt_off[4] = {};
  if (nfft == 512) {
    for (int j = 0; j < 4; ++j) {
      int klo = K, khi = -1;
      for (int m = 16 * j; m < 16 * j + 16; ++m) {
        const int wd = mel_off[m + 1] - mel_off[m];
        if (wd <= 0) continue;
        klo = std::min(klo, mel_lo[m]);
        khi = std::max(khi, mel_lo[m] + wd - 1);
      }
      const int ns = khi < klo ? 0 : (khi - klo + 1 + 3) / 4;
      mt_klo[j] = ns ? klo : 0;
      mt_ns[j] = ns;
      mt_off[j] = (int32_t)mel_mt.size();
      for (int st = 0; st < ns; ++st)
        for (int kk = 0; kk < 4; ++kk)
          for (int n = 0; n < 16; ++n) {
            const int k = klo + 4 * st + kk, m = 16 * j + n;
            mel_mt.push_back(k < K ? melW[(size_t)k * 64 + m] : 0.f);
          }
    }
  }

  auto bn_fold = [&](const std::string& p, int n, std::vector<double>& sc, std::vector<float>& mu,
                     std::vector<float>& bi) {
    const auto& g = get(p + ".weight");
    const auto& b = get(p + ".bias");
    const auto& m = get(p + ".running_mean");
    const auto& v = get(p + ".running_var");
    sc.resize(n);
    mu.resize(n);
    bi.resize(n);
    for (int i = 0; i < n; ++i) {
      sc[i] = (double)g[i] / std::sqrt((double)v[i] + 1e-5);
      mu[i] = m[i];
      bi[i] = b[i];
    }
  };
  std::vector<double> s0;
  std::vector<float> mu0, bi0, sc0f(64);
  bn_fold("bn0", 64, s0, mu0, bi0);
  for (int i = 0; i < 64; ++i) sc0f[i] = (float)s0[i];

  // ---- conv weights: fold BN, pack [Cin/4][9][khalf 2][Cout][ks 2] (exact:
  // channel 2 ks + khalf of a 4-channel chunk; the MFMA B fragments of both
  // k-steps are one 8-byte LDS read) ----
  const int ch[5] = {1, 64, 128, 256, 512};
  std::vector<float> packed[8], cbias[8], c1w(64 * 9), c1b(64);
  std::vector<uint16_t> packed_x3[8];
  std::vector<float> packed_wu[8], packed_wu43[8];
  for (int k = 1; k <= 4; ++k)
    for (int j = 1; j <= 2; ++j) {
      const std::string p = "conv_block" + std::to_string(k);
      const int cin = (j == 1) ? ch[k - 1] : ch[k], cout = ch[k];
      const auto& wt = get(p + ".conv" + std::to_string(j) + ".weight");
      std::vector<double> sc;
      std::vector<float> mu, bi;
      bn_fold(p + ".bn" + std::to_string(j), cout, sc, mu, bi);
      std::vector<float> bias(cout);
      for (int o = 0; o < cout; ++o) bias[o] = (float)((double)bi[o] - (double)mu[o] * sc[o]);
      if (k == 1 && j == 1) {
        for (int o = 0; o < 64; ++o)
          for (int t = 0; t < 9; ++t) c1w[o * 9 + t] = (float)(wt[(size_t)o * 9 + t] * sc[o]);
        c1b = bias;
        continue;
      }
      const int idx = 2 * (k - 1) + (j - 1);
      std::vector<float>& pk = packed[idx];
      pk.assign((size_t)cin * 9 * cout, 0.f);
      for (int o = 0; o < cout; ++o)
        for (int i = 0; i < cin; ++i)
          for (int t = 0; t < 9; ++t) {
            const int chunk = i / 4, kc = i % 4, ks = kc >> 1, kh = kc & 1;
            pk[((((size_t)chunk * 9 + t) * 2 + kh) * cout + o) * 2 + ks] =
                (float)(wt[((size_t)o * cin + i) * 9 + t] * sc[o]);
          }
      cbias[idx] = bias;
      // Winograd pack: U = G g G^T from the float64 BN-folded weights
      {
        std::vector<double> wf((size_t)cout * cin * 9);
        for (int o = 0; o < cout; ++o)
          for (size_t k = 0; k < (size_t)cin * 9; ++k) wf[(size_t)o * cin * 9 + k] = wt[(size_t)o * cin * 9 + k] * sc[o];
        packed_wu[idx].assign((size_t)cin * cout * 16, 0.f);
        pack_conv_wino(wf.data(), cin, cout, packed_wu[idx].data());
        {   // block 1's conv2 and blocks 2-4: the F(4x4,3x3) pack as well
          packed_wu43[idx].assign((size_t)2 * cin * cout * 36, 0.f);
          pack_conv_wino43(wf.data(), cin, cout, packed_wu43[idx].data());
        }
      }
      // 3xbf16 split pack: [Cout/BN][Cin/16][9][BN][4 slots x 8 bf16], slot c at c ^ ((n>>2)&3)
      {
        const int BN = (cout == 64) ? 64 : 128;
        std::vector<uint16_t>& px = packed_x3[idx];
        px.assign((size_t)cout * cin * 9 * 2, 0);
        auto rne = [](float x) -> uint32_t {
          uint32_t u;
          std::memcpy(&u, &x, 4);
          return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
        };
        for (int o = 0; o < cout; ++o)
          for (int i = 0; i < cin; ++i)
            for (int t = 0; t < 9; ++t) {
              const float x = (float)(wt[((size_t)o * cin + i) * 9 + t] * sc[o]);
              const uint32_t hb = rne(x);
              const uint32_t hbits = hb << 16;
              float hf;
              std::memcpy(&hf, &hbits, 4);
              const uint32_t lb = rne(x - hf);
              const int nt = o / BN, n = o % BN, chunk = i / 16, k = i % 16;
              const int sw = (n >> 2) & 3;
              const size_t rec = ((((size_t)nt * (cin / 16) + chunk) * 9 + t) * BN + n) * 32;
              px[rec + 8 * ((k / 8) ^ sw) + (k % 8)] = (uint16_t)hb;
              px[rec + 8 * ((2 + k / 8) ^ sw) + (k % 8)] = (uint16_t)lb;
            }
      }
    }

  // ---- head ----
  std::vector<float> w_ih, b_ih, whhT, bhh, wqkv, bqkv, wfc, bfc, whh_nat;
  // W [N][K] -> [N/BN][K/16][BN][4 slots x 8 bf16], slot c at c ^ ((n>>2)&3)
  // (the conv x3 layout with a single tap; linear_x3.hip)
  auto pack_linear_x3 = [](const std::vector<float>& W, int N, int K, int BN) {
    std::vector<uint16_t> px((size_t)N * K * 2, 0);
    auto rne = [](float x) -> uint32_t {
      uint32_t u;
      std::memcpy(&u, &x, 4);
      return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
    };
    for (int o = 0; o < N; ++o)
      for (int i = 0; i < K; ++i) {
        const float x = W[(size_t)o * K + i];
        const uint32_t hb = rne(x);
        const uint32_t hbits = hb << 16;
        float hf;
        std::memcpy(&hf, &hbits, 4);
        const uint32_t lb = rne(x - hf);
        const int nt = o / BN, n = o % BN, ks = i / 16, k = i % 16, sw = (n >> 2) & 3;
        const size_t rec = (((size_t)nt * (K / 16) + ks) * BN + n) * 32;
        px[rec + 8 * ((k / 8) ^ sw) + (k % 8)] = (uint16_t)hb;
        px[rec + 8 * ((2 + k / 8) ^ sw) + (k % 8)] = (uint16_t)lb;
      }
    return px;
  };
  if (is_gru(h)) {
    w_ih.resize(1536 * 512);
    b_ih.resize(1536);
    whhT.resize(2 * 256 * 768);
    bhh.resize(2 * 768);
    const char* sfx[2] = {"", "_reverse"};
    for (int d = 0; d < 2; ++d) {
      const auto& wih = get(std::string("gru.weight_ih_l0") + sfx[d]);
      const auto& whh = get(std::string("gru.weight_hh_l0") + sfx[d]);
      const auto& bi = get(std::string("gru.bias_ih_l0") + sfx[d]);
      const auto& bh = get(std::string("gru.bias_hh_l0") + sfx[d]);
      std::copy(wih.begin(), wih.end(), w_ih.begin() + (size_t)d * 768 * 512);
      std::copy(bi.begin(), bi.end(), b_ih.begin() + d * 768);
      std::copy(bh.begin(), bh.end(), bhh.begin() + d * 768);
      for (int r = 0; r < 768; ++r)
        for (int k = 0; k < 256; ++k) whhT[((size_t)d * 256 + k) * 768 + r] = whh[(size_t)r * 256 + k];
      whh_nat.insert(whh_nat.end(), whh.begin(), whh.end());
    }
  } else {
    wqkv.resize(1536 * 512);
    bqkv.resize(1536);
    const char* nm[3] = {"w_qs", "w_ks", "w_vs"};
    for (int i = 0; i < 3; ++i) {
      const auto& ww = get(std::string("multihead.") + nm[i] + ".weight");
      const auto& bb = get(std::string("multihead.") + nm[i] + ".bias");
      std::copy(ww.begin(), ww.end(), wqkv.begin() + (size_t)i * 512 * 512);
      std::copy(bb.begin(), bb.end(), bqkv.begin() + i * 512);
    }
    wfc = get("multihead.fc.weight");
    bfc = get("multihead.fc.bias");
  }
  std::vector<float> wac((size_t)h->nac * 512, 0.f), bac(h->nac, 0.f);
  {
    const auto& wa = get("att_block.att.weight");
    const auto& ba = get("att_block.att.bias");
    const auto& wc = get("att_block.cla.weight");
    const auto& bc = get("att_block.cla.bias");
    for (int c = 0; c < C; ++c) {
      std::copy(wa.begin() + (size_t)c * 512, wa.begin() + (size_t)(c + 1) * 512, wac.begin() + (size_t)c * 512);
      std::copy(wc.begin() + (size_t)c * 512, wc.begin() + (size_t)(c + 1) * 512,
                wac.begin() + (size_t)(C + c) * 512);
      bac[c] = ba[c];
      bac[C + c] = bc[c];
    }
  }

  // ---- gammatone tables (float64, numpy operation order: gamma_weights.cpp) ----
  std::vector<double> g_tw, g_win, g_wT;
  if (h->cfg.feature_type == SEDX_FEATURE_GAMMA) {
    // fft_gtgram (fftweight.py:151-152) + gtgram_strides (gtgram.py:23-40)
    const double fs = h->cfg.sample_rate;
    const double win_t = (double)h->cfg.window_size / fs, hop_t = (double)h->cfg.hop_size / fs;
    const int nfft_g = (int)std::pow(2.0, std::ceil(std::log2(2 * win_t * fs)));
    auto rhaz = [](double x) { return (x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0)) * std::floor(std::fabs(x) + 0.5); };
    const int nwin = (int)rhaz(win_t * fs), nhop = (int)rhaz(hop_t * fs);
    if (nfft_g != 512 && nfft_g != 1024 && nfft_g != 2048)
      return fail(h, SEDX_EINVAL, "gammatone nfft %d unsupported", nfft_g);
    h->g_nfft = nfft_g;
    h->g_nwin = nwin;
    h->g_hop = nhop;
    gamma_tables(fs, nfft_g, nwin, 64, h->cfg.fmin, g_wT, gamma_kp(nfft_g), g_tw, g_win);
  }

  // ---- upload: one blob ----
  struct Item {
    void** dst;
    const void* src;
    size_t bytes;
  };
  std::vector<Item> items;
  auto add = [&](void** dst, const void* src, size_t bytes) { items.push_back({dst, src, bytes}); };
  DevWeights& W = h->w;
  W = DevWeights();
  add((void**)&W.twiddle, tw.data(), tw.size() * 4);
  add((void**)&W.window, window.data(), window.size() * 4);
  add((void**)&W.mel_w, mel_w.data(), mel_w.size() * 4);
  add((void**)&W.mel_tab, mel_tab.data(), mel_tab.size() * 4);
  if (!mel_mt.empty() && mel_mt.size() <= (size_t)FE_MT_MAX_FLOATS) {
    add((void**)&W.mel_mt, mel_mt.data(), mel_mt.size() * 4);
    for (int j = 0; j < 4; ++j) {
      W.mt_klo[j] = mt_klo[j];
      W.mt_ns[j] = mt_ns[j];
      W.mt_off[j] = mt_off[j];
    }
    W.mt_floats = (int32_t)mel_mt.size();
  }
  W.mel_wmax = mel_wmax;
  add((void**)&W.mel_off, mel_off.data(), mel_off.size() * 4);
  add((void**)&W.mel_lo, mel_lo.data(), mel_lo.size() * 4);
  add((void**)&W.bn0_scale, sc0f.data(), 64 * 4);
  add((void**)&W.bn0_mean, mu0.data(), 64 * 4);
  add((void**)&W.bn0_bias, bi0.data(), 64 * 4);
  add((void**)&W.c1_w, c1w.data(), c1w.size() * 4);
  std::vector<float> c1wt(9 * 64);               // [tap][64]: channel pairs adjacent
  for (int o = 0; o < 64; ++o)
    for (int t = 0; t < 9; ++t) c1wt[t * 64 + o] = c1w[o * 9 + t];
  add((void**)&W.c1_wt, c1wt.data(), c1wt.size() * 4);
  add((void**)&W.c1_b, c1b.data(), c1b.size() * 4);
  std::vector<float> zeros(ZERO_BLOCK_FLOATS, 0.f);   // >= Cin + 4 floats: the Winograd halo DMA steps through it
  add((void**)&W.zero, zeros.data(), zeros.size() * 4);
  std::vector<float> trash(64 * 128, 0.f);
  add((void**)&W.trash, trash.data(), trash.size() * 4);
  for (int i = 1; i < 8; ++i) {
    add((void**)&W.wp[i], packed[i].data(), packed[i].size() * 4);
    add((void**)&W.cb[i], cbias[i].data(), cbias[i].size() * 4);
    add((void**)&W.wx3[i], packed_x3[i].data(), packed_x3[i].size() * 2);
    add((void**)&W.wu[i], packed_wu[i].data(), packed_wu[i].size() * 4);
    if (!packed_wu43[i].empty()) add((void**)&W.wu43[i], packed_wu43[i].data(), packed_wu43[i].size() * 4);
  }
  if (is_gru(h)) {
    add((void**)&W.w_ih, w_ih.data(), w_ih.size() * 4);
    add((void**)&W.b_ih, b_ih.data(), b_ih.size() * 4);
    add((void**)&W.whhT, whhT.data(), whhT.size() * 4);
    add((void**)&W.whh, whh_nat.data(), whh_nat.size() * 4);
    add((void**)&W.bhh, bhh.data(), bhh.size() * 4);
  } else {
    add((void**)&W.wqkv, wqkv.data(), wqkv.size() * 4);
    add((void**)&W.bqkv, bqkv.data(), bqkv.size() * 4);
    add((void**)&W.wfc, wfc.data(), wfc.size() * 4);
    add((void**)&W.bfc, bfc.data(), bfc.size() * 4);
  }
  add((void**)&W.wac, wac.data(), wac.size() * 4);
  add((void**)&W.bac, bac.data(), bac.size() * 4);
  std::vector<uint16_t> w_ih_x3, wqkv_x3, wfc_x3, wac_x3;
  if (is_gru(h)) {
    w_ih_x3 = pack_linear_x3(w_ih, 1536, 512, 128);
    add(&W.w_ih_x3, w_ih_x3.data(), w_ih_x3.size() * 2);
  } else {
    wqkv_x3 = pack_linear_x3(wqkv, 1536, 512, 128);
    wfc_x3 = pack_linear_x3(wfc, 512, 512, 128);
    add(&W.wqkv_x3, wqkv_x3.data(), wqkv_x3.size() * 2);
    add(&W.wfc_x3, wfc_x3.data(), wfc_x3.size() * 2);
  }
  wac_x3 = pack_linear_x3(wac, h->nac, 512, 64);
  add(&W.wac_x3, wac_x3.data(), wac_x3.size() * 2);
  if (!g_wT.empty()) {
    add((void**)&W.g_twiddle, g_tw.data(), g_tw.size() * 8);
    add((void**)&W.g_window, g_win.data(), g_win.size() * 8);
    add((void**)&W.g_weightsT, g_wT.data(), g_wT.size() * 8);
  }
  size_t total = 0;
  for (auto& it : items) total += (it.bytes + 255) & ~size_t(255);
  if (h->blob) {
    (void)hipFree(h->blob);
    h->blob = nullptr;
  }
  HIP_TRY(h, hipMalloc(&h->blob, total));
  h->blob_bytes = total;
  std::vector<char> host(total, 0);
  size_t off = 0;
  for (auto& it : items) {
    std::memcpy(host.data() + off, it.src, it.bytes);
    *it.dst = static_cast<char*>(h->blob) + off;
    off += (it.bytes + 255) & ~size_t(255);
  }
  HIP_TRY(h, hipMemcpy(h->blob, host.data(), total, hipMemcpyHostToDevice));
  if (!h->gru_err_host) {
    void* p = nullptr;
    HIP_TRY(h, hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
    h->gru_err_host = static_cast<unsigned*>(p);
    *h->gru_err_host = 0;
    void* d = nullptr;
    HIP_TRY(h, hipHostGetDevicePointer(&d, p, 0));
    h->gru_err_dev = static_cast<unsigned*>(d);
  }
  h->finalized = true;
  return SEDX_OK;
}

sedx_status sedx_set_profiling(sedx_handle* h, int32_t on) {
  if (!h) return SEDX_EINVAL;
  DeviceGuard dg(h->device);
  if (on && !h->ev[0])
    for (auto& e : h->ev) HIP_TRY(h, hipEventCreate(&e));
  if (on < 0 || on > 2) return fail(h, SEDX_EINVAL, "profiling mode %d (0 off, 1 last forward, 2 accumulate)", (int)on);
  if (h->profiling == 2) fold_ev_pool(h);
  // mode 2: event sets for the first 64 forwards up front, so a timed loop
  // does not create events on the host while it issues work
  while (on == 2 && h->ev_pool.size() < 64) {
    h->ev_pool.emplace_back();
    for (auto& e : h->ev_pool.back().ev) HIP_TRY(h, hipEventCreate(&e));
  }
  h->profiling = on;
  for (auto& r : h->ev_recorded) r = false;
  h->ev_used = 0;
  h->ev_cur = nullptr;
  for (int i = 0; i < SEDX_N_STAGES; ++i) {
    h->acc_ms[i] = 0.0;
    h->acc_n[i] = 0;
  }
  return SEDX_OK;
}

sedx_status sedx_set_pipelined(sedx_handle* h, int32_t on) {
  if (!h) return SEDX_EINVAL;
  DeviceGuard dg(h->device);
  if (on && !h->conv_done) HIP_TRY(h, hipEventCreateWithFlags(&h->conv_done, hipEventDisableTiming));
  if (on < 0 || on > 2) return fail(h, SEDX_EINVAL, "sedx_set_pipelined: on must be 0, 1 or 2");
  h->pipelined = on != 0;
  h->pipe_conv1_first = on == 2;
  h->conv_done_recorded = false;
  return SEDX_OK;
}

sedx_status sedx_stage_times(sedx_handle* h, float* ms, int32_t capacity, int32_t* n_stages) {
  if (!h || !n_stages) return SEDX_EINVAL;
  *n_stages = SEDX_N_STAGES;
  if (!h->profiling) return fail(h, SEDX_ESTATE, "profiling is off");
  DeviceGuard dg(h->device);
  if (sedx_status e = check_async_error(h)) return e;
  if (h->profiling == 2) {
    fold_ev_pool(h);
    for (int i = 0; i < SEDX_N_STAGES; ++i) {
      if (i < capacity) ms[i] = h->acc_n[i] ? (float)(h->acc_ms[i] / (double)h->acc_n[i]) : 0.f;
      h->acc_ms[i] = 0.0;
      h->acc_n[i] = 0;
    }
    return SEDX_OK;
  }
  for (int i = 0; i < SEDX_N_STAGES && i < capacity; ++i) {
    float v = 0.f;
    const int a = stage_begin(i), b = stage_end(i);
    if (h->ev_recorded[a] && h->ev_recorded[b]) {
      HIP_TRY(h, hipEventSynchronize(h->ev[b]));
      HIP_TRY(h, hipEventElapsedTime(&v, h->ev[a], h->ev[b]));
    }
    ms[i] = v;
  }
  return SEDX_OK;
}

sedx_status sedx_output_geometry(const sedx_handle* h, int64_t L_or_T, int64_t* out_frames,
                                 int64_t* seq_len) {
  if (!h || !out_frames || !seq_len) return SEDX_EINVAL;
  const int64_t T = (h->cfg.feature_type == SEDX_FEATURE_GAMMA) ? L_or_T : conv_T(h, L_or_T);
  const Geometry g = geometry_from_T(h, T);
  *out_frames = g.out_frames;
  *seq_len = g.T3;
  return SEDX_OK;
}

sedx_status sedx_workspace_size(const sedx_handle* h, int64_t B, int64_t L_or_T, size_t* bytes) {
  if (!h || !bytes || B <= 0) return SEDX_EINVAL;
  const int64_t T = (h->cfg.feature_type == SEDX_FEATURE_GAMMA) ? L_or_T : conv_T(h, L_or_T);
  *bytes = ws_layout(h, B, geometry_from_T(h, T)).total_bytes;
  return SEDX_OK;
}

static sedx_status forward_wave(sedx_handle* h, const float* d_wave, const int16_t* d_wave16, int64_t B,
                                int64_t L, float* d_framewise, float* d_clipwise, float* d_embedding,
                                void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!h) return SEDX_EINVAL;
  if (!h->finalized) return fail(h, SEDX_ESTATE, "weights not finalised");
  if (sedx_status e = check_async_error(h)) return e;
  if (h->cfg.feature_type != SEDX_FEATURE_LOGMEL)
    return fail(h, SEDX_EINVAL, "gamma models take features: use sedx_forward_features");
  if ((!d_wave && !d_wave16) || !d_framewise || !d_clipwise || B <= 0)
    return fail(h, SEDX_EINVAL, "null pointer or empty batch");
  const int n2 = h->cfg.window_size / 2;
  if (L <= n2)
    return fail(h, SEDX_EINVAL, "input of %lld samples is too short for reflect padding of %d",
                (long long)L, n2);
  const Geometry g = geometry_from_T(h, conv_T(h, L));
  if (g.T3 < 1) return fail(h, SEDX_EINVAL, "input too short for the 3 pooling stages");
  if (B * g.T > INT32_MAX / 64) return fail(h, SEDX_EINVAL, "batch too large");
  DeviceGuard dg(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const WsLayout l = ws_layout(h, B, g);
  float* ws = nullptr;
  sedx_status st = get_ws(h, l.total_bytes, d_workspace, workspace_bytes, &ws);
  if (st != SEDX_OK) return st;
  FrontendParams p{};
  p.audio = d_wave;
  p.audio_i16 = d_wave16;
  p.clip_stride = L;
  p.n_clips = (int32_t)B;
  p.n_win = 1;
  p.win_start = nullptr;
  p.clip_len = L;
  p.sig_len = L;
  p.T = (int32_t)g.T;
  p.hop = h->cfg.hop_size;
  p.twiddle = h->w.twiddle;
  p.window = h->w.window;
  p.mel_w = h->w.mel_w;
  p.mel_tab = h->w.mel_tab;
  set_mel_mt(p, h->w, h->mel_mfma);
  p.mel_wmax = h->w.mel_wmax;
  p.mel_off = h->w.mel_off;
  p.mel_lo = h->w.mel_lo;
  p.bn_scale = h->w.bn0_scale;
  p.bn_mean = h->w.bn0_mean;
  p.bn_bias = h->w.bn0_bias;
  p.out = ws + l.x0;
  mark(h, 0, s);
  launch_logmel(p, h->cfg.window_size, s);
  return run_body(h, B, g, ws, l, d_framewise, d_clipwise, d_embedding, s);
}

sedx_status sedx_forward(sedx_handle* h, const float* d_wave, int64_t B, int64_t L,
                         float* d_framewise, float* d_clipwise, float* d_embedding,
                         void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!d_wave) return fail(h, SEDX_EINVAL, "null waveform pointer");
  return forward_wave(h, d_wave, nullptr, B, L, d_framewise, d_clipwise, d_embedding, d_workspace,
                      workspace_bytes, stream);
}

sedx_status sedx_forward_i16(sedx_handle* h, const int16_t* d_wave, int64_t B, int64_t L,
                             float* d_framewise, float* d_clipwise, float* d_embedding,
                             void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!d_wave) return fail(h, SEDX_EINVAL, "null waveform pointer");
  return forward_wave(h, nullptr, d_wave, B, L, d_framewise, d_clipwise, d_embedding, d_workspace,
                      workspace_bytes, stream);
}

sedx_status sedx_forward_features(sedx_handle* h, const float* d_feat, int64_t B, int64_t T,
                                  float* d_framewise, float* d_clipwise, float* d_embedding,
                                  void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!h) return SEDX_EINVAL;
  if (!h->finalized) return fail(h, SEDX_ESTATE, "weights not finalised");
  if (sedx_status e = check_async_error(h)) return e;
  if (!d_feat || !d_framewise || !d_clipwise || B <= 0 || T <= 0)
    return fail(h, SEDX_EINVAL, "null pointer or empty batch");
  const Geometry g = geometry_from_T(h, T);
  if (g.T3 < 1) return fail(h, SEDX_EINVAL, "input too short for the 3 pooling stages");
  DeviceGuard dg(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const WsLayout l = ws_layout(h, B, g);
  float* ws = nullptr;
  sedx_status st = get_ws(h, l.total_bytes, d_workspace, workspace_bytes, &ws);
  if (st != SEDX_OK) return st;
  mark(h, 0, s);
  launch_features_bn0(d_feat, (int)B, (int)T, h->w.bn0_scale, h->w.bn0_mean, h->w.bn0_bias,
                      ws + l.x0, s);
  return run_body(h, B, g, ws, l, d_framewise, d_clipwise, d_embedding, s);
}

sedx_status sedx_gamma_features(sedx_handle* h, const float* d_audio, int64_t B, int64_t L,
                                float* d_feat, int64_t* T_out, void* d_workspace,
                                size_t workspace_bytes, void* stream) {
  if (!h) return SEDX_EINVAL;
  if (!h->finalized) return fail(h, SEDX_ESTATE, "weights not finalised");
  if (sedx_status e = check_async_error(h)) return e;
  if (h->cfg.feature_type != SEDX_FEATURE_GAMMA)
    return fail(h, SEDX_EINVAL, "handle was not created with feature_type=gamma");
  if (L < h->g_nfft) return fail(h, SEDX_EINVAL, "clip shorter than the gammatone FFT");
  const int64_t T = 1 + (L - h->g_nfft) / h->g_hop;
  if (T_out) *T_out = T;
  if (!d_feat) return SEDX_OK;   // geometry query
  if (!d_audio || B <= 0) return fail(h, SEDX_EINVAL, "null pointer or empty batch");
  if (B > INT32_MAX / 64 || B * T > INT32_MAX / 64) return fail(h, SEDX_EINVAL, "batch too large");
  const int64_t fill = (L - h->g_nfft + h->g_hop - 1) / h->g_hop;   // len(range(0, s-n, h))
  DeviceGuard dg(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t need = gamma_workspace_bytes(B, T, h->g_nfft);
  float* ws = nullptr;
  sedx_status st = get_ws(h, need, d_workspace, workspace_bytes, &ws);
  if (st != SEDX_OK) return st;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  char* base = reinterpret_cast<char*>(ws);
  GammaParams p{};
  p.audio = d_audio;
  p.L = L;
  p.B = (int32_t)B;
  p.T = (int32_t)T;
  p.T_fill = (int32_t)std::min<int64_t>(fill, T);
  p.hop = h->g_hop;
  p.nfft = h->g_nfft;
  p.kp = gamma_kp(h->g_nfft);
  p.twiddle = h->w.g_twiddle;
  p.window = h->w.g_window;
  p.weightsT = h->w.g_weightsT;
  p.mag = reinterpret_cast<double*>(base);
  base += al((size_t)B * T * p.kp * sizeof(double));
  p.db = reinterpret_cast<double*>(base);
  base += al((size_t)B * 64 * T * sizeof(double));
  p.mm = reinterpret_cast<unsigned long long*>(base);
  p.out = d_feat;
  launch_gamma(p, s, h->gamma_spec);
  return launch_status(h);
}

sedx_status sedx_gamma_workspace_size(const sedx_handle* h, int64_t B, int64_t L, size_t* bytes) {
  if (!h) return SEDX_EINVAL;
  sedx_handle* hm = const_cast<sedx_handle*>(h);   // sedx_last_error's message only
  if (!bytes || B <= 0) return fail(hm, SEDX_EINVAL, "null size pointer or empty batch");
  if (h->cfg.feature_type != SEDX_FEATURE_GAMMA)
    return fail(hm, SEDX_EINVAL, "handle was not created with feature_type=gamma");
  if (!h->finalized) return fail(hm, SEDX_ESTATE, "weights not finalised");
  if (L < h->g_nfft) return fail(hm, SEDX_EINVAL, "clip shorter than the gammatone FFT");
  *bytes = gamma_workspace_bytes(B, 1 + (L - h->g_nfft) / h->g_hop, h->g_nfft);
  return SEDX_OK;
}

// host-side failures of the window entry points (plan vectors) become
// status codes instead of exceptions crossing the C ABI
#define SEDX_HOST_TRY(h, body)                                                              \
  try {                                                                                     \
    body                                                                                    \
  } catch (const std::bad_alloc&) {                                                         \
    return fail(const_cast<sedx_handle*>(h), SEDX_ENOMEM, "host allocation failed (merge plan)"); \
  } catch (...) {                                                                           \
    return fail(const_cast<sedx_handle*>(h), SEDX_EINVAL, "host-side failure building the window plan"); \
  }

sedx_status sedx_window_geometry(const sedx_handle* h, int64_t L_clip, const sedx_window_spec* spec,
                                 int64_t* n_windows, int64_t* window_samples, int64_t* merged_frames) {
  if (!h) return SEDX_EINVAL;
  SEDX_HOST_TRY(h, {
    WinGeom wg;
    // the plan of the forward the spec names: avg_merge rejects a zero step
    sedx_status st = window_geometry(h, L_clip, spec, spec && spec->vote == 0, &wg);
    if (st != SEDX_OK) return st;
    if (n_windows) *n_windows = wg.n_win;
    if (window_samples) *window_samples = wg.full_len;
    if (merged_frames) *merged_frames = wg.plan.N;
    return SEDX_OK;
  })
}

// every window of every clip through the model (one batch per window group),
// then the merge by the host's plan (avg or vote)
static sedx_status forward_windows_impl(sedx_handle* h, const float* d_audio, int64_t n_clips, int64_t L_clip,
                                        const sedx_window_spec* spec, const double* h_vote_thres, float* d_merged,
                                        void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!h) return SEDX_EINVAL;
  if (!h->finalized) return fail(h, SEDX_ESTATE, "weights not finalised");
  if (sedx_status e = check_async_error(h)) return e;
  if (h->cfg.feature_type != SEDX_FEATURE_LOGMEL)
    return fail(h, SEDX_EINVAL, "windowed inference needs a logmel model");
  if (!d_audio || !d_merged || n_clips <= 0) return fail(h, SEDX_EINVAL, "null pointer or empty batch");
  if (spec && spec->vote != 0 && h_vote_thres == nullptr)
    return fail(h, SEDX_EINVAL, "spec.vote = 1: call sedx_forward_windows_vote");
  WinGeom wg;
  sedx_status st = window_geometry(h, L_clip, spec, h_vote_thres == nullptr, &wg);
  if (st != SEDX_OK) return st;
  // the frontend and conv launches index items with 32-bit sizes (as forward_wave)
  for (const auto& g : wg.groups)
    if (n_clips > INT32_MAX / g.nw || n_clips * g.nw * g.g.T > INT32_MAX / 64)
      return fail(h, SEDX_EINVAL, "batch too large: %lld clips x %d windows", (long long)n_clips, g.nw);
  if (n_clips * wg.plan.N > INT32_MAX / h->cfg.classes_num)
    return fail(h, SEDX_EINVAL, "merged output too large");
  DeviceGuard dg(h->device);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const WinLayout wl = win_layout(h, n_clips, wg);
  float* ws = nullptr;
  st = get_ws(h, wl.total_bytes, d_workspace, workspace_bytes, &ws);
  if (st != SEDX_OK) return st;
  const int C = h->cfg.classes_num;
  // tables: built on the host, one copy (the host vector is consumed by the
  // call: pageable-source hipMemcpyAsync stages it before returning)
  std::vector<char> blob(wl.table_bytes, 0);
  int64_t* t_start = reinterpret_cast<int64_t*>(blob.data() + wl.t_start);
  int64_t* t_wb = reinterpret_cast<int64_t*>(blob.data() + wl.t_wb);
  int64_t* t_wcs = reinterpret_cast<int64_t*>(blob.data() + wl.t_wcs);
  int32_t* t_off = reinterpret_cast<int32_t*>(blob.data() + wl.t_off);
  int2* t_src = reinterpret_cast<int2*>(blob.data() + wl.t_src);
  int32_t* t_div = reinterpret_cast<int32_t*>(blob.data() + wl.t_div);
  std::copy(wg.loop.start.begin(), wg.loop.start.end(), t_start);
  for (size_t gi = 0; gi < wg.groups.size(); ++gi) {
    const WinGroup& g = wg.groups[gi];
    for (int i = 0; i < g.nw; ++i) {
      t_wb[g.w0 + i] = (int64_t)(wl.fw_off[gi] - wl.model_bytes / sizeof(float)) + (int64_t)i * g.g.out_frames * C;
      t_wcs[g.w0 + i] = (int64_t)g.nw * g.g.out_frames * C;
    }
  }
  std::copy(wg.plan.off.begin(), wg.plan.off.end(), t_off);
  for (size_t j = 0; j < wg.plan.src.size(); ++j) {
    const int32_t id = wg.plan.src[j];
    const int w = (int)(std::upper_bound(wg.plan.win_base.begin(), wg.plan.win_base.end(), id) -
                        wg.plan.win_base.begin()) - 1;
    t_src[j] = make_int2(w, id - wg.plan.win_base[w]);
  }
  std::copy(wg.plan.div.begin(), wg.plan.div.end(), t_div);
  char* d_tables = reinterpret_cast<char*>(ws + wl.tables);
  HIP_TRY(h, hipMemcpyAsync(d_tables, blob.data(), blob.size(), hipMemcpyHostToDevice, s));
  double* vthr = reinterpret_cast<double*>(ws + wl.vthr);
  if (h_vote_thres) HIP_TRY(h, hipMemcpyAsync(vthr, h_vote_thres, C * sizeof(double), hipMemcpyHostToDevice, s));
  const int64_t* d_start = reinterpret_cast<const int64_t*>(d_tables + wl.t_start);
  mark(h, 0, s);
  for (size_t gi = 0; gi < wg.groups.size(); ++gi) {
    const WinGroup& g = wg.groups[gi];
    const WsLayout l = ws_layout(h, n_clips * g.nw, g.g);
    FrontendParams p{};
    p.audio = d_audio;
    p.clip_stride = L_clip;
    p.n_clips = (int32_t)n_clips;
    p.n_win = g.nw;
    p.win_start = d_start + g.w0;
    p.clip_len = wg.clip_len;
    p.sig_len = g.len;
    p.T = (int32_t)g.g.T;
    p.hop = h->cfg.hop_size;
    p.twiddle = h->w.twiddle;
    p.window = h->w.window;
    p.mel_w = h->w.mel_w;
    p.mel_tab = h->w.mel_tab;
    set_mel_mt(p, h->w, h->mel_mfma);
    p.mel_wmax = h->w.mel_wmax;
    p.mel_off = h->w.mel_off;
    p.mel_lo = h->w.mel_lo;
    p.bn_scale = h->w.bn0_scale;
    p.bn_mean = h->w.bn0_mean;
    p.bn_bias = h->w.bn0_bias;
    p.out = ws + l.x0;
    launch_logmel(p, h->cfg.window_size, s);
    st = run_body(h, n_clips * g.nw, g.g, ws, l, ws + wl.fw_off[gi], ws + wl.clip_off[gi], nullptr, s);
    if (st != SEDX_OK) return st;
  }
  MergeArgs a{};
  a.fw = ws + wl.model_bytes / sizeof(float);
  a.wb = reinterpret_cast<const int64_t*>(d_tables + wl.t_wb);
  a.wcs = reinterpret_cast<const int64_t*>(d_tables + wl.t_wcs);
  a.off = reinterpret_cast<const int32_t*>(d_tables + wl.t_off);
  a.src = reinterpret_cast<const int2*>(d_tables + wl.t_src);
  a.div = reinterpret_cast<const int32_t*>(d_tables + wl.t_div);
  a.vote_thr = h_vote_thres ? vthr : nullptr;
  a.n_clips = (int32_t)n_clips;
  a.N = (int32_t)wg.plan.N;
  a.C = C;
  a.merged = d_merged;
  launch_merge_plan(a, s);
  return launch_status(h);
}

sedx_status sedx_window_workspace_size(const sedx_handle* h, int64_t n_clips, int64_t L_clip,
                                       const sedx_window_spec* spec, size_t* bytes) {
  if (!h || !bytes || n_clips <= 0) return SEDX_EINVAL;
  SEDX_HOST_TRY(h, {
    WinGeom wg;
    sedx_status st = window_geometry(h, L_clip, spec, spec && spec->vote == 0, &wg);
    if (st != SEDX_OK) return st;
    *bytes = win_layout(h, n_clips, wg).total_bytes;
    return SEDX_OK;
  })
}

sedx_status sedx_forward_windows(sedx_handle* h, const float* d_audio, int64_t n_clips, int64_t L_clip,
                                 const sedx_window_spec* spec, float* d_merged, void* d_workspace,
                                 size_t workspace_bytes, void* stream) {
  if (!h) return SEDX_EINVAL;
  SEDX_HOST_TRY(h, {
    return forward_windows_impl(h, d_audio, n_clips, L_clip, spec, nullptr, d_merged, d_workspace, workspace_bytes,
                                stream);
  })
}

sedx_status sedx_forward_windows_vote(sedx_handle* h, const float* d_audio, int64_t n_clips, int64_t L_clip,
                                      const sedx_window_spec* spec, const double* bin_thres, float* d_votes,
                                      void* d_workspace, size_t workspace_bytes, void* stream) {
  if (!h) return SEDX_EINVAL;
  if (!bin_thres) return fail(h, SEDX_EINVAL, "vote mode needs the per-class binarisation thresholds");
  SEDX_HOST_TRY(h, {
    return forward_windows_impl(h, d_audio, n_clips, L_clip, spec, bin_thres, d_votes, d_workspace, workspace_bytes,
                                stream);
  })
}
#undef SEDX_HOST_TRY

sedx_status sedx_events_workspace_size(int64_t n_clips, int64_t T, int64_t C, size_t* bytes) {
  if (!bytes || n_clips < 0 || T < 0 || C <= 0) return SEDX_EINVAL;
  *bytes = events_workspace_bytes(n_clips * C, T, C);
  return SEDX_OK;
}

sedx_status sedx_events_device(const float* d_x, int64_t n_clips, int64_t T, int64_t C,
                               const double* high_thres, const double* low_thres,
                               int32_t use_low_thres, const int64_t* n_smooth, const int64_t* n_salt,
                               int32_t mode, double overlap_value, int32_t sample_duration,
                               int32_t* d_events, int64_t capacity, int64_t* d_info,
                               void* d_workspace, size_t workspace_bytes, void* stream) {
  if (n_clips < 0 || T < 0 || C <= 0 || !d_info || !n_smooth || !n_salt || (mode != 0 && mode != 1) ||
      (n_clips > 0 && !d_x) || (capacity > 0 && !d_events) || capacity < 0 ||
      (use_low_thres && !low_thres) || (mode == 0 && !high_thres))
    return SEDX_EINVAL;
  // int(100 * overlap_value) in float64 (vad.py:63)
  if (mode == 1 && !(std::fabs(100.0 * overlap_value) < 1e9)) return SEDX_EINVAL;
  const int64_t step = mode == 1 ? (int64_t)(100.0 * overlap_value) : 0;
  // step 0: range(0, N - 0, 0) raises; step < 0: the range is empty, no
  // frame is ever a candidate and the reference returns no events
  if (mode == 1 && (step == 0 || sample_duration <= 0)) return SEDX_EINVAL;
  if (T > events_max_frames()) return SEDX_EINVAL;   // a series' two bitmaps live in LDS
  const size_t need = events_workspace_bytes(n_clips * C, T, C);
  if (!d_workspace || workspace_bytes < need) return SEDX_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // per-class parameters -> one packed block in the workspace, one copy
  // (f32 high: the mode-0 compare is float32)
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  char* p = static_cast<char*>(d_workspace);
  int64_t* counts = reinterpret_cast<int64_t*>(p);
  p += al(n_clips * C * 8);
  int64_t* slots = reinterpret_cast<int64_t*>(p);
  p += al(n_clips * C * events_slot_cap(T) * 8);
  const size_t o_hi = 0, o_lo = al(C * 4), o_ns = o_lo + al(C * 8), o_salt = o_ns + al(C * 8);
  std::vector<char> blob(o_salt + C * 8, 0);
  for (int64_t k = 0; k < C; ++k) {
    reinterpret_cast<float*>(blob.data() + o_hi)[k] = high_thres ? (float)high_thres[k] : 0.f;
    reinterpret_cast<double*>(blob.data() + o_lo)[k] = use_low_thres ? low_thres[k] : 0.0;
    reinterpret_cast<int64_t*>(blob.data() + o_ns)[k] = n_smooth[k];
    reinterpret_cast<int64_t*>(blob.data() + o_salt)[k] = n_salt[k];
  }
  if (hipMemcpyAsync(p, blob.data(), blob.size(), hipMemcpyHostToDevice, s) != hipSuccess) return SEDX_EHIP;
  const float* d_hi = reinterpret_cast<const float*>(p + o_hi);
  const double* d_lo = reinterpret_cast<const double*>(p + o_lo);
  const int64_t* d_ns = reinterpret_cast<const int64_t*>(p + o_ns);
  const int64_t* d_nsalt = reinterpret_cast<const int64_t*>(p + o_salt);
  EventArgs a{d_x, n_clips, T, C, d_hi, d_lo, d_ns, d_nsalt, use_low_thres,
              step, (int64_t)sample_duration, counts, slots, events_slot_cap(T), d_info, d_events,
              capacity};
  launch_events(a, mode, s);
  if (take_launch_error() != hipSuccess) return SEDX_EHIP;
  return hipGetLastError() == hipSuccess ? SEDX_OK : SEDX_EHIP;
}

}  // extern "C"
