// Block 1's one-launch Winograd kernel (wino_block1_kernel: conv1 computed
// into conv2's halo staging + F(2x2,3x3) conv2 + 2x2 pool) stand-alone at the
// bench shape (B clips x 1001 frames x 64 bins), random operands:
// time per launch, an output checksum (a stamped build must match the plain
// one), and — in a SEDX_WINO_STAMPS build — the per-phase s_memtime split of
// the waves' cycles.  Ablation builds (SEDX_WINO_ABL) give wrong outputs and
// are timed only.  Built and run by tools/gpu_r04d.sh.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "../sound-event-detection_amd/csrc/sedx_internal.h"

namespace sedx {
#ifdef SEDX_WINO_STAMPS
void wino_stamps_rw(unsigned long long* h, bool reset);
#endif
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const char* tag = argc > 3 ? argv[3] : "plain";
  const int T = 1001;
  std::mt19937 rng(11);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> x0((size_t)B * T * 64), w1(64 * 9), b1(64), bias(64);
  for (auto& v : x0) v = nd(rng);
  for (auto& v : w1) v = nd(rng) * 0.3f;
  for (auto& v : b1) v = 0.1f * nd(rng);
  for (auto& v : bias) v = 0.1f * nd(rng);
  std::vector<double> w((size_t)64 * 64 * 9);
  const float ws = std::sqrt(2.f / (9 * 64));
  for (auto& v : w) v = (double)(float)(nd(rng) * ws);
  std::vector<float> U((size_t)64 * 64 * 16);
  sedx::pack_conv_wino(w.data(), 64, 64, U.data());
  const size_t nout = (size_t)B * (T / 2) * 32 * 64;
  float *d_x0, *d_w1, *d_b1, *d_U, *d_bias, *d_out, *d_zero, *d_trash;
  hipMalloc(&d_x0, x0.size() * 4);
  hipMalloc(&d_w1, w1.size() * 4);
  hipMalloc(&d_b1, b1.size() * 4);
  hipMalloc(&d_U, U.size() * 4);
  hipMalloc(&d_bias, bias.size() * 4);
  hipMalloc(&d_out, nout * 4);
  hipMalloc(&d_zero, sedx::ZERO_BLOCK_FLOATS * 4);
  hipMalloc(&d_trash, 64 * 128 * 4);
  hipMemset(d_zero, 0, sedx::ZERO_BLOCK_FLOATS * 4);
  hipMemcpy(d_x0, x0.data(), x0.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_w1, w1.data(), w1.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_b1, b1.data(), b1.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_U, U.data(), U.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_bias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice);
  hipMemset(d_out, 0xff, nout * 4);
  auto run = [&]() { sedx::launch_block1_wino(d_x0, B, T, d_w1, d_b1, d_U, d_bias, d_out, d_zero, d_trash, 0); };
  run();
  hipDeviceSynchronize();
  std::vector<float> out(nout);
  hipMemcpy(out.data(), d_out, nout * 4, hipMemcpyDeviceToHost);
  double sum = 0;
  unsigned long long hsh = 1469598103934665603ull;
  size_t nonfinite = 0;
  for (size_t i = 0; i < nout; ++i) {
    if (!std::isfinite(out[i])) ++nonfinite;
    sum += out[i];
    unsigned u;
    memcpy(&u, &out[i], 4);
    hsh = (hsh ^ u) * 1099511628211ull;
  }
#ifdef SEDX_WINO_STAMPS
  sedx::wino_stamps_rw(nullptr, true);
#endif
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) run();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%s B=%d  wino_block1 %.4f ms/launch  checksum %.6e  hash %016llx  nonfinite %zu  (err=%s, launch=%s)\n", tag,
         B, ms / reps, sum, hsh, nonfinite, hipGetErrorString(hipGetLastError()),
         hipGetErrorString(sedx::take_launch_error()));
#ifdef SEDX_WINO_STAMPS
  unsigned long long st[16];
  sedx::wino_stamps_rw(st, false);
  const char* names[] = {"prologue", "item top (chunk-0 reads + transform)", "chunk steps (MFMA + interleaved reads/transform/conv1)",
                         "barrier waits", "DMA issue (+X0 tile)", "window load", "epilogue"};
  const double tot = (double)st[7];
  printf("stamps: %llu waves sampled, %.0f cycles per wave (s_memtime)\n", st[8], tot / (st[8] ? st[8] : 1));
  double acc = 0;
  for (int i = 0; i < 7; ++i) {
    acc += st[i];
    printf("  %-58s %6.3f  (%.0f cycles/wave)\n", names[i], st[i] / tot, st[i] / (double)(st[8] ? st[8] : 1));
  }
  printf("  %-58s %6.3f\n", "unattributed", 1.0 - acc / tot);
#endif
  return nonfinite == 0 || argc > 4 ? 0 : 1;
}
