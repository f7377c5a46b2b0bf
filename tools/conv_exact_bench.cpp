// Stand-alone timing of the exact fp32 conv launches (conv.hip) at the bench
// shape (B clips x 10 s @ 16 kHz): block 1 fused (conv1 + conv2 + pool) and
// the six conv launches of blocks 2-4.  Random operands: time only (parity
// lives in tests/test_gpu_parity.py).  Built by tools/gpu_conv_exact.sh.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../sound-event-detection_amd/csrc/sedx_internal.h"
#ifdef SEDX_EXACT_STAMPS
namespace sedx { void exact_stamps_rw(unsigned long long* out8, bool reset); }
#endif

struct Layer { const char* name; int T, F, cin, cout, epi; };

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const char* only = argc > 3 ? argv[3] : nullptr;
  const Layer LM[] = {{"b1c2", 1001, 64, 64, 64, sedx::EPI_POOL2},  {"b2c1", 500, 32, 64, 128, sedx::EPI_STORE},
                      {"b2c2", 500, 32, 128, 128, sedx::EPI_POOL2}, {"b3c1", 250, 16, 128, 256, sedx::EPI_STORE},
                      {"b3c2", 250, 16, 256, 256, sedx::EPI_POOL2}, {"b4c1", 125, 8, 256, 512, sedx::EPI_STORE},
                      {"b4c2", 125, 8, 512, 512, sedx::EPI_FMEAN}};
  size_t max_in = (size_t)B * 1003 * 66, max_out = 0, max_w = 0;
  for (const Layer& l : LM) {
    max_in = std::max(max_in, (size_t)B * l.T * l.F * l.cin);
    max_out = std::max(max_out, (size_t)B * l.T * l.F * l.cout);
    max_w = std::max(max_w, (size_t)l.cin * l.cout * 9);
  }
  float *in, *out, *bias, *w, *w1, *b1, *zero;
  hipMalloc(&in, max_in * 4); hipMalloc(&out, max_out * 4); hipMalloc(&bias, 512 * 4);
  hipMalloc(&w, max_w * 4); hipMalloc(&w1, 64 * 9 * 4); hipMalloc(&b1, 64 * 4);
  hipMalloc(&zero, 256); hipMemset(zero, 0, 256);
  {
    std::vector<float> h(std::max(max_in, max_w));
    srand(1);
    for (auto& v : h) v = rand() / (float)RAND_MAX - 0.5f;
    hipMemcpy(in, h.data(), max_in * 4, hipMemcpyHostToDevice);
    for (auto& v : h) v *= 0.05f;
    hipMemcpy(w, h.data(), max_w * 4, hipMemcpyHostToDevice);
    hipMemcpy(w1, h.data(), 64 * 9 * 4, hipMemcpyHostToDevice);
    hipMemset(bias, 0, 512 * 4); hipMemset(b1, 0, 64 * 4);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  double tot_ms = 0, tot_f = 0;
  for (const Layer& l : LM) {
    if (only && strcmp(only, l.name) != 0) continue;
    auto go = [&]() {
      if (l.F == 64 && !getenv("CX_NOFUSE")) sedx::launch_block1_exact(in, B, l.T, w1, b1, w, bias, out, zero, 0);
      else sedx::launch_conv3x3(in, B, l.T, l.F, l.cin, l.cout, w, bias, out, l.epi, zero, 0);
    };
    go();
    hipDeviceSynchronize();
#ifdef SEDX_EXACT_STAMPS
    unsigned long long st[8];
    sedx::exact_stamps_rw(st, true);
#endif
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r) go();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    double fl = 2.0 * B * l.T * l.F * l.cin * l.cout * 9;
    if (l.F == 64) fl += 2.0 * B * l.T * 64 * 64 * 9;   // fused conv1
    tot_ms += ms; tot_f += fl;
    printf("%s  T=%4d F=%2d %3d->%3d  %.4f ms  %.1f TF/s  (%.3f of 157.3)\n", l.name, l.T, l.F, l.cin, l.cout, ms,
           fl / ms / 1e9, fl / ms / 1e9 / 157.3);
#ifdef SEDX_EXACT_STAMPS
    sedx::exact_stamps_rw(st, true);
    {
      const double tot = (double)st[0];
      printf("      stamps: waves %llu  barrier %.1f%%  conv1 %.1f%%  epilogue %.1f%%  (cycles/wave %.0f, clock %.2f GHz)\n",
             st[4], 100 * st[1] / tot, 100 * st[2] / tot, 100 * st[3] / tot, tot / (double)st[4],
             tot / (double)st[5] * 0.1);
    }
#endif
  }
  printf("total %.4f ms  %.1f TF/s  (err=%s, launch=%s)\n", tot_ms, tot_f / tot_ms / 1e9,
         hipGetErrorString(hipGetLastError()), hipGetErrorString(sedx::take_launch_error()));
  return 0;
}
