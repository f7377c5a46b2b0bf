// Stand-alone timing of the seven 3x3 conv layers (x3 path) at the bench
// shape (B clips x 10 s @ 16 kHz, 1001 frames).  Operand values are random:
// this measures time only (parity lives in tests/test_gpu_parity.py).
// Build variants with tools/gpu_conv_bench.sh (-DSEDX_CONV_STAMPS: phase split).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../sound-event-detection_amd/csrc/sedx_internal.h"

#ifdef SEDX_CONV_STAMPS
namespace sedx { void conv_stamps_rw(unsigned long long* out8, bool reset); }
#endif

struct Layer { const char* name; int T, F, cin, cout, epi; };

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const Layer LM[] = {{"b1c2", 1001, 64, 64, 64, sedx::EPI_POOL2},  {"b2c1", 500, 32, 64, 128, sedx::EPI_STORE},
                      {"b2c2", 500, 32, 128, 128, sedx::EPI_POOL2}, {"b3c1", 250, 16, 128, 256, sedx::EPI_STORE},
                      {"b3c2", 250, 16, 256, 256, sedx::EPI_POOL2}, {"b4c1", 125, 8, 256, 512, sedx::EPI_STORE},
                      {"b4c2", 125, 8, 512, 512, sedx::EPI_FMEAN}};
  // CB_SWEEP=1: K-length sweep at one shape (F=32, Cout 128, pooled), equal
  // FLOPs per layer (T scaled by 1/Cin): time per FLOP vs chunks per tile
  const Layer LS[] = {{"cin64", 1000, 32, 64, 128, sedx::EPI_POOL2},  {"cin128", 500, 32, 128, 128, sedx::EPI_POOL2},
                      {"cin256", 250, 32, 256, 128, sedx::EPI_POOL2}, {"cin512", 125, 32, 512, 128, sedx::EPI_POOL2},
                      {"s_cin64", 1000, 32, 64, 128, sedx::EPI_STORE}, {"s_cin256", 250, 32, 256, 128, sedx::EPI_STORE}};
  const bool sweep = getenv("CB_SWEEP") != nullptr;
  const Layer* L = sweep ? LS : LM;
  const int NL = sweep ? 6 : 7;
  size_t max_in = 0, max_w = 0;
  for (int li = 0; li < NL; ++li) {
    const Layer& l = L[li];
    max_in = std::max(max_in, (size_t)B * l.T * l.F * std::max(l.cin, l.cout));
    max_w = std::max(max_w, (size_t)l.cin * l.cout * 36);
  }
  float *in, *out, *bias;
  void* w;
  int* sched;   // per-launch tile-claim counters (zeroed before every launch)
  hipMalloc(&sched, 256 * 4 * 64);
  hipMalloc(&in, max_in * 4); hipMalloc(&out, max_in * 4); hipMalloc(&bias, 512 * 4); hipMalloc(&w, max_w);
  {
    std::vector<float> h(max_in);
    srand(1);
    for (auto& v : h) v = rand() / (float)RAND_MAX - 0.5f;
    hipMemcpy(in, h.data(), max_in * 4, hipMemcpyHostToDevice);
    std::vector<unsigned> hw(max_w / 4);
    for (auto& v : hw) v = ((rand() & 0x7fff) | 0x3c00u) * 0x10001u;   // small bf16 pairs
    hipMemcpy(w, hw.data(), max_w, hipMemcpyHostToDevice);
    hipMemset(bias, 0, 512 * 4);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  double tot_ms = 0, tot_f = 0;
  for (int li = 0; li < NL; ++li) {
    const Layer& l = L[li];
    hipMemsetAsync(sched, 0, 256 * 4, 0);
    sedx::launch_conv3x3_x3(in, B, l.T, l.F, l.cin, l.cout, w, bias, out, l.epi, sched, 0);
    hipDeviceSynchronize();
    hipMemsetAsync(sched, 0, 256 * 4 * 64, 0);
#ifdef SEDX_CONV_STAMPS
    unsigned long long st[8];
    sedx::conv_stamps_rw(st, true);
#endif
    hipEventRecord(e0, 0);
    for (int r = 0; r < reps; ++r)   // reps <= 64: one counter block per launch, zeroed up front
      sedx::launch_conv3x3_x3(in, B, l.T, l.F, l.cin, l.cout, w, bias, out, l.epi, sched + 256 * (r & 63), 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double fl = 2.0 * B * l.T * l.F * l.cin * l.cout * 9;
    tot_ms += ms; tot_f += fl;
    printf("%s  T=%4d F=%2d %3d->%3d  %.4f ms  %.1f TF/s\n", l.name, l.T, l.F, l.cin, l.cout, ms, fl / ms / 1e9);
#ifdef SEDX_CONV_STAMPS
    sedx::conv_stamps_rw(st, true);
    const double tot = (double)st[0];
    printf("      stamps: waves %llu  barrier %.1f%%  vm-wait %.1f%%  epilogue %.1f%%  (cycles/wave %.0f, clock %.2f GHz)\n",
           st[4], 100 * st[1] / tot, 100 * st[2] / tot, 100 * st[3] / tot, tot / (double)st[4],
           tot / (double)st[5] * 0.1);
#endif
  }
  printf("total %.4f ms  %.1f TF/s  (err=%s)\n", tot_ms, tot_f / tot_ms / 1e9, hipGetErrorString(hipGetLastError()));
  return 0;
}
