// Stand-alone micro-benchmark of the cooperative GRU recurrence
// (diagnostic build with -DSEDX_GRU_STAMPS: per-phase s_memtime sums of
// workgroup (pair 0, slice 0)).  Build: see tools/gpu_gru_bench.sh
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../sound-event-detection_amd/csrc/sedx_internal.h"

struct Sync {                         // must mirror GruSync in gru.hip
  unsigned err;
  unsigned pad0[63];
  unsigned ready[8][16];
  unsigned xcc[8][16];
  unsigned cnt[8][16];
  unsigned flag[8][16][16];
  unsigned long long stamps[8];
  unsigned mode;
};

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, T = argc > 2 ? atoi(argv[2]) : 125;
  const int reps = 20;
  std::vector<float> hG((size_t)B * T * 1536), hw(2 * 768 * 256), hb(2 * 768);
  srand(1);
  for (auto& v : hG) v = (rand() / (float)RAND_MAX - 0.5f);
  for (auto& v : hw) v = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  for (auto& v : hb) v = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
  float *G, *W, *Bb, *H;
  void* ws;
  hipMalloc(&G, hG.size() * 4); hipMalloc(&W, hw.size() * 4); hipMalloc(&Bb, hb.size() * 4);
  hipMalloc(&H, (size_t)B * T * 512 * 4);
  const size_t wsb = sedx::gru_coop_workspace_bytes(B);
  hipMalloc(&ws, wsb);
  hipMemcpy(G, hG.data(), hG.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(W, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(Bb, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  // variants: 0 = tagged 16-clip groups x 16 slices, 1 = tagged x 8 slices, 3 = coop on 16 slices,
  // 2 = the 32-clip flag kernel (fast = XCD-local hand-off allowed), 4 = K-split hand-off on 16 slices,
  // 5 = two interleaved 16-clip halves per workgroup (K-split structure)
  std::vector<float> ref;
  for (int exact = 1; exact >= 0; --exact)
    for (int variant = 0; variant < 6; ++variant)
    for (int fast = 0; fast < 2; ++fast) {
      if ((!exact || variant < 2 || variant >= 4) && !fast) continue;
      if (!exact && (variant < 2 || variant >= 3)) continue;
      sedx::launch_gru_coop(G, B, T, W, Bb, H, ws, exact, fast, variant, nullptr, 1u << 24, 0);
      hipDeviceSynchronize();
      if (exact) {   // every exact variant must give the same bits
        std::vector<float> out((size_t)B * T * 512);
        hipMemcpy(out.data(), H, out.size() * 4, hipMemcpyDeviceToHost);
        if (ref.empty()) ref = out;
        size_t bad = 0;
        for (size_t i = 0; i < out.size(); ++i) bad += out[i] != ref[i] && !(out[i] != out[i] && ref[i] != ref[i]);
        printf("B=%d exact variant %d fast %d: %zu of %zu outputs differ from variant 0\n", B, variant, fast, bad,
               out.size());
      }
      hipEventRecord(e0, 0);
      for (int r = 0; r < reps; ++r)
        sedx::launch_gru_coop(G, B, T, W, Bb, H, ws, exact, fast, variant, nullptr, 1u << 24, 0);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      Sync sy;
      hipMemcpy(&sy, ws, sizeof(Sync), hipMemcpyDeviceToHost);
      const double tot = (double)(sy.stamps[0] + sy.stamps[1] + sy.stamps[2] + sy.stamps[3]);
      printf("B=%d v%d %s %s: mode=%u err=%u  %.3f ms/launch  %.2f us/step | wait %.0f%% gather %.0f%% product %.0f%% "
             "gates+publish %.0f%% (s_memtime ticks/step %.0f)\n",
             B, variant, exact ? "exact" : "x3", fast ? "auto" : "global", sy.mode, sy.err, ms / reps, ms / reps * 1e3 / T,
             100 * sy.stamps[0] / tot, 100 * sy.stamps[1] / tot, 100 * sy.stamps[2] / tot, 100 * sy.stamps[3] / tot,
             tot / T);
    }
  return 0;
}
