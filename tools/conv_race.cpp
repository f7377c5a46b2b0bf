// Diagnostic: is each x3 conv layer (and the x3 linear) bit-deterministic
// when launches of two streams run concurrently?  Per layer: a serial
// reference output, then R rounds of the same launch issued alternately on
// two streams (each with its own input/output/claim buffers), every output
// compared bit for bit with the reference.  Random operands; timing only
// perturbs the schedule.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../sound-event-detection_amd/csrc/sedx_internal.h"

struct Layer { const char* name; int T, F, cin, cout, epi; };

static size_t out_floats(const Layer& l, int B) {
  if (l.epi == sedx::EPI_POOL2) return (size_t)B * (l.T / 2) * (l.F / 2) * l.cout;
  if (l.epi == sedx::EPI_FMEAN) return (size_t)B * l.T * l.cout;
  return (size_t)B * l.T * l.F * l.cout;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int R = argc > 2 ? atoi(argv[2]) : 6;
  const bool skip_layers = argc > 3 && atoi(argv[3]) == 1;
  const Layer L[] = {{"b2c1", 500, 32, 64, 128, sedx::EPI_STORE}, {"b2c2", 500, 32, 128, 128, sedx::EPI_POOL2},
                     {"b3c1", 250, 16, 128, 256, sedx::EPI_STORE}, {"b3c2", 250, 16, 256, 256, sedx::EPI_POOL2},
                     {"b4c1", 125, 8, 256, 512, sedx::EPI_STORE},  {"b4c2", 125, 8, 512, 512, sedx::EPI_FMEAN}};
  hipStream_t st[2];
  hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking);
  hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking);
  int* sched;
  hipMalloc(&sched, 2 * 64 * 256 * 4);
  int bad_total = 0;
  for (const Layer& l : L) {
    if (skip_layers) break;
    const size_t nin = (size_t)B * l.T * l.F * l.cin, nout = out_floats(l, B), nw = (size_t)l.cin * l.cout * 36 / 4;
    std::vector<float> h(nin);
    srand(7);
    for (auto& v : h) v = (rand() / (float)RAND_MAX - 0.3f) * 2.f;
    std::vector<unsigned> hw(nw);
    for (auto& v : hw) {
      const unsigned a = (rand() & 0x7f) | 0x3c00u | ((rand() & 1) << 15);   // bf16 ~ +-[1, 2)
      const unsigned b = (rand() & 0x7f) | 0x3800u | ((rand() & 1) << 15);
      v = a | (b << 16);
    }
    constexpr int NL = 16;           // launches per round, each with its own output
    float *in[2], *out[NL], *bias;
    void* w;
    for (int i = 0; i < 2; ++i) {
      hipMalloc(&in[i], nin * 4);
      hipMemcpy(in[i], h.data(), nin * 4, hipMemcpyHostToDevice);
    }
    for (int i = 0; i < NL; ++i) hipMalloc(&out[i], nout * 4);
    hipMalloc(&bias, l.cout * 4);
    hipMemset(bias, 0, l.cout * 4);
    hipMalloc(&w, nw * 4);
    hipMemcpy(w, hw.data(), nw * 4, hipMemcpyHostToDevice);
    // serial reference
    hipMemset(sched, 0, 256 * 4);
    sedx::launch_conv3x3_x3(in[0], B, l.T, l.F, l.cin, l.cout, w, bias, out[0], l.epi, sched, 0);
    hipDeviceSynchronize();
    std::vector<float> ref(nout), got(nout);
    hipMemcpy(ref.data(), out[0], nout * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    double worst = 0;
    for (int r = 0; r < R; ++r) {
      for (int i = 0; i < NL; ++i) hipMemset(out[i], 0xff, nout * 4);
      hipMemset(sched, 0, 2 * 64 * 256 * 4);
      hipDeviceSynchronize();
      for (int k = 0; k < NL; ++k)   // 8 launches per stream, interleaved issue
        sedx::launch_conv3x3_x3(in[k & 1], B, l.T, l.F, l.cin, l.cout, w, bias, out[k], l.epi,
                                sched + 256 * k, st[k & 1]);
      hipDeviceSynchronize();
      for (int i = 0; i < NL; ++i) {
        hipMemcpy(got.data(), out[i], nout * 4, hipMemcpyDeviceToHost);
        size_t nd = 0, first = 0;
        for (size_t j = 0; j < nout; ++j)
          if (memcmp(&got[j], &ref[j], 4) != 0) {
            if (!nd) first = j;
            ++nd;
            const double d = std::fabs((double)got[j] - ref[j]);
            if (d > worst || std::isnan(d)) worst = d;
          }
        if (nd) {
          ++bad;
          printf("  %s round %d stream %d: %zu of %zu differ (first %zu: %.9g vs %.9g)\n", l.name, r, i, nd,
                 nout, first, got[first], ref[first]);
        }
      }
    }
    printf("%s: %d of %d outputs differ, worst |d| %.3g (%s)\n", l.name, bad, NL * R, worst,
           hipGetErrorString(hipGetLastError()));
    fflush(stdout);
    bad_total += bad;
    for (int i = 0; i < 2; ++i) hipFree(in[i]);
    for (int i = 0; i < NL; ++i) hipFree(out[i]);
    hipFree(bias); hipFree(w);
  }
  // ---- block 1 fused (pad_x0 + conv1-in-staging + conv2 + pool) and linear_x3 ----
  {
    const int T = 1001;
    const size_t nx0 = (size_t)B * T * 64, nxp = sedx::block1_pad_floats(B, T), nout = (size_t)B * 500 * 32 * 64;
    const size_t nw = (size_t)64 * 64 * 36 / 4;
    std::vector<float> h(nx0), w1(9 * 64), b1(64);
    srand(11);
    for (auto& v : h) v = (rand() / (float)RAND_MAX - 0.5f) * 4.f;
    for (auto& v : w1) v = (rand() / (float)RAND_MAX - 0.5f);
    for (auto& v : b1) v = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
    std::vector<unsigned> hw(nw);
    for (auto& v : hw) {
      const unsigned a = (rand() & 0x7f) | 0x3c00u | ((rand() & 1) << 15);
      const unsigned b = (rand() & 0x7f) | 0x3800u | ((rand() & 1) << 15);
      v = a | (b << 16);
    }
    constexpr int NL = 8;
    float *x0, *xp[NL], *out[NL], *dw1, *db1, *bias;
    void* w;
    hipMalloc(&x0, nx0 * 4);
    hipMemcpy(x0, h.data(), nx0 * 4, hipMemcpyHostToDevice);
    for (int i = 0; i < NL; ++i) { hipMalloc(&xp[i], nxp * 4); hipMalloc(&out[i], nout * 4); }
    hipMalloc(&dw1, 9 * 64 * 4); hipMemcpy(dw1, w1.data(), 9 * 64 * 4, hipMemcpyHostToDevice);
    hipMalloc(&db1, 64 * 4); hipMemcpy(db1, b1.data(), 64 * 4, hipMemcpyHostToDevice);
    hipMalloc(&bias, 64 * 4); hipMemset(bias, 0, 64 * 4);
    hipMalloc(&w, nw * 4); hipMemcpy(w, hw.data(), nw * 4, hipMemcpyHostToDevice);
    hipMemset(sched, 0, 256 * 4);
    sedx::launch_block1_fused_x3(x0, B, T, xp[0], dw1, db1, w, bias, out[0], sched, 0);
    hipDeviceSynchronize();
    std::vector<float> ref(nout), got(nout);
    hipMemcpy(ref.data(), out[0], nout * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < R; ++r) {
      for (int i = 0; i < NL; ++i) { hipMemset(out[i], 0xff, nout * 4); hipMemset(xp[i], 0xff, nxp * 4); }
      hipMemset(sched, 0, 2 * 64 * 256 * 4);
      hipDeviceSynchronize();
      for (int k = 0; k < NL; ++k)
        sedx::launch_block1_fused_x3(x0, B, T, xp[k], dw1, db1, w, bias, out[k], sched + 256 * k, st[k & 1]);
      hipDeviceSynchronize();
      for (int i = 0; i < NL; ++i) {
        hipMemcpy(got.data(), out[i], nout * 4, hipMemcpyDeviceToHost);
        size_t nd = 0, first = 0;
        for (size_t j = 0; j < nout; ++j)
          if (memcmp(&got[j], &ref[j], 4) != 0) { if (!nd) first = j; ++nd; }
        if (nd) {
          ++bad;
          printf("  b1fused round %d launch %d: %zu of %zu differ (first %zu: %.9g vs %.9g)\n", r, i, nd, nout,
                 first, got[first], ref[first]);
        }
      }
    }
    printf("b1fused: %d of %d outputs differ (%s)\n", bad, NL * R, hipGetErrorString(hipGetLastError()));
    bad_total += bad;
  }
  {
    // linear_x3: the GRU input projection shape (M = 32 x 125, K 512, N 1536, BN 128)
    const int M = B * 125, K = 512, N = 1536, BN = 128;
    std::vector<float> a((size_t)M * K);
    srand(13);
    for (auto& v : a) v = rand() / (float)RAND_MAX - 0.5f;
    std::vector<unsigned> hw((size_t)N * K * 4 / 4);
    for (auto& v : hw) v = (((rand() & 0x7f) | 0x3c00u) | (((rand() & 0x7f) | 0x3800u) << 16));
    constexpr int NL = 16;
    float *A, *C[NL], *bias;
    void* w;
    hipMalloc(&A, a.size() * 4); hipMemcpy(A, a.data(), a.size() * 4, hipMemcpyHostToDevice);
    for (int i = 0; i < NL; ++i) hipMalloc(&C[i], (size_t)M * N * 4);
    hipMalloc(&bias, N * 4); hipMemset(bias, 0, N * 4);
    hipMalloc(&w, hw.size() * 4); hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
    sedx::launch_linear_x3(A, M, K, w, N, BN, bias, C[0], 0, 0);
    hipDeviceSynchronize();
    std::vector<float> ref((size_t)M * N), got((size_t)M * N);
    hipMemcpy(ref.data(), C[0], ref.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < R; ++r) {
      for (int i = 0; i < NL; ++i) hipMemset(C[i], 0xff, (size_t)M * N * 4);
      hipDeviceSynchronize();
      for (int k = 0; k < NL; ++k) sedx::launch_linear_x3(A, M, K, w, N, BN, bias, C[k], 0, st[k & 1]);
      hipDeviceSynchronize();
      for (int i = 0; i < NL; ++i) {
        hipMemcpy(got.data(), C[i], got.size() * 4, hipMemcpyDeviceToHost);
        if (memcmp(got.data(), ref.data(), got.size() * 4) != 0) ++bad;
      }
    }
    printf("linear_x3: %d of %d outputs differ (%s)\n", bad, NL * R, hipGetErrorString(hipGetLastError()));
    bad_total += bad;
  }
  printf("total differing outputs: %d\n", bad_total);
  return 0;
}
