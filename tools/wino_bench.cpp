// Winograd F(2x2,3x3) fp32 conv (conv_wino.hip) against the direct exact
// fp32 conv (conv.hip) at the bench shapes (B clips x 10 s @ 16 kHz, blocks
// 2-4): same random operands for both, outputs compared with each other and
// with a float64 reference on sampled output elements; then each timed.
// Built by tools/gpu_wino.sh.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "../sound-event-detection_amd/csrc/sedx_internal.h"

struct Layer { const char* name; int T, F, cin, cout, epi; };

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const char* only = argc > 3 ? argv[3] : nullptr;
  const Layer LM[] = {{"b2c1", 500, 32, 64, 128, sedx::EPI_STORE}, {"b2c2", 500, 32, 128, 128, sedx::EPI_POOL2},
                      {"b3c1", 250, 16, 128, 256, sedx::EPI_STORE}, {"b3c2", 250, 16, 256, 256, sedx::EPI_POOL2},
                      {"b4c1", 125, 8, 256, 512, sedx::EPI_STORE},  {"b4c2", 125, 8, 512, 512, sedx::EPI_FMEAN}};
  float *d_in, *d_o1, *d_o2, *d_bias, *d_wp, *d_u, *d_zero;
  size_t max_in = 0, max_out = 0, max_w = 0;
  for (const Layer& l : LM) {
    max_in = std::max(max_in, (size_t)B * l.T * l.F * l.cin);
    max_out = std::max(max_out, (size_t)B * l.T * l.F * l.cout);
    max_w = std::max(max_w, (size_t)l.cin * l.cout * 16);
  }
  hipMalloc(&d_in, max_in * 4); hipMalloc(&d_o1, max_out * 4); hipMalloc(&d_o2, max_out * 4);
  hipMalloc(&d_bias, 512 * 4); hipMalloc(&d_wp, max_w * 4); hipMalloc(&d_u, max_w * 4);
  hipMalloc(&d_zero, 4096); hipMemset(d_zero, 0, 4096);
  float* d_trash;
  hipMalloc(&d_trash, 64 * 128 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  double tot_d = 0, tot_w = 0, tot_f = 0;
  bool ok = true;
  for (const Layer& l : LM) {
    if (only && strcmp(only, l.name) != 0) continue;
    const size_t nin = (size_t)B * l.T * l.F * l.cin;
    // post-ReLU-like inputs (non-negative, some zeros), He-scaled weights
    std::vector<float> in(nin), bias(l.cout);
    for (auto& v : in) v = std::max(0.f, nd(rng));
    std::vector<double> w((size_t)l.cout * l.cin * 9);
    const float ws = std::sqrt(2.f / (9 * l.cin));
    for (auto& v : w) v = (double)(float)(nd(rng) * ws);
    for (auto& v : bias) v = 0.1f * nd(rng);
    std::vector<float> wp((size_t)l.cin * 9 * l.cout), U((size_t)l.cin * l.cout * 16);
    for (int o = 0; o < l.cout; ++o)
      for (int i = 0; i < l.cin; ++i)
        for (int t = 0; t < 9; ++t) {
          const int chunk = i / 4, kc = i % 4, ks = kc >> 1, kh = kc & 1;
          wp[((((size_t)chunk * 9 + t) * 2 + kh) * l.cout + o) * 2 + ks] = (float)w[((size_t)o * l.cin + i) * 9 + t];
        }
    sedx::pack_conv_wino(w.data(), l.cin, l.cout, U.data());
    hipMemcpy(d_in, in.data(), nin * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_bias, bias.data(), l.cout * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_wp, wp.data(), wp.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_u, U.data(), U.size() * 4, hipMemcpyHostToDevice);
    const int To = l.epi == sedx::EPI_POOL2 ? l.T / 2 : l.T;
    const int Fo = l.epi == sedx::EPI_POOL2 ? l.F / 2 : (l.epi == sedx::EPI_FMEAN ? 1 : l.F);
    const size_t nout = (size_t)B * To * Fo * l.cout;
    hipMemset(d_o1, 0xff, nout * 4);
    hipMemset(d_o2, 0xff, nout * 4);
    auto direct = [&]() { sedx::launch_conv3x3(d_in, B, l.T, l.F, l.cin, l.cout, d_wp, d_bias, d_o1, l.epi, d_zero, 0); };
    auto wino = [&]() { sedx::launch_conv3x3_wino(d_in, B, l.T, l.F, l.cin, l.cout, d_u, d_bias, d_o2, l.epi, d_zero, d_trash, 0); };
    direct();
    wino();
    hipDeviceSynchronize();
    std::vector<float> o1(nout), o2(nout);
    hipMemcpy(o1.data(), d_o1, nout * 4, hipMemcpyDeviceToHost);
    hipMemcpy(o2.data(), d_o2, nout * 4, hipMemcpyDeviceToHost);
    double dmax = 0, omax = 0;
    size_t nan = 0;
    for (size_t i = 0; i < nout; ++i) {
      if (!std::isfinite(o2[i]) || !std::isfinite(o1[i])) { ++nan; continue; }
      dmax = std::max(dmax, (double)std::fabs(o1[i] - o2[i]));
      omax = std::max(omax, (double)std::fabs(o1[i]));
    }
    // float64 reference at sampled outputs (conv + bias + ReLU, then the epilogue)
    auto conv_px = [&](int b, int t, int f, int o) {
      double s = 0;
      for (int dt = 0; dt < 3; ++dt)
        for (int df = 0; df < 3; ++df) {
          const int tt = t + dt - 1, ff = f + df - 1;
          if (tt < 0 || tt >= l.T || ff < 0 || ff >= l.F) continue;
          const float* x = &in[(((size_t)b * l.T + tt) * l.F + ff) * l.cin];
          for (int i = 0; i < l.cin; ++i) s += (double)x[i] * w[((size_t)o * l.cin + i) * 9 + dt * 3 + df];
        }
      return std::max(0.0, s + bias[o]);
    };
    double e1max = 0, e2max = 0;
    std::uniform_int_distribution<size_t> pick(0, nout - 1);
    for (int k = 0; k < 300; ++k) {
      size_t idx = k < 4 ? (k % 2 ? nout - 1 - k : k) : pick(rng);
      const int o = idx % l.cout;
      size_t r = idx / l.cout;
      const int fo = r % Fo;
      r /= Fo;
      const int to = r % To, b = (int)(r / To);
      double ref;
      if (l.epi == sedx::EPI_POOL2)
        ref = (conv_px(b, 2 * to, 2 * fo, o) + conv_px(b, 2 * to, 2 * fo + 1, o) + conv_px(b, 2 * to + 1, 2 * fo, o) +
               conv_px(b, 2 * to + 1, 2 * fo + 1, o)) * 0.25;
      else if (l.epi == sedx::EPI_FMEAN) {
        ref = 0;
        for (int f = 0; f < l.F; ++f) ref += conv_px(b, to, f, o);
        ref /= l.F;
      } else
        ref = conv_px(b, to, fo, o);
      e1max = std::max(e1max, std::fabs(o1[idx] - ref));
      e2max = std::max(e2max, std::fabs(o2[idx] - ref));
    }
    const bool lok = nan == 0 && dmax < 1e-4 * std::max(1.0, omax) && e2max < 1e-4 * std::max(1.0, omax);
    ok = ok && lok;
    auto timeit = [&](auto fn) {
      hipEventRecord(e0, 0);
      for (int r = 0; r < reps; ++r) fn();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      return ms / reps;
    };
    const float md = timeit(direct), mw = timeit(wino);
    const double fl = 2.0 * B * l.T * l.F * l.cin * l.cout * 9;
    const double flw = fl * 16.0 / 36.0;   // matrix-pipe FLOPs of the Winograd form
    tot_d += md; tot_w += mw; tot_f += fl;
    printf("%s B=%d  direct %.4f ms (%.1f TF/s)  wino %.4f ms (%.1f eff TF/s, MFMA %.1f TF/s = %.3f of 157.3)  x%.2f  "
           "|d-w| %.2e  |d-ref| %.2e |w-ref| %.2e  max|o| %.2f  nonfinite %zu  %s\n",
           l.name, B, md, fl / md / 1e9, mw, fl / mw / 1e9, flw / mw / 1e9, flw / mw / 1e9 / 157.3, md / mw, dmax, e1max,
           e2max, omax, nan, lok ? "OK" : "MISMATCH");
  }
  printf("total direct %.4f ms  wino %.4f ms  (x%.2f; eff %.1f TF/s)  %s  (err=%s, launch=%s)\n", tot_d, tot_w,
         tot_d / tot_w, tot_f / tot_w / 1e9, ok ? "ALL OK" : "MISMATCH", hipGetErrorString(hipGetLastError()),
         hipGetErrorString(sedx::take_launch_error()));
  return ok ? 0 : 1;
}
