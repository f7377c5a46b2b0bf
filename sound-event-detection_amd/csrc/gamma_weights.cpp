// Host-side gammatone tables for the float64 gammatone frontend, in the
// reference's numpy operation order (this file is compiled with
// -ffp-contract=off so no a*b+c is fused):
//   erb_point / erb_space          utils/gammatone/filters.py:21-72
//   make_erb_filters (width = 1)   utils/gammatone/filters.py:90-193
//   fft_weights                    utils/gammatone/fftweight.py:63-123
//   specgram_window                utils/gammatone/fftweight.py:15-30
// Complex arithmetic follows numpy's float64 complex loops: product
// (ar br - ai bi, ar bi + ai br) with a real operand promoted to x + 0j,
// Smith's division, integer powers by repeated squaring, abs = hypot.
#include <cmath>
#include <vector>

#include "sedx_internal.h"

namespace sedx {
namespace {

struct Z {
  double r, i;
};
Z zr(double x) { return Z{x, 0.0}; }
Z mul(Z a, Z b) { return Z{a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
Z add(Z a, Z b) { return Z{a.r + b.r, a.i + b.i}; }
Z sub(Z a, Z b) { return Z{a.r - b.r, a.i - b.i}; }
// numpy CDOUBLE_divide (Smith)
Z div(Z a, Z b) {
  const double abr = std::fabs(b.r), abi = std::fabs(b.i);
  if (abr >= abi) {
    const double rat = b.i / b.r, scl = 1.0 / (b.r + b.i * rat);
    return Z{(a.r + a.i * rat) * scl, (a.i - a.r * rat) * scl};
  }
  const double rat = b.r / b.i, scl = 1.0 / (b.i + b.r * rat);
  return Z{(a.r * rat + a.i) * scl, (a.i * rat - a.r) * scl};
}
// numpy npy_cexp for a finite argument
Z zexp(Z a) {
  const double x = std::exp(a.r);
  return Z{x * std::cos(a.i), x * std::sin(a.i)};
}
// numpy complex ** 4 (binary powering, p starts at 1 + 0j)
Z pow4(Z a) {
  const Z a2 = mul(a, a);
  const Z a4 = mul(a2, a2);
  return mul(Z{1.0, 0.0}, a4);
}
double zabs(Z a) { return std::hypot(a.r, a.i); }

}  // namespace

void gamma_tables(double fs, int nfft, int nwin, int nfilts, double fmin, std::vector<double>& weightsT,
                  int kp, std::vector<double>& twiddle, std::vector<double>& window) {
  const double ear_q = 9.26449, min_bw = 24.7;
  const double fmax = fs / 2;
  const int NB = nfft / 2 + 1;
  // erb_space(fmin, fmax, nfilts)[::-1]
  std::vector<double> cf(nfilts);
  for (int i = 0; i < nfilts; ++i) {
    const double fraction = (double)(i + 1) / (double)nfilts;
    const double e = -ear_q * min_bw +
                     std::exp(fraction * (-std::log(fmax + ear_q * min_bw) + std::log(fmin + ear_q * min_bw))) *
                         (fmax + ear_q * min_bw);
    cf[nfilts - 1 - i] = e;
  }
  // ucirc = exp(1j * 2 * pi * arange(0, nfft/2 + 1) / nfft)
  std::vector<Z> ucirc(NB);
  for (int k = 0; k < NB; ++k) {
    const double im = (2.0 * M_PI) * (double)k;
    ucirc[k] = zexp(div(Z{0.0, im}, zr((double)nfft)));
  }
  weightsT.assign((size_t)kp * nfilts, 0.0);
  const double T = 1 / fs;
  const double rt_pos = std::sqrt(3 + std::pow(2.0, 1.5)), rt_neg = std::sqrt(3 - std::pow(2.0, 1.5));
  for (int c = 0; c < nfilts; ++c) {
    // make_erb_filters
    const double erb = cf[c] / ear_q + min_bw;
    const double B = 1.019 * 2 * M_PI * erb;
    const double arg = 2 * cf[c] * M_PI * T;
    const Z vec = zexp(mul(Z{0.0, 2.0}, zr(arg)));
    const double B2 = std::exp(-2 * B * T);
    const double common = -T * std::exp(-(B * T));
    const double k11 = std::cos(arg) + rt_pos * std::sin(arg);
    const double k12 = std::cos(arg) - rt_pos * std::sin(arg);
    const double k13 = std::cos(arg) + rt_neg * std::sin(arg);
    const double k14 = std::cos(arg) - rt_neg * std::sin(arg);
    const double A11 = common * k11, A12 = common * k12, A13 = common * k13, A14 = common * k14;
    const Z gain_arg = zexp(sub(mul(Z{0.0, 1.0}, zr(arg)), zr(B * T)));
    const double ebt = std::exp(B * T);
    const Z den = add(zr(-1 / ebt + 1), mul(vec, zr(1 - ebt)));
    const Z q = div(zr(T * ebt), den);
    Z prod = sub(vec, mul(gain_arg, zr(k11)));
    prod = mul(prod, sub(vec, mul(gain_arg, zr(k12))));
    prod = mul(prod, sub(vec, mul(gain_arg, zr(k13))));
    prod = mul(prod, sub(vec, mul(gain_arg, zr(k14))));
    prod = mul(prod, pow4(q));
    const double gain = zabs(prod);
    // fft_weights
    const double r = std::sqrt(B2);
    const double theta = 2 * M_PI * cf[c] / fs;
    const Z pole = mul(zr(r), zexp(mul(Z{0.0, 1.0}, zr(theta))));
    const Z pconj = Z{pole.r, -pole.i};
    for (int k = 0; k < NB; ++k) {
      const Z u = ucirc[k];
      const double den4 = std::pow(zabs(mul(mul(zr(fs), sub(pole, u)), sub(pconj, u))), -4.0);
      const double w = zabs(add(u, zr(A11 * fs))) * zabs(add(u, zr(A12 * fs))) * zabs(add(u, zr(A13 * fs))) *
                       zabs(add(u, zr(A14 * fs))) * den4 / gain;
      weightsT[(size_t)k * nfilts + c] = w;
    }
  }
  // FFT twiddles exp(-2 pi i m / nfft)
  twiddle.resize(2 * (size_t)nfft);
  for (int m = 0; m < nfft; ++m) {
    twiddle[2 * m] = std::cos(-2.0 * M_PI * m / nfft);
    twiddle[2 * m + 1] = std::sin(-2.0 * M_PI * m / nfft);
  }
  // specgram_window: Hann of width nwin centred in nfft
  window.assign(nfft, 0.0);
  const int halflen = nwin / 2, halff = nfft / 2;
  const int act = halff < halflen ? halff : halflen;
  for (int i = 0; i < act; ++i) {
    const double v = 0.5 * (1 + std::cos(M_PI * (double)i / halflen));
    window[halff + i] = v;
    window[halff - i] = v;
  }
}

}  // namespace sedx
