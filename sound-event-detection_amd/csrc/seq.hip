// Sequence + head kernels for gfx950:
//   linear_kernel   C = act(A W^T + b) on fp32 MFMA 32x32x2 (GRU input projection
//                   both directions, MHA q|k|v projection, MHA fc + ReLU, AttBlock
//                   att|cla 1x1 convs)
//   gru_kernel      bi-GRU recurrence, one workgroup per (clip, direction)
//                   (torch nn.GRU semantics, pytorch/models.py:614-615,670)
//   mha_kernel      per (clip, head) softmax(q k^T / 8) v, exact two-pass softmax
//                   (ScaledDotProductAttention, pytorch/models.py:805-820)
//   att_head_kernel AttBlock finish (clamp, exp, normalise over T, sigmoid,
//                   weighted sum) + x8 frame repeat + GRU last-frame padding
//                   (pytorch/models.py:161-175, :84-95, :65-81)
//   merge_plan_kernel  overlap-add of window predictions + avg_merge divisors (host plan)
//                   (utils/utilities.py:405-446)
#include "sedx_internal.h"

namespace sedx {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
template <int ACT>
__global__ __launch_bounds__(256) void linear_kernel(const float* __restrict__ A, int M, int K,
                                                     const float* __restrict__ W, int N,
                                                     const float* __restrict__ bias,
                                                     float* __restrict__ C) {
  // 128 x 64 tile, 4 waves of 32 rows x 64 columns; K in slices of 16 staged
  // through a 2-slot LDS ring, the next slice's global loads in flight (in
  // registers) while the current slice's MFMAs run: one barrier per slice
  constexpr int BM = 128, BN = 64, BK = 16;
  __shared__ float As[2][BK][BM + 4];
  __shared__ float Ws[2][BK][BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kh = lane >> 5;
  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
  // per thread: 2 float4 of the A slice (128 rows x 4 quads), 1 of the W slice
  float4 ra[2], rw;
  auto load = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int i = tid + 256 * e;
      const int m = i % BM, q = i / BM;
      const int row = min(m0 + m, M - 1);   // rows past M: any valid row, never stored
      ra[e] = *reinterpret_cast<const float4*>(A + (int64_t)row * K + k0 + 4 * q);
    }
    const int n = tid % BN, q = tid / BN;
    rw = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + n) * K + k0 + 4 * q);
  };
  auto store = [&](int slot) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int i = tid + 256 * e;
      const int m = i % BM, q = i / BM;
      As[slot][4 * q + 0][m] = ra[e].x; As[slot][4 * q + 1][m] = ra[e].y;
      As[slot][4 * q + 2][m] = ra[e].z; As[slot][4 * q + 3][m] = ra[e].w;
    }
    const int n = tid % BN, q = tid / BN;
    Ws[slot][4 * q + 0][n] = rw.x; Ws[slot][4 * q + 1][n] = rw.y;
    Ws[slot][4 * q + 2][n] = rw.z; Ws[slot][4 * q + 3][n] = rw.w;
  };
  const int nk = K / BK;
  load(0);
  store(0);
  if (nk > 1) load(BK);
  __syncthreads();
  for (int it = 0; it < nk; ++it) {
    const int slot = it & 1;
#pragma unroll
    for (int ks = 0; ks < BK / 2; ++ks) {
      const float a = As[slot][2 * ks + kh][wave * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float bb = Ws[slot][2 * ks + kh][j * 32 + (lane & 31)];
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc[j], 0, 0, 0);
      }
    }
    if (it + 1 < nk) {
      store(slot ^ 1);                     // slot ^ 1 was last read in it - 1 (barrier below it)
      if (it + 2 < nk) load((it + 2) * BK);
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + j * 32 + (lane & 31);
    const float bv = bias ? bias[n] : 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
      if (m < M) {
        float v = acc[j][r] + bv;
        if (ACT == 1) v = fmaxf(v, 0.0f);
        C[(int64_t)m * N + n] = v;
      }
    }
  }
}

// Small-M shape (single clips, the head's 64 columns): one wave per 32 x 32
// output tile, A / W fragments straight from global (L2) as float4 rows, 32 k
// in flight per wave, no LDS and no barriers.  Every output's MFMA sequence
// (k ascending in pairs, zero start, + bias, act) is linear_kernel's, so the
// two shapes give identical bits.
//
// KS = 4 (the AttBlock att|cla projection, N <= 64, at every M): four waves
// per tile, wave q chaining K quarter q, the quarters summed in order
// ((q0 + q1) + q2) + q3 — a different (fixed) summation order, used for
// every call of that projection, so results stay batch-size independent.
template <int ACT, int KS>
__global__ __launch_bounds__(64 * KS) void linear_small_kernel(const float* __restrict__ A, int M, int K,
                                                               const float* __restrict__ W, int N,
                                                               const float* __restrict__ bias,
                                                               float* __restrict__ C) {
  const int lane = threadIdx.x & 63, i = lane & 31, kh = lane >> 5, wq_ = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  const int KQ = K / KS;   // this wave's K range: [wq_ KQ, (wq_ + 1) KQ)
  const float4* ap = reinterpret_cast<const float4*>(A + (int64_t)min(m0 + i, M - 1) * K + wq_ * KQ);
  const float4* wq = reinterpret_cast<const float4*>(W + (int64_t)(n0 + i) * K + wq_ * KQ);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  constexpr int Q = 16;  // float4 per row per round (64 k); two rounds in registers
  float4 xa0[Q], xw0[Q], xa1[Q], xw1[Q];
  const int nr = KQ / (4 * Q);
  auto load = [&](float4* xa, float4* xw, int rd) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      xa[q] = ap[rd * Q + q];
      xw[q] = wq[rd * Q + q];
    }
  };
  // k-step 2q: k = 4q + kh (element kh); k-step 2q + 1: k = 4q + 2 + kh
  auto mma = [&](const float4* xa, const float4* xw) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float4 a = xa[q], b = xw[q];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kh ? a.y : a.x, kh ? b.y : b.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(kh ? a.w : a.z, kh ? b.w : b.z, acc, 0, 0, 0);
    }
  };
  load(xa0, xw0, 0);
  for (int rd = 0; rd < nr; rd += 2) {   // static buffer names: no dynamic register indexing
    if (rd + 1 < nr) load(xa1, xw1, rd + 1);
    mma(xa0, xw0);
    if (rd + 1 < nr) {
      if (rd + 2 < nr) load(xa0, xw0, rd + 2);
      mma(xa1, xw1);
    }
  }
  if constexpr (KS > 1) {
    __shared__ float part[KS - 1][32][33];
    if (wq_ > 0)
#pragma unroll
      for (int r = 0; r < 16; ++r) part[wq_ - 1][(r & 3) + 8 * (r >> 2) + 4 * kh][i] = acc[r];
    __syncthreads();
    if (wq_ > 0) return;
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int q = 0; q < KS - 1; ++q) acc[r] += part[q][(r & 3) + 8 * (r >> 2) + 4 * kh][i];
  }
  const int n = n0 + i;
  const float bv = bias ? bias[n] : 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
    if (m < M) {
      float v = acc[r] + bv;
      if (ACT == 1) v = fmaxf(v, 0.0f);
      C[(int64_t)m * N + n] = v;
    }
  }
}

void launch_linear(const float* A, int M, int K, const float* W, int N, const float* bias,
                   float* C, int act, hipStream_t s) {
  dim3 grid((M + 127) / 128, N / 64);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const dim3 g2((M + 31) / 32, N / 32);
  if (N <= 64 && act == 0 && K % 256 == 0 && N % 32 == 0)   // the head projection, every M
    return launch_kernel(linear_small_kernel<0, 4>, g2, 256, s, A, M, K, W, N, bias, C);
  if ((int64_t)grid.x * grid.y < ncu && K % 64 == 0 && N % 32 == 0) {
    if (act == 1)
      launch_kernel(linear_small_kernel<1, 1>, g2, 64, s, A, M, K, W, N, bias, C);
    else
      launch_kernel(linear_small_kernel<0, 1>, g2, 64, s, A, M, K, W, N, bias, C);
    return;
  }
  if (act == 1)
    launch_kernel(linear_kernel<1>, grid, 256, s, A, M, K, W, N, bias, C);
  else
    launch_kernel(linear_kernel<0>, grid, 256, s, A, M, K, W, N, bias, C);
}

// ---------------------------------------------------------------------------
// bi-GRU: thread j owns hidden unit j of one (clip, direction); W_hh^T is
// streamed from L2 each step (coalesced across j), h lives in LDS.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ __launch_bounds__(256) void gru_kernel(const float* __restrict__ G, int T,
                                                  const float* __restrict__ whhT,
                                                  const float* __restrict__ bhh,
                                                  float* __restrict__ H) {
  __shared__ float h[256];
  const int j = threadIdx.x;
  const int b = blockIdx.x;
  const int dir = blockIdx.y;
  const float* W = whhT + (int64_t)dir * 256 * 768;
  const float br = bhh[dir * 768 + j], bz = bhh[dir * 768 + 256 + j], bn = bhh[dir * 768 + 512 + j];
  h[j] = 0.0f;
  float hj = 0.0f;
  __syncthreads();
  for (int s = 0; s < T; ++s) {
    const int t = dir == 0 ? s : T - 1 - s;
    const float* g = G + ((int64_t)b * T + t) * 1536 + dir * 768;
    const float gr = g[j], gz = g[256 + j], gn = g[512 + j];
    float ar = 0.f, az = 0.f, an = 0.f;
#pragma unroll 8
    for (int k = 0; k < 256; ++k) {
      const float hk = h[k];
      const float* wk = W + k * 768;
      ar = fmaf(hk, wk[j], ar);
      az = fmaf(hk, wk[256 + j], az);
      an = fmaf(hk, wk[512 + j], an);
    }
    const float r = sigmoidf_(gr + (ar + br));
    const float z = sigmoidf_(gz + (az + bz));
    const float n = tanhf(gn + r * (an + bn));
    hj = n + z * (hj - n);                 // ATen GRU cell: (1-z) n + z h
    __syncthreads();
    h[j] = hj;
    H[((int64_t)b * T + t) * 512 + dir * 256 + j] = hj;
    __syncthreads();
  }
}

void launch_gru(const float* G, int B, int T, const float* whhT, const float* bhh, float* H,
                hipStream_t s) {
  hipLaunchKernelGGL(gru_kernel, dim3(B, 2), dim3(256), 0, s, G, T, whhT, bhh, H);
}

// (the cooperative multi-CU recurrence lives in gru.hip)

// ---------------------------------------------------------------------------
// MHA core.  grid (ceil(T/32), B*8), 128 threads: 4 lanes per query row
// (lane quarter g = lane & 3 owns dims 16g..16g+15), so a row's serial dot /
// p.v chain is 16 long instead of 64 and a single clip fills 32x more
// threads.  q.k = the 4 partial dots summed in a fixed order (quad shuffles);
// exact two-pass softmax as before.  XCD-aware grid: the nqb query blocks of
// one (clip, head) are workgroups n, n + 8, ... of one XCD, so that head's
// K / V rows (read by every query block, K twice) come from HBM once per
// clip-head instead of once per query block (round-robin dispatch put the
// blocks of a head on different XCDs: 111 MB per B = 32 launch against 33 MB
// algorithmic, profiles/r03c_config3_kernel_summary.md).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(128) void mha_kernel(const float* __restrict__ QKV, int T, int nqb,
                                                  float* __restrict__ O) {
  constexpr int KC = 64, DG = 16;
  __shared__ float Ks[KC][68];
  __shared__ float Vs[KC][68];
  const int n = blockIdx.x, j = n >> 3;
  const int qb = j % nqb;
  const int bh = (j / nqb) * 8 + (n & 7);   // heads per clip = 8: B * 8 is a multiple of the 8 XCDs
  const int b = bh >> 3, head = bh & 7;
  const int g = threadIdx.x & 3;
  const int qi = qb * 32 + (threadIdx.x >> 2);
  const bool valid = qi < T;
  const float* base = QKV + (int64_t)b * T * 1536;
  float q[DG], o[DG];
#pragma unroll
  for (int d = 0; d < DG; ++d) {
    q[d] = valid ? base[(int64_t)qi * 1536 + head * 64 + DG * g + d] : 0.0f;
    o[d] = 0.0f;
  }
  // q.k of this row with key row jj: partial dots over 16 dims, then
  // ((p0 + p1) + (p2 + p3)) by two quad shuffles (every lane gets the sum)
  auto dot = [&](int jj) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < DG; ++d) s = fmaf(q[d], Ks[jj][DG * g + d], s);
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    return s;
  };
  auto stage = [&](int c0, int nk, bool v) {
    __syncthreads();
    for (int i = threadIdx.x; i < nk * 64; i += 128) {
      const int64_t r = (int64_t)(c0 + (i >> 6)) * 1536 + head * 64 + (i & 63);
      Ks[i >> 6][i & 63] = base[r + 512];
      if (v) Vs[i >> 6][i & 63] = base[r + 1024];
    }
    __syncthreads();
  };
  // pass 1: row max of q.k / 8
  float mx = -INFINITY;
  for (int c0 = 0; c0 < T; c0 += KC) {
    const int nk = min(KC, T - c0);
    stage(c0, nk, false);
    for (int jj = 0; jj < nk; ++jj) mx = fmaxf(mx, dot(jj) / 8.0f);
  }
  // pass 2: exp, sum, p.v
  float l = 0.f;
  for (int c0 = 0; c0 < T; c0 += KC) {
    const int nk = min(KC, T - c0);
    stage(c0, nk, true);
    for (int jj = 0; jj < nk; ++jj) {
      const float p = expf(dot(jj) / 8.0f - mx);
      l += p;
#pragma unroll
      for (int d = 0; d < DG; ++d) o[d] = fmaf(p, Vs[jj][DG * g + d], o[d]);
    }
  }
  if (valid) {
    const float inv = 1.0f / l;
    float* dst = O + ((int64_t)b * T + qi) * 512 + head * 64 + DG * g;
#pragma unroll
    for (int d = 0; d < DG; ++d) dst[d] = o[d] * inv;
  }
}

void launch_mha(const float* QKV, int B, int T, float* O, hipStream_t s) {
  const int nqb = (T + 31) / 32;
  if (B <= 0 || T <= 0 || (int64_t)nqb * B * 8 > INT32_MAX) return note_launch_error(hipErrorInvalidValue);
  hipLaunchKernelGGL(mha_kernel, dim3((unsigned)(nqb * B * 8)), dim3(128), 0, s, QKV, T, nqb, O);
}

// ---------------------------------------------------------------------------
// AttBlock finish (pytorch/models.py:161-175, :84-95, :65-81).  One clip per
// block; thread = (class slot c = tid / 8, t-lane l = tid % 8): each thread
// walks t = l, l+8, ... and the 8 lanes of a class reduce with shuffles, so
// the T-long sums are 8-way parallel instead of one serial loop per class.
// cla is staged per 128-frame chunk in LDS for the coalesced framewise
// (x8 repeat) and embedding writes.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float att_exp_(float a) {
  return expf(fminf(fmaxf(a, -10.0f), 10.0f)) + 1e-6f;
}
__device__ __forceinline__ float sum8_(float v) {      // over the 8 lanes of a class
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  return v;
}

// One workgroup per clip; the clip's att / cla logits are staged into LDS
// 128 frames at a time by independent coalesced loads (a 10 s clip's 125
// frames once, for both passes) instead of per-lane dependent global loads.
__global__ __launch_bounds__(256) void att_head_kernel(const float* __restrict__ logits, int T,
                                                       int C, int ldl, int out_frames,
                                                       float* __restrict__ fw,
                                                       float* __restrict__ clip,
                                                       float* __restrict__ emb) {
  constexpr int TC = 128;
  __shared__ float s_att[TC][33];
  __shared__ float s_cla[TC][33];             // cla logits, then sigmoid(cla)
  __shared__ float s_last[32];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int cs = tid >> 3, l = tid & 7;
  const float* lg = logits + (int64_t)b * T * ldl;
  for (int c0 = 0; c0 < C; c0 += 32) {
    const int nc = min(32, C - c0);
    const bool act = cs < nc;
    const int c = c0 + cs;
    // (index maps by shifts and masks: no integer division in the loops)
    auto stage = [&](int t0, int nt) {
      __syncthreads();
      const int j = tid & 63, half = j >> 5, cc = j & 31;
      if (cc < nc)
        for (int t = tid >> 6; t < nt; t += 4) {
          const float v = lg[(int64_t)(t0 + t) * ldl + half * C + c0 + cc];
          if (half)
            s_cla[t][cc] = v;
          else
            s_att[t][cc] = v;
        }
      __syncthreads();
    };
    // pass 1: sum over t of exp(clamp(att)) + 1e-6 (lane l: t = l, l + 8, ...)
    float sum = 0.f;
    for (int t0 = 0; t0 < T; t0 += TC) {
      const int nt = min(TC, T - t0);
      stage(t0, nt);
      if (act)
        for (int t = l; t < nt; t += 8) sum += att_exp_(s_att[t][cs]);
    }
    sum = sum8_(sum);
    const float inv_tot = 1.0f / sum;
    // pass 2: clipwise = sum_t norm_att * sigmoid(cla); sigmoid(cla) -> outputs
    float acc = 0.f;
    for (int t0 = 0; t0 < T; t0 += TC) {
      const int nt = min(TC, T - t0);
      if (T > TC) stage(t0, nt);             // else still staged from pass 1
      if (act)
        for (int t = l; t < nt; t += 8) {
          const float cl = 1.0f / (1.0f + expf(-s_cla[t][cs]));
          acc += (att_exp_(s_att[t][cs]) * inv_tot) * cl;
          s_cla[t][cs] = cl;
        }
      __syncthreads();
      if ((tid & 31) < nc)
        for (int fr = tid >> 5; fr < nt * 8; fr += 8)
          fw[((int64_t)b * out_frames + 8 * t0 + fr) * C + c0 + (tid & 31)] = s_cla[fr >> 3][tid & 31];
      if (emb)
        for (int cc = tid >> 7; cc < nc; cc += 2)
          if ((tid & 127) < nt) emb[((int64_t)b * C + c0 + cc) * T + t0 + (tid & 127)] = s_cla[tid & 127][cc];
      if (t0 + nt == T && tid < nc) s_last[tid] = s_cla[nt - 1][tid];
    }
    acc = sum8_(acc);
    if (act && l == 0) clip[(int64_t)b * C + c] = acc;
    __syncthreads();
    const int npad = out_frames - 8 * T;          // GRU: last frame repeated
    if ((tid & 31) < nc)
      for (int f = 8 * T + (tid >> 5); f < 8 * T + npad; f += 8)
        fw[((int64_t)b * out_frames + f) * C + c0 + (tid & 31)] = s_last[tid & 31];
  }
}

void launch_att_head(const float* logits, int B, int T, int C, int ldl, int out_frames,
                     float* framewise, float* clipwise, float* emb_cla, hipStream_t s) {
  hipLaunchKernelGGL(att_head_kernel, dim3(B), dim3(256), 0, s, logits, T, C, ldl, out_frames,
                     framewise, clipwise, emb_cla);
}

__global__ __launch_bounds__(256) void transpose_btd_kernel(const float* __restrict__ E, int T,
                                                            int D, float* __restrict__ out) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int t0 = blockIdx.x * 32, d0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, d = d0 + tx;
    tile[i][tx] = (t < T && d < D) ? E[((int64_t)b * T + t) * D + d] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int d = d0 + i, t = t0 + tx;
    if (t < T && d < D) out[((int64_t)b * D + d) * T + t] = tile[tx][i];
  }
}

void launch_transpose_btd(const float* E, int B, int T, int D, float* out, hipStream_t s) {
  hipLaunchKernelGGL(transpose_btd_kernel, dim3((T + 31) / 32, (D + 31) / 32, B), dim3(256), 0, s,
                     E, T, D, out);
}

// ---------------------------------------------------------------------------
// merge (utilities.py:405-446) by the host's plan (windows.cpp
// build_merge_plan): merged[c][f][k] = left fold, in the plan's order, of the
// window values numpy added into frame f, then / div[f].  One thread per
// (clip, frame, class); a frame reads O(sample_duration / step) values.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void merge_plan_kernel(MergeArgs a) {
  const int64_t total = (int64_t)a.n_clips * a.N * a.C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int k = (int)(i % a.C);
    const int64_t cf = i / a.C;
    const int f = (int)(cf % a.N);
    const int64_t c = cf / a.N;
    float s = 0.f;
    const int j0 = a.off[f], j1 = a.off[f + 1];
    for (int j = j0; j < j1; ++j) {
      const int2 e = a.src[j];
      float v = a.fw[a.wb[e.x] + c * a.wcs[e.x] + (int64_t)e.y * a.C + k];
      // binarize_pred: float64 0/1 (a float32 element compared with a float64
      // threshold is compared in float64); sums of 0/1 are exact in f32
      if (a.vote_thr) v = ((double)v > a.vote_thr[k]) ? 1.0f : 0.0f;
      s = j == j0 ? v : s + v;                 // prev_overlap + curr_overlap, window order
    }
    const int d = a.div[f];
    a.merged[i] = d > 1 ? s / (float)d : s;    // float32 /= int (utilities.py:435)
  }
}

void launch_merge_plan(const MergeArgs& a, hipStream_t s) {
  const int64_t total = (int64_t)a.n_clips * a.N * a.C;
  if (total <= 0) return;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(merge_plan_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
}

}  // namespace sedx
