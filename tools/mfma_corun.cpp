// Diagnostic: do co-resident MFMA waves change the results of another
// kernel's VALU / transcendental / LDS work?  Probes (non-MFMA) run on
// stream 0 while mfma_spin (bf16 MFMA only, no memory traffic) runs on
// stream 1; every probe output is compared bit for bit with a serial run.
//   probe 0: VALU fma + v_log_f32 / v_exp_f32 / v_rcp_f32 chains, no LDS
//   probe 1: LDS ring traffic (ds_write_b64 / ds_read_b64 + barriers), integer math only
//   probe 2: VALU fma only (no transcendental), no LDS
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void mfma_spin(float* out, int iters) {
  __shared__ uint4 big[4608];
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(0.5f - i * 0.01f); }
  f32x16 acc = {};
  for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  if (threadIdx.x == 0 && acc[0] == 12345.f) big[0] = make_uint4(1, 2, 3, 4);
  __syncthreads();
  if (acc[3] == -1.f) out[blockIdx.x] = acc[0] + (float)big[threadIdx.x].x;
}

__global__ __launch_bounds__(256) void probe_trans(float* out, int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  float x = 1.0f + gid * 1e-6f, y = 0.5f;
  for (int it = 0; it < iters; ++it) {
    x = __logf(x * x + 1.5f);          // v_log_f32
    y = fmaf(y, 0.75f, __expf(-x));     // v_exp_f32
    x = x + __frcp_rn(1.0f + y);        // v_rcp_f32
  }
  out[gid] = x + y;
}

__global__ __launch_bounds__(256) void probe_lds(float* out, int iters) {
  __shared__ uint2 ring[2][256];
  const int t = threadIdx.x;
  uint2 v = make_uint2(blockIdx.x * 977u + t, t * 31u + 7u);
  for (int it = 0; it < iters; ++it) {
    ring[it & 1][t] = v;
    __syncthreads();
    const uint2 w = ring[it & 1][(t * 37 + it) & 255];
    v.x = v.x * 1664525u + w.y;
    v.y ^= w.x + (unsigned)it;
  }
  out[blockIdx.x * 256 + t] = __uint_as_float((v.x ^ v.y) & 0x3fffffffu);
}

__global__ __launch_bounds__(256) void probe_valu(float* out, int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  float x = 1.0f + gid * 1e-6f, y = 0.5f;
  for (int it = 0; it < iters; ++it) {
    x = fmaf(x, 0.999f, y * 1e-3f);
    y = fmaf(y, 1.0001f, -x * 1e-4f);
  }
  out[gid] = x + y;
}

// packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) chains, no LDS
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void probe_pk(float* out, int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  f32x2 x = {1.0f + gid * 1e-6f, 0.5f - gid * 1e-7f}, y = {0.25f, -0.125f};
  const f32x2 c = {0.999f, 1.0001f}, d = {1e-3f, -2e-3f};
  for (int it = 0; it < iters; ++it) {
    x = __builtin_elementwise_fma(x, c, y * d);
    y = y * c + x * d;
  }
  out[gid] = x.x + x.y * 3.0f + y.x * 5.0f + y.y * 7.0f;
}

// probe 4: packed fp32 results written to LDS and read back by other lanes
// (the FFT frontend's pattern: v_pk_* arithmetic feeding ds_write, then
// cross-lane ds_read), wave-local hand-offs only
__global__ __launch_bounds__(256) void probe_pk_lds(float* out, int iters) {
  __shared__ f32x2 ring[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  f32x2 x = {1.0f + gid * 1e-6f, 0.5f - gid * 1e-7f}, y = {0.25f, -0.125f};
  const f32x2 c = {0.999f, 1.0001f}, d = {1e-3f, -2e-3f};
  for (int it = 0; it < iters; ++it) {
    x = __builtin_elementwise_fma(x, c, y * d);
    ring[w][lane] = x;                       // ds_write_b64 of a v_pk result
    __builtin_amdgcn_s_waitcnt(0xc07f);      // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    const f32x2 o = ring[w][(lane * 37 + it) & 63];
    y = y * c + o * d;
    __builtin_amdgcn_wave_barrier();
  }
  out[gid] = x.x + x.y * 3.0f + y.x * 5.0f + y.y * 7.0f;
}

// probe 5: packed fp32 under a PARTIAL exec mask — a lane-dependent trip
// count (lane l runs 8 + (l & 31) iterations, like the mel band sums whose
// widths grow with the band), so the last iterations of each wave run with
// only the upper lanes of each 32-lane half active
__global__ __launch_bounds__(256) void probe_pk_div(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  f32x2 x = {1.0f + gid * 1e-6f, 0.5f - gid * 1e-7f}, y = {0.25f, -0.125f};
  const f32x2 c = {0.999f, 1.0001f}, d = {1e-3f, -2e-3f};
  for (int it = 0; it < iters; ++it) {
    const int n = 8 + (lane & 31);
    for (int k = 0; k < n; ++k) {
      x = __builtin_elementwise_fma(x, c, y * d);
      y = y * c + x * d;
    }
  }
  out[gid] = x.x + x.y * 3.0f + y.x * 5.0f + y.y * 7.0f;
}

// logmel-like gather: reflect-padded 64-bit sample indices, global loads
__global__ __launch_bounds__(256) void probe_gather(const float* __restrict__ audio, int64_t L, int64_t T,
                                                    int64_t total, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t fr = (int64_t)blockIdx.x * 4 + wave; fr < total; fr += (int64_t)gridDim.x * 4) {
    const int64_t item = fr / T;
    const int t = (int)(fr - item * T);
    const float* src = audio + item * L;
    const int64_t pos0 = (int64_t)t * 160 - 256;
    float acc = 0.f;
    for (int m = lane; m < 256; m += 64) {
      for (int e = 0; e < 2; ++e) {
        int64_t j = pos0 + 2 * m + e;
        if (j < 0) j = -j;
        if (j >= L) j = 2 * (L - 1) - j;
        acc = fmaf(src[j], (float)(m + 1), acc);
      }
    }
    out[fr * 64 + lane] = acc;
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 10;
  hipStream_t st[2];
  hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking);
  hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking);
  const int blocks = 4096, n = blocks * 256;
  float *ref, *out, *dummy;
  hipMalloc(&ref, n * 4); hipMalloc(&out, n * 4); hipMalloc(&dummy, 1 << 20);
  std::vector<float> a(n), b(n);
  const int64_t Lg = 160000, Tg = 1001, totalg = 32 * Tg;
  float* audio;
  hipMalloc(&audio, 32 * Lg * 4);
  {
    std::vector<float> h(32 * Lg);
    srand(5);
    for (auto& v : h) v = rand() / (float)RAND_MAX - 0.5f;
    hipMemcpy(audio, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  }
  float *gref, *gout;
  hipMalloc(&gref, totalg * 64 * 4); hipMalloc(&gout, totalg * 64 * 4);
  if (0) {
    hipLaunchKernelGGL(probe_gather, dim3(1024), dim3(256), 0, 0, audio, Lg, Tg, totalg, gref);
    hipDeviceSynchronize();
    std::vector<float> ga(totalg * 64), gb(totalg * 64);
    hipMemcpy(ga.data(), gref, ga.size() * 4, hipMemcpyDeviceToHost);
    int bad_runs = 0;
    size_t bad_vals = 0;
    for (int r = 0; r < R * 8; ++r) {
      hipLaunchKernelGGL(mfma_spin, dim3(512), dim3(256), 0, st[1], dummy, 20000);
      hipLaunchKernelGGL(probe_gather, dim3(1024), dim3(256), 0, st[0], audio, Lg, Tg, totalg, gout);
      hipStreamSynchronize(st[0]);
      hipMemcpy(gb.data(), gout, gb.size() * 4, hipMemcpyDeviceToHost);
      size_t nd = 0;
      for (size_t i = 0; i < ga.size(); ++i) nd += memcmp(&ga[i], &gb[i], 4) != 0;
      bad_runs += nd > 0;
      bad_vals += nd;
      hipDeviceSynchronize();
    }
    printf("probe gather (64-bit reflect indices + global loads): %d of %d runs beside mfma_spin differ, %zu values\n",
           bad_runs, R * 8, bad_vals);
    fflush(stdout);
  }
  for (int probe = 5; probe >= 0; --probe) {
    auto launch = [&](float* o, hipStream_t s) {
      if (probe == 5) hipLaunchKernelGGL(probe_pk_div, dim3(blocks), dim3(256), 0, s, o, 20);
      else if (probe == 4) hipLaunchKernelGGL(probe_pk_lds, dim3(blocks), dim3(256), 0, s, o, 400);
      else if (probe == 3) hipLaunchKernelGGL(probe_pk, dim3(blocks), dim3(256), 0, s, o, 400);
      else if (probe == 0) hipLaunchKernelGGL(probe_trans, dim3(blocks), dim3(256), 0, s, o, 200);
      else if (probe == 1) hipLaunchKernelGGL(probe_lds, dim3(blocks), dim3(256), 0, s, o, 200);
      else hipLaunchKernelGGL(probe_valu, dim3(blocks), dim3(256), 0, s, o, 400);
    };
    launch(ref, 0);
    hipDeviceSynchronize();
    hipMemcpy(a.data(), ref, n * 4, hipMemcpyDeviceToHost);
    int bad_runs = 0;
    size_t bad_vals = 0;
    for (int r = 0; r < R; ++r) {
      for (int k = 0; k < 8; ++k) {
        hipLaunchKernelGGL(mfma_spin, dim3(512), dim3(256), 0, st[1], dummy, 20000);
        launch(out, st[0]);
        hipStreamSynchronize(st[0]);
        hipMemcpy(b.data(), out, n * 4, hipMemcpyDeviceToHost);
        size_t nd = 0;
        for (int i = 0; i < n; ++i) nd += memcmp(&a[i], &b[i], 4) != 0;
        bad_runs += nd > 0;
        bad_vals += nd;
      }
      hipDeviceSynchronize();
    }
    printf("probe %d (%s): %d of %d runs beside mfma_spin differ, %zu values (%s)\n", probe,
           probe == 5 ? "packed fp32, partial exec (divergent trip counts)" : probe == 4 ? "packed fp32 -> LDS -> other lanes" : probe == 3 ? "packed fp32" : probe == 0 ? "VALU+trans" : probe == 1 ? "LDS" : "VALU fma", bad_runs, 8 * R, bad_vals,
           hipGetErrorString(hipGetLastError()));
    fflush(stdout);
  }
  return 0;
}
