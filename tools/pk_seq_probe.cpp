// Probe for the packed-FP32 corruption (DESIGN §4 "Packed FP32 beside MFMA"):
// the exact instruction sequence of the failing loop, pinned with inline asm,
// run beside an MFMA-only co-runner on a second stream and compared with a
// solo run.
//
// The failing kernel of profiles/r03_pk_fp32_evidence.log is
// tools/fe_race.cpp lm_variant<0> built WITH packed FP32.  Its wrong outputs
// are mel bands 21-31 or 53-63 of one frame: with that probe's synthetic mel
// (band m reads bins 2m .. 2m+7) exactly the bands whose bins meet 48-63 or
// 112-127 = the power values of lanes 48-63 (the wave's last 16 lanes) in
// the first or second iteration of the power loop (k = lane + 64 i).  That
// loop's memory operations and waits are identical in the packed and the
// non-packed builds (3 ds_read_b64, s_waitcnt lgkmcnt(0), ds_write_b32):
// only the arithmetic differs.  Its packed arithmetic (gfx950 ISA of the
// packed build, registers renamed v26:27 -> v60:61, v52:53 -> v62:63,
// v54:55 -> v64:65, v56:57 -> v66:67, v58:59 -> v68:69):
//
//   variant 0  the packed sequence as the compiler emitted it (s_nop 0
//              between dependent packed ops; v_mov_b32 v69 writes the high
//              half of the pair the next v_pk_fma_f32 reads)
//   variant 1  the same with s_nop 4 after every VALU write that a packed
//              op reads next (more wait states, same arithmetic)
//   variant 2  the non-packed build's scalar sequence (same values)
//   variant 3  variant 0 with its operands from registers (no ds_read)
//   variants 4-9  ONE packed instruction on register operands: v_pk_add_f32,
//              v_pk_mul_f32, v_pk_fma_f32 (no modifiers), v_pk_mul_f32 with
//              op_sel, v_pk_fma_f32 with an inline constant and op_sel_hi,
//              v_pk_add_f32 with neg_lo / neg_hi
//   variants 10-15  the operand-half selects alone: v_pk_mul_f32 op_sel:[0,1]
//              (low result from src1's high half), op_sel_hi:[0,0] (high
//              result from both low halves), v_pk_add_f32 and v_pk_fma_f32
//              with variant 7's selects, v_pk_mul_f32 op_sel:[1,0] and
//              op_sel_hi:[1,0]
//
// Every thread folds its power values into a hash; a run beside the
// co-runner is bad when any hash differs from the solo run's.
//   usage: pk_seq_probe <variant|-1 for all> <runs>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void mfma_spin(float* out, int iters) {
  __shared__ uint4 big[4608];
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(threadIdx.x * 0.001f + i);
    b[i] = (__bf16)(0.5f - i * 0.01f);
  }
  f32x16 acc = {};
  for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  if (threadIdx.x == 0 && acc[0] == 12345.f) big[0] = make_uint4(1, 2, 3, 4);
  __syncthreads();
  if (acc[3] == -1.f) out[blockIdx.x] = acc[0] + (float)big[threadIdx.x].x;
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#define PK_CLOBBER "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "memory"
// variants 4-9: one packed FP32 instruction on register operands (v[60:61]
// = tw, v[62:63] = z1, v[64:65] = z2), result lo + hi
#define PK_SINGLE(OPSTR)                                                                    \
  asm volatile("v_mov_b32 v60, %1\n\tv_mov_b32 v61, %2\n\tv_mov_b32 v62, %3\n\t"            \
               "v_mov_b32 v63, %4\n\tv_mov_b32 v64, %5\n\tv_mov_b32 v65, %6\n\ts_nop 4\n\t" OPSTR \
               "\n\ts_nop 4\n\tv_add_f32 %0, v66, v67"                                      \
               : "=v"(pw)                                                                     \
               : "v"(tw.x), "v"(tw.y), "v"(z1.x), "v"(z1.y), "v"(z2.x), "v"(z2.y)             \
               : PK_CLOBBER)
template <int V>
__device__ __forceinline__ float power_seq(uint32_t a_tw, uint32_t a_z1, uint32_t a_z2, float2 tw, float2 z1,
                                           float2 z2) {
  float pw;
  if constexpr (V == 0) {
    asm volatile(
        "ds_read_b64 v[60:61], %1\n\t"
        "ds_read_b64 v[62:63], %2\n\t"
        "ds_read_b64 v[64:65], %3\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_pk_add_f32 v[66:67], v[62:63], v[64:65]\n\t"
        "v_pk_add_f32 v[62:63], v[62:63], v[64:65] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_mov_b32 v64, v66\n\t"
        "v_mul_f32 v62, -0.5, v62\n\t"
        "v_mov_b32 v65, v63\n\t"
        "v_mul_f32 v66, 0.5, v67\n\t"
        "v_pk_mul_f32 v[62:63], v[62:63], v[60:61] op_sel:[0,1] op_sel_hi:[0,0]\n\t"
        "v_pk_fma_f32 v[68:69], v[60:61], v[66:67], v[62:63] neg_lo:[0,0,1] neg_hi:[0,0,1]\n\t"
        "v_pk_fma_f32 v[60:61], v[60:61], v[66:67], v[62:63] op_sel_hi:[1,0,1]\n\t"
        "s_nop 0\n\t"
        "v_mov_b32 v69, v61\n\t"
        "v_pk_fma_f32 v[60:61], v[64:65], 0.5, v[68:69] op_sel_hi:[1,0,1]\n\t"
        "s_nop 0\n\t"
        "v_pk_mul_f32 v[60:61], v[60:61], v[60:61]\n\t"
        "s_nop 0\n\t"
        "v_add_f32 %0, v60, v61"
        : "=v"(pw)
        : "v"(a_tw), "v"(a_z1), "v"(a_z2)
        : PK_CLOBBER);
  } else if constexpr (V == 1) {
    asm volatile(
        "ds_read_b64 v[60:61], %1\n\t"
        "ds_read_b64 v[62:63], %2\n\t"
        "ds_read_b64 v[64:65], %3\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_pk_add_f32 v[66:67], v[62:63], v[64:65]\n\t"
        "v_pk_add_f32 v[62:63], v[62:63], v[64:65] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "s_nop 4\n\t"
        "v_mov_b32 v64, v66\n\t"
        "v_mul_f32 v62, -0.5, v62\n\t"
        "v_mov_b32 v65, v63\n\t"
        "v_mul_f32 v66, 0.5, v67\n\t"
        "s_nop 4\n\t"
        "v_pk_mul_f32 v[62:63], v[62:63], v[60:61] op_sel:[0,1] op_sel_hi:[0,0]\n\t"
        "s_nop 4\n\t"
        "v_pk_fma_f32 v[68:69], v[60:61], v[66:67], v[62:63] neg_lo:[0,0,1] neg_hi:[0,0,1]\n\t"
        "v_pk_fma_f32 v[60:61], v[60:61], v[66:67], v[62:63] op_sel_hi:[1,0,1]\n\t"
        "s_nop 4\n\t"
        "v_mov_b32 v69, v61\n\t"
        "s_nop 4\n\t"
        "v_pk_fma_f32 v[60:61], v[64:65], 0.5, v[68:69] op_sel_hi:[1,0,1]\n\t"
        "s_nop 4\n\t"
        "v_pk_mul_f32 v[60:61], v[60:61], v[60:61]\n\t"
        "s_nop 4\n\t"
        "v_add_f32 %0, v60, v61"
        : "=v"(pw)
        : "v"(a_tw), "v"(a_z1), "v"(a_z2)
        : PK_CLOBBER);
  } else if constexpr (V == 2) {
    // the non-packed build's sequence (v26 v27 tw, v52 v53 A, v54 v55 Bz)
    asm volatile(
        "ds_read_b64 v[60:61], %1\n\t"
        "ds_read_b64 v[62:63], %2\n\t"
        "ds_read_b64 v[64:65], %3\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_add_f32 v66, v62, v64\n\t"
        "v_sub_f32 v67, v63, v65\n\t"
        "v_add_f32 v63, v63, v65\n\t"
        "v_sub_f32 v62, v62, v64\n\t"
        "v_mul_f32 v63, 0.5, v63\n\t"
        "v_mul_f32 v62, -0.5, v62\n\t"
        "v_mul_f32 v64, v62, v61\n\t"
        "v_mul_f32 v61, v61, v63\n\t"
        "v_fmac_f32 v61, v60, v62\n\t"
        "v_fma_f32 v63, v60, v63, -v64\n\t"
        "v_fmac_f32 v61, 0.5, v67\n\t"
        "v_fmac_f32 v63, 0.5, v66\n\t"
        "v_mul_f32 v66, v61, v61\n\t"
        "v_fmac_f32 v66, v63, v63\n\t"
        "v_mov_b32 %0, v66"
        : "=v"(pw)
        : "v"(a_tw), "v"(a_z1), "v"(a_z2)
        : PK_CLOBBER);
  } else if constexpr (V == 4) {
    PK_SINGLE("v_pk_add_f32 v[66:67], v[62:63], v[64:65]");
  } else if constexpr (V == 5) {
    PK_SINGLE("v_pk_mul_f32 v[66:67], v[62:63], v[64:65]");
  } else if constexpr (V == 6) {
    PK_SINGLE("v_pk_fma_f32 v[66:67], v[60:61], v[62:63], v[64:65]");
  } else if constexpr (V == 7) {
    PK_SINGLE("v_pk_mul_f32 v[66:67], v[62:63], v[60:61] op_sel:[0,1] op_sel_hi:[0,0]");
  } else if constexpr (V == 8) {
    PK_SINGLE("v_pk_fma_f32 v[66:67], v[64:65], 0.5, v[62:63] op_sel_hi:[1,0,1]");
  } else if constexpr (V == 9) {
    PK_SINGLE("v_pk_add_f32 v[66:67], v[62:63], v[64:65] neg_lo:[0,1] neg_hi:[0,1]");
  } else if constexpr (V == 10) {
    PK_SINGLE("v_pk_mul_f32 v[66:67], v[62:63], v[60:61] op_sel:[0,1]");
  } else if constexpr (V == 11) {
    PK_SINGLE("v_pk_mul_f32 v[66:67], v[62:63], v[60:61] op_sel_hi:[0,0]");
  } else if constexpr (V == 12) {
    PK_SINGLE("v_pk_add_f32 v[66:67], v[62:63], v[60:61] op_sel:[0,1] op_sel_hi:[0,0]");
  } else if constexpr (V == 13) {
    PK_SINGLE("v_pk_fma_f32 v[66:67], v[62:63], v[60:61], v[64:65] op_sel:[0,1,0] op_sel_hi:[0,0,1]");
  } else if constexpr (V == 14) {
    PK_SINGLE("v_pk_mul_f32 v[66:67], v[62:63], v[60:61] op_sel:[1,0] op_sel_hi:[1,1]");
  } else if constexpr (V == 15) {
    PK_SINGLE("v_pk_mul_f32 v[66:67], v[62:63], v[60:61] op_sel_hi:[1,0]");
  } else {
    asm volatile(
        "v_mov_b32 v60, %1\n\t"
        "v_mov_b32 v61, %2\n\t"
        "v_mov_b32 v62, %3\n\t"
        "v_mov_b32 v63, %4\n\t"
        "v_mov_b32 v64, %5\n\t"
        "v_mov_b32 v65, %6\n\t"
        "s_nop 4\n\t"
        "v_pk_add_f32 v[66:67], v[62:63], v[64:65]\n\t"
        "v_pk_add_f32 v[62:63], v[62:63], v[64:65] neg_lo:[0,1] neg_hi:[0,1]\n\t"
        "v_mov_b32 v64, v66\n\t"
        "v_mul_f32 v62, -0.5, v62\n\t"
        "v_mov_b32 v65, v63\n\t"
        "v_mul_f32 v66, 0.5, v67\n\t"
        "v_pk_mul_f32 v[62:63], v[62:63], v[60:61] op_sel:[0,1] op_sel_hi:[0,0]\n\t"
        "v_pk_fma_f32 v[68:69], v[60:61], v[66:67], v[62:63] neg_lo:[0,0,1] neg_hi:[0,0,1]\n\t"
        "v_pk_fma_f32 v[60:61], v[60:61], v[66:67], v[62:63] op_sel_hi:[1,0,1]\n\t"
        "s_nop 0\n\t"
        "v_mov_b32 v69, v61\n\t"
        "v_pk_fma_f32 v[60:61], v[64:65], 0.5, v[68:69] op_sel_hi:[1,0,1]\n\t"
        "s_nop 0\n\t"
        "v_pk_mul_f32 v[60:61], v[60:61], v[60:61]\n\t"
        "s_nop 0\n\t"
        "v_add_f32 %0, v60, v61"
        : "=v"(pw)
        : "v"(tw.x), "v"(tw.y), "v"(z1.x), "v"(z1.y), "v"(z2.x), "v"(z2.y)
        : PK_CLOBBER);
    (void)a_tw;
    (void)a_z1;
    (void)a_z2;
  }
  return pw;
}
#pragma clang diagnostic pop

// per wave: Z [256] float2 and the twiddles in LDS; the power loop of
// lm_variant<0> (k = lane + 64 i, i = 0..3, full EXEC) repeated `iters` times
// with inputs perturbed per pass; each thread hashes its power values
template <int V>
__global__ __launch_bounds__(256) void seq_probe(const float2* __restrict__ in, unsigned* __restrict__ out, int iters) {
  __shared__ float2 s_tw[512];
  __shared__ float2 s_z[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 512; i += 256) s_tw[i] = in[i];
  for (int i = lane; i < 256; i += 64) s_z[wave][i] = in[512 + ((blockIdx.x * 4 + wave) * 256 + i) % 65536];
  __syncthreads();
  unsigned h = 2166136261u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = lane + 64 * i;
      const uint32_t a_tw = (uint32_t)(size_t)(__attribute__((address_space(3))) float2*)(s_tw + k);
      const uint32_t a_z1 = (uint32_t)(size_t)(__attribute__((address_space(3))) float2*)(&s_z[wave][k & 255]);
      const uint32_t a_z2 = (uint32_t)(size_t)(__attribute__((address_space(3))) float2*)(&s_z[wave][(256 - k) & 255]);
      float2 tw = make_float2(0.f, 0.f), z1 = tw, z2 = tw;
      if constexpr (V >= 3) {
        tw = s_tw[k];
        z1 = s_z[wave][k & 255];
        z2 = s_z[wave][(256 - k) & 255];
      }
      const float pw = power_seq<V>(a_tw, a_z1, a_z2, tw, z1, z2);
      h = (h ^ __float_as_uint(pw)) * 16777619u;
    }
    // perturb this wave's Z for the next pass (wave-local, in order)
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < 256; i += 64) {
      float2 z = s_z[wave][i];
      s_z[wave][i] = make_float2(z.y * 0.999f + 1e-3f, z.x * 1.001f - 1e-3f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  out[blockIdx.x * 256 + tid] = h;
}

template <int V>
static void launch(const float2* in, unsigned* out, int blocks, int iters, hipStream_t s) {
  hipLaunchKernelGGL(seq_probe<V>, dim3(blocks), dim3(256), 0, s, in, out, iters);
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  const int runs = argc > 2 ? atoi(argv[2]) : 32;
  const int blocks = 4096, iters = 64;
  std::vector<float2> hin(512 + 65536);
  srand(7);
  for (auto& v : hin) v = make_float2((rand() / (float)RAND_MAX - 0.5f) * 4.f, (rand() / (float)RAND_MAX - 0.5f) * 4.f);
  float2* din;
  unsigned *dref, *dout;
  float* dspin;
  hipMalloc(&din, hin.size() * sizeof(float2));
  hipMemcpy(din, hin.data(), hin.size() * sizeof(float2), hipMemcpyHostToDevice);
  const size_t n = (size_t)blocks * 256;
  hipMalloc(&dref, n * 4);
  hipMalloc(&dout, n * 4);
  hipMalloc(&dspin, 4096 * 4);
  hipStream_t st[2];
  hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking);
  hipStreamCreateWithFlags(&st[1], hipStreamNonBlocking);
  std::vector<unsigned> ref(n), got(n);
  for (int v = 0; v < 16; ++v) {
    if (only >= 0 && v != only) continue;
    auto run = [&](unsigned* o, hipStream_t s) {
      switch (v) {
        case 0: launch<0>(din, o, blocks, iters, s); break;
        case 1: launch<1>(din, o, blocks, iters, s); break;
        case 2: launch<2>(din, o, blocks, iters, s); break;
        case 3: launch<3>(din, o, blocks, iters, s); break;
        case 4: launch<4>(din, o, blocks, iters, s); break;
        case 5: launch<5>(din, o, blocks, iters, s); break;
        case 6: launch<6>(din, o, blocks, iters, s); break;
        case 7: launch<7>(din, o, blocks, iters, s); break;
        case 8: launch<8>(din, o, blocks, iters, s); break;
        case 9: launch<9>(din, o, blocks, iters, s); break;
        case 10: launch<10>(din, o, blocks, iters, s); break;
        case 11: launch<11>(din, o, blocks, iters, s); break;
        case 12: launch<12>(din, o, blocks, iters, s); break;
        case 13: launch<13>(din, o, blocks, iters, s); break;
        case 14: launch<14>(din, o, blocks, iters, s); break;
        default: launch<15>(din, o, blocks, iters, s); break;
      }
    };
    run(dref, 0);
    hipDeviceSynchronize();
    hipMemcpy(ref.data(), dref, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    size_t bad_threads = 0;
    int lanes_hit[64] = {};
    for (int r = 0; r < runs; ++r) {
      hipMemset(dout, 0, n * 4);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(mfma_spin, dim3(512), dim3(256), 0, st[1], dspin, 4000);
      run(dout, st[0]);
      hipLaunchKernelGGL(mfma_spin, dim3(512), dim3(256), 0, st[1], dspin, 4000);
      hipDeviceSynchronize();
      hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost);
      size_t nd = 0;
      for (size_t j = 0; j < n; ++j)
        if (got[j] != ref[j]) {
          ++nd;
          ++lanes_hit[j & 63];
        }
      if (nd) ++bad;
      bad_threads += nd;
    }
    printf("variant %d: %d of %d runs beside mfma_spin differ, %zu thread hashes (%s)", v, bad, runs, bad_threads,
           hipGetErrorString(hipGetLastError()));
    if (bad_threads) {
      printf("; lanes hit:");
      for (int l = 0; l < 64; ++l)
        if (lanes_hit[l]) printf(" %d", l);
    }
    printf("\n");
  }
  return 0;
}
