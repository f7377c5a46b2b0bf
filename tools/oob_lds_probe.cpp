// Probe: does an out-of-range buffer_load_dword / _dwordx4 ... offen lds
// (raw buffer, voffset >= num_records) write zeros into LDS, and does soffset
// take part in the range check?  The F(4,3) Winograd halo staging
// (csrc/conv_wino43.hip) relies on the zero fill for pixels outside the clip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(const float* src, int nbytes, int soff_bytes, unsigned* out) {
  __shared__ unsigned sm[2048];
  const int l = threadIdx.x;
  for (int i = l; i < 2048; i += 64) sm[i] = 0xDEADBEEFu;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nbytes, 0x00020000);
  // lanes 0..31 in range, 32..47 far out (0x80000000), 48..63 just past the end
  unsigned vo = l < 32 ? 4u * l : (l < 48 ? 0x80000000u : (unsigned)nbytes + 4u * (l - 48));
  const unsigned m0a = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) unsigned*)sm);
  const unsigned m0b = m0a + 256 * 4;
  const int so = __builtin_amdgcn_readfirstlane(soff_bytes);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, %3 offen offset:4 lds" ::"v"(vo), "s"(r), "s"(m0a), "s"(so) : "memory");
  unsigned vo4 = l < 32 ? 16u * l : (l < 48 ? 0x80000000u : (unsigned)nbytes + 16u * (l - 48));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds" ::"v"(vo4), "s"(r), "s"(m0b), "s"(so) : "memory");
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  for (int i = l; i < 512; i += 64) out[i] = sm[i];
}

int main() {
  const int n = 4096;
  std::vector<float> h(n);
  for (int i = 0; i < n; ++i) h[i] = (float)(i + 1);
  float* d;
  unsigned* o;
  hipMalloc(&d, n * 4 + 4096);
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  hipMemset((char*)d + n * 4, 0x7f, 4096);   // bytes past num_records are NOT zero
  hipMalloc(&o, 512 * 4);
  for (int so : {0, 64}) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 256 * 4, so, o);
    std::vector<unsigned> r(512);
    hipMemcpy(r.data(), o, 512 * 4, hipMemcpyDeviceToHost);
    printf("soffset %d\n dword: ", so);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
      const float v = *reinterpret_cast<float*>(&r[l]);
      printf("%g%s", v, l % 16 == 15 ? "\n        " : " ");
      if (l >= 32 && r[l] != 0) ++bad;
    }
    printf("\n dwordx4 (first dword of each lane): ");
    for (int l = 0; l < 64; ++l) {
      const float v = *reinterpret_cast<float*>(&r[256 + 4 * l]);
      printf("%g%s", v, l % 16 == 15 ? "\n        " : " ");
      if (l >= 32) for (int q = 0; q < 4; ++q) bad += r[256 + 4 * l + q] != 0;
    }
    printf("\n out-of-range lanes not zero: %d\n", bad);
  }
  hipFree(d);
  hipFree(o);
  return 0;
}
