// ilp_probe.hip -- cycles per v_mad_u64_u32 per wave at 1 and 2 waves per
// SIMD (config 2 = 64K signatures = 1024 waves = one wave per SIMD) for 1, 2
// and 4 independent accumulation chains.  Each iteration is ONE inline-asm
// block of 96 mads (separate asm statements get an s_nop each).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define M0 "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\t"
#define M1 "v_mad_u64_u32 %1, vcc, %4, %5, %1\n\t"
#define M2 "v_mad_u64_u32 %2, vcc, %4, %5, %2\n\t"
#define M3 "v_mad_u64_u32 %3, vcc, %4, %5, %3\n\t"
#define X8(s) s s s s s s s s
#define X24(s) X8(s) X8(s) X8(s)
#define X96(s) X24(s) X24(s) X24(s) X24(s)
template<int ILP>
__global__ void __launch_bounds__(256) k(uint32_t* out, unsigned long long* cyc, uint32_t seed, int iters) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a = threadIdx.x ^ seed, b = seed * 3u + 1u;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
    if (ILP == 1) asm volatile(X96(M0) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a), "v"(b) : "vcc");
    else if (ILP == 2) asm volatile(X24(M0 M1) X24(M0 M1) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a), "v"(b) : "vcc");
    else asm volatile(X24(M0 M1 M2 M3) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = (uint32_t)(a0 ^ a1 ^ a2 ^ a3);
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (s == 0x12345678u) out[threadIdx.x] = s;
}
template<int ILP>
int run(int waves_per_simd) {
  uint32_t* d; unsigned long long* c; CHECK(hipMalloc(&d, 4096)); CHECK(hipMalloc(&c, 8));
  int iters = 200; int blocks = 256 * waves_per_simd;
  for (int rep = 0; rep < 2; rep++) {
    CHECK(hipMemset(c, 0, 8));
    hipLaunchKernelGGL(k<ILP>, dim3(blocks), dim3(256), 0, 0, d, c, 7u, iters);
    CHECK(hipDeviceSynchronize());
  }
  unsigned long long h; CHECK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
  printf("{\"waves_per_simd\": %d, \"ilp\": %d, \"cyc_per_mad_per_wave\": %.2f}\n", waves_per_simd, ILP, (double)h / (blocks * 4.0) / (iters * 96.0));
  CHECK(hipFree(d)); CHECK(hipFree(c)); return 0;
}
int main() {
  for (int w = 1; w <= 4; w *= 2) { run<1>(w); run<2>(w); run<4>(w); }
  return 0;
}
