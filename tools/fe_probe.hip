// fe_probe.hip -- per-wave cycles of the verify kernel's field / group
// building blocks at 1, 2 and 4 waves per SIMD (config 2 runs at 1):
// fe_sq chain (the decode's pow22523 body), fe_mul chain, ge_dbl chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../firedancer_amd/csrc/fd_f25519_dev.h"
#include "../firedancer_amd/csrc/fd_curve25519_dev.h"
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256, 2) k_sq(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a; for (int i = 0; i < 10; i++) a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_sq(a, a);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1];
}
__global__ void __launch_bounds__(256, 2) k_mul(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a, b; for (int i = 0; i < 10; i++) { a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; b.v[i] = (threadIdx.x * 7u + i * 131u) & 0x1ffffffu; }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_mul(a, a, b);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1];
}
__global__ void __launch_bounds__(256, 2) k_pow(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a; for (int i = 0; i < 10; i++) a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_pow22523(a, a);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1];
}
__global__ void __launch_bounds__(256, 2) k_dbl(uint32_t* out, unsigned long long* cyc, int iters) {
  ge_p3 p; for (int i = 0; i < 10; i++) { p.X.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; p.Y.v[i] = (i * 31u) & 0x1ffffffu; p.Z.v[i] = i == 0; p.T.v[i] = 0; }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) ge_dbl(p, p, false);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (p.X.v[0] == 0x12345678u) out[threadIdx.x] = p.Y.v[1];
}
__global__ void __launch_bounds__(256, 2) k_sq2(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a, b; for (int i = 0; i < 10; i++) { a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; b.v[i] = (threadIdx.x * 7u + i * 131u) & 0x1ffffffu; }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_sq2(a, a, b, b);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1] + b.v[2];
}
__global__ void __launch_bounds__(256, 2) k_mul2(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a, b, c, d; for (int i = 0; i < 10; i++) { a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; b.v[i] = (threadIdx.x * 7u + i * 131u) & 0x1ffffffu; c.v[i] = (i * 5u) & 0x1ffffffu; d.v[i] = (threadIdx.x + i) & 0x1ffffffu; }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) fe_mul2(a, a, b, c, c, a);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1] + c.v[2] + d.v[0];
}
__global__ void __launch_bounds__(256, 2) k_mulv(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a, b; for (int i = 0; i < 10; i++) { a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; b.v[i] = (threadIdx.x * 7u + i * 131u) & 0x1ffffffu; }
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int it = 0; it < iters; it++) { fe t; fe_mul(t, a, b); b = a; a = t; }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1];
}
typedef void (*kfn)(uint32_t*, unsigned long long*, int);
int run(const char* name, kfn f, int w, int iters, double per) {
  uint32_t* d; unsigned long long* c; CHECK(hipMalloc(&d, 4096)); CHECK(hipMalloc(&c, 8));
  int blocks = 256 * w;
  for (int rep = 0; rep < 2; rep++) { CHECK(hipMemset(c, 0, 8)); hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, c, iters); CHECK(hipDeviceSynchronize()); }
  unsigned long long h; CHECK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_op_per_wave\": %.1f}\n", name, w, (double)h / (blocks * 4.0) / (iters * per));
  CHECK(hipFree(d)); CHECK(hipFree(c)); return 0;
}
int main() {
  for (int w = 1; w <= 2; w++) {
    run("fe_sq", k_sq, w, 2000, 1.0); run("fe_mul", k_mul, w, 2000, 1.0); run("fe_mul (both operands vary)", k_mulv, w, 2000, 1.0);
    run("fe_sq2 (per pair)", k_sq2, w, 2000, 1.0); run("fe_mul2 (per pair)", k_mul2, w, 2000, 1.0);
    run("fe_pow22523", k_pow, w, 20, 1.0); run("ge_dbl(no T)", k_dbl, w, 500, 1.0);
  }
  return 0;
}
