// issue_probe.hip -- per-wave issue cost (cycles per instruction) of the VALU
// instructions the verify kernel is made of, at 1 and 2 waves per SIMD.
// Each iteration is ONE inline-asm block of 96 instructions over 4
// independent registers (separate asm statements would get s_nop padding).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define X8(s) s s s s s s s s
#define X24(s) X8(s) X8(s) X8(s)
#define BODY(I0, I1, I2, I3) X24(I0 "\n\t" I1 "\n\t" I2 "\n\t" I3 "\n\t")
#define KERNEL(NAME, I0, I1, I2, I3)                                                              \
__global__ void __launch_bounds__(256) NAME(uint32_t* out, unsigned long long* cyc, uint32_t seed, int iters) { \
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a = threadIdx.x ^ seed, b = seed * 3u + 1u; \
  uint64_t t0 = __builtin_amdgcn_s_memtime();                                                     \
  for (int it = 0; it < iters; it++)                                                              \
    asm volatile(BODY(I0, I1, I2, I3) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a), "v"(b) : "vcc", "s40", "s41"); \
  uint64_t t1 = __builtin_amdgcn_s_memtime();                                                     \
  uint32_t s = (uint32_t)(a0 ^ a1 ^ a2 ^ a3);                                                     \
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));                     \
  if (s == 0x12345678u) out[threadIdx.x] = s; }
#define KERNEL32(NAME, I0, I1, I2, I3)                                                            \
__global__ void __launch_bounds__(256) NAME(uint32_t* out, unsigned long long* cyc, uint32_t seed, int iters) { \
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3; uint32_t a = threadIdx.x ^ seed, b = seed * 3u + 1u; \
  uint64_t t0 = __builtin_amdgcn_s_memtime();                                                     \
  for (int it = 0; it < iters; it++)                                                              \
    asm volatile(BODY(I0, I1, I2, I3) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a), "v"(b) : "vcc", "s40", "s41"); \
  uint64_t t1 = __builtin_amdgcn_s_memtime();                                                     \
  uint32_t s = a0 ^ a1 ^ a2 ^ a3;                                                                 \
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));                     \
  if (s == 0x12345678u) out[threadIdx.x] = s; }
KERNEL(k_mad,    "v_mad_u64_u32 %0, vcc, %4, %5, %0", "v_mad_u64_u32 %1, vcc, %4, %5, %1", "v_mad_u64_u32 %2, vcc, %4, %5, %2", "v_mad_u64_u32 %3, vcc, %4, %5, %3")
KERNEL32(k_and,    "v_and_b32 %0, %4, %0", "v_and_b32 %1, %4, %1", "v_and_b32 %2, %4, %2", "v_and_b32 %3, %4, %3")
KERNEL(k_shr64,  "v_lshrrev_b64 %0, 26, %0", "v_lshrrev_b64 %1, 25, %1", "v_lshrrev_b64 %2, 26, %2", "v_lshrrev_b64 %3, 25, %3")
KERNEL32(k_mullo,  "v_mul_lo_u32 %0, %4, %0", "v_mul_lo_u32 %1, %4, %1", "v_mul_lo_u32 %2, %4, %2", "v_mul_lo_u32 %3, %4, %3")
KERNEL32(k_add,    "v_add_u32 %0, %4, %0", "v_add_u32 %1, %4, %1", "v_add_u32 %2, %4, %2", "v_add_u32 %3, %4, %3")
KERNEL(k_lshladd64, "v_lshl_add_u64 %0, %0, 1, %1", "v_lshl_add_u64 %1, %1, 1, %2", "v_lshl_add_u64 %2, %2, 1, %3", "v_lshl_add_u64 %3, %3, 1, %0")
KERNEL32(k_cnd,    "v_cndmask_b32 %0, %0, %4, vcc", "v_cndmask_b32 %1, %1, %4, vcc", "v_cndmask_b32 %2, %2, %4, vcc", "v_cndmask_b32 %3, %3, %4, vcc")
KERNEL(k_mad_shr, "v_mad_u64_u32 %0, vcc, %4, %5, %0", "v_lshrrev_b64 %1, 26, %1", "v_mad_u64_u32 %2, vcc, %4, %5, %2", "v_lshrrev_b64 %3, 25, %3")
KERNEL(k_fma64,  "v_fma_f64 %0, %0, %0, %1", "v_fma_f64 %1, %1, %1, %2", "v_fma_f64 %2, %2, %2, %3", "v_fma_f64 %3, %3, %3, %0")
KERNEL32(k_dpp,   "v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v_mov_b32_dpp %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v_mov_b32_dpp %2, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v_mov_b32_dpp %3, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
KERNEL32(k_adddpp, "v_add_u32_dpp %0, %4, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v_add_u32_dpp %1, %4, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v_add_u32_dpp %2, %4, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "v_add_u32_dpp %3, %4, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
KERNEL32(k_cnd64, "v_cndmask_b32_e64 %0, %0, %4, s[40:41]", "v_cndmask_b32_e64 %1, %1, %4, s[40:41]", "v_cndmask_b32_e64 %2, %2, %4, s[42:43]", "v_cndmask_b32_e64 %3, %3, %4, s[42:43]")
KERNEL32(k_bfi,   "v_bfi_b32 %0, %4, %0, %5", "v_bfi_b32 %1, %4, %1, %5", "v_bfi_b32 %2, %4, %2, %5", "v_bfi_b32 %3, %4, %3, %5")
KERNEL32(k_swap,  "v_permlane32_swap_b32 %0, %1", "v_permlane32_swap_b32 %2, %3", "v_permlane32_swap_b32 %1, %0", "v_permlane32_swap_b32 %3, %2")
KERNEL32(k_cmpcnd, "v_cmp_lt_u32 vcc, %4, %0", "v_cndmask_b32 %1, %1, %0, vcc", "v_cndmask_b32 %2, %2, %1, vcc", "v_cndmask_b32 %3, %3, %2, vcc")
KERNEL32(k_cmpcnd64, "v_cmp_lt_u32_e64 s[40:41], %4, %0", "v_cndmask_b32_e64 %1, %1, %0, s[40:41]", "v_cndmask_b32_e64 %2, %2, %1, s[40:41]", "v_cndmask_b32_e64 %3, %3, %2, s[40:41]")
KERNEL32(k_cnd64vcc, "v_cndmask_b32_e64 %0, %0, %4, vcc", "v_cndmask_b32_e64 %1, %1, %4, vcc", "v_cndmask_b32_e64 %2, %2, %4, vcc", "v_cndmask_b32_e64 %3, %3, %4, vcc")
KERNEL32(k_addco, "v_add_co_u32 %0, vcc, %4, %0", "v_addc_co_u32 %1, vcc, %4, %1, vcc", "v_add_co_u32 %2, vcc, %4, %2", "v_addc_co_u32 %3, vcc, %4, %3, vcc")
typedef void (*kfn)(uint32_t*, unsigned long long*, uint32_t, int);
int run(const char* name, kfn f, int w) {
  uint32_t* d; unsigned long long* c; CHECK(hipMalloc(&d, 4096)); CHECK(hipMalloc(&c, 8));
  int iters = 200, blocks = 256 * w;
  for (int rep = 0; rep < 2; rep++) { CHECK(hipMemset(c, 0, 8)); hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, c, 7u, iters); CHECK(hipDeviceSynchronize()); }
  unsigned long long h; CHECK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
  printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_instr_per_wave\": %.2f}\n", name, w, (double)h / (blocks * 4.0) / (iters * 96.0));
  CHECK(hipFree(d)); CHECK(hipFree(c)); return 0;
}
int main() {
  for (int w = 1; w <= 2; w++) {
    run("v_mad_u64_u32", k_mad, w); run("v_and_b32", k_and, w); run("v_lshrrev_b64", k_shr64, w); run("v_mul_lo_u32", k_mullo, w);
    run("v_add_u32", k_add, w); run("v_lshl_add_u64", k_lshladd64, w); run("v_cndmask_b32", k_cnd, w); run("mad+shr64 alternating", k_mad_shr, w);
    run("v_fma_f64", k_fma64, w);
    run("v_mov_b32_dpp quad_perm", k_dpp, w); run("v_add_u32_dpp quad_perm", k_adddpp, w); run("v_cndmask_b32_e64 sgpr", k_cnd64, w);
    run("v_bfi_b32", k_bfi, w); run("v_permlane32_swap", k_swap, w);
    run("v_cmp(vcc)+3 v_cndmask_e32", k_cmpcnd, w); run("v_cndmask_b32_e64 vcc", k_cnd64vcc, w); run("v_add_co/v_addc_co vcc", k_addco, w); run("v_cmp(sgpr)+3 v_cndmask_e64", k_cmpcnd64, w);
  }
  return 0;
}
