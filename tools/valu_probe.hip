// valu_probe.hip -- measures the gfx950 issue rate of the integer/VALU
// instructions the Ed25519 field arithmetic can be built from, so that the
// INT32 VALU roofline used by bench.py is a MEASURED number (SURVEY.md §8(d):
// "r must be measured by a microbenchmark on the box").
//
// Each kernel runs ILP independent chains of one instruction in an unrolled
// loop; every CU gets WAVES_PER_SIMD*4 waves.  Output: one JSON object with,
// per instruction, wave-instructions per CU per cycle and lane-ops/s for the
// whole chip at the measured shader clock (s_memtime / s_memrealtime ratio).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/valu_probe tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

#ifndef PROBE_ILP
#define PROBE_ILP 12
#endif
constexpr int ILP   = PROBE_ILP;
constexpr int ITERS = 16384 / ILP * 12 / 4;

// clk[0] = sum over waves of s_memtime delta, clk[1] = sum of s_memrealtime delta
#define PROLOGUE \
  uint64_t t0 = __builtin_amdgcn_s_memtime(); uint64_t r0 = __builtin_amdgcn_s_memrealtime();
#define EPILOGUE(SINK) \
  uint64_t t1 = __builtin_amdgcn_s_memtime(); uint64_t r1 = __builtin_amdgcn_s_memrealtime(); \
  if ((threadIdx.x & 63) == 0) { atomicAdd((unsigned long long*)&clk[0], (unsigned long long)(t1 - t0)); \
                                  atomicAdd((unsigned long long*)&clk[1], (unsigned long long)(r1 - r0)); } \
  if (SINK == 0x12345678u) out[blockIdx.x * blockDim.x + threadIdx.x] = SINK;

__global__ void k_mad_u64_u32(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint64_t acc[ILP]; uint32_t a = threadIdx.x ^ seed, b = seed * 3u + 1u;
#pragma unroll
  for (int i = 0; i < ILP; i++) acc[i] = (uint64_t)(a + i) << 7;
  PROLOGUE
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(cc) : "v"(a), "v"(b));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < ILP; i++) s ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32);
  EPILOGUE(s)
}

#define K32(NAME, ASM)                                                                  \
__global__ void NAME(uint32_t* out, uint64_t* clk, uint32_t seed) {                       \
  uint32_t acc[ILP]; uint32_t a = threadIdx.x ^ seed, b = seed * 3u + 1u;                \
  _Pragma("unroll") for (int i = 0; i < ILP; i++) acc[i] = a + i * 77u;                  \
  PROLOGUE                                                                               \
  for (int it = 0; it < ITERS; it++) {                                                   \
    _Pragma("unroll") for (int i = 0; i < ILP; i++) {                                    \
      asm volatile(ASM : "+v"(acc[i]) : "v"(a), "v"(b));                                 \
    }                                                                                    \
  }                                                                                      \
  uint32_t s = 0; _Pragma("unroll") for (int i = 0; i < ILP; i++) s ^= acc[i];           \
  EPILOGUE(s)                                                                            \
}

K32(k_mul_lo_u32,      "v_mul_lo_u32 %0, %1, %0")
K32(k_mul_hi_u32,      "v_mul_hi_u32 %0, %1, %0")
K32(k_mad_u32_u24,     "v_mad_u32_u24 %0, %1, %2, %0")
K32(k_mul_hi_u32_u24,  "v_mul_hi_u32_u24 %0, %1, %0")
K32(k_add_u32,         "v_add_u32 %0, %1, %0")
K32(k_add3_u32,        "v_add3_u32 %0, %1, %2, %0")
K32(k_alignbit_b32,    "v_alignbit_b32 %0, %1, %0, 7")
K32(k_perm_b32,        "v_perm_b32 %0, %1, %0, %2")
K32(k_xor_b32,         "v_xor_b32 %0, %1, %0")
K32(k_bfi_b32,         "v_bfi_b32 %0, %1, %2, %0")
K32(k_lshl_add_u32,    "v_lshl_add_u32 %0, %1, 3, %0")
K32(k_add_u32_e64,     "v_add_u32_e64 %0, %1, %0")
K32(k_mul_u32_u24,     "v_mul_u32_u24 %0, %1, %0")
K32(k_and_b32,         "v_and_b32 %0, %1, %0")
K32(k_lshrrev_b32,     "v_lshrrev_b32 %0, %1, %0")
K32(k_xor_b32_e64,     "v_xor_b32_e64 %0, %1, %0")
K32(k_add_co_vcc_pair, "v_add_co_u32_e32 %0, vcc, %1, %0\n\tv_addc_co_u32_e32 %0, vcc, %2, %0, vcc")
K32(k_cndmask_vcc,     "v_cndmask_b32_e32 %0, %1, %0, vcc")

// add with carry chain: v_add_co_u32 then v_addc_co_u32 through vcc-like SGPR pair
__global__ void k_add_co_addc(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t lo[ILP], hi[ILP]; uint32_t a = threadIdx.x ^ seed;
#pragma unroll
  for (int i = 0; i < ILP; i++) { lo[i] = a + i; hi[i] = a * 5u + i; }
  PROLOGUE
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) {
      uint64_t cc;
      asm volatile("v_add_co_u32 %0, %2, %0, %3\n\tv_addc_co_u32 %1, %2, %1, %3, %2"
                   : "+v"(lo[i]), "+v"(hi[i]), "=&s"(cc) : "v"(a));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < ILP; i++) s ^= lo[i] ^ hi[i];
  EPILOGUE(s)
}

__global__ void k_fma_f64(uint32_t* out, uint64_t* clk, uint32_t seed) {
  double acc[ILP]; double a = 1.0 + 1e-9 * (threadIdx.x ^ seed), b = 0.999999;
#pragma unroll
  for (int i = 0; i < ILP; i++) acc[i] = 1.0 + i;
  PROLOGUE
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ILP; i++) s += acc[i];
  uint32_t si = (uint32_t)__double_as_longlong(s);
  EPILOGUE(si)
}

__global__ void k_fma_f32(uint32_t* out, uint64_t* clk, uint32_t seed) {
  float acc[ILP]; float a = 1.0f + 1e-6f * (threadIdx.x ^ seed), b = 0.9999f;
#pragma unroll
  for (int i = 0; i < ILP; i++) acc[i] = 1.0f + i;
  PROLOGUE
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < ILP; i++) s += acc[i];
  uint32_t si = __float_as_uint(s);
  EPILOGUE(si)
}

__global__ void k_lshrrev_b64(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint64_t acc[ILP]; uint32_t a = (threadIdx.x ^ seed) & 7;
#pragma unroll
  for (int i = 0; i < ILP; i++) acc[i] = 0x123456789ull * (i + 1);
  PROLOGUE
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(acc[i]) : "v"(a));
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < ILP; i++) s ^= (uint32_t)acc[i];
  EPILOGUE(s)
}

// mixed stream typical of a product-scanning field multiply: mad + addc pairs
__global__ void k_mad_addc_pair(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint64_t acc[ILP]; uint32_t c2[ILP]; uint32_t a = threadIdx.x ^ seed, b = seed * 3u + 1u;
#pragma unroll
  for (int i = 0; i < ILP; i++) { acc[i] = (uint64_t)(a + i) << 7; c2[i] = i; }
  PROLOGUE
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, %2, %1"
                   : "+v"(acc[i]), "=&s"(cc), "+v"(c2[i]) : "v"(a), "v"(b));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < ILP; i++) s ^= (uint32_t)acc[i] ^ c2[i];
  EPILOGUE(s)
}

typedef void (*kfn)(uint32_t*, uint64_t*, uint32_t);
struct Probe { const char* name; kfn fn; int instr_per_chain_step; };

int main(int argc, char** argv) {
  Probe probes[] = {
    {"v_mad_u64_u32", k_mad_u64_u32, 1}, {"v_mul_lo_u32", k_mul_lo_u32, 1}, {"v_mul_hi_u32", k_mul_hi_u32, 1},
    {"v_mad_u32_u24", k_mad_u32_u24, 1}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 1},
    {"v_add_u32", k_add_u32, 1}, {"v_add3_u32", k_add3_u32, 1}, {"v_alignbit_b32", k_alignbit_b32, 1},
    {"v_perm_b32", k_perm_b32, 1}, {"v_xor_b32", k_xor_b32, 1}, {"v_bfi_b32", k_bfi_b32, 1},
    {"v_lshl_add_u32", k_lshl_add_u32, 1}, {"v_add_co+v_addc_co(pair)", k_add_co_addc, 2},
    {"v_fma_f64", k_fma_f64, 1}, {"v_fma_f32", k_fma_f32, 1}, {"v_lshrrev_b64", k_lshrrev_b64, 1},
    {"v_mad_u64_u32+v_addc(pair)", k_mad_addc_pair, 2},
    {"v_add_u32_e64", k_add_u32_e64, 1}, {"v_mul_u32_u24", k_mul_u32_u24, 1}, {"v_and_b32", k_and_b32, 1},
    {"v_lshrrev_b32", k_lshrrev_b32, 1}, {"v_xor_b32_e64", k_xor_b32_e64, 1},
    {"v_add_co_e32+v_addc_e32(vcc pair)", k_add_co_vcc_pair, 2}, {"v_cndmask_b32_e32", k_cndmask_vcc, 1},
  };
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  uint32_t* out; uint64_t* clk;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * cus * 8 * 1024));
  CHECK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"ilp\": %d, \"iters\": %d, \"probes\": [\n",
         prop.gcnArchName, cus, prop.clockRate, ILP, ITERS);
  int first = 1;
  int wps_list[] = {2, 4, 8};
  for (auto& p : probes) {
    for (int wps : wps_list) {
      int threads = 256;                       // 4 waves per workgroup
      int blocks = cus * wps;                  // wps workgroups/CU -> wps waves/SIMD
      hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(threads), 0, 0, out, clk, 1u);   // warm-up
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemset(clk, 0, 16));
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(p.fn, dim3(blocks), dim3(threads), 0, 0, out, clk, 1u);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
      uint64_t hclk[2]; CHECK(hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost));
      double ghz = hclk[1] ? (double)hclk[0] / (double)hclk[1] * 0.1 : 0.0;   // memrealtime = 100 MHz
      double wave_instr = (double)blocks * (threads / 64) * ITERS * ILP * p.instr_per_chain_step;
      double lane_ops_s = wave_instr * 64.0 / (ms * 1e-3);
      double cyc = ms * 1e-3 * ghz * 1e9;
      double wi_per_cu_cyc = wave_instr / cus / cyc;
      printf("%s  {\"instr\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ghz\": %.3f, "
             "\"wave_instr_per_cu_per_clk\": %.4f, \"lane_ops_per_cu_per_clk\": %.2f, \"chip_lane_ops_per_s\": %.4e}",
             first ? "" : ",\n", p.name, wps, ms, ghz, wi_per_cu_cyc, wi_per_cu_cyc * 64.0, lane_ops_s);
      first = 0;
    }
  }
  printf("\n]}\n");
  return 0;
}
