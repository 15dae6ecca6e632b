// cu_probe.hip -- which CUs do N workgroups land on? (placement of a 1-wave-per-SIMD grid)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <set>
#include <map>
__global__ void __launch_bounds__(256, 2) k(uint32_t* out, int spin) {
  __shared__ uint32_t lds[10240];
  lds[threadIdx.x] = threadIdx.x;
  uint32_t hwid, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < (uint64_t)spin) {}
  if (threadIdx.x % 64 == 0) out[(blockIdx.x * 4 + threadIdx.x / 64) * 2] = hwid, out[(blockIdx.x * 4 + threadIdx.x / 64) * 2 + 1] = xcc + lds[threadIdx.x] * 0;
}
int main() {
  int nb[] = {256, 512, 1024};
  for (int b : nb) {
    uint32_t* d; hipMalloc(&d, b * 4 * 8);
    hipLaunchKernelGGL(k, dim3(b), dim3(256), 0, 0, d, 200000);
    hipDeviceSynchronize();
    uint32_t* h = new uint32_t[b * 8];
    hipMemcpy(h, d, b * 4 * 8, hipMemcpyDeviceToHost);
    std::map<uint64_t, int> cu, simd;
    for (int i = 0; i < b * 4; i++) {
      uint32_t hw = h[2 * i], x = h[2 * i + 1];
      uint32_t wave = hw & 15, simdid = (hw >> 4) & 3, cuid = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      uint64_t key = ((uint64_t)x << 20) | (se << 12) | (sh << 8) | cuid;
      cu[key]++; simd[(key << 4) | simdid]++;
    }
    int maxw = 0; for (auto& kv : simd) maxw = kv.second > maxw ? kv.second : maxw;
    printf("blocks=%d distinct_CUs=%zu distinct_SIMDs=%zu max_waves_per_SIMD=%d\n", b, cu.size(), simd.size(), maxw);
    hipFree(d);
  }
}
