// bank_probe.hip -- does VGPR bank placement change v_mad_u64_u32 issue on
// gfx950?  (dev tool; run under rocprofv3 --pmc SQ_INSTS_VALU
// SQ_BUSY_CU_CYCLES, tools/pmc_probe.py).  Each kernel runs a dependent
// MAC chain (the accumulator pair is the addend of the next MAC, as in the
// field products) with fixed physical registers: the two 32-bit operands
// in banks distinct from the accumulator's ("spread") or in the
// accumulator's low bank ("same"); and 4 independent chains ("ilp4").
// One wave per SIMD (256 workgroups of 256 threads).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

extern "C" __global__ void __launch_bounds__( 256 ) k_spread( uint32_t * out, int iters ) {
  uint32_t r;
  asm volatile( "v_mov_b32 v0, %1\n v_mov_b32 v1, 0\n v_mov_b32 v2, 3\n v_mov_b32 v3, %1\n"
                "s_mov_b32 s40, %2\n"
                "1:\n"
                REP64( "v_mad_u64_u32 v[0:1], vcc, v2, v3, v[0:1]\n" )
                "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n"
                "v_mov_b32 %0, v0\n"
                : "=v"(r) : "v"(threadIdx.x), "s"(iters) : "v0", "v1", "v2", "v3", "s40", "vcc", "scc" );
  if( r == 0x12345u ) out[ threadIdx.x ] = r;
}
extern "C" __global__ void __launch_bounds__( 256 ) k_same( uint32_t * out, int iters ) {
  uint32_t r;
  asm volatile( "v_mov_b32 v0, %1\n v_mov_b32 v1, 0\n v_mov_b32 v4, 3\n v_mov_b32 v8, %1\n"
                "s_mov_b32 s40, %2\n"
                "1:\n"
                REP64( "v_mad_u64_u32 v[0:1], vcc, v4, v8, v[0:1]\n" )
                "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n"
                "v_mov_b32 %0, v0\n"
                : "=v"(r) : "v"(threadIdx.x), "s"(iters) : "v0", "v1", "v4", "v8", "s40", "vcc", "scc" );
  if( r == 0x12345u ) out[ threadIdx.x ] = r;
}
extern "C" __global__ void __launch_bounds__( 256 ) k_ilp4( uint32_t * out, int iters ) {
  uint32_t r;
  asm volatile( "v_mov_b32 v0, %1\n v_mov_b32 v1, 0\n v_mov_b32 v2, 3\n v_mov_b32 v3, %1\n"
                "v_mov_b32 v4, %1\n v_mov_b32 v5, 0\n v_mov_b32 v6, %1\n v_mov_b32 v7, 0\n v_mov_b32 v8, %1\n v_mov_b32 v9, 0\n"
                "s_mov_b32 s40, %2\n"
                "1:\n"
                REP8( "v_mad_u64_u32 v[0:1], vcc, v2, v3, v[0:1]\n v_mad_u64_u32 v[4:5], vcc, v2, v3, v[4:5]\n"
                      "v_mad_u64_u32 v[6:7], vcc, v2, v3, v[6:7]\n v_mad_u64_u32 v[8:9], vcc, v2, v3, v[8:9]\n"
                      "v_mad_u64_u32 v[0:1], vcc, v2, v3, v[0:1]\n v_mad_u64_u32 v[4:5], vcc, v2, v3, v[4:5]\n"
                      "v_mad_u64_u32 v[6:7], vcc, v2, v3, v[6:7]\n v_mad_u64_u32 v[8:9], vcc, v2, v3, v[8:9]\n" )
                "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n"
                "v_add_u32 %0, v0, v4\n"
                : "=v"(r) : "v"(threadIdx.x), "s"(iters) : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "s40", "vcc", "scc" );
  if( r == 0x12345u ) out[ threadIdx.x ] = r;
}
extern "C" __global__ void __launch_bounds__( 256 ) k_ilp4_nosdst( uint32_t * out, int iters ) {
  uint32_t r;
  asm volatile( "v_mov_b32 v0, %1\n v_mov_b32 v1, 0\n v_mov_b32 v2, 3\n v_mov_b32 v3, %1\n"
                "v_mov_b32 v4, %1\n v_mov_b32 v5, 0\n v_mov_b32 v6, %1\n v_mov_b32 v7, 0\n v_mov_b32 v8, %1\n v_mov_b32 v9, 0\n"
                "s_mov_b32 s40, %2\n"
                "1:\n"
                REP8( "v_mad_u64_u32 v[0:1], s[42:43], v2, v3, v[0:1]\n v_mad_u64_u32 v[4:5], s[44:45], v2, v3, v[4:5]\n"
                      "v_mad_u64_u32 v[6:7], s[46:47], v2, v3, v[6:7]\n v_mad_u64_u32 v[8:9], s[48:49], v2, v3, v[8:9]\n"
                      "v_mad_u64_u32 v[0:1], s[42:43], v2, v3, v[0:1]\n v_mad_u64_u32 v[4:5], s[44:45], v2, v3, v[4:5]\n"
                      "v_mad_u64_u32 v[6:7], s[46:47], v2, v3, v[6:7]\n v_mad_u64_u32 v[8:9], s[48:49], v2, v3, v[8:9]\n" )
                "s_sub_u32 s40, s40, 1\n s_cmp_lg_u32 s40, 0\n s_cbranch_scc1 1b\n"
                "v_add_u32 %0, v0, v4\n"
                : "=v"(r) : "v"(threadIdx.x), "s"(iters) : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9",
                  "s40", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "scc" );
  if( r == 0x12345u ) out[ threadIdx.x ] = r;
}

int main() {
  uint32_t * d; hipMalloc( &d, 1 << 16 );
  for( int rep=0; rep<2; rep++ ) {
    hipLaunchKernelGGL( k_spread, dim3( 256 ), dim3( 256 ), 0, 0, d, 512 );
    hipLaunchKernelGGL( k_same, dim3( 256 ), dim3( 256 ), 0, 0, d, 512 );
    hipLaunchKernelGGL( k_ilp4, dim3( 256 ), dim3( 256 ), 0, 0, d, 512 );
    hipLaunchKernelGGL( k_ilp4_nosdst, dim3( 256 ), dim3( 256 ), 0, 0, d, 512 );
  }
  hipDeviceSynchronize();
  printf( "done\n" );
  return 0;
}
