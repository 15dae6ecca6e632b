// pair_probe.hip -- which gfx950 VALU instruction pairs issue in the same
// quad-cycle from two waves of one SIMD (dev tool; run under rocprofv3
// --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU2, summarized by
// tools/pmc_probe.py).  512-thread workgroups, one per CU: waves 0-3 run
// loop kind A, waves 4-7 loop kind B (wave i and i+4 share SIMD i); kind
// -1 = the wave exits at once.  Each loop: ILP independent chains of one
// instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define ILP 8
#define ITERS 4096

template<int K> __device__ __forceinline__ void body( uint32_t (&x)[ ILP ], uint64_t (&y)[ ILP ], uint32_t a ) {
#pragma unroll
  for( int i=0; i<ILP; i++ ) {
    if constexpr( K == 0 ) asm volatile( "v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(y[i]) : "v"(a), "v"(x[i]) : "vcc" );
    if constexpr( K == 1 ) asm volatile( "v_add_u32 %0, %1, %0" : "+v"(x[i]) : "v"(a) );
    if constexpr( K == 2 ) asm volatile( "v_xor_b32 %0, %1, %0" : "+v"(x[i]) : "v"(a) );
    if constexpr( K == 3 ) asm volatile( "v_and_b32 %0, %1, %0" : "+v"(x[i]) : "v"(a) );
    if constexpr( K == 4 ) asm volatile( "v_lshrrev_b64 %0, 26, %0" : "+v"(y[i]) );
    if constexpr( K == 5 ) asm volatile( "v_mul_lo_u32 %0, %1, %0" : "+v"(x[i]) : "v"(a) );
    if constexpr( K == 6 ) asm volatile( "v_lshl_add_u64 %0, %0, 0, %1" : "+v"(y[i]) : "v"(y[(i+1)%ILP]) );
    if constexpr( K == 7 ) asm volatile( "v_alignbit_b32 %0, %1, %0, 7" : "+v"(x[i]) : "v"(a) );
    if constexpr( K == 8 ) asm volatile( "v_cndmask_b32_e64 %0, %1, %0, vcc" : "+v"(x[i]) : "v"(a) : "vcc" );
  }
}

template<int K> __device__ void run( uint32_t * out, uint32_t seed ) {
  uint32_t x[ ILP ]; uint64_t y[ ILP ];
  uint32_t a = threadIdx.x ^ seed;
#pragma unroll
  for( int i=0; i<ILP; i++ ) { x[i] = a * (i + 3); y[i] = (uint64_t)x[i] << 5; }
  for( int it=0; it<ITERS; it++ ) body<K>( x, y, a );
  uint32_t s = 0;
#pragma unroll
  for( int i=0; i<ILP; i++ ) s ^= x[i] ^ (uint32_t)y[i] ^ (uint32_t)(y[i] >> 32);
  if( s == 0x12345678u ) out[ threadIdx.x ] = s;
}

__device__ void dispatch( int k, uint32_t * out, uint32_t seed ) {
  switch( k ) {
    case 0: run<0>( out, seed ); break; case 1: run<1>( out, seed ); break; case 2: run<2>( out, seed ); break;
    case 3: run<3>( out, seed ); break; case 4: run<4>( out, seed ); break; case 5: run<5>( out, seed ); break;
    case 6: run<6>( out, seed ); break; case 7: run<7>( out, seed ); break; case 8: run<8>( out, seed ); break;
    default: break;
  }
}

extern "C" __global__ void __launch_bounds__( 512 ) k_pair( uint32_t * out, uint32_t seed, int ka, int kb ) {
  int role = __builtin_amdgcn_readfirstlane( (int)threadIdx.x >> 8 );
  dispatch( role ? kb : ka, out, seed );
}

int main( int argc, char ** argv ) {
  static const char * nm[ 9 ] = { "mad_u64_u32", "add_u32", "xor_b32", "and_b32", "lshrrev_b64", "mul_lo_u32", "lshl_add_u64", "alignbit", "cndmask_e64" };
  int pairs[][ 2 ] = { {0,-1}, {1,-1}, {0,0}, {1,1}, {2,2}, {0,1}, {0,2}, {0,3}, {5,1}, {4,1}, {6,1}, {7,1}, {8,1}, {4,4}, {6,6}, {0,4}, {0,6} };
  uint32_t * d; hipMalloc( &d, 1 << 16 );
  for( auto & p : pairs ) {
    for( int rep=0; rep<2; rep++ ) hipLaunchKernelGGL( k_pair, dim3( 256 ), dim3( 512 ), 0, 0, d, 7u, p[0], p[1] );
    hipDeviceSynchronize();
    printf( "{\"a\": \"%s\", \"b\": \"%s\"}\n", nm[ p[0] ], p[1] >= 0 ? nm[ p[1] ] : "-" );
  }
  hipFree( d );
  return 0;
}
