// rcp_probe.hip -- relative error of the hardware f64 reciprocal (v_rcp_f64)
// and of one Newton step on it, over 2^32 mantissas of y in [1, 2): bounds the
// quotient estimate of the Lehmer step (fd_lattice_dev.h, lat_rcp).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/rcp_probe tools/rcp_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <math.h>
#include <string.h>

__global__ void probe( unsigned long long * out, uint64_t base, uint32_t per ) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double m0 = 0.0, m1 = 0.0;
  for( uint32_t i=0; i<per; i++ ) {
    uint64_t idx = base + tid * per + i;
    /* top 32 mantissa bits enumerate, low 20 a hash of them */
    uint64_t h = idx * 0x9e3779b97f4a7c15ull; h ^= h >> 29;
    uint64_t bits = 0x3ff0000000000000ull | ((idx & 0xffffffffull) << 20) | (h & 0xfffffull);
    double y = __longlong_as_double( (long long)bits );
    double r = __builtin_amdgcn_rcp( y );
    double e0 = fabs( fma( r, y, -1.0 ) );
    double r1 = r * fma( -y, r, 2.0 );
    double e1 = fabs( fma( r1, y, -1.0 ) );
    m0 = fmax( m0, e0 ); m1 = fmax( m1, e1 );
  }
  atomicMax( out + 0, (unsigned long long)__double_as_longlong( m0 ) );
  atomicMax( out + 1, (unsigned long long)__double_as_longlong( m1 ) );
}

int main() {
  unsigned long long * d; unsigned long long h[ 2 ] = { 0, 0 };
  if( hipMalloc( &d, 16 ) != hipSuccess ) return 1;
  if( hipMemcpy( d, h, 16, hipMemcpyHostToDevice ) != hipSuccess ) return 1;
  uint32_t per = 256, threads = 256, blocks = 16384;           /* 2^30 per launch */
  for( int l=0; l<4; l++ ) {
    hipLaunchKernelGGL( probe, dim3( blocks ), dim3( threads ), 0, 0, d, (uint64_t)l << 30, per );
    if( hipDeviceSynchronize() != hipSuccess ) return 2;
    fprintf( stderr, "launch %d done\n", l );
  }
  if( hipMemcpy( h, d, 16, hipMemcpyDeviceToHost ) != hipSuccess ) return 3;
  double e0, e1; memcpy( &e0, &h[0], 8 ); memcpy( &e1, &h[1], 8 );
  printf( "{\"samples\": %llu, \"rcp_max_rel_err\": %.6e, \"log2\": %.2f, \"rcp_newton1_max_rel_err\": %.6e, \"log2_1\": %.2f}\n",
          4ull << 30, e0, log2( e0 ), e1, e1 > 0 ? log2( e1 ) : -999.0 );
  return 0;
}
