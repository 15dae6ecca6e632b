// fe_probe2.hip -- one wave per SIMD (config 2's geometry): cycles per group
// operation for the verify kernel's doubling and cached addition, as built
// now (each field product alone between scheduling fences) and with the
// independent products of each formula issued two at a time (fe_sq2 /
// fe_mul2: two MAC chains interleaved instruction by instruction, so a
// dependent v_mad_u64_u32 never waits on its predecessor with nothing else
// to issue).  Also the decode's squaring chain single vs two chains at once.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/fe_probe2 tools/fe_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../firedancer_amd/csrc/fd_f25519_dev.h"
#include "../firedancer_amd/csrc/fd_curve25519_dev.h"
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

#ifndef WPE
#define WPE 1
#endif

__device__ __forceinline__ void ge_dbl_il( ge_p3 & r, ge_p3 const & p, bool want_t ) {
  fe XX, YY, ZZ, AA, s, H, G, E, Fn;
  fe_sq2( XX, p.X, YY, p.Y );
  FE_FENCE();
  fe_add( s, p.X, p.Y );
  fe_sq2( ZZ, p.Z, AA, s );
  FE_FENCE();
  fe_add_r( H, YY, XX );
  fe_sub( G, YY, XX );
  fe_sub( E, AA, H );
  fe_add( s, ZZ, ZZ ); fe_add( s, s, XX );
  fe_sub( Fn, s, YY );
  fe_mul2( r.X, Fn, E, r.Y, H, G );
  FE_FENCE();
  if( want_t ) fe_mul2( r.Z, Fn, G, r.T, H, E );
  else fe_mul( r.Z, Fn, G );
  FE_FENCE();
}

__device__ __forceinline__ void ge_add_cached_il( ge_p3 & r, ge_p3 const & p, ge_cached const & q, bool want_t ) {
  fe a, b, PP, MM, TT, D, E, F, G, H;
  fe_add( a, p.Y, p.X );
  fe_sub( b, p.Y, p.X );
  fe_mul2( PP, a, q.YpX, MM, b, q.YmX );
  FE_FENCE();
  fe_mul2( TT, p.T, q.T2d, D, p.Z, q.Z2 );
  FE_FENCE();
  fe_sub( E, PP, MM );
  fe_add( H, PP, MM );
  fe_add( G, D, TT );
  fe_sub( F, D, TT );
  fe_mul2( r.X, E, F, r.Y, G, H );
  FE_FENCE();
  if( want_t ) fe_mul2( r.Z, G, F, r.T, E, H );
  else fe_mul( r.Z, G, F );
  FE_FENCE();
}

#define INIT_P( p ) for (int i = 0; i < 10; i++) { p.X.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; \
  p.Y.v[i] = (i * 31u + threadIdx.x) & 0x1ffffffu; p.Z.v[i] = i == 0; p.T.v[i] = (i * 7u) & 0x1ffffu; }
#define INIT_Q( q ) for (int i = 0; i < 10; i++) { q.YpX.v[i] = (threadIdx.x * 3u + i * 99u) & 0x1ffffffu; \
  q.YmX.v[i] = (i * 5u + 1u) & 0x1ffffffu; q.T2d.v[i] = (threadIdx.x + i) & 0x1ffffffu; q.Z2.v[i] = i == 0 ? 2u : 0u; }
#define TIMED( body ) \
  uint64_t t0 = __builtin_amdgcn_s_memtime(); \
  _Pragma("unroll 1") for (int it = 0; it < iters; it++) { body; } \
  uint64_t t1 = __builtin_amdgcn_s_memtime(); \
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));

__global__ void __launch_bounds__(256, WPE) k_dbl(uint32_t* out, unsigned long long* cyc, int iters) {
  ge_p3 p; INIT_P( p );
  TIMED( ge_dbl( p, p, false ); ge_dbl( p, p, false ); ge_dbl( p, p, false ); ge_dbl( p, p, true ) )
  if (p.X.v[0] == 0x12345678u) out[threadIdx.x] = p.Y.v[1] + p.T.v[2];
}
__global__ void __launch_bounds__(256, WPE) k_dbl_il(uint32_t* out, unsigned long long* cyc, int iters) {
  ge_p3 p; INIT_P( p );
  TIMED( ge_dbl_il( p, p, false ); ge_dbl_il( p, p, false ); ge_dbl_il( p, p, false ); ge_dbl_il( p, p, true ) )
  if (p.X.v[0] == 0x12345678u) out[threadIdx.x] = p.Y.v[1] + p.T.v[2];
}
__global__ void __launch_bounds__(256, WPE) k_add(uint32_t* out, unsigned long long* cyc, int iters) {
  ge_p3 p; INIT_P( p ); ge_cached q; INIT_Q( q );
  TIMED( ge_add_cached( p, p, q, true ); ge_add_cached( p, p, q, false ); q.YpX.v[0] ^= p.X.v[3] & 1u; p.T = p.X )
  if (p.X.v[0] == 0x12345678u) out[threadIdx.x] = p.Y.v[1] + p.T.v[2];
}
__global__ void __launch_bounds__(256, WPE) k_add_il(uint32_t* out, unsigned long long* cyc, int iters) {
  ge_p3 p; INIT_P( p ); ge_cached q; INIT_Q( q );
  TIMED( ge_add_cached_il( p, p, q, true ); ge_add_cached_il( p, p, q, false ); q.YpX.v[0] ^= p.X.v[3] & 1u; p.T = p.X )
  if (p.X.v[0] == 0x12345678u) out[threadIdx.x] = p.Y.v[1] + p.T.v[2];
}
__global__ void __launch_bounds__(256, WPE) k_sqchain(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a, b; for (int i = 0; i < 10; i++) { a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; b.v[i] = (threadIdx.x * 5u + i) & 0x1ffffffu; }
  TIMED( fe_sq( a, a ); fe_sq( a, a ); fe_sq( b, b ); fe_sq( b, b ) )
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1] + b.v[1];
}
__global__ void __launch_bounds__(256, WPE) k_sqchain2(uint32_t* out, unsigned long long* cyc, int iters) {
  fe a, b; for (int i = 0; i < 10; i++) { a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu; b.v[i] = (threadIdx.x * 5u + i) & 0x1ffffffu; }
  TIMED( fe_sq2( a, a, b, b ); fe_sq2( a, a, b, b ) )
  if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1] + b.v[1];
}

/* the same doubling loop with only lanes 0..ACT-1 of each wave active (EXEC
   upper bits clear for the whole loop): does a half-empty wave64 issue in
   one 32-lane pass on gfx950's SIMD32? */
template<int ACT>
__global__ void __launch_bounds__(256, WPE) k_dbl_part(uint32_t* out, unsigned long long* cyc, int iters) {
  if ((int)(threadIdx.x & 63) >= ACT) return;
  ge_p3 p; INIT_P( p );
  TIMED( ge_dbl( p, p, false ); ge_dbl( p, p, false ); ge_dbl( p, p, false ); ge_dbl( p, p, true ) )
  if (p.X.v[0] == 0x12345678u) out[threadIdx.x] = p.Y.v[1] + p.T.v[2];
}

/* Co-running roles on one SIMD (the pipelined-kernel question): a block of
   4*NW waves; waves 0-3 (one per SIMD) run the doubling loop (the chain) at
   priority PRIO, waves 4.. run the squaring loop (the decode).  cyc[0] sums
   the chain waves' cycles per dbl, cyc[1] the others' per sq. */
template<int NW, int PRIO>
__global__ void __launch_bounds__(256 * NW, 1) k_mix(uint32_t* out, unsigned long long* cyc, int iters) {
  int w = threadIdx.x >> 6;
  if (w < 4) {
    if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
    ge_p3 p; INIT_P( p );
    uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < iters; it++) { ge_dbl( p, p, false ); ge_dbl( p, p, false ); ge_dbl( p, p, false ); ge_dbl( p, p, true ); }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) atomicAdd(&cyc[0], (unsigned long long)(t1 - t0));
    if (p.X.v[0] == 0x12345678u) out[threadIdx.x] = p.Y.v[1] + p.T.v[2];
  } else {
    fe a; for (int i = 0; i < 10; i++) a.v[i] = (threadIdx.x * 77u + i * 1313u) & 0x1ffffffu;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    int n = iters * 40;   /* about as long as the chain waves' loop alone */
#pragma unroll 1
    for (int it = 0; it < n; it++) { fe_sq( a, a ); }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) atomicAdd(&cyc[1], (unsigned long long)(t1 - t0));
    if (a.v[0] == 0x12345678u) out[threadIdx.x] = a.v[1];
  }
}

int run_mix(const char* name, void (*f)(uint32_t*, unsigned long long*, int), int nw, int iters) {
  uint32_t* d; unsigned long long* c; CHECK(hipMalloc(&d, 1 << 16)); CHECK(hipMalloc(&c, 16));
  for (int rep = 0; rep < 2; rep++) { CHECK(hipMemset(c, 0, 16)); hipLaunchKernelGGL(f, dim3(256), dim3(256 * nw), 0, 0, d, c, iters); CHECK(hipDeviceSynchronize()); }
  unsigned long long h[2]; CHECK(hipMemcpy(h, c, 16, hipMemcpyDeviceToHost));
  double dbl = (double)h[0] / (256 * 4.0) / (iters * 4.0);
  double sq = nw > 1 ? (double)h[1] / (256 * 4.0 * (nw - 1)) / (iters * 40.0) : 0.0;
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"chain_cyc_per_dbl\": %.1f, \"other_cyc_per_sq\": %.1f}\n", name, nw, dbl, sq);
  CHECK(hipFree(d)); CHECK(hipFree(c)); return 0;
}

typedef void (*kfn)(uint32_t*, unsigned long long*, int);
int run(const char* name, kfn f, int iters, double per) {
  uint32_t* d; unsigned long long* c; CHECK(hipMalloc(&d, 4096)); CHECK(hipMalloc(&c, 8));
  int blocks = 256 * WPE;     // WPE waves per SIMD
  for (int rep = 0; rep < 2; rep++) { CHECK(hipMemset(c, 0, 8)); hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, c, iters); CHECK(hipDeviceSynchronize()); }
  unsigned long long h; CHECK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cyc_per_op_per_wave\": %.1f}\n", name, WPE, (double)h / (blocks * 4.0) / (iters * per));
  CHECK(hipFree(d)); CHECK(hipFree(c)); return 0;
}
int main(int argc, char** argv) {
  if (argc > 1) {
    run_mix("chain alone", k_mix<1, 0>, 1, 100);
    run_mix("chain + 1 sq wave, prio 0", k_mix<2, 0>, 2, 100);
    run_mix("chain + 1 sq wave, chain prio 3", k_mix<2, 3>, 2, 100);
    run_mix("chain + 2 sq waves, chain prio 3", k_mix<3, 3>, 3, 100);
    run_mix("chain + 3 sq waves, chain prio 3", k_mix<4, 3>, 4, 100);
    run_mix("chain + 3 sq waves, prio 0", k_mix<4, 0>, 4, 100);
    return 0;
  }
  run("ge_dbl x4 (3 no-T + 1 T), per dbl", k_dbl, 200, 4.0);
  run("ge_dbl interleaved, per dbl", k_dbl_il, 200, 4.0);
  run("ge_dbl, 32 of 64 lanes active, per dbl", k_dbl_part<32>, 200, 4.0);
  run("ge_dbl, 16 of 64 lanes active, per dbl", k_dbl_part<16>, 200, 4.0);
  run("ge_add_cached (T + no-T), per add", k_add, 400, 2.0);
  run("ge_add_cached interleaved, per add", k_add_il, 400, 2.0);
  run("fe_sq chains a,b alone, per sq", k_sqchain, 1000, 4.0);
  run("fe_sq2 chains a,b together, per sq", k_sqchain2, 1000, 4.0);
  return 0;
}
