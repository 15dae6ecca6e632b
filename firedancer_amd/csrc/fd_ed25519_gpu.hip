/* fd_ed25519_gpu.hip -- MI355X (gfx950) Ed25519 batch verifier: kernels and
   the C ABI declared in include/fd_ed25519_gpu.h.

   One signature per lane.  The verify kernel does, per lane:
     S < l check -> decode A, R (sqrt-ratio ladder) -> small-order checks ->
     SHA-512(R || A || M) with M streamed from HBM -> reduce mod l ->
     signed fixed-window recoding of k (4-bit) and S (8-bit) ->
     table of [0..8](-A) in a per-lane HBM/L2 scratch -> joint double-scalar
     multiplication [k](-A) + [S]B with the [0..128]B affine table in LDS ->
     projective compare against R.
   Semantics follow fd_ed25519_verify (src/ballet/ed25519/fd_ed25519_user.c:
   134-229) with the FD_HAS_AVX512 error mapping (SURVEY.md §8(a) A-spec).

   Host side: a context owns, per device, a stream, the B table, descriptor /
   arena / code staging buffers and the A-table scratch.  Batches are sharded
   contiguously over the context's devices; no collective is needed (every
   signature is independent). */

#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#include "../../include/fd_ed25519_gpu.h"
#include "fd_f25519_dev.h"
#include "fd_curve25519_dev.h"
#include "fd_sha512_dev.h"
#include "fd_scalar_dev.h"
#include "fd_lattice_dev.h"

#define FD_VERIFY_BLOCK   256          /* threads per workgroup: 4 waves              */
#ifndef FD_VERIFY_WAVES_PER_EU
#define FD_VERIFY_WAVES_PER_EU 2       /* -> <= 256 VGPR+AGPR per lane                */
#endif
#define FD_BTAB_N         129          /* [0..128]P                                   */
#define FD_BTAB_STRIDE    32           /* u32 per entry: 3 x 10 limbs + pad           */
#define FD_BTAB_WORDS     (2 * FD_BTAB_N * FD_BTAB_STRIDE)   /* P = B and P = 2^128 B */
#define FD_BTAB_LOADS     ((FD_BTAB_WORDS/4 + FD_VERIFY_BLOCK - 1) / FD_VERIFY_BLOCK)   /* uint4 per thread */
#define FD_BTAB_ALLOC     (FD_BTAB_LOADS * FD_VERIFY_BLOCK * 4)                       /* padded u32 */
#define FD_VTAB_N         9            /* [0..8](-Q), Q = A or R                      */
#define FD_VTAB_WORDS     40           /* u32 per entry (4 fe)                        */
#define FD_NDIG_MAX       64           /* 4-bit windows of a <= 256-bit scalar        */

/* LDS digit rows ([row][slot] bytes) */
#define FD_ROW_U          0            /* signed 4-bit digits of u (sign folded in)   */
#define FD_ROW_V          64           /* signed 4-bit digits of v                    */
#define FD_ROW_W          128          /* signed 8-bit digits of w = v S mod l (32)   */
#define FD_ROW_NW         160          /* lane 0 of each wave: the wave's window count */
#define FD_ROWS           161

/* Diagnostic build only (-DFD_PHASE_STAMPS, tools/Makefile): s_memtime at
   phase boundaries, per-wave deltas summed into args.stamps.  The product
   build compiles none of it. */
#ifdef FD_PHASE_STAMPS
#define FD_NSTAMP 8
#define STAMP( i ) do { FE_FENCE(); _st[ i ] = __builtin_amdgcn_s_memtime(); FE_FENCE(); } while( 0 )
#else
#define STAMP( i ) do {} while( 0 )
#endif

/* ------------------------------------------------------------------ loads */

/* n little-endian words starting at an arbitrary byte offset off (read
   through aligned dwords, clamped to the readable arena). */
template<int N>
__device__ __forceinline__ void load_words( uint32_t out[ N ], uint8_t const * arena, uint32_t off, uint32_t lim_dw ) {
  uint32_t const * a32 = (uint32_t const *)arena;
  uint32_t dw = off >> 2, sh = off & 3u;
  uint32_t prev = a32[ min( dw, lim_dw ) ];
#pragma unroll
  for( int i=0; i<N; i++ ) {
    uint32_t nxt = a32[ min( dw+1u+(uint32_t)i, lim_dw ) ];
    out[i] = __builtin_amdgcn_alignbyte( nxt, prev, sh );
    prev = nxt;
  }
}

/* ------------------------------------------------------------------ B tables */

__device__ void ge_affine_precomp( ge_precomp & q, ge_p3 & p ) {
  fe zi, x, y, xy, d2;
  fe_invert( zi, p.Z );
  fe_mul( x, p.X, zi ); fe_mul( y, p.Y, zi );
  fe_const_d2( d2 );
  fe_add_r( q.YpX, y, x ); fe_sub_r( q.YmX, y, x ); fe_mul( xy, x, y ); fe_mul( q.T2d, xy, d2 );
  p.X = x; p.Y = y; fe_set1( p.Z ); p.T = xy;
}

/* Device init: thread (t, i) computes [i]P_t, P_0 = B, P_1 = 2^128 B, and
   stores its affine precomputed form (Y+X, Y-X, 2dXY) at
   btab[(t*FD_BTAB_N + i)*FD_BTAB_STRIDE ...].  B decoded from its standard
   encoding (y = 4/5, x even). */
__global__ void fd_ed25519_btab_init( uint32_t * btab ) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if( g >= 2*FD_BTAB_N ) return;
  int t = g / FD_BTAB_N, i = g % FD_BTAB_N;
  uint32_t benc[ 8 ];
  benc[0] = 0x66666658u;
#pragma unroll
  for( int j=1; j<8; j++ ) benc[j] = 0x66666666u;
  ge_p3 B; ge_decode( B, benc, true );
  if( t ) {
    for( int j=0; j<128; j++ ) ge_dbl( B, B, true );
  }
  ge_precomp Bp; ge_affine_precomp( Bp, B );
  ge_p3 acc; ge_identity( acc );
  for( int bit=7; bit>=0; bit-- ) {
    ge_dbl( acc, acc, true );
    if( (i >> bit) & 1 ) ge_madd( acc, acc, Bp, true );
  }
  ge_precomp o; ge_affine_precomp( o, acc );
  uint32_t * e = btab + g * FD_BTAB_STRIDE;
  for( int j=0; j<10; j++ ) { e[j] = o.YpX.v[j]; e[10+j] = o.YmX.v[j]; e[20+j] = o.T2d.v[j]; }
  e[30] = 0u; e[31] = 0u;
}

/* ------------------------------------------------------------------ verify */

struct verify_args {
  uint8_t const *           arena;
  uint64_t                  arena_sz;
  fd_ed25519_desc_t const * desc;
  uint64_t                  n;
  int8_t *                  out;
  uint32_t const *          btab;      /* FD_BTAB_WORDS u32                        */
  uint32_t *                vtab;      /* FD_VTAB_N * FD_VTAB_WORDS * vtab_cap u32 */
  uint64_t                  vtab_cap;  /* tables                                   */
  int                       ref_codes;
  unsigned long long *      stamps;    /* FD_PHASE_STAMPS builds only: per-phase cycle sums */
};

/* Raw message dwords of SHA block b: dword (msg_off>>2) + 32b - 16 + i,
   i < 33, clamped to the readable arena (block 0's first 16 are unused:
   R || A come from registers). */
__device__ __forceinline__ void sha_fetch( uint32_t raw[ 33 ], uint32_t const * a32, uint32_t msg_off, uint32_t b,
                                           uint32_t lim_dw ) {
  int32_t start = (int32_t)(msg_off >> 2) + 32*(int32_t)b - 16;
#pragma unroll
  for( int i=0; i<33; i++ ) raw[i] = a32[ min( (uint32_t)max( start + i, 0 ), lim_dw ) ];
}

/* SHA-512(R || A || M) mod l.  R, A: 8 LE words each; the message is
   streamed from HBM, each block's dwords fetched one block ahead so the
   load latency hides behind the previous compression. */
__device__ __forceinline__ void hash_ram( uint32_t k[ 8 ], uint32_t const Rw[ 8 ], uint32_t const Aw[ 8 ],
                                          uint8_t const * arena, uint32_t msg_off, uint32_t msg_sz, uint32_t lim_dw ) {
  uint64_t h[ 8 ]; sha512_init_state( h );
  uint32_t total = 64u + msg_sz;
  uint32_t nblk = (total + 17u + 127u) >> 7;
  uint32_t const * a32 = (uint32_t const *)arena;
  uint32_t sh = msg_off & 3u;
  uint32_t nxt[ 33 ];
  sha_fetch( nxt, a32, msg_off, 0u, lim_dw );
  for( uint32_t b=0; b<nblk; b++ ) {
    uint32_t raw[ 33 ];
#pragma unroll
    for( int i=0; i<33; i++ ) raw[i] = nxt[i];
    if( b + 1u < nblk ) sha_fetch( nxt, a32, msg_off, b + 1u, lim_dw );
    uint64_t W[ 16 ];
#pragma unroll
    for( int j=0; j<16; j++ ) {
      uint32_t hi, lo;                                  /* big-endian halves */
      if( b == 0 && j < 8 ) {
        uint32_t const * src = (j < 4) ? Rw : Aw;
        int jj = j & 3;
        hi = sha_bswap32( src[2*jj] ); lo = sha_bswap32( src[2*jj+1] );
      } else {
        int32_t m = (int32_t)((b << 7) + 8u*(uint32_t)j) - 64;     /* message byte index of the word's first byte */
        uint32_t w0 = __builtin_amdgcn_alignbyte( raw[2*j+1], raw[2*j],   sh );   /* bytes m..m+3 LE */
        uint32_t w1 = __builtin_amdgcn_alignbyte( raw[2*j+2], raw[2*j+1], sh );   /* bytes m+4..m+7  */
        hi = sha_bswap32( w0 ); lo = sha_bswap32( w1 );
        /* padding: keep bytes < msg_sz, 0x80 at msg_sz, zeros after */
        int32_t rem0 = (int32_t)msg_sz - m;             /* valid bytes from m   */
        int32_t rem1 = rem0 - 4;
        uint32_t keep0 = rem0 >= 4 ? 0xffffffffu : (rem0 <= 0 ? 0u : ~(0xffffffffu >> (8*rem0)));
        uint32_t keep1 = rem1 >= 4 ? 0xffffffffu : (rem1 <= 0 ? 0u : ~(0xffffffffu >> (8*rem1)));
        uint32_t pad0  = (rem0 >= 0 && rem0 < 4) ? (0x80000000u >> (8*rem0)) : 0u;
        uint32_t pad1  = (rem1 >= 0 && rem1 < 4) ? (0x80000000u >> (8*rem1)) : 0u;
        hi = (hi & keep0) | pad0;
        lo = (lo & keep1) | pad1;
        if( b == nblk-1u && j == 15 ) { hi = total >> 29; lo = total << 3; }
        if( b == nblk-1u && j == 14 ) { hi = 0u; lo = 0u; }
      }
      W[j] = ((uint64_t)hi << 32) | lo;
    }
    sha512_compress( h, W );
  }
  uint32_t dg[ 16 ];
#pragma unroll
  for( int i=0; i<8; i++ ) { dg[2*i] = sha_bswap32( (uint32_t)(h[i] >> 32) ); dg[2*i+1] = sha_bswap32( (uint32_t)h[i] ); }
  sc_reduce512( k, dg );
}

/* Variable-base table layout: entry e of thread t = 40 words (Y+X, Y-X,
   2dT, 2Z; 10 limbs each) split into a 128-byte record main[e][t][32] (one
   cache line, read with 8 x 16-B loads) and a 32-byte record tail[e][t][8]
   (4 threads per line), so a thread's entry is fetched with no over-read
   whatever entry its digit selects. */
__device__ __forceinline__ void vtab_ptrs( uint32_t const * vtab, uint64_t cap, uint64_t t, uint32_t e,
                                           uint4 const ** m, uint4 const ** tl ) {
  uint64_t idx = (uint64_t)e * cap + t;
  *m  = (uint4 const *)(vtab + idx * 32u);
  *tl = (uint4 const *)(vtab + (uint64_t)FD_VTAB_N * cap * 32u + idx * 8u);
}

__device__ __forceinline__ void vtab_store( uint32_t * vtab, uint64_t cap, uint64_t t, int e, ge_cached const & c ) {
  uint32_t w[ 40 ];
#pragma unroll
  for( int j=0; j<10; j++ ) { w[j] = c.YpX.v[j]; w[10+j] = c.YmX.v[j]; w[20+j] = c.T2d.v[j]; w[30+j] = c.Z2.v[j]; }
  uint4 const * mc; uint4 const * tc;
  vtab_ptrs( vtab, cap, t, (uint32_t)e, &mc, &tc );
  uint4 * m = (uint4 *)mc; uint4 * tl = (uint4 *)tc;
#pragma unroll
  for( int j=0; j<8; j++ ) m[j] = make_uint4( w[4*j], w[4*j+1], w[4*j+2], w[4*j+3] );
#pragma unroll
  for( int j=0; j<2; j++ ) tl[j] = make_uint4( w[32+4*j], w[33+4*j], w[34+4*j], w[35+4*j] );
}

/* Table [0..8](-Q) for an affine Q (Z = 1), cached form (replaces the
   reference's -A table of fd_ed25519_double_scalar_mul_base,
   fd_curve25519.c:136-144, and the neg of fd_ed25519_user.c:215). */
__device__ __forceinline__ void vtab_build( uint32_t * vtab, uint64_t cap, uint64_t t, ge_p3 const & Q ) {
  ge_p3 nQ = Q;
  { fe x; fe_neg( x, Q.X ); fe_carry( nQ.X, x ); fe_neg( x, Q.T ); fe_carry( nQ.T, x ); }
  ge_cached c;
  ge_p3 id; ge_identity( id );
  ge_to_cached( c, id );  vtab_store( vtab, cap, t, 0, c );
  ge_to_cached( c, nQ );  vtab_store( vtab, cap, t, 1, c );
  ge_precomp nQp;
  { fe d2; fe_const_d2( d2 ); fe_add_r( nQp.YpX, nQ.Y, nQ.X ); fe_sub_r( nQp.YmX, nQ.Y, nQ.X ); fe_mul( nQp.T2d, nQ.T, d2 ); }
  FE_FENCE();
  ge_p3 P;
  ge_dbl( P, nQ, true ); ge_to_cached( c, P ); vtab_store( vtab, cap, t, 2, c );
#pragma unroll 1
  for( int e=3; e<=8; e++ ) { ge_madd( P, P, nQp, true ); ge_to_cached( c, P ); vtab_store( vtab, cap, t, e, c ); FE_FENCE(); }
}

/* Issue the loads of entry |d| (biased digit db = d + 8) into raw words;
   vtab_finish (at the use point) applies the sign. */
__device__ __forceinline__ void vtab_fetch( uint32_t w[ 40 ], uint32_t const * vtab, uint64_t cap, uint64_t t, uint32_t db ) {
  uint32_t e = min( db < 8u ? 8u - db : db - 8u, 8u );
  uint4 const * m; uint4 const * tl;
  vtab_ptrs( vtab, cap, t, e, &m, &tl );
#pragma unroll
  for( int j=0; j<8; j++ ) { uint4 v = m[j]; w[4*j] = v.x; w[4*j+1] = v.y; w[4*j+2] = v.z; w[4*j+3] = v.w; }
#pragma unroll
  for( int j=0; j<2; j++ ) { uint4 v = tl[j]; w[32+4*j] = v.x; w[33+4*j] = v.y; w[34+4*j] = v.z; w[35+4*j] = v.w; }
}

__device__ __forceinline__ void vtab_finish( ge_cached & c, uint32_t const w[ 40 ], uint32_t db ) {
  bool neg = db < 8u;
  fe tv, tn;
#pragma unroll
  for( int j=0; j<10; j++ ) { tv.v[j] = w[20+j]; c.Z2.v[j] = w[30+j]; }
  fe_neg( tn, tv );
#pragma unroll
  for( int j=0; j<10; j++ ) {
    c.YpX.v[j] = neg ? w[10+j] : w[j];
    c.YmX.v[j] = neg ? w[j]    : w[10+j];
    c.T2d.v[j] = neg ? tn.v[j] : tv.v[j];
  }
}

__device__ __forceinline__ void btab_load( ge_precomp & q, uint32_t const * lds_btab, uint32_t db ) {
  bool neg = db < 128u;
  uint32_t e = neg ? 128u - db : db - 128u;
  uint4 const * p = (uint4 const *)(lds_btab + e * FD_BTAB_STRIDE);
  uint32_t w[ 32 ];
#pragma unroll
  for( int j=0; j<8; j++ ) { uint4 v = p[j]; w[4*j] = v.x; w[4*j+1] = v.y; w[4*j+2] = v.z; w[4*j+3] = v.w; }
  fe t, tn;
#pragma unroll
  for( int j=0; j<10; j++ ) t.v[j] = w[20+j];
  fe_neg( tn, t );
#pragma unroll
  for( int j=0; j<10; j++ ) {
    q.YpX.v[j] = neg ? w[10+j] : w[j];
    q.YmX.v[j] = neg ? w[j]    : w[10+j];
    q.T2d.v[j] = neg ? tn.v[j] : t.v[j];
  }
}

/* acc = [u](-A) + [v](-R) + [w_lo]B + [w_hi](2^128 B) over nw 4-bit windows
   (wave-uniform; one shared doubling chain -- Straus).  u / v digits from
   LDS rows (biased by 8, sign of u folded in), w digits (biased by 128)
   at every other window.  Table entries are fetched one step ahead: A's for
   the next window before the doublings, R's before A's addition. */
__device__ __forceinline__ void dsm_loop( ge_p3 & acc, uint32_t const * vtab, uint64_t cap, uint64_t ta, uint64_t tr,
                                          uint8_t const * dig, uint32_t const * lds_bt, int nw ) {
  ge_identity( acc );
  uint32_t raw[ 40 ];
  uint32_t dba = dig[ (FD_ROW_U + nw-1)*FD_VERIFY_BLOCK ];
  vtab_fetch( raw, vtab, cap, ta, dba );
#pragma unroll 1
  for( int i=nw-1; i>=0; i-- ) {
    if( i < nw-1 ) {
#pragma unroll 1
      for( int j=0; j<4; j++ ) { ge_dbl( acc, acc, j == 3 ); FE_FENCE(); }
    }
    bool bq = ((i & 1) == 0) && (i <= 30);
    ge_cached q;
    vtab_finish( q, raw, dba );
    uint32_t dbr = dig[ (FD_ROW_V + i)*FD_VERIFY_BLOCK ];
    vtab_fetch( raw, vtab, cap, tr, dbr );
    FE_FENCE();
    ge_add_cached( acc, acc, q, true );
    FE_FENCE();
    vtab_finish( q, raw, dbr );
    if( i > 0 ) { dba = dig[ (FD_ROW_U + i-1)*FD_VERIFY_BLOCK ]; vtab_fetch( raw, vtab, cap, ta, dba ); }
    FE_FENCE();
    ge_add_cached( acc, acc, q, bq );
    FE_FENCE();
    if( bq ) {
      ge_precomp bp;
      btab_load( bp, lds_bt, dig[ (FD_ROW_W + (i>>1))*FD_VERIFY_BLOCK ] );
      FE_FENCE();
      ge_madd( acc, acc, bp, true );
      FE_FENCE();
      btab_load( bp, lds_bt + FD_BTAB_N*FD_BTAB_STRIDE, dig[ (FD_ROW_W + 16 + (i>>1))*FD_VERIFY_BLOCK ] );
      FE_FENCE();
      ge_madd( acc, acc, bp, false );
      FE_FENCE();
    }
  }
}

__device__ __forceinline__ int bitlen8( uint32_t const x[ 8 ] ) {
  int b = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) b = x[j] ? 32*j + 32 - __clz( (int)x[j] ) : b;
  return b;
}

/* Signed 4-bit recoding of x (< 2^(4 nw - 1)) into nw LDS rows (biased by 8,
   negated when neg): digits in [-8, 7] below the top one, top digit in
   [0, 8] (its top nibble <= 7 plus the incoming carry, never wrapped). */
__device__ __forceinline__ void recode4_lds( uint8_t * row, uint32_t const x[ 8 ], int neg, int nw ) {
  int c = 0;
#pragma unroll
  for( int i=0; i<FD_NDIG_MAX; i++ ) {
    if( i < nw ) {
      int d = (int)((x[i>>3] >> (4*(i&7))) & 15u) + c;
      c = d >= 8 && i < nw-1;           /* the top digit keeps its carry: d in [0, 8] */
      d -= c << 4;
      row[ i*FD_VERIFY_BLOCK ] = (uint8_t)((neg ? -d : d) + 8);
    }
  }
}

/* One signature per lane:
     S check -> k = SHA-512(R||A||M) mod l -> (u, v) short vector of k mod 8l,
     w = v S mod l, digits -> LDS -> decode A and R, small-order checks,
     tables [0..8](-A), [0..8](-R) -> Q = [u](-A) + [v](-R) + [w]B -> Q == O
   (Q = [v]([S]B - [k]A - R), fd_lattice_dev.h).  The reported code follows
   the reference's check order (fd_ed25519_user.c:157-228): S, decode A,
   decode R, small-order A, small-order R, equation. */
__global__ void __launch_bounds__( FD_VERIFY_BLOCK, FD_VERIFY_WAVES_PER_EU )
fd_ed25519_verify_kernel( verify_args args ) {
  __shared__ uint4    s_btab4[ FD_BTAB_WORDS / 4 ];
  __shared__ uint8_t  s_dig[ FD_ROWS * FD_VERIFY_BLOCK ];

  int tid = (int)threadIdx.x;
#ifdef FD_PHASE_STAMPS
  uint64_t _st[ FD_NSTAMP ] = { 0, 0, 0, 0, 0, 0, 0, 0 };
#endif
  STAMP( 0 );
  uint64_t gid = (uint64_t)blockIdx.x * FD_VERIFY_BLOCK + (uint64_t)tid;
  uint64_t cap = args.vtab_cap;
  uint32_t const * s_btab = (uint32_t const *)s_btab4;
  /* Every lane stays to the wave-wide window count below (no early exit):
     lanes past n or with a bad descriptor take the no-work path.  The
     descriptor / signature / key loads are issued before the B-table copy
     so their latency overlaps it. */
  bool valid = gid < args.n;
  fd_ed25519_desc_t d; d.sig_off = 0u; d.pub_off = 0u; d.msg_off = 0u; d.msg_sz = 0u; d.txn_idx = 0u;
  if( valid ) d = args.desc[ gid ];
  uint64_t asz = args.arena_sz;
  bool desc_ok = valid && (uint64_t)d.sig_off + 64u <= asz && (uint64_t)d.pub_off + 32u <= asz &&
                 (uint64_t)d.msg_off + d.msg_sz <= asz;
  uint32_t lim_dw = (uint32_t)((asz + 3u) >> 2) + 1u;   /* last readable dword (arena padded by 8 bytes) */

  uint32_t sig[ 16 ], pub[ 8 ];
#pragma unroll
  for( int j=0; j<16; j++ ) sig[j] = 0u;
#pragma unroll
  for( int j=0; j<8; j++ ) pub[j] = 0u;
  if( desc_ok ) {
    load_words<16>( sig, args.arena, d.sig_off, lim_dw );
    load_words<8> ( pub, args.arena, d.pub_off, lim_dw );
  }

  {
    /* all of this thread's table loads in flight at once (the device copy is
       padded to FD_BTAB_LOADS full rounds), then the LDS stores */
    uint4 const * g = (uint4 const *)args.btab;
    uint4 t[ FD_BTAB_LOADS ];
#pragma unroll
    for( int r=0; r<FD_BTAB_LOADS; r++ ) t[r] = g[ tid + r*FD_VERIFY_BLOCK ];
#pragma unroll
    for( int r=0; r<FD_BTAB_LOADS; r++ ) {
      int i = tid + r*FD_VERIFY_BLOCK;
      if( r < FD_BTAB_LOADS-1 || i < FD_BTAB_WORDS/4 ) s_btab4[i] = t[r];
    }
  }
  __syncthreads();
  STAMP( 1 );

  bool bad_s = desc_ok && !sc_lt_l( sig + 8 );                           /* :157-159 */
  bool live  = desc_ok && !bad_s;

  /* k, lattice vector, w and digits (before the decodes: only digits stay live) */
  uint8_t * drow = s_dig + tid;
  {
    uint32_t u[ 8 ], v[ 8 ];
    int un = 0, nbits = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = 0u; v[j] = 0u; }
    if( live ) {
      uint32_t k[ 8 ];
      hash_ram( k, sig, pub, args.arena, d.msg_off, d.msg_sz, lim_dw );  /* :203-206 */
      FE_FENCE();
      STAMP( 2 );
      lat_short_vector( k, u, v, &un );
      FE_FENCE();
      uint32_t pr[ 16 ];                                                 /* w = v S mod l */
#pragma unroll
      for( int j=0; j<16; j++ ) pr[j] = 0u;
#pragma unroll
      for( int i=0; i<8; i++ ) {
        uint64_t c = 0;
#pragma unroll
        for( int j=0; j<8; j++ ) { uint64_t t = (uint64_t)v[i] * sig[8+j] + pr[i+j] + c; pr[i+j] = (uint32_t)t; c = t >> 32; }
        pr[i+8] = (uint32_t)c;
      }
      uint32_t w[ 8 ];
      sc_reduce512( w, pr );
      uint8_t ds[ 32 ];
      sc_recode_w8( ds, w );
#pragma unroll
      for( int i=0; i<32; i++ ) drow[ (FD_ROW_W + i)*FD_VERIFY_BLOCK ] = ds[i];
      nbits = max( bitlen8( u ), bitlen8( v ) );
    }
    /* wave-uniform window count: x < 2^(4 nw - 1) for every lane's u, v */
#pragma unroll
    for( int o=32; o>=1; o>>=1 ) nbits = max( nbits, __shfl_xor( nbits, o ) );
    int nw = min( FD_NDIG_MAX, max( 32, (nbits + 4) >> 2 ) );
    recode4_lds( drow + FD_ROW_U*FD_VERIFY_BLOCK, u, un, nw );
    recode4_lds( drow + FD_ROW_V*FD_VERIFY_BLOCK, v, 0,  nw );
    if( (tid & 63) == 0 ) drow[ FD_ROW_NW*FD_VERIFY_BLOCK ] = (uint8_t)nw;
  }
  FE_FENCE();

  /* decode A then R (:162 frombytes_2x), small order (:193-198), tables */
  STAMP( 3 );
  int st[ 2 ] = { 0, 0 };
  if( live ) {
#pragma unroll 1
    for( int q=0; q<2; q++ ) {
      uint32_t enc[ 8 ];
#pragma unroll
      for( int j=0; j<8; j++ ) enc[j] = q ? sig[j] : pub[j];
      ge_p3 Q;
      int ok = ge_decode( Q, enc, !args.ref_codes );
      int sm = ge_affine_small_order( Q );
      FE_FENCE();
      if( ok && !sm ) vtab_build( args.vtab, cap, (uint64_t)q*cap/2u + gid, Q );
      int s = (ok ? 1 : 0) | (sm ? 2 : 0);
      if( q ) st[1] = s; else st[0] = s;
      FE_FENCE();
    }
  }
  int stA = st[0], stR = st[1];
  STAMP( 4 );

  if( !valid ) return;
  int code;
  if     ( !desc_ok    ) code = FD_ED25519_GPU_CODE_BAD_DESC;
  else if( bad_s       ) code = FD_ED25519_ERR_SIG;
  else if( !(stA & 1)  ) code = args.ref_codes ? FD_ED25519_ERR_PUBKEY : FD_ED25519_ERR_SIG;   /* :190-192 */
  else if( !(stR & 1)  ) code = FD_ED25519_ERR_SIG;
  else if( stA & 2     ) code = FD_ED25519_ERR_PUBKEY;                                        /* :193-195 */
  else if( stR & 2     ) code = FD_ED25519_ERR_SIG;                                           /* :196-198 */
  else                   code = 0;

  if( code == 0 ) {
    int nw = s_dig[ FD_ROW_NW*FD_VERIFY_BLOCK + (tid & ~63) ];
    ge_p3 acc;
    dsm_loop( acc, args.vtab, cap, gid, cap/2u + gid, drow, s_btab, nw );
    STAMP( 5 );
    /* Q == O  <=>  X == 0 and Y == Z (the reference's projective compare, :225-228, on [v]D) */
    fe dl;
    int ex = fe_is_zero( acc.X );
    fe_sub( dl, acc.Y, acc.Z ); fe_carry( dl, dl );
    int ey = fe_is_zero( dl );
    code = (ex & ey) ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  }
  args.out[ gid ] = (int8_t)code;
#ifdef FD_PHASE_STAMPS
  STAMP( 6 );
  if( args.stamps && (tid & 63) == 0 ) {
    /* 0-1 prologue+table copy, 1-2 SHA (live lanes), 2-3 lattice+digits, 3-4 decodes+tables, 4-5 loop, 5-6 tail */
    for( int i=0; i<6; i++ ) atomicAdd( &args.stamps[i], (unsigned long long)(_st[i+1] - _st[i]) );
    atomicAdd( &args.stamps[7], 1ull );
  }
#endif
}

/* Self-test kernel (tests only, fd_ed25519_gpu_test_lattice): the device
   lattice reduction on caller-supplied k, one per lane. */
__global__ void fd_ed25519_lattice_test_kernel( uint32_t const * k, uint32_t * out, uint64_t n ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t kk[ 8 ], u[ 8 ], v[ 8 ];
  int un = 0, it = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) { kk[j] = i < n ? k[ i*8u + (uint64_t)j ] : 0u; u[j] = 0u; v[j] = 0u; }
  if( i < n ) it = lat_short_vector( kk, u, v, &un );
  if( i < n ) {
    uint32_t * o = out + i*18u;
#pragma unroll
    for( int j=0; j<8; j++ ) { o[j] = u[j]; o[8+j] = v[j]; }
    o[16] = (uint32_t)un; o[17] = (uint32_t)it;
  }
}

/* ------------------------------------------------------------------ host side */

#define FD_MAX_DEV 16

struct fd_dev_state {
  int          dev;
  hipStream_t  stream;
  hipEvent_t   done;
  uint32_t *   btab;        /* device */
  uint32_t *   vtab;        /* device, FD_VTAB_N*FD_VTAB_WORDS*vtab_cap u32 */
  uint64_t     vtab_cap;    /* tables (2 per signature) */
  uint64_t     sig_cap;     /* signatures per launch     */
  unsigned long long * stamps; /* FD_PHASE_STAMPS builds only */
  uint8_t *    d_arena;  uint64_t arena_cap;
  fd_ed25519_desc_t * d_desc; uint64_t desc_cap;
  int8_t *     d_out;
  int          busy;
};

struct fd_ed25519_gpu {
  int          ndev;
  uint64_t     max_batch;
  int          ref_codes;
  fd_dev_state d[ FD_MAX_DEV ];
  /* pending async batch */
  int8_t *     pend_out;
  uint64_t     pend_cnt;
  int          pend_active;
};

#define HIPCK( x ) do { hipError_t _e = (x); if( _e != hipSuccess ) { \
    fprintf( stderr, "fd_ed25519_gpu: %s failed: %s (%s:%d)\n", #x, hipGetErrorString( _e ), __FILE__, __LINE__ ); \
    return FD_ED25519_GPU_ERR_LAUNCH; } } while( 0 )

static uint64_t align_up( uint64_t x, uint64_t a ) { return (x + a - 1u) / a * a; }

static int dev_reserve( fd_dev_state * s, uint64_t arena_sz, uint64_t cnt ) {
  HIPCK( hipSetDevice( s->dev ) );
  uint64_t need_arena = align_up( arena_sz, 4u ) + 16u;
  if( need_arena > s->arena_cap ) {
    if( s->d_arena ) HIPCK( hipFree( s->d_arena ) );
    s->arena_cap = align_up( need_arena * 5u / 4u, 1u << 20 );
    if( hipMalloc( &s->d_arena, s->arena_cap ) != hipSuccess ) { s->d_arena = NULL; s->arena_cap = 0; return FD_ED25519_GPU_ERR_OOM; }
  }
  if( cnt > s->desc_cap ) {
    if( s->d_desc ) HIPCK( hipFree( s->d_desc ) );
    if( s->d_out )  HIPCK( hipFree( s->d_out ) );
    s->desc_cap = align_up( cnt, 4096u );
    if( hipMalloc( &s->d_desc, s->desc_cap * sizeof(fd_ed25519_desc_t) ) != hipSuccess ||
        hipMalloc( &s->d_out, s->desc_cap ) != hipSuccess ) { s->desc_cap = 0; return FD_ED25519_GPU_ERR_OOM; }
  }
  return FD_ED25519_GPU_OK;
}

/* Enqueue kernels over [0, cnt) of device-resident descriptors, chunked to
   the A-table scratch capacity. */
static int dev_launch( fd_ed25519_gpu_t * ctx, fd_dev_state * s, uint8_t const * d_arena, uint64_t arena_sz,
                       fd_ed25519_desc_t const * d_desc, uint64_t cnt, int8_t * d_out, hipStream_t st ) {
  HIPCK( hipSetDevice( s->dev ) );
  for( uint64_t off=0; off<cnt; off+=s->sig_cap ) {
    uint64_t m = cnt - off < s->sig_cap ? cnt - off : s->sig_cap;
    verify_args a;
    a.arena = d_arena; a.arena_sz = arena_sz; a.desc = d_desc + off; a.n = m; a.out = d_out + off;
    a.btab = s->btab; a.vtab = s->vtab; a.vtab_cap = s->vtab_cap; a.ref_codes = ctx->ref_codes;
    a.stamps = s->stamps;
    uint32_t blocks = (uint32_t)((m + FD_VERIFY_BLOCK - 1u) / FD_VERIFY_BLOCK);
    hipLaunchKernelGGL( fd_ed25519_verify_kernel, dim3( blocks ), dim3( FD_VERIFY_BLOCK ), 0, st, a );
    HIPCK( hipGetLastError() );
  }
  return FD_ED25519_GPU_OK;
}

extern "C" {

fd_ed25519_gpu_t *
fd_ed25519_gpu_new( uint64_t device_mask, uint64_t max_batch ) {
  int cnt = 0;
  if( hipGetDeviceCount( &cnt ) != hipSuccess || cnt <= 0 ) return NULL;
  fd_ed25519_gpu_t * ctx = (fd_ed25519_gpu_t *)calloc( 1, sizeof(fd_ed25519_gpu_t) );
  if( !ctx ) return NULL;
  if( !max_batch ) max_batch = 1u << 18;
  ctx->max_batch = max_batch;
  if( !device_mask ) { int cur = 0; hipGetDevice( &cur ); device_mask = 1ull << cur; }
  for( int i=0; i<cnt && i<FD_MAX_DEV; i++ ) {
    if( !((device_mask >> i) & 1u) ) continue;
    fd_dev_state * s = &ctx->d[ ctx->ndev ];
    s->dev = i;
    if( hipSetDevice( i ) != hipSuccess ) goto fail;
    if( hipStreamCreateWithFlags( &s->stream, hipStreamNonBlocking ) != hipSuccess ) goto fail;
    if( hipEventCreateWithFlags( &s->done, hipEventDisableTiming ) != hipSuccess ) goto fail;
    if( hipMalloc( &s->btab, FD_BTAB_ALLOC * sizeof(uint32_t) ) != hipSuccess ) goto fail;
    if( hipMemsetAsync( s->btab, 0, FD_BTAB_ALLOC * sizeof(uint32_t), s->stream ) != hipSuccess ) goto fail;
    s->sig_cap  = align_up( max_batch, FD_VERIFY_BLOCK );
    s->vtab_cap = 2u * s->sig_cap;   /* tables of -A at [0, sig_cap), of -R at [sig_cap, 2 sig_cap) */
    if( hipMalloc( &s->vtab, (uint64_t)FD_VTAB_N * FD_VTAB_WORDS * s->vtab_cap * sizeof(uint32_t) ) != hipSuccess ) goto fail;
#ifdef FD_PHASE_STAMPS
    if( hipMalloc( &s->stamps, 8 * sizeof(unsigned long long) ) != hipSuccess ) goto fail;
    hipMemset( s->stamps, 0, 8 * sizeof(unsigned long long) );
#endif
    ctx->ndev++;
    hipLaunchKernelGGL( fd_ed25519_btab_init, dim3( (2*FD_BTAB_N + 63)/64 ), dim3( 64 ), 0, s->stream, s->btab );
    if( hipStreamSynchronize( s->stream ) != hipSuccess ) goto fail;
  }
  if( !ctx->ndev ) goto fail;
  return ctx;
fail:
  fd_ed25519_gpu_delete( ctx );
  return NULL;
}

void
fd_ed25519_gpu_delete( fd_ed25519_gpu_t * ctx ) {
  if( !ctx ) return;
  for( int i=0; i<FD_MAX_DEV; i++ ) {
    fd_dev_state * s = &ctx->d[i];
    if( !s->stream && !s->btab ) continue;
    hipSetDevice( s->dev );
    if( s->stream ) hipStreamSynchronize( s->stream );
    if( s->btab )    hipFree( s->btab );
    if( s->vtab )    hipFree( s->vtab );
#ifdef FD_PHASE_STAMPS
    if( s->stamps ) {
      unsigned long long h[ 8 ];
      if( hipMemcpy( h, s->stamps, sizeof(h), hipMemcpyDeviceToHost ) == hipSuccess && h[7] ) {
        char const * nm[ 6 ] = { "prologue", "sha", "lattice", "decode+tab", "loop", "tail" };
        unsigned long long tot = 0; for( int i=0; i<6; i++ ) tot += h[i];
        for( int i=0; i<6; i++ ) fprintf( stderr, "stamp %-10s %12.0f cyc/wave  %5.1f%%\n", nm[i], (double)h[i]/(double)h[7], 100.0*(double)h[i]/(double)tot );
      }
      hipFree( s->stamps );
    }
#endif
    if( s->d_arena ) hipFree( s->d_arena );
    if( s->d_desc )  hipFree( s->d_desc );
    if( s->d_out )   hipFree( s->d_out );
    if( s->done )    hipEventDestroy( s->done );
    if( s->stream )  hipStreamDestroy( s->stream );
  }
  free( ctx );
}

int fd_ed25519_gpu_device_cnt( fd_ed25519_gpu_t const * ctx ) { return ctx ? ctx->ndev : 0; }

int
fd_ed25519_gpu_set_codes( fd_ed25519_gpu_t * ctx, int flavour ) {
  if( !ctx || (flavour != FD_ED25519_GPU_CODES_AVX512 && flavour != FD_ED25519_GPU_CODES_REF) ) return FD_ED25519_GPU_ERR_ARG;
  ctx->ref_codes = flavour;
  return FD_ED25519_GPU_OK;
}

static int
check_descs( uint64_t arena_sz, fd_ed25519_desc_t const * desc, uint64_t n ) {
  for( uint64_t i=0; i<n; i++ ) {
    fd_ed25519_desc_t const * d = desc + i;
    if( (uint64_t)d->sig_off + 64u > arena_sz || (uint64_t)d->pub_off + 32u > arena_sz ||
        (uint64_t)d->msg_off + d->msg_sz > arena_sz ) return FD_ED25519_GPU_ERR_ARG;
  }
  return FD_ED25519_GPU_OK;
}

int
fd_ed25519_gpu_submit( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                       fd_ed25519_desc_t const * desc, uint64_t desc_cnt, int8_t * out_code ) {
  if( !ctx ) return FD_ED25519_GPU_ERR_ARG;
  if( ctx->pend_active ) return FD_ED25519_GPU_ERR_BUSY;
  if( desc_cnt && (!arena || !desc || !out_code) ) return FD_ED25519_GPU_ERR_ARG;
  if( arena_sz > 0xffffffffull + 1ull ) return FD_ED25519_GPU_ERR_ARG;
  int err = check_descs( arena_sz, desc, desc_cnt );
  if( err ) return err;
  ctx->pend_out = out_code; ctx->pend_cnt = desc_cnt; ctx->pend_active = 1;
  for( int i=0; i<ctx->ndev; i++ ) {
    fd_dev_state * s = &ctx->d[i];
    uint64_t lo = desc_cnt * (uint64_t)i / (uint64_t)ctx->ndev;
    uint64_t hi = desc_cnt * (uint64_t)(i+1) / (uint64_t)ctx->ndev;
    uint64_t m = hi - lo;
    s->busy = 0;
    if( !m ) continue;
    if( (err = dev_reserve( s, arena_sz, m )) ) { ctx->pend_active = 0; return err; }
    /* Each device gets the whole arena (descriptors index it freely). */
    HIPCK( hipMemcpyAsync( s->d_arena, arena, arena_sz, hipMemcpyHostToDevice, s->stream ) );
    HIPCK( hipMemcpyAsync( s->d_desc, desc + lo, m * sizeof(fd_ed25519_desc_t), hipMemcpyHostToDevice, s->stream ) );
    if( (err = dev_launch( ctx, s, s->d_arena, arena_sz, s->d_desc, m, s->d_out, s->stream )) ) { ctx->pend_active = 0; return err; }
    HIPCK( hipMemcpyAsync( out_code + lo, s->d_out, m, hipMemcpyDeviceToHost, s->stream ) );
    HIPCK( hipEventRecord( s->done, s->stream ) );
    s->busy = 1;
  }
  return FD_ED25519_GPU_OK;
}

int
fd_ed25519_gpu_poll( fd_ed25519_gpu_t * ctx ) {
  if( !ctx ) return FD_ED25519_GPU_ERR_ARG;
  if( !ctx->pend_active ) return FD_ED25519_GPU_OK;
  for( int i=0; i<ctx->ndev; i++ ) {
    fd_dev_state * s = &ctx->d[i];
    if( !s->busy ) continue;
    hipSetDevice( s->dev );
    hipError_t e = hipEventQuery( s->done );
    if( e == hipErrorNotReady ) return FD_ED25519_GPU_PENDING;
    if( e != hipSuccess ) { ctx->pend_active = 0; return FD_ED25519_GPU_ERR_LAUNCH; }
    s->busy = 0;
  }
  ctx->pend_active = 0;
  return FD_ED25519_GPU_OK;
}

int
fd_ed25519_verify_batch_gpu( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                             fd_ed25519_desc_t const * desc, uint64_t desc_cnt, int8_t * out_code ) {
  int err = fd_ed25519_gpu_submit( ctx, arena, arena_sz, desc, desc_cnt, out_code );
  if( err ) return err;
  for( int i=0; i<ctx->ndev; i++ ) {
    fd_dev_state * s = &ctx->d[i];
    if( !s->busy ) continue;
    hipSetDevice( s->dev );
    if( hipEventSynchronize( s->done ) != hipSuccess ) { ctx->pend_active = 0; return FD_ED25519_GPU_ERR_LAUNCH; }
  }
  return fd_ed25519_gpu_poll( ctx );
}

int
fd_ed25519_verify_batch_gpu_dev( fd_ed25519_gpu_t * ctx, int dev_idx, uint8_t const * d_arena, uint64_t arena_sz,
                                 fd_ed25519_desc_t const * d_desc, uint64_t desc_cnt, int8_t * d_out, void * stream ) {
  if( !ctx || dev_idx < 0 || dev_idx >= ctx->ndev ) return FD_ED25519_GPU_ERR_ARG;
  if( !desc_cnt ) return FD_ED25519_GPU_OK;
  if( !d_arena || !d_desc || !d_out ) return FD_ED25519_GPU_ERR_ARG;
  fd_dev_state * s = &ctx->d[ dev_idx ];
  hipStream_t st = stream ? (hipStream_t)stream : s->stream;
  return dev_launch( ctx, s, d_arena, arena_sz, d_desc, desc_cnt, d_out, st );
}

int
fd_ed25519_gpu_verify( fd_ed25519_gpu_t * ctx, uint8_t const * msg, uint64_t msg_sz,
                       uint8_t const sig[ 64 ], uint8_t const pub[ 32 ], int * out ) {
  if( !ctx || !out || !sig || !pub || (msg_sz && !msg) || msg_sz > 0xffffu ) return FD_ED25519_GPU_ERR_ARG;
  uint64_t sz = 96u + msg_sz;
  uint8_t * arena = (uint8_t *)malloc( sz + 16u );
  if( !arena ) return FD_ED25519_GPU_ERR_OOM;
  memcpy( arena, sig, 64 ); memcpy( arena + 64, pub, 32 ); if( msg_sz ) memcpy( arena + 96, msg, msg_sz );
  fd_ed25519_desc_t d = { 0u, 64u, 96u, (uint16_t)msg_sz, 0u };
  int8_t code = 0;
  int err = fd_ed25519_verify_batch_gpu( ctx, arena, sz, &d, 1u, &code );
  free( arena );
  if( err ) return err;
  *out = code;
  return FD_ED25519_GPU_OK;
}

int
fd_ed25519_gpu_verify_batch_single_msg( fd_ed25519_gpu_t * ctx, uint8_t const * msg, uint64_t msg_sz,
                                        uint8_t const * sigs, uint8_t const * pubs, uint64_t n, int * out ) {
  if( !ctx || !out || (msg_sz && !msg) || msg_sz > 0xffffu ) return FD_ED25519_GPU_ERR_ARG;
  if( n == 0u || n > 16u ) { *out = FD_ED25519_ERR_SIG; return FD_ED25519_GPU_OK; }   /* fd_ed25519_user.c:238-240 */
  if( !sigs || !pubs ) return FD_ED25519_GPU_ERR_ARG;
  uint64_t sz = 96u * n + msg_sz;
  uint8_t * arena = (uint8_t *)malloc( sz + 16u );
  if( !arena ) return FD_ED25519_GPU_ERR_OOM;
  memcpy( arena, sigs, 64u * n ); memcpy( arena + 64u * n, pubs, 32u * n );
  if( msg_sz ) memcpy( arena + 96u * n, msg, msg_sz );
  fd_ed25519_desc_t d[ 16 ];
  for( uint64_t j=0; j<n; j++ ) {
    d[j].sig_off = (uint32_t)(64u * j); d[j].pub_off = (uint32_t)(64u * n + 32u * j);
    d[j].msg_off = (uint32_t)(96u * n); d[j].msg_sz = (uint16_t)msg_sz; d[j].txn_idx = 0u;
  }
  int8_t codes[ 16 ];
  int err = fd_ed25519_verify_batch_gpu( ctx, arena, sz, d, n, codes );
  free( arena );
  if( err ) return err;
  int8_t t;
  fd_ed25519_gpu_txn_reduce( codes, d, n, &t, 1u );
  *out = t;
  return FD_ED25519_GPU_OK;
}

int64_t
fd_ed25519_gpu_txn_reduce( int8_t const * out_code, fd_ed25519_desc_t const * desc, uint64_t n,
                           int8_t * out_txn_code, uint64_t out_cap ) {
  int64_t t = 0;
  uint64_t i = 0;
  while( i < n ) {
    uint64_t j = i;
    while( j < n && desc[j].txn_idx == desc[i].txn_idx ) j++;
    int8_t code = FD_ED25519_SUCCESS;
    if( j - i > 16u ) code = FD_ED25519_ERR_SIG;
    else {
      int8_t first_p1 = 0, any_msg = 0;
      for( uint64_t k=i; k<j; k++ ) {
        int8_t c = out_code[k];
        if( c == FD_ED25519_ERR_MSG ) any_msg = 1;
        else if( c != FD_ED25519_SUCCESS && !first_p1 ) first_p1 = c;
      }
      code = first_p1 ? first_p1 : (any_msg ? (int8_t)FD_ED25519_ERR_MSG : (int8_t)FD_ED25519_SUCCESS);
    }
    if( (uint64_t)t < out_cap ) out_txn_code[t] = code;
    t++;
    i = j;
  }
  return t;
}

int
fd_ed25519_gpu_test_lattice( fd_ed25519_gpu_t * ctx, uint32_t const * k, uint64_t n, uint32_t * out ) {
  if( !ctx || !k || !out || !n ) return FD_ED25519_GPU_ERR_ARG;
  fd_dev_state * s = &ctx->d[0];
  HIPCK( hipSetDevice( s->dev ) );
  uint32_t * dk = NULL; uint32_t * dout = NULL;
  HIPCK( hipMalloc( &dk, n * 32u ) );
  if( hipMalloc( &dout, n * 72u ) != hipSuccess ) { hipFree( dk ); return FD_ED25519_GPU_ERR_OOM; }
  int err = FD_ED25519_GPU_OK;
  if( hipMemcpy( dk, k, n * 32u, hipMemcpyHostToDevice ) != hipSuccess ) err = FD_ED25519_GPU_ERR_LAUNCH;
  if( !err ) {
    hipLaunchKernelGGL( fd_ed25519_lattice_test_kernel, dim3( (uint32_t)((n + 255u) / 256u) ), dim3( 256 ), 0, s->stream, dk, dout, n );
    if( hipGetLastError() != hipSuccess || hipStreamSynchronize( s->stream ) != hipSuccess ) err = FD_ED25519_GPU_ERR_LAUNCH;
  }
  if( !err && hipMemcpy( out, dout, n * 72u, hipMemcpyDeviceToHost ) != hipSuccess ) err = FD_ED25519_GPU_ERR_LAUNCH;
  hipFree( dk ); hipFree( dout );
  return err;
}

char const *
fd_ed25519_gpu_strerror( int err ) {
  switch( err ) {
  case FD_ED25519_SUCCESS:         return "success";
  case FD_ED25519_ERR_SIG:         return "bad signature";
  case FD_ED25519_ERR_PUBKEY:      return "bad public key";
  case FD_ED25519_ERR_MSG:         return "bad message";
  case FD_ED25519_GPU_PENDING:     return "pending";
  case FD_ED25519_GPU_ERR_NODEV:   return "no gpu device";
  case FD_ED25519_GPU_ERR_OOM:     return "gpu out of memory";
  case FD_ED25519_GPU_ERR_LAUNCH:  return "gpu launch/runtime failure";
  case FD_ED25519_GPU_ERR_ARG:     return "bad argument";
  case FD_ED25519_GPU_ERR_BUSY:    return "batch already in flight";
  case FD_ED25519_GPU_CODE_BAD_DESC: return "descriptor outside arena";
  default: break;
  }
  return "unknown";
}

} /* extern "C" */
