/* fd_ed25519_gpu_kern.hip -- MI355X (gfx950) Ed25519 batch verifier: the
   device code.  Built to gfx950 assembly, passed through the peephole
   rewriter tools/asm_peephole.py, assembled into a code object that the host
   runtime (fd_ed25519_gpu_host.cpp) embeds, loads and launches by name.

   One signature per lane:
     S < l check -> k = SHA-512(R || A || M) mod l (M streamed from HBM) ->
     short vector (u, v) of the lattice {u = v k mod 8l}, w = v S mod l
     (fd_lattice_dev.h) -> decode A and R (sqrt-ratio ladder), small-order
     checks -> per-lane tables [0..8](-A), [0..8](-R) in HBM ->
     Q = [u](-A) + [v](-R) in ONE ~130-doubling Straus chain, then + [w]B
     as 11 mixed additions from the fixed-base comb table
     [0..2^22](2^(23 k) B), k < 11 (5.9 GB in HBM, built once per context)
     -> Q == O.
   Semantics follow fd_ed25519_verify (src/ballet/ed25519/fd_ed25519_user.c:
   134-229) with the FD_HAS_AVX512 error mapping (SURVEY.md §8(a) A-spec). */

#include <hip/hip_runtime.h>

#include "fd_ed25519_gpu_abi.h"
#include "fd_f25519_dev.h"
#include "fd_curve25519_dev.h"
#include "fd_sha512_dev.h"
#include "fd_sha256_dev.h"
#include "fd_scalar_dev.h"
#include "fd_lattice_dev.h"
#include "fd_diag.h"

/* Round-4 instruction cuts, each a build switch for same-process A/Bs
   (tools/ab_b2b.py; -DFD_OPT_X=0 builds the previous form):
     FIRSTWIN  the chain's first window takes its entry as the point
               (ge_from_cached) instead of adding it to the identity;
     COMBCHK   the last comb addition folded into the final compare
               (comb_lds_eq);
     IDROW     1: row 0 of every variable-base table pre-filled with the
               identity (fd_vtab_id_fill at allocation) instead of a shared
               record selected per fetch (0); 2 (round 5): a zero digit
               reads row 0 of table 0 through one min in the index, so every
               zero digit of the chip hits the same two L2-resident lines
               (1 fetched each signature's own row 0: +8.6 % HBM bytes). */
#ifndef FD_OPT_FIRSTWIN
#define FD_OPT_FIRSTWIN 1
#endif
#ifndef FD_OPT_COMBCHK
#define FD_OPT_COMBCHK 1
#endif
#ifndef FD_OPT_IDROW
#define FD_OPT_IDROW 2
#endif
/*   TAIL1     (round 5, with IDROW 2) entry 1 is -Q with Q affine, so its 2Z
               is 2 and its 32-B tail (2Z's limbs 2..9) is zero like the
               identity row's: a digit of magnitude <= 1 reads the tail of
               row 0 of table 0 (L2-resident), and entry 1's tail is never
               stored. */
#ifndef FD_OPT_TAIL1
#define FD_OPT_TAIL1 1
#endif
/*   APARSE    (round 5) the pipelined kernel's phase A can parse its frag
               batch in the launch (pipe_aparse); 0 compiles that path out
               (an A/B of what its code costs the launches that do not use it;
               such a build runs frag batches only with FD_ED25519_GPU_APARSE=0). */
#ifndef FD_OPT_APARSE
#define FD_OPT_APARSE 1
#endif
/*   APRIO     (round 6) the pipe kernel's phase-A waves are the youngest on
               their SIMD, so the arbiter (oldest first) gives them the issue
               slots phases C and B leave: a SHA block's 33 dword loads (and
               the signature's and key's 26) came out spread over many
               microseconds, and the L2 -- streaming ~4 MB of table reads per
               XCD every ~15 us -- had dropped a window's two lines before the
               window's last loads reached them: 4.2 KB of HBM reads per
               verify for 312 B in the steady state, 322 B with phase A alone
               (tools/phase_bytes.py).  APRIO issues each window's loads at
               the top wave priority (s_setprio 3 around them, back to 0
               after), so they leave within a few hundred cycles. */
#ifndef FD_OPT_APRIO
#define FD_OPT_APRIO 1
#endif
/*   X4        (round 6) the arena windows (a SHA block's 33 dwords, the
               signature's 17, the key's 9) as 16-byte loads from their
               dword-aligned start (gfx950 takes a dwordx4 at any 4-byte
               alignment) at immediate offsets from one base: 9 / 5 / 3 load
               instructions and no per-dword address arithmetic, when the
               whole window lies inside the readable arena for every lane of
               the wave (else the clamped dword loads). */
/*   BNOT      (round 6) phase B's chain segment ends without T (phase C
               starts with a doubling, which does not read it): one product
               fewer and 40 bytes fewer of partial sum each way per verify. */
#ifndef FD_OPT_BNOT
#define FD_OPT_BNOT 1
#endif
#ifndef FD_OPT_X4
#define FD_OPT_X4 1
#endif

/* Diagnostic build only (-DFD_PHASE_STAMPS, tools/Makefile): s_memtime at
   phase boundaries, per-wave deltas summed into args.stamps.  The product
   build compiles none of it. */
#ifdef FD_PHASE_STAMPS
#define FD_NSTAMP 8
#define FD_TL_BASE 8      /* pipe-kernel timeline: 4 u64 per wave after the sums (single-lane kernel: 2 per wave) */
#define FD_STAMP_WORDS_DEV (8u + 4096u * 12u * 4u)   /* = the host's FD_STAMP_WORDS */
#define STAMP( i ) do { FE_FENCE(); if( _st ) _st[ i ] = __builtin_amdgcn_s_memtime(); FE_FENCE(); } while( 0 )
#else
#define STAMP( i ) do {} while( 0 )
#endif

/* ------------------------------------------------------------------ loads */

/* n little-endian words starting at an arbitrary byte offset off (read
   through aligned dwords, clamped to the readable arena). */
typedef unsigned int fd_u4a4 __attribute__(( ext_vector_type( 4 ), aligned( 4 ) ));   /* 16-byte load, 4-byte alignment */

/* raw[0 .. M) = a32[dw .. dw + M) (M = 4 k + 1) as k dwordx4 + 1 dword
   from one base address (FD_OPT_X4's fast path; the caller checked the
   range) */
template<int M>
__device__ __forceinline__ void load_x4( uint32_t raw[ M ], uint32_t const * a32, uint32_t dw ) {
  static_assert( (M & 3) == 1, "M = 4 k + 1" );
  uint32_t const * p = a32 + dw;
#pragma unroll
  for( int j=0; j<M/4; j++ ) {
    fd_u4a4 v = *(fd_u4a4 const *)(p + 4*j);
    raw[4*j] = v.x; raw[4*j+1] = v.y; raw[4*j+2] = v.z; raw[4*j+3] = v.w;
  }
  raw[M-1] = p[M-1];
}

template<int N>
__device__ __forceinline__ void load_words( uint32_t out[ N ], uint8_t const * arena, uint32_t off, uint32_t lim_dw ) {
  uint32_t const * a32 = (uint32_t const *)arena;
  uint32_t dw = off >> 2, sh = off & 3u;
#if FD_OPT_X4
  if constexpr( (N & 3) == 0 ) {
    if( __all( dw + (uint32_t)N <= lim_dw ) ) {
      uint32_t raw[ N + 1 ];
      load_x4<N + 1>( raw, a32, dw );
#pragma unroll
      for( int i=0; i<N; i++ ) out[i] = __builtin_amdgcn_alignbyte( raw[i+1], raw[i], sh );
      return;
    }
  }
#endif
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

/* Bases of the fixed-base comb table: thread k < FD_CTAB_POS computes
   B_k = [2^(23 k)] B (23 k doublings of B, decoded from its standard
   encoding: y = 4/5, x even) and stores its affine precomputed form (Y+X,
   Y-X, 2dXY; 30 words) at cbase[30 k].  Runs once per device at context
   creation, before fd_ed25519_ctab_init. */
extern "C" __global__ void __launch_bounds__( 64 ) fd_ed25519_ctab_base( uint32_t * cbase ) {
  uint32_t k = threadIdx.x;
  if( k >= (uint32_t)FD_CTAB_POS ) return;
  uint32_t benc[ 8 ];
  benc[0] = 0x66666658u;
#pragma unroll
  for( int i=1; i<8; i++ ) benc[i] = 0x66666666u;
  ge_p3 B; ge_decode( B, benc, true );
#pragma unroll 1
  for( uint32_t i=0; i<(uint32_t)FD_CTAB_BITS*k; i++ ) ge_dbl( B, B, false );
  ge_precomp Bp; ge_affine_precomp( Bp, B );
#pragma unroll
  for( int i=0; i<10; i++ ) { cbase[30*k + i] = Bp.YpX.v[i]; cbase[30*k + 10 + i] = Bp.YmX.v[i]; cbase[30*k + 20 + i] = Bp.T2d.v[i]; }
}

/* The fixed-base comb table: thread g = k FD_CTAB_N + j computes [j] B_k
   (23-bit double-and-add from the affine base, j <= 2^22) and stores its
   affine precomputed form (Y+X, Y-X, 2dXY) at ctab[g FD_CTAB_STRIDE ...]
   (entry 0: the identity, Y+X = Y-X = 1, 2dXY = 0).  11 x (2^22+1)
   entries, 5.9 GB; runs once per device at context creation (~0.1 s). */
extern "C" __global__ void __launch_bounds__( 256 ) fd_ed25519_ctab_init( uint32_t * ctab, uint32_t const * cbase ) {
  uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( g >= (uint64_t)FD_CTAB_POS * FD_CTAB_N ) return;
  uint32_t k = (uint32_t)(g / FD_CTAB_N), j = (uint32_t)(g % FD_CTAB_N);
  ge_precomp Bp;
#pragma unroll
  for( int i=0; i<10; i++ ) { Bp.YpX.v[i] = cbase[30*k + i]; Bp.YmX.v[i] = cbase[30*k + 10 + i]; Bp.T2d.v[i] = cbase[30*k + 20 + i]; }
  ge_p3 acc; ge_identity( acc );
#pragma unroll 1
  for( int bit=FD_CTAB_BITS-1; bit>=0; bit-- ) {
    ge_dbl( acc, acc, true );
    if( (j >> bit) & 1u ) ge_madd( acc, acc, Bp, true );
  }
  ge_precomp o; ge_affine_precomp( o, acc );
  uint4 * e = (uint4 *)(ctab + g * FD_CTAB_STRIDE);
  uint32_t w[ 32 ];
#pragma unroll
  for( int i=0; i<10; i++ ) { w[i] = o.YpX.v[i]; w[10+i] = o.YmX.v[i]; w[20+i] = o.T2d.v[i]; }
  w[30] = 0u; w[31] = 0u;
#pragma unroll
  for( int i=0; i<8; i++ ) e[i] = make_uint4( w[4*i], w[4*i+1], w[4*i+2], w[4*i+3] );
}

/* ------------------------------------------------------------------ verify */

/* struct verify_args: fd_ed25519_gpu_abi.h */

/* Raw message dwords of SHA block b: dword (msg_off>>2) + 32b - 16 + i,
   i < 33, clamped to the readable arena (block 0's first 16 are unused:
   R || A come from registers). */
__device__ __forceinline__ void sha_fetch( uint32_t raw[ 33 ], uint32_t const * a32, uint32_t msg_off, uint32_t b,
                                           uint32_t lim_dw ) {
  int32_t start = (int32_t)(msg_off >> 2) + 32*(int32_t)b - 16;
#if FD_DIAG_NO_ARENA_ON
  (void)a32; (void)lim_dw;
#pragma unroll
  for( int i=0; i<33; i++ ) raw[i] = fd_diag_hash( (uint64_t)msg_off, (uint32_t)(start + i) );
#else
#if FD_OPT_X4
  if( __all( start >= 0 && (uint32_t)start + 32u <= lim_dw ) ) { load_x4<33>( raw, a32, (uint32_t)start ); return; }
#endif
#pragma unroll
  for( int i=0; i<33; i++ ) raw[i] = a32[ min( (uint32_t)max( start + i, 0 ), lim_dw ) ];
#endif
}

/* SHA-512(R || A || M) mod l.  R, A: 8 LE words each; the message is
   streamed from HBM, each block's dwords fetched one block ahead so the
   load latency hides behind the previous compression. */
template<bool FASTBLK>
__device__ __forceinline__ void hash_ram( uint32_t k[ 8 ], uint32_t const Rw[ 8 ], uint32_t const Aw[ 8 ],
                                          uint8_t const * arena, uint32_t msg_off, uint32_t msg_sz, uint32_t lim_dw ) {
  uint64_t h[ 8 ]; sha512_init_state( h );
  uint32_t total = 64u + msg_sz;
  uint32_t nblk = (total + 17u + 127u) >> 7;
  uint32_t const * a32 = (uint32_t const *)arena;
  uint32_t sh = msg_off & 3u;
  /* the <false> instantiation is the pipe kernel's phase A (FD_OPT_APRIO) */
  constexpr bool APRIO = !FASTBLK && FD_OPT_APRIO;
  uint32_t nxt[ 33 ];
  if( APRIO ) { FE_FENCE(); __builtin_amdgcn_s_setprio( 3 ); FE_FENCE(); }
  sha_fetch( nxt, a32, msg_off, 0u, lim_dw );
  if( APRIO ) { FE_FENCE(); __builtin_amdgcn_s_setprio( 0 ); FE_FENCE(); }
  for( uint32_t b=0; b<nblk; b++ ) {
    uint32_t raw[ 33 ];
#pragma unroll
    for( int i=0; i<33; i++ ) raw[i] = nxt[i];
    if( APRIO ) { FE_FENCE(); __builtin_amdgcn_s_setprio( 3 ); FE_FENCE(); }
    if( b + 1u < nblk ) sha_fetch( nxt, a32, msg_off, b + 1u, lim_dw );
    if( APRIO ) { FE_FENCE(); __builtin_amdgcn_s_setprio( 0 ); FE_FENCE(); }
    uint64_t W[ 16 ];
    /* a block whose message bytes all lie before msg_sz on every lane of
       the wave (every block but the last one or two) needs no padding
       masks: the wave-uniform fast form assembles just the bytes (not in
       the pipe kernel's phase A: its extra registers spill there) */
    if( FASTBLK && __all( (b << 7) + 64u <= msg_sz ) ) {
#pragma unroll
      for( int j=0; j<16; j++ ) {
        uint32_t hi, lo;
        if( b == 0 && j < 8 ) {
          uint32_t const * src = (j < 4) ? Rw : Aw;
          int jj = j & 3;
          hi = sha_bswap32( src[2*jj] ); lo = sha_bswap32( src[2*jj+1] );
        } else {
          hi = sha_bswap32( __builtin_amdgcn_alignbyte( raw[2*j+1], raw[2*j],   sh ) );
          lo = sha_bswap32( __builtin_amdgcn_alignbyte( raw[2*j+2], raw[2*j+1], sh ) );
        }
        W[j] = ((uint64_t)hi << 32) | lo;
      }
    } else {
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
   whatever entry its digit selects.  One record per |d|: the digit's sign is
   applied at the use point (vtab_finish).  (Storing both signs instead --
   twice the table writes for no selects at the 66 uses -- measured 8 %
   slower: the kernel runs power-limited, and the table traffic costs clock;
   DESIGN.md §4.)  The diagnostic variants of those measurements (wrong
   results by design) hook in through fd_diag.h. */
__device__ __forceinline__ void vtab_ptrs( uint32_t const * vtab, uint64_t cap, uint64_t t, uint32_t e,
                                           uint4 const ** m, uint4 const ** tl ) {
#if FD_OPT_IDROW == 2
  /* digit 0 -> row 0 of table 0 (every row 0 is the identity): one min
     (e << 28 exceeds e cap + t for e >= 1, as cap < 2^26 -- host-checked),
     so all zero digits of the chip read the same two L2-hot lines */
  uint32_t i32 = min( (uint32_t)e * (uint32_t)cap + (uint32_t)t, e << 28 );
  uint64_t idx = i32;
#if FD_OPT_TAIL1
  uint64_t tdx = min( i32, (e << 28) - (1u << 28) );   /* e <= 1: 0; e >= 2: (e-1) 2^28 > e cap + t */
#else
  uint64_t tdx = idx;
#endif
#else
  uint64_t idx = (uint64_t)e * cap + t, tdx = idx;
#endif
  *m  = (uint4 const *)(vtab + idx * 32u);
  *tl = (uint4 const *)(vtab + (uint64_t)FD_VTAB_N * cap * 32u + tdx * 8u);
#if !FD_OPT_IDROW
  if( !e ) {   /* the identity: one shared record after both regions (written by the host) */
    uint32_t const * id = vtab + (uint64_t)FD_VTAB_N * cap * 40u;
    *m = (uint4 const *)id; *tl = (uint4 const *)(id + 32);
  }
#endif
}

/* Row 0 of every table = the identity in cached form (Y+X = 1, Y-X = 1,
   2dT = 0, 2Z = 2; FD_VW layout): written once when the table scratch is
   allocated (no kernel ever stores row 0), so a fetch of digit 0 needs no
   select of a shared record.  One thread per table. */
extern "C" __global__ void __launch_bounds__( 256 ) fd_vtab_id_fill( uint32_t * vtab, uint64_t cap ) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( t >= cap ) return;
  uint4 * m  = (uint4 *)(vtab + t * 32u);
  uint4 * tl = (uint4 *)(vtab + (uint64_t)FD_VTAB_N * cap * 32u + t * 8u);
#pragma unroll
  for( int j=0; j<8; j++ ) {
    uint32_t w[ 4 ];
#pragma unroll
    for( int i=0; i<4; i++ ) {
      int k = 4*j + i;
      w[i] = (k == FD_VW( 0, 0 ) || k == FD_VW( 1, 0 )) ? 1u : (k == FD_VW( 3, 0 ) ? 2u : 0u);
    }
    m[j] = make_uint4( w[0], w[1], w[2], w[3] );
  }
  tl[0] = make_uint4( 0u, 0u, 0u, 0u ); tl[1] = make_uint4( 0u, 0u, 0u, 0u );
}

/* Entry |d| of a biased digit db = d + 8 (db <= 16 by construction; clamped
   to the table all the same): one v_sad_u32 (|db - 8| + 0) and a min. */
__device__ __forceinline__ uint32_t vtab_entry( uint32_t db ) {
  uint32_t e;
  asm( "v_sad_u32 %0, %1, 8, 0" : "=v"(e) : "v"(db) );
  return min( e, 8u );
}

__device__ __forceinline__ void vtab_store( uint32_t * vtab, uint64_t cap, uint64_t t, int e, ge_cached const & c,
                                            bool tail = true ) {
  uint32_t w[ 40 ];
#pragma unroll
  for( int j=0; j<10; j++ ) {
    w[FD_VW(0,j)] = c.YpX.v[j]; w[FD_VW(1,j)] = c.YmX.v[j]; w[FD_VW(2,j)] = c.T2d.v[j]; w[FD_VW(3,j)] = c.Z2.v[j];
  }
  uint4 const * mc; uint4 const * tc;
  vtab_ptrs( vtab, cap, t, (uint32_t)e, &mc, &tc );
  uint4 * m = (uint4 *)mc; uint4 * tl = (uint4 *)tc;
  FD_DIAG_VTAB_STORE( m, tl, w );
#pragma unroll
  for( int j=0; j<8; j++ ) m[j] = make_uint4( w[4*j], w[4*j+1], w[4*j+2], w[4*j+3] );
#if FD_VTAB_TAIL
  if( tail ) {
#pragma unroll
    for( int j=0; j<2; j++ ) tl[j] = make_uint4( w[32+4*j], w[33+4*j], w[34+4*j], w[35+4*j] );
  }
#endif
}

/* Table [0..8](-Q) for an affine Q (Z = 1), cached form (replaces the
   reference's -A table of fd_ed25519_double_scalar_mul_base,
   fd_curve25519.c:136-144, and the neg of fd_ed25519_user.c:215). */
__device__ __forceinline__ void vtab_build( uint32_t * vtab, uint64_t cap, uint64_t t, ge_p3 const & Q ) {
  ge_p3 nQ = Q;
  { fe x; fe_neg( x, Q.X ); fe_carry( nQ.X, x ); fe_neg( x, Q.T ); fe_carry( nQ.T, x ); }
  ge_cached c;
  ge_to_cached( c, nQ );  vtab_store( vtab, cap, t, 1, c, !(FD_OPT_IDROW == 2 && FD_OPT_TAIL1) );   /* tail: 2Z = 2, read from row 0 */
  /* -Q's affine form for the mixed additions is the cached entry without 2Z:
     Y+X and Y-X uncarried (M: ge_madd takes them only as second operands of
     fe_mul), 2dT the same product */
  ge_precomp nQp;
  nQp.YpX = c.YpX; nQp.YmX = c.YmX; nQp.T2d = c.T2d;
  ge_p3 P;
  ge_dbl( P, nQ, true ); ge_to_cached( c, P ); vtab_store( vtab, cap, t, 2, c );
#pragma unroll 1
  for( int e=3; e<=8; e++ ) { ge_madd( P, P, nQp, true ); ge_to_cached( c, P ); vtab_store( vtab, cap, t, e, c ); FE_FENCE(); }
}

/* Issue the loads of entry |d| (biased digit db = d + 8) into raw words;
   vtab_finish (at the use point) applies the sign. */
__device__ __forceinline__ void vtab_fetch( uint32_t w[ 40 ], uint32_t const * vtab, uint64_t cap, uint64_t t, uint32_t db ) {
  uint32_t e = vtab_entry( db );
  uint4 const * m; uint4 const * tl;
  vtab_ptrs( vtab, cap, t, e, &m, &tl );
#pragma unroll
  for( int j=0; j<8; j++ ) { uint4 v = m[j]; w[4*j] = v.x; w[4*j+1] = v.y; w[4*j+2] = v.z; w[4*j+3] = v.w; }
#pragma unroll
  for( int j=0; j<2; j++ ) { uint4 v = tl[j]; w[32+4*j] = v.x; w[33+4*j] = v.y; w[34+4*j] = v.z; w[35+4*j] = v.w; }
}

__device__ __forceinline__ void vtab_finish( ge_cached & c, uint32_t const w[ 40 ], uint32_t db ) {
  bool neg = db < 8u;
  fe tv;
#pragma unroll
  for( int j=0; j<10; j++ ) { tv.v[j] = w[FD_VW(2,j)]; c.Z2.v[j] = w[FD_VW(3,j)]; }
  fe_cneg( c.T2d, tv, neg );
#pragma unroll
  for( int j=0; j<10; j++ ) {
    c.YpX.v[j] = neg ? w[FD_VW(1,j)] : w[FD_VW(0,j)];
    c.YmX.v[j] = neg ? w[FD_VW(0,j)] : w[FD_VW(1,j)];
  }
}

/* Comb-table entry |d| of position k (signed 23-bit digit d): loads issued
   here, sign applied by ctab_finish at the use point. */
__device__ __forceinline__ void ctab_fetch( uint32_t w[ 32 ], uint32_t const * ctab, int k, int d ) {
  uint32_t e = min( (uint32_t)(d < 0 ? -d : d), FD_CTAB_HALF );    /* |d| <= 2^22 by construction; never past the table */
  uint4 const * p = (uint4 const *)(ctab + ((uint64_t)k * FD_CTAB_N + e) * FD_CTAB_STRIDE);
#pragma unroll
  for( int j=0; j<8; j++ ) { uint4 v = p[j]; w[4*j] = v.x; w[4*j+1] = v.y; w[4*j+2] = v.z; w[4*j+3] = v.w; }
}

__device__ __forceinline__ void ctab_finish( ge_precomp & q, uint32_t const w[ 32 ], int d ) {
  bool neg = d < 0;
  fe t;
#pragma unroll
  for( int j=0; j<10; j++ ) t.v[j] = w[20+j];
  fe_cneg( q.T2d, t, neg );
#pragma unroll
  for( int j=0; j<10; j++ ) {
    q.YpX.v[j] = neg ? w[10+j] : w[j];
    q.YmX.v[j] = neg ? w[j]    : w[10+j];
  }
}

__device__ __forceinline__ int wdig( uint8_t const * dig, int k ) {
  uint32_t b0 = dig[ (FD_ROW_W + 3*k)*FD_VERIFY_BLOCK ], b1 = dig[ (FD_ROW_W + 3*k + 1)*FD_VERIFY_BLOCK ];
  uint32_t b2 = dig[ (FD_ROW_W + 3*k + 2)*FD_VERIFY_BLOCK ];
  return ((int)((b0 | (b1 << 8) | (b2 << 16)) << 8)) >> 8;      /* 24-bit two's complement */
}

/* acc = [u](-A) + [v](-R) over nw 4-bit windows (wave-uniform; one shared
   doubling chain -- Straus), then + [w]B as 11 mixed additions of comb-table
   entries (no doublings: entry k already carries its 2^(23 k)).  u / v
   digits from LDS rows (biased by 8, sign of u folded in), w digits signed
   23-bit (three byte rows each).  Table entries are fetched one step ahead: A's for the next window
   before the doublings, R's before A's addition, the first comb entry during
   the last window. */
template<bool COMB>
__device__ __forceinline__ void dsm_loop( ge_p3 & acc, uint32_t const * vtab, uint64_t cap, uint64_t ta, uint64_t tr,
                                          uint8_t const * dig, uint32_t const * ctab, int nw, int wn ) {
  ge_identity( acc );
  uint32_t raw[ 40 ];
  uint32_t craw[ 32 ];
  uint32_t dba = dig[ (FD_ROW_U + nw-1)*FD_VERIFY_BLOCK ];
  vtab_fetch( raw, vtab, cap, ta, dba );
#pragma unroll 1
  for( int i=nw-1; i>=0; i-- ) {
    if( i < nw-1 ) {
      /* T only on the last doubling (the adds need it); a runtime want_t in
         a rolled loop would compute it on all four.  Window nw-2 is wn bits
         wide (recode_p_lds) */
      int nd = i == nw-2 ? wn : 4;
#pragma unroll 1
      for( int j=1; j<nd; j++ ) { ge_dbl( acc, acc, false ); FE_FENCE(); }
      ge_dbl( acc, acc, true );
      FE_FENCE();
    }
    ge_cached q;
    vtab_finish( q, raw, dba );
    uint32_t dbr = dig[ (FD_ROW_V + i)*FD_VERIFY_BLOCK ];
    vtab_fetch( raw, vtab, cap, tr, dbr );
    FE_FENCE();
    ge_add_cached( acc, acc, q, true );
    FE_FENCE();
    vtab_finish( q, raw, dbr );
    if( i > 0 ) { dba = dig[ (FD_ROW_U + i-1)*FD_VERIFY_BLOCK ]; vtab_fetch( raw, vtab, cap, ta, dba ); }
    else if( COMB ) ctab_fetch( craw, ctab, 0, wdig( dig, 0 ) );
    FE_FENCE();
    ge_add_cached( acc, acc, q, i == 0 );
    FE_FENCE();
  }
  if( !COMB ) return;
#pragma unroll 1
  for( int k=0; k<FD_CTAB_POS; k++ ) {
    ge_precomp bp;
    ctab_finish( bp, craw, wdig( dig, k ) );
    if( k + 1 < FD_CTAB_POS ) ctab_fetch( craw, ctab, k + 1, wdig( dig, k + 1 ) );
    FE_FENCE();
    ge_madd( acc, acc, bp, k + 1 < FD_CTAB_POS );
    FE_FENCE();
  }
}

/* c = [w]B alone: the 11 comb-table additions of dsm_loop from the identity
   (the pair kernel's second wave computes it beside the chain). */
__device__ __forceinline__ void comb_only( ge_p3 & c, uint8_t const * dig, uint32_t const * ctab ) {
  ge_identity( c );
  uint32_t craw[ 32 ];
  ctab_fetch( craw, ctab, 0, wdig( dig, 0 ) );
#pragma unroll 1
  for( int k=0; k<FD_CTAB_POS; k++ ) {
    ge_precomp bp;
    ctab_finish( bp, craw, wdig( dig, k ) );
    if( k + 1 < FD_CTAB_POS ) ctab_fetch( craw, ctab, k + 1, wdig( dig, k + 1 ) );
    FE_FENCE();
    ge_madd( c, c, bp, true );
    FE_FENCE();
  }
}

__device__ __forceinline__ int bitlen8( uint32_t const x[ 8 ] ) {
  int b = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) b = x[j] ? 32*j + 32 - __clz( (int)x[j] ) : b;
  return b;
}


/* The pipe's top-digit position for the wave (its longest scalar has nbits
   bits): P = nbits - 3, within [124, 252]. */
__device__ __forceinline__ int wave_top_pos( int nbits ) {
#pragma unroll
  for( int o=32; o>=1; o>>=1 ) nbits = max( nbits, __shfl_xor( nbits, o ) );
  return recode_p_top( nbits );
}

/* recode_p_lds: ybias_p's digits into nw LDS byte rows (biased by 8, negated
   when neg) for the one-shot kernels' Straus loop (dsm_loop): windows
   0 .. nw-3 4-bit, window nw-2 wn bits, the top digit at bit P. */
__device__ __forceinline__ void recode_p_lds( uint8_t * row, uint32_t const x[ 8 ], int neg, int P, uint64_t stride ) {
  uint32_t y[ 8 ];
  ybias_p( y, x, P );
  int nw = ((P + 3) >> 2) + 1;
#pragma unroll
  for( int i=0; i<FD_NDIG_MAX-1; i++ ) {
    if( i < nw-1 ) {
      uint32_t db = recode_p_low( y, i, P );
      row[ (uint64_t)i*stride ] = (uint8_t)(neg ? 16u - db : db);
    }
  }
  uint32_t db = recode_p_hi( y, P );
  row[ (uint64_t)(nw-1)*stride ] = (uint8_t)(neg ? 16u - db : db);
}

/* k = SHA-512(R||A||M) mod l (:203-206), the lattice vector (u, v, sign
   of u) of k (fd_lattice_dev.h) and w = v S mod l, for a live lane; *nbits =
   the longer of u, v in bits. */
template<bool FASTBLK>
__device__ __forceinline__ void verify_prep_scalars( uint32_t u[ 8 ], uint32_t v[ 8 ], int * un, uint32_t w[ 8 ], int * nbits,
                                                     uint32_t const sig[ 16 ], uint32_t const pub[ 8 ], verify_args const & args,
                                                     fd_ed25519_desc_t const & d, uint32_t lim_dw
#ifdef FD_PHASE_STAMPS
                                                     , uint64_t * _st
#endif
                                                     , uint32_t const * krow = nullptr   /* k precomputed (wave-uniform) */
                                                     ) {
  uint32_t k[ 8 ];
  if( krow ) {
    uint4 k0 = ((uint4 const *)krow)[0], k1 = ((uint4 const *)krow)[1];
    k[0] = k0.x; k[1] = k0.y; k[2] = k0.z; k[3] = k0.w; k[4] = k1.x; k[5] = k1.y; k[6] = k1.z; k[7] = k1.w;
  } else {
    hash_ram<FASTBLK>( k, sig, pub, args.arena, d.msg_off, d.msg_sz, lim_dw );
  }
  FE_FENCE();
  STAMP( 2 );
  lat_short_vector( k, u, v, un );
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
  sc_reduce512( w, pr );
  *nbits = max( bitlen8( u ), bitlen8( v ) );
}


/* k, the lattice vector, w = v S mod l and their digits into this lane's
   column drow (rows FD_ROW_U / _V / _W, row r at drow[r * stride], LDS with
   stride FD_VERIFY_BLOCK; FD_ROW_NW: the wave-uniform top-digit position P
   of recode_p_lds, written by lane 0 of each wave).  Lanes that are not live write zero digits (every
   lane takes part in the wave max). */
__device__ __forceinline__ void verify_prep_digits( uint8_t * drow, uint64_t stride, int tid, bool live, uint32_t const sig[ 16 ],
                                                    uint32_t const pub[ 8 ], verify_args const & args,
                                                    fd_ed25519_desc_t const & d, uint32_t lim_dw
#ifdef FD_PHASE_STAMPS
                                                    , uint64_t * _st
#endif
                                                    ) {
  uint32_t u[ 8 ], v[ 8 ];
  int un = 0, nbits = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) { u[j] = 0u; v[j] = 0u; }
  if( live ) {
    uint32_t w[ 8 ];
    verify_prep_scalars<true>( u, v, &un, w, &nbits, sig, pub, args, d, lim_dw
#ifdef FD_PHASE_STAMPS
                         , _st
#endif
                         );
    /* signed 23-bit comb digits (fd_scalar_dev.h comb_digit), three bytes each */
    uint32_t yw[ 8 ];
    comb_bias( yw, w );
#pragma unroll
    for( int k=0; k<FD_CTAB_POS; k++ ) {
      int dd = comb_digit( yw, k );
      drow[ (uint64_t)(FD_ROW_W + 3*k    )*stride ] = (uint8_t)(dd & 255);
      drow[ (uint64_t)(FD_ROW_W + 3*k + 1)*stride ] = (uint8_t)((dd >> 8) & 255);
      drow[ (uint64_t)(FD_ROW_W + 3*k + 2)*stride ] = (uint8_t)((dd >> 16) & 255);
    }
  }
  int P = wave_top_pos( nbits );
  recode_p_lds( drow + FD_ROW_U*stride, u, un, P, stride );
  recode_p_lds( drow + FD_ROW_V*stride, v, 0,  P, stride );
  if( (tid & 63) == 0 ) drow[ FD_ROW_NW*stride ] = (uint8_t)P;     /* the wave's top-digit position */
}

/* The verify code from the check results, in the reference's order
   (fd_ed25519_user.c:157-228): 0 means every check before the equation
   passed. */
__device__ __forceinline__ int verify_precode( verify_args const & args, bool desc_ok, bool bad_s, int stA, int stR ) {
  int code;
  if     ( !desc_ok    ) code = FD_ED25519_GPU_CODE_BAD_DESC;
  else if( bad_s       ) code = FD_ED25519_ERR_SIG;
  else if( !(stA & 1)  ) code = args.ref_codes ? FD_ED25519_ERR_PUBKEY : FD_ED25519_ERR_SIG;   /* :190-192 */
  else if( !(stR & 1)  ) code = FD_ED25519_ERR_SIG;
  else if( stA & 2     ) code = FD_ED25519_ERR_PUBKEY;                                        /* :193-195 */
  else if( stR & 2     ) code = FD_ED25519_ERR_SIG;                                           /* :196-198 */
  else                   code = 0;
  return code;
}

/* The equation for a lane whose checks passed: Q = [u](-A) + [v](-R) + [w]B
   (tables ta / tr of vtab, digits in this lane's LDS column drow, the
   wave's window count in s_dig) and Q == O -> SUCCESS / ERR_MSG. */
__device__ __forceinline__ int verify_equation( verify_args const & args, uint8_t const * drow, uint8_t const * s_dig,
                                                int tid, uint64_t ta, uint64_t tr,
                                                uint32_t const * s_wb  /* NULL: add [w]B here; else its cached form in LDS ([word][256]) */
#ifdef FD_PHASE_STAMPS
                                                , uint64_t * _st
#endif
                                                ) {
  uint64_t cap = args.vtab_cap;
  int P = __builtin_amdgcn_readfirstlane( (int)s_dig[ FD_ROW_NW*FD_VERIFY_BLOCK + (tid & ~63) ] );
  int nw = ((P + 3) >> 2) + 1, wn = P - 4*(nw - 2);  /* recode_p_lds's windows */
  ge_p3 acc;
  if( !s_wb ) dsm_loop<true>( acc, args.vtab, cap, ta, tr, drow, args.ctab, nw, wn );
  else {
    dsm_loop<false>( acc, args.vtab, cap, ta, tr, drow, args.ctab, nw, wn );
    ge_cached c;
#pragma unroll
    for( int j=0; j<10; j++ ) {
      c.YpX.v[j] = s_wb[ (j     )*FD_VERIFY_BLOCK + tid ]; c.YmX.v[j] = s_wb[ (10 + j)*FD_VERIFY_BLOCK + tid ];
      c.T2d.v[j] = s_wb[ (20 + j)*FD_VERIFY_BLOCK + tid ]; c.Z2.v[j]  = s_wb[ (30 + j)*FD_VERIFY_BLOCK + tid ];
    }
    FE_FENCE();
    ge_add_cached( acc, acc, c, false );
    FE_FENCE();
  }
  STAMP( 5 );
  /* Q == O  <=>  X == 0 and Y == Z (the reference's projective compare, :225-228, on [v]D) */
  fe dl;
  int ex = fe_is_zero( acc.X );
  fe_sub( dl, acc.Y, acc.Z ); fe_carry( dl, dl );
  int ey = fe_is_zero( dl );
  return (ex & ey) ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
}

/* The verify code: the checks, then for lanes at 0 the equation
   (tables at vtab[gid] / vtab[cap/2 + gid]). */
__device__ __forceinline__ int verify_tail( verify_args const & args, bool desc_ok, bool bad_s, int stA, int stR,
                                            uint8_t const * drow, uint8_t const * s_dig, int tid, uint64_t gid,
                                            uint32_t const * s_wb
#ifdef FD_PHASE_STAMPS
                                            , uint64_t * _st
#endif
                                            ) {
  int code = verify_precode( args, desc_ok, bad_s, stA, stR );
  if( code == 0 ) code = verify_equation( args, drow, s_dig, tid, gid, args.vtab_cap/2u + gid, s_wb
#ifdef FD_PHASE_STAMPS
                                          , _st
#endif
                                          );
  return code;
}

/* ------------------------------------------------------------------ LDS-DMA chain */

typedef __attribute__((address_space(3))) void lds_void_t;

/* N 16-byte chunks of one per-lane record at g into the wave's LDS buffer
   chunks buf[j][64] by LDS-DMA from ONE address: chunk j's 16 j bytes are
   the instruction's immediate offset, which the DMA adds to the LDS address
   as well, so its LDS base (M0) is taken 16 j bytes lower -- no address
   arithmetic per chunk.  (The offset must be a constant: a template.) */
template<int J, int N>
__device__ __forceinline__ void glds_chunks( void const * g, uint4 * buf ) {
  if constexpr( J < N ) {
    __builtin_amdgcn_global_load_lds( g, (lds_void_t *)((char *)(buf + 64*J) - 16*J), 16, 16*J, 0 );
    glds_chunks<J+1, N>( g, buf );
  }
}
template<int N>
__device__ __forceinline__ void glds_record( void const * g, uint4 * buf ) { glds_chunks<0, N>( g, buf ); }

/* One table entry (10 x 16 B per lane) into the wave's LDS buffer
   buf[10][64] by LDS-DMA. */
__device__ __forceinline__ void vtab_fetch_lds( uint4 * buf, uint32_t const * vtab, uint64_t cap, uint64_t t, uint32_t db ) {
  uint32_t e = vtab_entry( db );
  FD_DIAG_FETCH_ENTRY( e );
  uint4 const * m; uint4 const * tl;
  vtab_ptrs( vtab, cap, t, e, &m, &tl );
  glds_record<8>( m, buf );
#if FD_VTAB_TAIL
  glds_record<2>( tl, buf + 64*8 );
#endif
}

/* Comb-table entry |d| of position k into buf[8][64]. */
__device__ __forceinline__ void ctab_fetch_lds( uint4 * buf, uint32_t const * ctab, int k, int d ) {
  uint32_t e = min( (uint32_t)(d < 0 ? -d : d), FD_CTAB_HALF );
  uint4 const * p = (uint4 const *)(ctab + ((uint64_t)k * FD_CTAB_N + e) * FD_CTAB_STRIDE);
  glds_record<8>( p, buf );
}

/* The wave's LDS-DMA has landed (this wave's only vector-memory operations
   in flight are its own table fetches). */
__device__ __forceinline__ void dma_wait( void ) {
  FE_FENCE();
  __builtin_amdgcn_s_waitcnt( 0x0f70 );      /* vmcnt(0) */
  FE_FENCE();
}

template<int N>
__device__ __forceinline__ void lds_words( uint32_t w[ 4*N ], uint4 const * buf, int lane ) {
#pragma unroll
  for( int j=0; j<N; j++ ) { uint4 v = buf[ 64*j + lane ]; w[4*j] = v.x; w[4*j+1] = v.y; w[4*j+2] = v.z; w[4*j+3] = v.w; }
}

/* A table entry (NC = 10 16-B chunks) out of the wave's LDS buffer with the
   digit's sign applied to Y+X / Y-X by the read address (FD_VW: chunk c < 5
   holds two limbs of each, 8 bytes apart): w gets Y+X, Y-X (already swapped
   for a negative digit), then 2dT and 2Z in plain order (words 20..39).
   (The comb and key tables keep the plain order: their VGPR readers'
   selects between two words of one 16-B load were compiled into dynamic
   indexing, +1.2K instructions per comb addition in the pair kernel.) */
template<int NC>
__device__ __forceinline__ void lds_entry_words( uint32_t w[ 4*NC ], uint4 const * buf, int lane, bool neg ) {
  char const * b = (char const *)(buf + lane);
  uint32_t sp = neg ? 8u : 0u;
  uint2 const * pp = (uint2 const *)(b + sp);
  uint2 const * pm = (uint2 const *)(b + (8u - sp));
#pragma unroll
  for( int c=0; c<5; c++ ) {
    uint2 x = pp[ c*128 ]; w[2*c] = x.x; w[2*c+1] = x.y;
    uint2 y = pm[ c*128 ]; w[10+2*c] = y.x; w[11+2*c] = y.y;
  }
#pragma unroll
  for( int j=5; j<NC; j++ ) { uint4 v = buf[ 64*j + lane ]; w[4*j] = v.x; w[4*j+1] = v.y; w[4*j+2] = v.z; w[4*j+3] = v.w; }
}

/* The cached entry from lds_entry_words' words: 2dT negated for a negative
   digit (Y+X / Y-X came swapped). */
__device__ __forceinline__ void lds_entry_finish( ge_cached & c, uint32_t const w[ 40 ], bool neg ) {
  fe tv;
#pragma unroll
  for( int j=0; j<10; j++ ) { c.YpX.v[j] = w[j]; c.YmX.v[j] = w[10+j]; tv.v[j] = w[20+j]; c.Z2.v[j] = w[30+j]; }
  fe_cneg( c.T2d, tv, neg );
}

/* Biased digit i (0..16, d_i + 8) of a scalar recoded by ybias_p, held in
   the wave's LDS column block y[8][64] (wave-uniform top position P = 4 (nw-2)
   + wn): windows below nw-2 are nibbles biased by 8, window nw-2 is wn bits
   (1..4) biased by 2^(wn-1), the top digit sits at bit P (it may straddle
   two words); negated when neg. */
__device__ __forceinline__ uint32_t ydig_p( uint32_t const * y, int lane, int i, int nw, int wn, bool neg ) {
  uint32_t db;
  if( i == nw-1 ) {
    int P = 4*(nw-2) + wn, q = P >> 5;
    uint64_t two = (uint64_t)y[ q*64 + lane ] | (q < 7 ? (uint64_t)y[ (q+1)*64 + lane ] << 32 : 0ull);
    db = ((uint32_t)(two >> (P & 31)) & 15u) + 8u;         /* the top digit (<= 8) */
  } else {
    db = (y[ (i >> 3)*64 + lane ] >> (4*(i & 7))) & 15u;
    if( i == nw-2 ) db = (db & ((1u << wn) - 1u)) + 8u - (1u << (wn - 1));
  }
  return neg ? 16u - db : db;
}

/* Windows hi-1 .. lo of the Straus chain acc = [u](-A) + [v](-R) (dsm_loop's
   order: four doublings unless it is the chain's first window, then A's and
   R's entries); entries staged in buf one addition ahead; T computed at the
   last window of the segment (the next phase starts with a doubling or the
   comb). */
__device__ __forceinline__ void chain_seg( ge_p3 & acc, uint4 * buf, uint32_t const * yu, uint32_t const * yv, int lane,
                                           bool uneg, uint32_t const * vtab, uint64_t cap, uint64_t ta, uint64_t tr,
                                           int nw, int hi, int lo, int wn, bool last_t = true ) {
  uint32_t dba = ydig_p( yu, lane, hi-1, nw, wn, uneg );
  vtab_fetch_lds( buf, vtab, cap, ta, dba );
  uint32_t dbr = 0u;
  bool skip_a = false;
#if FD_OPT_FIRSTWIN
  if( hi == nw ) {
    /* the chain's first window (every caller starts a chain at hi = nw
       from the identity): A's entry becomes the point itself
       (ge_from_cached, ~1/4 of an addition), outside the loop so the loop
       body's registers do not grow */
    ge_cached q;
    dma_wait();
    uint32_t w[ 40 ];
    lds_entry_words<10>( w, buf, lane, dba < 8u );
    dbr = ydig_p( yv, lane, hi-1, nw, wn, false );
    FE_FENCE();
    vtab_fetch_lds( buf, vtab, cap, tr, dbr );
    lds_entry_finish( q, w, dba < 8u );
    FE_FENCE();
    ge_from_cached( acc, q );
    FE_FENCE();
    skip_a = true;
  }
#endif
#pragma unroll 1
  for( int i=hi-1; i>=lo; i-- ) {
    if( !skip_a ) {
      if( i < nw-1 ) {
        int nd = i == nw-2 ? wn : 4;                /* window nw-2 is wn bits wide (ybias_p) */
#pragma unroll 1
        for( int j=1; j<nd; j++ ) { ge_dbl( acc, acc, false ); FE_FENCE(); }
        ge_dbl( acc, acc, true );
        FE_FENCE();
      }
      ge_cached q;
      {
        dma_wait();
        uint32_t w[ 40 ];
        lds_entry_words<10>( w, buf, lane, dba < 8u );
        dbr = ydig_p( yv, lane, i, nw, wn, false );
        FE_FENCE();
        vtab_fetch_lds( buf, vtab, cap, tr, dbr );   /* LDS reads issued before the DMA see the old bytes */
        lds_entry_finish( q, w, dba < 8u );
      }
      FE_FENCE();
      ge_add_cached( acc, acc, q, true );
      FE_FENCE();
    }
    skip_a = false;
    ge_cached q;
    {
      dma_wait();
      uint32_t w[ 40 ];
      lds_entry_words<10>( w, buf, lane, dbr < 8u );
      if( i > lo ) dba = ydig_p( yu, lane, i-1, nw, wn, uneg );
      FE_FENCE();
      if( i > lo ) vtab_fetch_lds( buf, vtab, cap, ta, dba );
      lds_entry_finish( q, w, dbr < 8u );
    }
    FE_FENCE();
    ge_add_cached( acc, acc, q, i == lo && last_t );
    FE_FENCE();
  }
}

/* acc += [w]B: the 11 comb-table additions, w's biased digits in yw
   (FD_COMB_POS_RUN: fd_diag.h). */
__device__ __forceinline__ void comb_lds( ge_p3 & acc, uint4 * buf, uint32_t const * yw, int lane, uint32_t const * ctab ) {
#define FD_WDIG( k ) comb_digit_w( yw[ ((23*(k)) >> 5)*64 + lane ], ((23*(k)) >> 5) < 7 ? yw[ (((23*(k)) >> 5) + 1)*64 + lane ] : 0u, (k) )
  int d = FD_WDIG( 0 );
  ctab_fetch_lds( buf, ctab, 0, d );
#pragma unroll 1
  for( int k=0; k<FD_COMB_POS_RUN; k++ ) {
    ge_precomp bp;
    {
      dma_wait();
      uint32_t w[ 32 ];
      lds_words<8>( w, buf, lane );
      int dn = k + 1 < FD_COMB_POS_RUN ? FD_WDIG( k + 1 ) : 0;
      FE_FENCE();
      if( k + 1 < FD_COMB_POS_RUN ) ctab_fetch_lds( buf, ctab, k + 1, dn );
      ctab_finish( bp, w, d );
      d = dn;
    }
    FE_FENCE();
    ge_madd( acc, acc, bp, k + 1 < FD_COMB_POS_RUN );
    FE_FENCE();
  }
#undef FD_WDIG
}

/* acc + [w]B == O, the comb additions of comb_lds but the last: Q = acc + C
   with C = [d_10] B_10 is O iff acc = -C = (-x_C, y_C), i.e. (affine C,
   projective acc, Z != 0 on the curve) 2X + (Y+X - (Y-X))_C Z = 0 and
   2Y - (Y+X + Y-X)_C Z = 0: two products and the two zero tests instead
   of the last mixed addition (7 products), the previous one's T and the
   projective compare.  C's sign flips x_C only, so it is applied to the
   first product.  Comb entries are R (ctab_init: carried sums). */
__device__ __forceinline__ int comb_lds_eq( ge_p3 & acc, uint4 * buf, uint32_t const * yw, int lane, uint32_t const * ctab ) {
#define FD_WDIG( k ) comb_digit_w( yw[ ((23*(k)) >> 5)*64 + lane ], ((23*(k)) >> 5) < 7 ? yw[ (((23*(k)) >> 5) + 1)*64 + lane ] : 0u, (k) )
  int d = FD_WDIG( 0 );
  ctab_fetch_lds( buf, ctab, 0, d );
#pragma unroll 1
  for( int k=0; k<FD_COMB_POS_RUN-1; k++ ) {       /* (FD_COMB_POS_RUN: fd_diag.h) */
    ge_precomp bp;
    {
      dma_wait();
      uint32_t w[ 32 ];
      lds_words<8>( w, buf, lane );
      int dn = FD_WDIG( k + 1 );
      FE_FENCE();
      ctab_fetch_lds( buf, ctab, k + 1, dn );
      ctab_finish( bp, w, d );
      d = dn;
    }
    FE_FENCE();
    ge_madd( acc, acc, bp, k + 2 < FD_COMB_POS_RUN );
    FE_FENCE();
  }
#undef FD_WDIG
  dma_wait();
  fe yp, ym, t1, t2, e;
  {
    uint32_t w[ 32 ];
    lds_words<8>( w, buf, lane );
#pragma unroll
    for( int j=0; j<10; j++ ) { yp.v[j] = w[j]; ym.v[j] = w[10+j]; }
  }
  fe_sub( e, yp, ym );                  /* M: 2 x_C of the unsigned entry */
  fe_mul( t1, e, acc.Z );
  FE_FENCE();
  fe_add( e, yp, ym );                  /* M: 2 y_C */
  fe_mul( t2, e, acc.Z );
  FE_FENCE();
  fe_cneg( t1, t1, d < 0 );
  fe_lshl1_add( e, acc.X, t1 );         /* 2X + 2 x_C Z */
  fe_carry( e, e );
  int ex = fe_is_zero( e );
  fe_add( yp, acc.Y, acc.Y );
  fe_sub( e, yp, t2 );                  /* 2Y - 2 y_C Z */
  fe_carry( e, e );
  int ey = fe_is_zero( e );
  return ex & ey;
}

/* One signature per lane:
     S check -> k = SHA-512(R||A||M) mod l -> (u, v) short vector of k mod 8l,
     w = v S mod l, digits -> LDS -> decode A and R, small-order checks,
     tables [0..8](-A), [0..8](-R) -> Q = [u](-A) + [v](-R) + [w]B -> Q == O
   (Q = [v]([S]B - [k]A - R), fd_lattice_dev.h).  The reported code follows
   the reference's check order (fd_ed25519_user.c:157-228): S, decode A,
   decode R, small-order A, small-order R, equation. */
extern "C" __global__ void __launch_bounds__( 64 * FD_SL_WAVES, FD_SL_WAVES_PER_EU )
fd_ed25519_verify_kernel( verify_args args ) {
  __shared__ uint4    s_buf[ FD_SL_WAVES ][ 10*64 ];     /* a table / comb entry per wave (LDS-DMA) */
  __shared__ uint32_t s_y[ FD_SL_WAVES ][ 24*64 ];       /* per wave: biased u, v, w (8 words each) */

  int tid = (int)threadIdx.x;
  int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane( tid >> 6 );
#ifdef FD_PHASE_STAMPS
  uint64_t _st[ FD_NSTAMP ] = { 0, 0, 0, 0, 0, 0, 0, 0 };
  uint64_t _rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  STAMP( 0 );
  uint64_t gid = (uint64_t)blockIdx.x * (64u * FD_SL_WAVES) + (uint64_t)tid;
  uint64_t cap = args.vtab_cap;
  /* List form (hot-key cache split): the count is known on the device only;
     whole waves past it leave at once (wave-uniform). */
  uint64_t nn = args.cnt ? (uint64_t)*args.cnt : args.n;
  if( (gid & ~(uint64_t)63) >= nn ) return;
  /* Every lane stays to the wave-wide window count below (no early exit):
     lanes past n or with a bad descriptor take the no-work path.  The
     descriptor / signature / key loads are issued first. */
  bool valid = gid < nn;
  uint64_t di = valid ? (args.idx ? (uint64_t)args.idx[ gid ] : gid) : 0u;
  fd_ed25519_desc_t d; d.sig_off = 0u; d.pub_off = 0u; d.msg_off = 0u; d.msg_sz = 0u; d.txn_idx = 0u;
  if( valid ) d = args.desc[ di ];
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
  STAMP( 1 );

  bool bad_s = desc_ok && !sc_lt_l( sig + 8 );                           /* :157-159 */
  bool live  = desc_ok && !bad_s;

  /* k, the lattice vector (u, v), w; their biased digits into this lane's
     LDS column (before the decodes: only they and the sign of u stay live) */
  uint32_t * y = s_y[ wv ];
  int un = 0, nwin = 124;          /* the top-digit position P (ybias_p) */
  {
    uint32_t u[ 8 ], v[ 8 ], w[ 8 ];
    int nbits = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = 0u; v[j] = 0u; w[j] = 0u; }
    if( live ) verify_prep_scalars<true>( u, v, &un, w, &nbits, sig, pub, args, d, lim_dw
#ifdef FD_PHASE_STAMPS
                                    , _st
#endif
                                    );
    int P = wave_top_pos( nbits );                  /* the chain's doublings (ybias_p) */
    uint32_t t[ 8 ];
    ybias_p( t, u, P );
#pragma unroll
    for( int j=0; j<8; j++ ) y[ j*64 + lane ] = t[j];
    ybias_p( t, v, P );
#pragma unroll
    for( int j=0; j<8; j++ ) y[ (8 + j)*64 + lane ] = t[j];
    comb_bias( t, w );
#pragma unroll
    for( int j=0; j<8; j++ ) y[ (16 + j)*64 + lane ] = t[j];
    nwin = P;
  }
  FE_FENCE();

  /* decode A then R (:162 frombytes_2x), small order (:193-198), tables;
     the two encodings wait in the wave's (still idle) LDS-DMA buffer, so
     they hold no registers across the decodes */
  STAMP( 3 );
  uint32_t * encs = (uint32_t *)s_buf[ wv ];
#pragma unroll
  for( int j=0; j<8; j++ ) { encs[ j*64 + lane ] = pub[j]; encs[ (8 + j)*64 + lane ] = sig[j]; }
  int st[ 2 ] = { 0, 0 };
  if( live ) {
#pragma unroll 1
    for( int q=0; q<2; q++ ) {
      uint32_t enc[ 8 ];
#pragma unroll
      for( int j=0; j<8; j++ ) enc[j] = encs[ (8*q + j)*64 + lane ];
      ge_p3 Q;
      int sm;
      int ok = ge_decode_small( Q, enc, !args.ref_codes, &sm );
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
  int code = verify_precode( args, desc_ok, bad_s, stA, stR );
  if( code == 0 ) {
    /* Q = [u](-A) + [v](-R) + [w]B, Q == O  (:225-228 on [v]D) */
    int P = __builtin_amdgcn_readfirstlane( nwin );
    int nw = ((P + 3) >> 2) + 1, wn = P - 4*(nw - 2);  /* ybias_p's windows */
    ge_p3 acc; ge_identity( acc );
    chain_seg( acc, s_buf[ wv ], y, y + 8*64, lane, un != 0, args.vtab, cap, gid, cap/2u + gid, nw, nw, 0, wn );
#if FD_OPT_COMBCHK
    int eq = comb_lds_eq( acc, s_buf[ wv ], y + 16*64, lane, args.ctab );
    STAMP( 5 );
#else
    comb_lds( acc, s_buf[ wv ], y + 16*64, lane, args.ctab );
    STAMP( 5 );
    fe dl;
    int ex = fe_is_zero( acc.X );
    fe_sub( dl, acc.Y, acc.Z ); fe_carry( dl, dl );
    int eq = ex & fe_is_zero( dl );
#endif
    code = eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  }
  args.out[ di ] = (int8_t)code;
#ifdef FD_PHASE_STAMPS
  STAMP( 6 );
  if( args.stamps && (tid & 63) == 0 ) {
    /* 0-1 prologue, 1-2 SHA (live lanes), 2-3 lattice+digits, 3-4 decodes+tables, 4-5 chain+comb, 5-6 compare */
    for( int i=0; i<6; i++ ) atomicAdd( &args.stamps[i], (unsigned long long)(_st[i+1] - _st[i]) );
    atomicAdd( &args.stamps[7], 1ull );
    /* the wave's clock (MI355X_MICROARCH.md DVFS item 6): s_memtime cycles and
       s_memrealtime ticks (100 MHz) from start to end, per wave of the launch */
    uint64_t gw = (uint64_t)blockIdx.x * FD_SL_WAVES + (uint64_t)wv;
    if( FD_TL_BASE + 2u*gw + 1u < FD_STAMP_WORDS_DEV ) {
      args.stamps[ FD_TL_BASE + 2u*gw ] = _st[6] - _st[0];
      args.stamps[ FD_TL_BASE + 2u*gw + 1u ] = __builtin_amdgcn_s_memrealtime() - _rt0;
    }
  }
#endif
}

/* Pair form of the verify kernel, for batches of at most one 256-signature
   workgroup per CU (config 2's 64K = one wave per SIMD): a 512-thread
   workgroup gives every signature two lanes in two waves of the same SIMD
   pair slot -- waves 0-3 (role 0) and waves 4-7 (role 1) hold signatures
   [256 b, 256 b + 256).  Role 0 does the S check, SHA-512, lattice and
   digits while role 1 waits at the first barrier; then BOTH run the same
   decode + table code at once -- role 0 on A, role 1 on R -- so that phase
   has two waves per SIMD (the single-wave kernel issues one VALU op per ~4.9
   cycles per SIMD; two waves of the same code fill more of the issue slots;
   same code, so no extra instruction-cache footprint); role 1 leaves the
   status of R in LDS, computes [w]B (the 11 comb additions) beside role 0's
   chain and hands it over in LDS (cached form) at the second barrier; role 0
   runs the Straus chain and adds it.  Bit-identical results to
   fd_ed25519_verify_kernel (same functions, same order of checks).
   Measured at 64K, launches of both kernels alternated in one process
   (tools/ab_kernels.py): 0.672 ms vs 0.683 ms for the single-lane kernel
   (FD_ED25519_GPU_PAIR=0); the decode pairing alone 0.678.  Waves go to SIMDs round-robin (wave i -> SIMD
   i mod 4): pairing roles by odd/even wave instead put two chain waves on
   one SIMD and ran 1.44x slower.  Starting R's decode during role 0's
   SHA-512 (different code side by side) gained nothing over this order. */
extern "C" __global__ void __launch_bounds__( 2 * FD_VERIFY_BLOCK, 2 )
fd_ed25519_verify_pair_kernel( verify_args args ) {
  __shared__ uint8_t  s_dig[ FD_ROWS * FD_VERIFY_BLOCK ];
  __shared__ uint8_t  s_stR[ FD_VERIFY_BLOCK ];
  __shared__ uint32_t s_wb[ FD_VTAB_WORDS * FD_VERIFY_BLOCK ];   /* [w]B, cached form, from role 1 */

  int role = (int)threadIdx.x >> 8;                  /* wave-uniform */
  int tid  = (int)threadIdx.x & (FD_VERIFY_BLOCK - 1);
  uint64_t gid = (uint64_t)blockIdx.x * FD_VERIFY_BLOCK + (uint64_t)tid;
  uint64_t cap = args.vtab_cap;
  uint64_t nn  = args.n;
  /* no early return before the barriers: waves past n skip the work only */
  bool wave_live = (gid & ~(uint64_t)63) < nn;
  bool valid = gid < nn;
  fd_ed25519_desc_t d; d.sig_off = 0u; d.pub_off = 0u; d.msg_off = 0u; d.msg_sz = 0u; d.txn_idx = 0u;
  if( valid ) d = args.desc[ gid ];
  uint64_t asz = args.arena_sz;
  bool desc_ok = valid && (uint64_t)d.sig_off + 64u <= asz && (uint64_t)d.pub_off + 32u <= asz &&
                 (uint64_t)d.msg_off + d.msg_sz <= asz;
  uint32_t lim_dw = (uint32_t)((asz + 3u) >> 2) + 1u;

  uint32_t sig[ 16 ], pub[ 8 ];
#pragma unroll
  for( int j=0; j<16; j++ ) sig[j] = 0u;
#pragma unroll
  for( int j=0; j<8; j++ ) pub[j] = 0u;
  if( desc_ok ) {
    load_words<16>( sig, args.arena, d.sig_off, lim_dw );
    if( !role ) load_words<8>( pub, args.arena, d.pub_off, lim_dw );
  }
  bool bad_s = desc_ok && !sc_lt_l( sig + 8 );                           /* :157-159 */
  bool live  = desc_ok && !bad_s;
  uint8_t * drow = s_dig + tid;

  if( !role && wave_live ) {
    verify_prep_digits( drow, FD_VERIFY_BLOCK, tid, live, sig, pub, args, d, lim_dw
#ifdef FD_PHASE_STAMPS
                        , nullptr
#endif
                        );
  }
  FE_FENCE();
  __syncthreads();

  /* role 0: A = pub, role 1: R = sig[0:32] -- one decode + table each, at once */
  int stq = 0;
  if( live ) {
    uint32_t enc[ 8 ];
#pragma unroll
    for( int j=0; j<8; j++ ) enc[j] = role ? sig[j] : pub[j];
    ge_p3 Q;
    int sm;
    int ok = ge_decode_small( Q, enc, !args.ref_codes, &sm );
    FE_FENCE();
    if( ok && !sm ) vtab_build( args.vtab, cap, (uint64_t)role*cap/2u + gid, Q );
    stq = (ok ? 1 : 0) | (sm ? 2 : 0);
    FE_FENCE();
  }
  if( role ) s_stR[ tid ] = (uint8_t)stq;
  if( role ) {
    /* [w]B beside role 0's chain (11 comb additions; w digits came before
       the first barrier) */
    ge_p3 c;
    ge_cached cc;
    comb_only( c, drow, args.ctab );
    ge_to_cached( cc, c );
#pragma unroll
    for( int j=0; j<10; j++ ) {
      s_wb[ (j     )*FD_VERIFY_BLOCK + tid ] = cc.YpX.v[j]; s_wb[ (10 + j)*FD_VERIFY_BLOCK + tid ] = cc.YmX.v[j];
      s_wb[ (20 + j)*FD_VERIFY_BLOCK + tid ] = cc.T2d.v[j]; s_wb[ (30 + j)*FD_VERIFY_BLOCK + tid ] = cc.Z2.v[j];
    }
  }
  __syncthreads();
  if( role || !valid ) return;

  int code = verify_tail( args, desc_ok, bad_s, stq, (int)s_stR[ tid ], drow, s_dig, tid, gid, s_wb
#ifdef FD_PHASE_STAMPS
                          , nullptr
#endif
                          );
  args.out[ gid ] = (int8_t)code;
}

/* Pipelined form (throughput): one launch runs three phases of three
   consecutive batches side by side, in the three 256-thread thirds of
   768-thread workgroups (waves i, i+4, i+8 share SIMD i: three waves per
   SIMD, none of them idle):
     waves 8-11 (phase A), batch j:   descriptor / S checks, SHA-512, lattice
       vector (u, v), w = v S mod l;
     waves 4-7  (phase B), batch j-1: decode A, small-order A, A's table,
       decode R, small-order R, R's table, the check-order code, then the
       TOP kb windows of the Straus chain;
     waves 0-3  (phase C), batch j-2: the remaining windows, the 11 comb
       additions of [w]B and the compare.
   Why: config 2 is one 64-signature wave per SIMD; a single wave issues a
   VALU instruction per ~4.6 cycles, the SIMD takes one per ~4.05 from
   several (tools/fe_probe2.hip, profiles/r02/probes).  The SIMD's arbiter
   serves the oldest wave first, so the phases run nearly one after the
   other (C, then B, then A in the leftover issue slots) and the launch ends
   with the last one alone (profiles/r02/s3/stamps_*): phase A -- the
   youngest wave, whose code waits on memory most -- is kept short (A's
   decode and table moved to phase B: -1.6 %; R's moved to phase A instead:
   +4.8 %).
   A batch crosses the launches in HBM: phase A leaves R's and A's
   encodings, the digit scalars (u, v, w plus their recoding bias, so each
   consumer reads its signed digits straight off the bits), a status byte
   per slot and the window count per wave; phase B leaves the partial sum
   (X, Y, Z, T) and the code of the checks.  The chain phases stage their table entries
   in LDS by LDS-DMA (global_load_lds_dwordx4), one entry ahead, instead
   of in 40 VGPRs: 168 VGPRs are the budget of three waves per SIMD.  Same
   device functions and check order as fd_ed25519_verify_kernel:
   bit-identical codes. */
/* SHA-512 block count of R || A || M (the length-order key, clamped). */
__device__ __forceinline__ uint32_t len_bucket( fd_ed25519_desc_t const & d ) {
  uint32_t b = (64u + (uint32_t)d.msg_sz + 17u + 127u) >> 7;
  return min( b, (uint32_t)FD_LEN_NB - 1u );
}

/* Phase A's descriptor order inside a full workgroup (256 descriptors): a
   wave runs the SHA-512 loop for its longest message, so the four phase-A
   waves of a workgroup take the 256 descriptors ordered by block count (a
   counting sort over the four waves' ballots, through LDS) instead of 64
   consecutive ones each.  With Uniform{0..1232}-B messages a wave's longest
   is then the 1/4..4/4 quantile of 256 instead of the maximum every time.
   Returns the descriptor index (within the workgroup) slot t = w*64 + lane
   takes.  The four waves wait for each other on LDS counters zeroed by the
   workgroup's barrier at kernel start (bounded waits: all four are resident
   in the workgroup, so they arrive).  An expired wait stores errv (the
   batch's pipe counter + 1) into *err, the batch's word of the host-mapped
   error ring. */
__device__ __forceinline__ uint32_t pipe_len_order( uint32_t key, int w, int lane, uint32_t * wh, uint32_t * perm,
                                                    uint32_t * flag, uint32_t * err, uint32_t errv ) {
  uint64_t below = (1ull << lane) - 1ull;
  uint32_t mine = 0, rank = 0;
#pragma unroll 1
  for( uint32_t b=0; b<(uint32_t)FD_LEN_NB; b++ ) {
    uint64_t m = __ballot( key == b );
    if( lane == (int)b ) mine = (uint32_t)__popcll( m );
    if( key == b ) rank = (uint32_t)__popcll( m & below );
  }
  if( lane < FD_LEN_NB ) wh[ w*FD_LEN_NB + lane ] = mine;
  __builtin_amdgcn_fence( __ATOMIC_RELEASE, "workgroup" );
  if( lane == 0 ) __hip_atomic_fetch_add( &flag[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP );
  uint32_t i;
  for( i=0; i<FD_LSORT_SPIN && __hip_atomic_load( &flag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP ) < 4u; i++ )
    __builtin_amdgcn_s_sleep( 1 );
  /* an expired wait (impossible while the four waves are co-resident, as
     one workgroup's waves are) leaves the counts partial: the order below is
     then not a permutation, so the launch reports it (the host turns the
     error word into FD_ED25519_GPU_ERR_LAUNCH) instead of returning codes */
  int late = __hip_atomic_load( &flag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP ) < 4u;
  __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "workgroup" );
  uint32_t pos = rank;
#pragma unroll 1
  for( uint32_t b=0; b<(uint32_t)FD_LEN_NB; b++ ) {
    uint32_t c0 = wh[ b ], c1 = wh[ FD_LEN_NB + b ], c2 = wh[ 2*FD_LEN_NB + b ], c3 = wh[ 3*FD_LEN_NB + b ];
    uint32_t tot = c0 + c1 + c2 + c3;
    uint32_t pre = (w > 0 ? c0 : 0u) + (w > 1 ? c1 : 0u) + (w > 2 ? c2 : 0u);
    pos += b < key ? tot : (b == key ? pre : 0u);
  }
  perm[ pos & (FD_VERIFY_BLOCK - 1u) ] = (uint32_t)(w*64 + lane);
  __builtin_amdgcn_fence( __ATOMIC_RELEASE, "workgroup" );
  if( lane == 0 ) __hip_atomic_fetch_add( &flag[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP );
  for( i=0; i<FD_LSORT_SPIN && __hip_atomic_load( &flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP ) < 4u; i++ )
    __builtin_amdgcn_s_sleep( 1 );
  late |= __hip_atomic_load( &flag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP ) < 4u;
  __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "workgroup" );
  if( late && lane == 0 && err ) __hip_atomic_store( err, errv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
  return perm[ w*64 + lane ] & (FD_VERIFY_BLOCK - 1u);   /* in the workgroup's range whatever happened */
}

#define FD_PIPE_ST_VALID  0x80      /* phase A status byte                    */
#define FD_PIPE_ST_DESC   0x01      /* descriptor inside the arena            */
#define FD_PIPE_ST_BADS   0x02      /* S >= l                                 */
#define FD_PIPE_ST_UNEG   0x10      /* the lattice u is negated               */

/* The wave's digit scalars (words [w0, w0 + nwords) of the hand-off, row
   stride cap) into its LDS column block y[nwords][64]. */
__device__ __forceinline__ void hand_to_lds( uint32_t * y, uint32_t const * hand, uint64_t cap, uint64_t gid, int lane,
                                             int w0, int nwords ) {
  /* all loads first, then the LDS stores: one memory round trip at the
     wave's start instead of one per word (a rolled loop waited for each) */
  uint32_t t[ 24 ];
#if FD_DIAG_NO_HAND_ON
  (void)hand; (void)cap;
#pragma unroll
  for( int j=0; j<24; j++ ) t[j] = j < nwords ? fd_diag_hash( gid, (uint32_t)(w0 + j) ) & (j % 8 == 7 ? 0x0fffffffu : ~0u) : 0u;
#else
#pragma unroll
  for( int j=0; j<24; j++ ) t[j] = j < nwords ? hand[ (uint64_t)(w0 + j)*cap + gid ] : 0u;
#endif
#pragma unroll
  for( int j=0; j<24; j++ ) if( j < nwords ) y[ j*64 + lane ] = t[j];
}

__device__ __forceinline__ uint32_t pipe_aparse( fparse_args const & a, uint32_t * s_ap, int wv, int lane );
__device__ __forceinline__ fd_ed25519_desc_t desc_ld_coh( fd_ed25519_desc_t const * p );

extern "C" __global__ void __launch_bounds__( 3 * FD_VERIFY_BLOCK, 1 )
fd_ed25519_verify_pipe_kernel( pipe_args a ) {
  __shared__ uint4    s_buf[ 2 ][ 4 ][ 10*64 ];       /* phase C / B: a table entry per wave      */
  __shared__ uint32_t s_y[ 2 ][ 4 ][ 24*64 ];         /* phase C / B: u, v, w digit scalars       */
  __shared__ uint32_t s_lo[ 4*FD_LEN_NB + FD_VERIFY_BLOCK + 2 ];   /* phase A: length order (pipe_len_order) */
  __shared__ uint32_t s_ap[ 8 ];                                    /* phase A: in-launch parse (pipe_aparse) */
  if( threadIdx.x < 2 ) s_lo[ 4*FD_LEN_NB + FD_VERIFY_BLOCK + threadIdx.x ] = 0u;
  if( threadIdx.x < 8 ) s_ap[ threadIdx.x ] = 0u;
  __syncthreads();
  /* 0: phase C, 1: phase B, 2: phase A -- the thirds' waves are created in
     this order and the SIMD's arbiter favours the oldest (the other five
     orders measured 2.5-5 % slower) */
  int role = __builtin_amdgcn_readfirstlane( (int)threadIdx.x >> 8 );
  int tid  = (int)threadIdx.x & (FD_VERIFY_BLOCK - 1);
  int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane( tid >> 6 );
  uint64_t gid = (uint64_t)blockIdx.x * FD_VERIFY_BLOCK + (uint64_t)tid;
  uint64_t cap = a.sig_cap;
  verify_args const & args = a.v;
  uint64_t vcap = args.vtab_cap;
  switch( (int)(a.prio >> (2*role)) & 3 ) {            /* wave priority (age decides among equals) */
    case 1:  __builtin_amdgcn_s_setprio( 1 ); break;
    case 2:  __builtin_amdgcn_s_setprio( 2 ); break;
    case 3:  __builtin_amdgcn_s_setprio( 3 ); break;
    default: break;
  }
#ifdef FD_PHASE_STAMPS
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
  /* per-wave timeline of the launch (the last one before the context closes):
     start / end on the constant-rate clock, HW_ID and XCC_ID, cycles */
#define FD_TL_STAMP() do {                                                                              \
    if( args.stamps && lane == 0 ) {                                                                    \
      unsigned long long * tl = args.stamps + FD_TL_BASE + ((uint64_t)blockIdx.x * 12u + (uint64_t)(role*4 + wv)) * 4u; \
      uint64_t rt1 = __builtin_amdgcn_s_memrealtime();                                                  \
      uint32_t hw = __builtin_amdgcn_s_getreg( (31 << 11) | 4 ), xcc = __builtin_amdgcn_s_getreg( (15 << 11) | 20 ); \
      tl[0] = rt0; tl[1] = rt1; tl[2] = ((uint64_t)xcc << 32) | hw; tl[3] = __builtin_amdgcn_s_memtime() - t0; \
    } } while( 0 )
#else
#define FD_TL_STAMP() do {} while( 0 )
#endif

  if( role == 2 ) {
    /* ---- phase A, batch j ---- */
    uint64_t nn = args.n;                                               /* args.cnt: a device-side count <= n */
#if FD_OPT_APARSE
    if( a.aparse )                   /* the batch's frags parsed in this launch: the count this workgroup may use */
      nn = min( nn, (uint64_t)__builtin_amdgcn_readfirstlane( (int)pipe_aparse( a.fp, s_ap, wv, lane ) ) );
    else
#endif
    if( args.cnt ) nn = min( nn, (uint64_t)__builtin_amdgcn_readfirstlane( (int)*args.cnt ) );
    uint64_t b0 = (uint64_t)blockIdx.x * FD_VERIFY_BLOCK, di = gid;   /* di: the descriptor this lane verifies */
#if FD_DIAG_NO_ARENA_ON
    fd_ed25519_desc_t dsyn; dsyn.sig_off = 0u; dsyn.pub_off = 64u; dsyn.msg_off = 96u; dsyn.msg_sz = 200u; dsyn.txn_idx = 0u;
#define FD_PIPE_DESC( i ) dsyn
#else
#define FD_PIPE_DESC( i ) (a.aparse ? desc_ld_coh( args.desc + (i) ) : args.desc[ (i) ])
#endif
    if( a.lsort && b0 + FD_VERIFY_BLOCK <= nn )                       /* full workgroups only: all four waves here */
      di = b0 + pipe_len_order( len_bucket( FD_PIPE_DESC( gid ) ), wv, lane, s_lo, s_lo + 4*FD_LEN_NB,
                                s_lo + 4*FD_LEN_NB + FD_VERIFY_BLOCK,
                                a.err ? a.err + (a.seq % FD_PIPE_ERR_RING) : nullptr, (uint32_t)a.seq + 1u );
    if( (gid & ~(uint64_t)63) >= nn ) {
      if( gid < args.n ) a.st_a[ gid ] = 0u;             /* past a device-side count: no batch slot */
      return;
    }
    bool valid = gid < nn;
    fd_ed25519_desc_t d; d.sig_off = 0u; d.pub_off = 0u; d.msg_off = 0u; d.msg_sz = 0u; d.txn_idx = 0u;
    if( valid ) d = FD_PIPE_DESC( di );
#undef FD_PIPE_DESC
    uint64_t asz = args.arena_sz;
    bool desc_ok = valid && (uint64_t)d.sig_off + 64u <= asz && (uint64_t)d.pub_off + 32u <= asz &&
                   (uint64_t)d.msg_off + d.msg_sz <= asz;
    uint32_t lim_dw = (uint32_t)((asz + 3u) >> 2) + 1u;
    uint32_t sig[ 16 ], pub[ 8 ];
#pragma unroll
    for( int j=0; j<16; j++ ) sig[j] = 0u;
#pragma unroll
    for( int j=0; j<8; j++ ) pub[j] = 0u;
    if( desc_ok ) {
#if FD_DIAG_NO_ARENA_ON
#pragma unroll
      for( int j=0; j<8; j++ ) { sig[j] = fd_diag_bp_word( j ); pub[j] = fd_diag_bp_word( j ); }
#pragma unroll
      for( int j=0; j<8; j++ ) sig[8+j] = j < 7 ? fd_diag_hash( gid, 100u + (uint32_t)j ) : 0x0fffffffu & fd_diag_hash( gid, 107u );
#else
#if FD_OPT_APRIO
      FE_FENCE(); __builtin_amdgcn_s_setprio( 3 ); FE_FENCE();
#endif
      load_words<16>( sig, args.arena, d.sig_off, lim_dw );
      load_words<8> ( pub, args.arena, d.pub_off, lim_dw );
#if FD_OPT_APRIO
      FE_FENCE(); __builtin_amdgcn_s_setprio( 0 ); FE_FENCE();
#endif
#endif
    }
    bool bad_s = desc_ok && !sc_lt_l( sig + 8 );                         /* :157-159 */
    bool live  = desc_ok && !bad_s;
    uint32_t u[ 8 ], v[ 8 ], w[ 8 ];
    int un = 0, nbits = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = 0u; v[j] = 0u; w[j] = 0u; }
    if( live ) verify_prep_scalars<false>( u, v, &un, w, &nbits, sig, pub, args, d, lim_dw
#ifdef FD_PHASE_STAMPS
                                    , nullptr
#endif
                                    , a.kpre ? a.kpre + 8u*di : nullptr );
    FE_FENCE();
    int P = wave_top_pos( nbits );                  /* the chain's doublings (ybias_p) */
    if( valid ) {
      uint32_t * h = a.hand_a + gid;
#if FD_DIAG_NO_HAND_ON
      /* every hand-off word folded into one store that never happens */
      uint32_t sink = 0u;
#define FD_HAND_ST( row, v ) (sink ^= (v))
#else
#define FD_HAND_ST( row, v ) (h[ (uint64_t)(row)*cap ] = (v))
#endif
      uint32_t y[ 8 ];
#pragma unroll
      for( int j=0; j<8; j++ ) FD_HAND_ST( FD_PH_R + j, sig[j] );
      ybias_p( y, u, P );
#pragma unroll
      for( int j=0; j<8; j++ ) FD_HAND_ST( FD_PH_YU + j, y[j] );
      ybias_p( y, v, P );
#pragma unroll
      for( int j=0; j<8; j++ ) FD_HAND_ST( FD_PH_YV + j, y[j] );
      comb_bias( y, w );
#pragma unroll
      for( int j=0; j<8; j++ ) FD_HAND_ST( FD_PH_YW + j, y[j] );
#pragma unroll
      for( int j=0; j<8; j++ ) FD_HAND_ST( FD_PH_A + j, pub[j] );
      FD_HAND_ST( FD_PH_IDX, (uint32_t)di );
      if( a.first_a ) {
        uint32_t f0 = a.aparse ? __hip_atomic_load( (uint32_t *)a.first_a + d.txn_idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT )
                               : a.first_a[ d.txn_idx ];
        FD_HAND_ST( FD_PH_FRAG, (uint32_t)d.txn_idx | ((uint32_t)(di - f0) << 16) );
      }
#undef FD_HAND_ST
#if FD_DIAG_NO_HAND_ON
      if( sink == 0xdeadbeefu && di == 0xffffffffu ) h[ 0 ] = sink;
#endif
    }
    if( lane == 0 ) a.nw_a[ gid >> 6 ] = (uint8_t)P;     /* the wave's top-digit position */
    FE_FENCE();
    if( gid < args.n )
      a.st_a[ gid ] = !valid ? (uint8_t)0 : (uint8_t)(FD_PIPE_ST_VALID | (desc_ok ? FD_PIPE_ST_DESC : 0) | (bad_s ? FD_PIPE_ST_BADS : 0) |
                                (un ? FD_PIPE_ST_UNEG : 0));
#ifdef FD_PHASE_STAMPS
    if( args.stamps && lane == 0 ) { atomicAdd( &args.stamps[2], (unsigned long long)(__builtin_amdgcn_s_memtime() - t0) ); atomicAdd( &args.stamps[5], 1ull ); }
#endif
    FD_TL_STAMP();
    return;
  }

  /* ---- phases B (batch j-1) and C (batch j-2): one copy of the chain code
     for both (two copies of its ~30 KB window loop would not share the
     instruction cache) ---- */
  uint4 *    buf = s_buf[ role ][ wv ];
  uint32_t * y   = s_y[ role ][ wv ];
  bool phb = role == 1;
  FD_DIAG_PHASE_BC_ENTRY();
  uint64_t nx = phb ? a.n_b : a.n_c;
  if( (gid & ~(uint64_t)63) >= nx ) return;
  uint64_t set = phb ? a.set_b : a.set_c;
  uint32_t const * hand = phb ? a.hand_b : a.hand_c;
  int ps = gid < nx ? (int)(phb ? a.st_b : a.st_c)[ gid ] : 0;
  bool valid = (ps & FD_PIPE_ST_VALID) != 0;            /* phase A marked the batch's slots */
  /* the status bits read after the decodes travel as wave ballots (SGPR
     pairs): kept as the byte, ps was the kernel's one spilled VGPR */
  uint64_t m_uneg = __ballot( (ps & FD_PIPE_ST_UNEG) != 0 );
  uint64_t m_desc = __ballot( (ps & FD_PIPE_ST_DESC) != 0 ), m_bads = __ballot( (ps & FD_PIPE_ST_BADS) != 0 );
  if( !__ballot( valid ) ) return;                      /* a wave past a device-side count */
  int code;
  if( phb ) {
    bool desc_ok = (m_desc >> lane) & 1u, bad_s = (m_bads >> lane) & 1u;
    int stA = 0, stR = 0;
    if( desc_ok && !bad_s ) {                         /* A: decode, small order, table */
      uint32_t enc[ 8 ];
#pragma unroll
      for( int j=0; j<8; j++ ) enc[j] = FD_DIAG_NO_HAND_ON ? fd_diag_bp_word( j ) : hand[ (uint64_t)(FD_PH_A + j)*cap + gid ];
      ge_p3 Q;
      int sm;
      int ok = ge_decode_small( Q, enc, !args.ref_codes, &sm );
      FE_FENCE();
      if( ok && !sm ) vtab_build( args.vtab, vcap, (2u*set)*cap + gid, Q );
      stA = (ok ? 1 : 0) | (sm ? 2 : 0);
      FE_FENCE();
    }
    /* A's status as two wave ballots (SGPRs) and R's encoding addressed from
       an opaque copy of gid: neither a status VGPR nor the hand-off address
       stays live across R's decode (both were spilled at 168 VGPRs) */
    uint64_t m_aok = __ballot( (stA & 1) != 0 ), m_asm = __ballot( (stA & 2) != 0 );
    uint64_t gr = gid;
    asm volatile( "" : "+v"(gr) );
    if( desc_ok && !bad_s ) {                         /* R = sig[0:32]: decode, small order, table */
      uint32_t enc[ 8 ];
#pragma unroll
      for( int j=0; j<8; j++ ) enc[j] = FD_DIAG_NO_HAND_ON ? fd_diag_bp_word( j ) : hand[ (uint64_t)(FD_PH_R + j)*cap + gr ];
      ge_p3 Q;
      int sm;
      int ok = ge_decode_small( Q, enc, !args.ref_codes, &sm );
      FE_FENCE();
      bool aok = (m_aok >> lane) & 1u, asm_ = (m_asm >> lane) & 1u;
      if( ok && !sm && aok && !asm_ ) vtab_build( args.vtab, vcap, (2u*set + 1u)*cap + gid, Q );
      stR = (ok ? 1 : 0) | (sm ? 2 : 0);
      FE_FENCE();
    }
    stA = (int)((m_aok >> lane) & 1u) | (int)(((m_asm >> lane) & 1u) << 1);
    FD_DIAG_AFTER_TABLES();
    code = verify_precode( args, desc_ok, bad_s, stA, stR );
    if( valid && !FD_DIAG_NO_HAND_ON ) a.code_b[ gid ] = (int8_t)code;
  } else {
    code = valid && !FD_DIAG_NO_HAND_ON ? (int)a.code_c[ gid ] : 0;
  }
  bool run = valid && code == 0;
  int P = __builtin_amdgcn_readfirstlane( (int)(phb ? a.nw_b : a.nw_c)[ gid >> 6 ] );
  int nw = ((P + 3) >> 2) + 1, wn = P - 4*(nw - 2);    /* ybias_p's windows */
  int split = max( nw - (int)a.kb, 0 );
  int hi = phb ? nw : split, lo = phb ? split : 0;
  ge_p3 acc;
  if( run ) {
    hand_to_lds( y, hand, cap, gid, lane, FD_PH_YU, phb ? 16 : 24 );
    if( phb || FD_DIAG_NO_HAND_ON ) ge_identity( acc );
    else {
      uint32_t const * o = a.acc_c + gid;
#pragma unroll
      for( int j=0; j<10; j++ ) {
        acc.X.v[j] = o[ (uint64_t)j*cap ]; acc.Y.v[j] = o[ (uint64_t)(10+j)*cap ];
        acc.Z.v[j] = o[ (uint64_t)(20+j)*cap ];
        if( !FD_OPT_BNOT ) acc.T.v[j] = o[ (uint64_t)(30+j)*cap ];    /* BNOT: the first doubling writes T before any read */
      }
    }
    FE_FENCE();
    if( hi > lo )
      chain_seg( acc, buf, y, y + 8*64, lane, ((m_uneg >> lane) & 1u) != 0, args.vtab, vcap,
                 (2u*set)*cap + gid, (2u*set + 1u)*cap + gid, nw, hi, lo, wn, !(FD_OPT_BNOT && phb) );
    FE_FENCE();
    if( phb ) {
      uint32_t * o = a.acc_b + gid;
#if FD_DIAG_NO_HAND_ON
      /* the partial sum folded into one store that never happens */
      uint32_t sink = 0u;
#pragma unroll
      for( int j=0; j<10; j++ ) sink ^= acc.X.v[j] ^ acc.Y.v[j] ^ acc.Z.v[j] ^ (FD_OPT_BNOT ? 0u : acc.T.v[j]);
      if( sink == 0xdeadbeefu && acc.X.v[0] == 0xdeadbeefu ) o[ 0 ] = sink;
#else
#pragma unroll
      for( int j=0; j<10; j++ ) {
        o[ (uint64_t)j*cap ] = acc.X.v[j]; o[ (uint64_t)(10+j)*cap ] = acc.Y.v[j];
        o[ (uint64_t)(20+j)*cap ] = acc.Z.v[j];
        if( !FD_OPT_BNOT ) o[ (uint64_t)(30+j)*cap ] = acc.T.v[j];
      }
#endif
    } else {
#if FD_OPT_COMBCHK
      /* [w]B and Q == O (:225-228 on [v]D) folded into the last comb entry */
      int eq = comb_lds_eq( acc, buf, y + 16*64, lane, args.ctab );
#else
      comb_lds( acc, buf, y + 16*64, lane, args.ctab );
      /* Q == O  <=>  X == 0 and Y == Z (:225-228 on [v]D) */
      fe dl;
      int ex = fe_is_zero( acc.X );
      fe_sub( dl, acc.Y, acc.Z ); fe_carry( dl, dl );
      int eq = ex & fe_is_zero( dl );
#endif
      code = eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
    }
  }
  if( !phb && valid ) {
    uint32_t di = FD_DIAG_NO_HAND_ON ? (uint32_t)gid : hand[ (uint64_t)FD_PH_IDX*cap + gid ];
    a.out_c[ di ] = (int8_t)code;
    if( a.fold_c ) {
      /* frag batch: the code's class into its field of the frag's fold word
         and the count down, one relaxed atomic (no fence: the word is its own
         record); the add that ends the count writes the frag's record */
      uint32_t fw = hand[ (uint64_t)FD_PH_FRAG*cap + gid ];
      uint32_t fi = fw & 0xffffu, k = fw >> 16;
      uint64_t cls = code == FD_ED25519_SUCCESS ? 0u : code == FD_ED25519_ERR_MSG ? 1u : code == FD_ED25519_ERR_SIG ? 2u :
                     code == FD_ED25519_ERR_PUBKEY ? 3u : 4u;
      uint64_t delta = (cls << (FD_FOLD_SH + 3u*k)) - 1u;
      uint64_t old = __hip_atomic_fetch_add( a.fold_c + fi, delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
      if( (old & 0xffu) == 1u ) {
        uint64_t w = (old + delta) >> FD_FOLD_SH;
        int st = FD_ED25519_SUCCESS, any_msg = 0;
#pragma unroll 1
        for( int j=0; j<16; j++, w >>= 3 ) {       /* first phase-1 error by index, else ERR_MSG, else SUCCESS */
          uint32_t c = (uint32_t)w & 7u;
          if( c == 1u ) any_msg = 1;
          else if( c ) { st = c == 2u ? FD_ED25519_ERR_SIG : c == 3u ? FD_ED25519_ERR_PUBKEY : FD_ED25519_GPU_CODE_BAD_DESC; break; }
        }
        if( st == FD_ED25519_SUCCESS && any_msg ) st = FD_ED25519_ERR_MSG;
        uint64_t tag = a.ftag_c[ fi ];
        ((uint4 *)a.frec_c)[ fi ] = make_uint4( (uint32_t)tag, (uint32_t)(tag >> 32), (uint32_t)(int32_t)st, 0u );
      }
    }
  }
#ifdef FD_PHASE_STAMPS
  if( args.stamps && lane == 0 ) { atomicAdd( &args.stamps[phb ? 1 : 0], (unsigned long long)(__builtin_amdgcn_s_memtime() - t0) ); atomicAdd( &args.stamps[phb ? 6 : 7], 1ull ); }
#endif
  FD_TL_STAMP();
}

/* ------------------------------------------------------------------ SHA-512 batch */

/* Batched SHA-512, one message per lane (replaces fd_sha512_batch_init /
   _add / _fini, src/ballet/sha512/fd_sha512.h:223-408, and fd_sha512_hash
   fd_sha512.c:399).  Messages are (off, sz) pairs into one arena; digest i
   goes to out[64 i .. 64 i + 63].  Each block's dwords are fetched one block
   ahead (the fetch of block b covers message bytes [128 b, 128 b + 128) plus
   the misalignment word). */
__device__ __forceinline__ void sha_fetch_msg( uint32_t raw[ 33 ], uint32_t const * a32, uint32_t off, uint32_t b,
                                               uint32_t lim_dw ) {
  uint32_t start = (off >> 2) + 32u*b;
#pragma unroll
  for( int i=0; i<33; i++ ) raw[i] = a32[ min( start + (uint32_t)i, lim_dw ) ];
}

extern "C" __global__ void __launch_bounds__( 256 )
fd_sha512_batch_kernel( uint8_t const * arena, uint64_t arena_sz, fd_sha512_gpu_msg_t const * msg, uint64_t n,
                        uint8_t * out ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  fd_sha512_gpu_msg_t m = msg[ i ];
  uint32_t lim_dw = (uint32_t)((arena_sz + 3u) >> 2) + 1u;
  uint32_t const * a32 = (uint32_t const *)arena;
  uint32_t sz = m.sz, sh = m.off & 3u;
  uint32_t nblk = (sz + 17u + 127u) >> 7;
  uint64_t h[ 8 ]; sha512_init_state( h );
  uint32_t nxt[ 33 ];
  sha_fetch_msg( nxt, a32, m.off, 0u, lim_dw );
  for( uint32_t b=0; b<nblk; b++ ) {
    uint32_t raw[ 33 ];
#pragma unroll
    for( int j=0; j<33; j++ ) raw[j] = nxt[j];
    if( b + 1u < nblk ) sha_fetch_msg( nxt, a32, m.off, b + 1u, lim_dw );
    uint64_t W[ 16 ];
#pragma unroll
    for( int j=0; j<16; j++ ) {
      int32_t mo = (int32_t)((b << 7) + 8u*(uint32_t)j);            /* message byte of the word's first byte */
      uint32_t w0 = __builtin_amdgcn_alignbyte( raw[2*j+1], raw[2*j],   sh );
      uint32_t w1 = __builtin_amdgcn_alignbyte( raw[2*j+2], raw[2*j+1], sh );
      uint32_t hi = sha_bswap32( w0 ), lo = sha_bswap32( w1 );
      int32_t rem0 = (int32_t)sz - mo, rem1 = rem0 - 4;
      uint32_t keep0 = rem0 >= 4 ? 0xffffffffu : (rem0 <= 0 ? 0u : ~(0xffffffffu >> (8*rem0)));
      uint32_t keep1 = rem1 >= 4 ? 0xffffffffu : (rem1 <= 0 ? 0u : ~(0xffffffffu >> (8*rem1)));
      uint32_t pad0  = (rem0 >= 0 && rem0 < 4) ? (0x80000000u >> (8*rem0)) : 0u;
      uint32_t pad1  = (rem1 >= 0 && rem1 < 4) ? (0x80000000u >> (8*rem1)) : 0u;
      hi = (hi & keep0) | pad0;
      lo = (lo & keep1) | pad1;
      if( b == nblk-1u && j == 15 ) { hi = sz >> 29; lo = sz << 3; }
      if( b == nblk-1u && j == 14 ) { hi = 0u; lo = 0u; }
      W[j] = ((uint64_t)hi << 32) | lo;
    }
    sha512_compress( h, W );
  }
  uint4 * o = (uint4 *)(out + 64u*i);
#pragma unroll
  for( int q=0; q<4; q++ )
    o[q] = make_uint4( sha_bswap32( (uint32_t)(h[2*q]   >> 32) ), sha_bswap32( (uint32_t)h[2*q]   ),
                       sha_bswap32( (uint32_t)(h[2*q+1] >> 32) ), sha_bswap32( (uint32_t)h[2*q+1] ) );
}

/* ------------------------------------------------------------------ SHA-256 batch */

/* Batched SHA-256, one message per lane (replaces fd_sha256_hash,
   src/ballet/sha256/fd_sha256.c, and the fd_sha256_batch_* API of
   src/ballet/sha256/fd_sha256.h): digest i = SHA-256( arena[off, off + sz) )
   to out[32 i .. 32 i + 31]. */
extern "C" __global__ void __launch_bounds__( 256 )
fd_sha256_batch_kernel( uint8_t const * arena, uint64_t arena_sz, fd_sha512_gpu_msg_t const * msg, uint64_t n,
                        uint8_t * out ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  fd_sha512_gpu_msg_t m = msg[ i ];
  uint32_t lim_dw = (uint32_t)((arena_sz + 3u) >> 2) + 1u;
  uint32_t const pw[ 8 ] = { 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u };
  uint32_t h[ 8 ];
  sha256_span( h, pw, 0u, arena, m.off, m.sz, lim_dw );
  uint4 * o = (uint4 *)(out + 32u*i);
  o[0] = make_uint4( s256_bswap( h[0] ), s256_bswap( h[1] ), s256_bswap( h[2] ), s256_bswap( h[3] ) );
  o[1] = make_uint4( s256_bswap( h[4] ), s256_bswap( h[5] ), s256_bswap( h[6] ), s256_bswap( h[7] ) );
}

/* The shred Merkle roots of the FEC resolver's signature check
   (src/disco/shred/fd_fec_resolver.c:334-399; fd_bmtree_hash_leaf /
   fd_bmtree_commitp_insert_with_proof, src/ballet/bmtree/fd_bmtree.c:
   385-420), one shred per lane: the leaf over the protected bytes (~18
   blocks), then per proof layer one node hash of 26 + 20 + 20 bytes (two
   blocks), left / right by the index bit; the 32-byte root is written into
   the device arena where the verify kernel reads it as the message. */
extern "C" __global__ void __launch_bounds__( 256 )
fd_shred_root_kernel( shred_root_args a ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= a.n ) return;
  fd_shred_job_t j = a.job[ i ];
  uint32_t lim_dw = (uint32_t)((a.arena_sz + 3u) >> 2) + 1u;
  uint32_t const leaf[ 8 ] = { 0x00534f4cu, 0x414e415fu, 0x4d45524bu, 0x4c455f53u,      /* "\0SOLANA_MERKLE_SHREDS_LEAF" */
                               0x48524544u, 0x535f4c45u, 0x41460000u, 0x00000000u };
  uint32_t h[ 8 ];
  sha256_span( h, leaf, 26u, a.arena, j.leaf_off, j.leaf_len, lim_dw );
  uint32_t const np[ 7 ] = { 0x01534f4cu, 0x414e415fu, 0x4d45524bu, 0x4c455f53u,      /* "\1SOLANA_MERKLE_SHREDS_NODE" */
                             0x48524544u, 0x535f4e4fu, 0x44450000u };
#pragma unroll 1
  for( uint32_t l=0; l<j.depth; l++ ) {
    uint32_t sib[ 5 ];
    load_words<5>( sib, a.arena, j.proof_off + 20u*l, lim_dw );
    uint32_t nd[ 5 ], L[ 5 ], R[ 5 ];
    int right = (j.idx >> l) & 1u;                 /* this node is the right child */
#pragma unroll
    for( int k=0; k<5; k++ ) {
      nd[k] = h[k];                                /* a node is the hash's first 20 bytes */
      uint32_t sk = s256_bswap( sib[k] );
      L[k] = right ? sk : nd[k];
      R[k] = right ? nd[k] : sk;
    }
    uint32_t W[ 16 ];
#pragma unroll
    for( int k=0; k<6; k++ ) W[k] = np[k];
    W[6]  = np[6] | (L[0] >> 16);
#pragma unroll
    for( int k=0; k<4; k++ ) W[7+k] = (L[k] << 16) | (L[k+1] >> 16);
    W[11] = (L[4] << 16) | (R[0] >> 16);
#pragma unroll
    for( int k=0; k<4; k++ ) W[12+k] = (R[k] << 16) | (R[k+1] >> 16);
    sha256_init_state( h );
    sha256_compress( h, W );
    W[0] = (R[4] << 16) | 0x8000u;
#pragma unroll
    for( int k=1; k<15; k++ ) W[k] = 0u;
    W[15] = 66u * 8u;
    sha256_compress( h, W );
  }
  uint8_t * o = a.arena + j.out_off;
#pragma unroll
  for( int k=0; k<8; k++ ) {
    o[4*k] = (uint8_t)(h[k] >> 24); o[4*k+1] = (uint8_t)(h[k] >> 16); o[4*k+2] = (uint8_t)(h[k] >> 8); o[4*k+3] = (uint8_t)h[k];
  }
}

/* ------------------------------------------------------------------ hot-key cache */

/* Build the comb tables of newly cached keys, one key per lane: decode A
   under both builds' rules, small-order status, then [j](2^(w p) (-A)) for
   p < FD_KTAB_POS, j in [1, FD_KTAB_ENT] as affine precomputed records (one
   inversion each: this runs once per key, at fd_ed25519_gpu_keycache_add). */
extern "C" __global__ void __launch_bounds__( 256 )
fd_ed25519_ktab_build_kernel( uint32_t * ktab, uint32_t * kmeta, uint32_t const * pubs, uint32_t const * slots,
                              uint64_t n ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  uint32_t pub[ 8 ];
#pragma unroll
  for( int j=0; j<8; j++ ) pub[j] = pubs[ i*8u + (uint64_t)j ];
  uint64_t slot = slots[ i ];
  ge_p3 A, A2;
  int sm, sm2;
  int ok_ref = ge_decode_small( A, pub, false, &sm );
  int ok_avx = ge_decode_small( A2, pub, true, &sm2 );
  uint32_t * m = kmeta + slot * FD_KMETA_WORDS;
#pragma unroll
  for( int j=0; j<8; j++ ) m[j] = pub[j];
  m[8] = (ok_ref ? FD_KST_OK_REF : 0u) | (ok_avx ? FD_KST_OK_AVX : 0u) | (sm ? FD_KST_SMALL : 0u);
  if( !ok_ref || sm ) return;                       /* such a key never reaches the equation */
  ge_p3 base = A;
  { fe x; fe_neg( x, A.X ); fe_carry( base.X, x ); fe_neg( x, A.T ); fe_carry( base.T, x ); }
  uint32_t * kt = ktab + slot * (uint64_t)FD_KTAB_WORDS;
#pragma unroll 1
  for( int p=0; p<FD_KTAB_POS; p++ ) {
    ge_precomp bp; ge_affine_precomp( bp, base );   /* base := affine */
    ge_p3 P = base;
#pragma unroll 1
    for( int j=1; j<=FD_KTAB_ENT; j++ ) {
      if( j == 2 ) ge_dbl( P, base, true );
      else if( j > 2 ) ge_madd( P, P, bp, true );
      ge_precomp e;
      if( j == 1 ) e = bp;
      else ge_affine_precomp( e, P );
      uint32_t * r = kt + (uint64_t)(p*FD_KTAB_ENT + (j-1)) * 32u;
#pragma unroll
      for( int w=0; w<10; w++ ) { r[w] = e.YpX.v[w]; r[10+w] = e.YmX.v[w]; r[20+w] = e.T2d.v[w]; }
      r[30] = 0u; r[31] = 0u;
    }
    ge_dbl( P, P, true );                           /* [2^w] base: the next position's base */
    base = P;
  }
}

/* Split a batch by key: descriptors whose public key is cached go to the
   hit list (with its slot), the rest (and out-of-arena descriptors) to the
   miss list.  One lane per descriptor; list appends are wave-aggregated. */
extern "C" __global__ void __launch_bounds__( 256 )
fd_ed25519_kcache_part_kernel( kpart_args a ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t nn = a.ncnt ? min( a.n, (uint64_t)*a.ncnt ) : a.n;
  if( (i & ~(uint64_t)63) >= nn ) return;
  bool valid = i < nn;
  int64_t slot = -1;
  if( valid ) {
    fd_ed25519_desc_t d = a.desc[ i ];
    if( (uint64_t)d.pub_off + 32u <= a.arena_sz ) {
      uint32_t lim_dw = (uint32_t)((a.arena_sz + 3u) >> 2) + 1u;
      uint32_t pub[ 8 ];
      load_words<8>( pub, a.arena, d.pub_off, lim_dw );
      uint64_t h = fd_kcache_hash( pub[0], pub[1], a.seed ) & a.hmask;
      for( uint64_t probe=0; probe<=a.hmask; probe++ ) {
        uint32_t e = a.khash[ h ];
        if( !e ) break;
        uint32_t const * m = a.kmeta + (uint64_t)(e - 1u) * FD_KMETA_WORDS;
        uint32_t diff = 0u;
#pragma unroll
        for( int j=0; j<8; j++ ) diff |= m[j] ^ pub[j];
        if( !diff ) { slot = (int64_t)(e - 1u); break; }
        h = (h + 1u) & a.hmask;
      }
    }
  }
  bool hit = valid && slot >= 0, miss = valid && slot < 0;
  uint64_t bh = __ballot( hit ), bm = __ballot( miss );
  uint32_t lane = threadIdx.x & 63u;
  uint64_t below = lane ? (~0ull >> (64u - lane)) : 0ull;
  uint32_t base_h = 0u, base_m = 0u;
  if( lane == 0u ) {
    if( bh ) base_h = atomicAdd( &a.counts[0], (uint32_t)__popcll( bh ) );
    if( bm ) base_m = atomicAdd( &a.counts[1], (uint32_t)__popcll( bm ) );
  }
  base_h = __shfl( base_h, 0 ); base_m = __shfl( base_m, 0 );
  if( hit )  { uint32_t o = base_h + (uint32_t)__popcll( bh & below ); a.hit_idx[ o ] = (uint32_t)i; a.hit_slot[ o ] = (uint32_t)slot; }
  if( miss ) { uint32_t o = base_m + (uint32_t)__popcll( bm & below ); a.miss_idx[ o ] = (uint32_t)i; }
}

/* ------------------------------------------------------------------ length buckets */

/* Descriptor order by SHA-512 block count inside segments of FD_LEN_SEG
   consecutive descriptors (one 1024-thread workgroup per segment, counting
   sort in LDS): waves then hash messages of one block count, and a wave's
   lanes still read arena bytes from one segment (a global sort scattered
   them over the whole arena: the message loads then missed the TLB and the
   1M-signature launch took 1.9x as long). */
extern "C" __global__ void __launch_bounds__( 1024 )
fd_len_sort_kernel( len_args a ) {
  __shared__ uint32_t h[ FD_LEN_NB ], cur[ FD_LEN_NB ];
  uint64_t lo = (uint64_t)blockIdx.x * FD_LEN_SEG;
  if( lo >= a.n ) return;
  uint32_t m = (uint32_t)min( (uint64_t)FD_LEN_SEG, a.n - lo );
  uint32_t tid = threadIdx.x;
  if( tid < FD_LEN_NB ) h[ tid ] = 0u;
  __syncthreads();
  for( uint32_t j=tid; j<m; j+=1024u ) atomicAdd( &h[ len_bucket( a.desc[ lo + j ] ) ], 1u );
  __syncthreads();
  if( tid == 0u ) {   /* longest first: the segment's last workgroups are its shortest (a shorter launch tail) */
    uint32_t c = 0u;
    for( int k=FD_LEN_NB-1; k>=0; k-- ) { cur[k] = c; c += h[k]; }
  }
  __syncthreads();
  for( uint32_t j=tid; j<m; j+=1024u ) {
    uint32_t o = atomicAdd( &cur[ len_bucket( a.desc[ lo + j ] ) ], 1u );
    a.idx[ lo + o ] = (uint32_t)(lo + j);
  }
}

/* k = SHA-512(R || A || M) mod l ahead of the pipelined kernel (kpre_args,
   fd_ed25519_gpu_abi.h): lane i hashes descriptor idx[i] (length order, so a
   wave's messages have similar block counts) with the one-shot kernels'
   hash (message fetched a block ahead, interior blocks without padding
   masks) and stores k at k[8 di].  Descriptors outside the arena get no
   hash (phase A never reads their k). */
extern "C" __global__ void __launch_bounds__( 256 )
fd_ed25519_kpre_kernel( kpre_args a ) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if( (i & ~(uint64_t)63) >= a.n ) return;                      /* whole waves past n */
  bool valid = i < a.n;
  uint64_t di = valid ? (a.idx ? (uint64_t)a.idx[ i ] : i) : 0u;
  fd_ed25519_desc_t d; d.sig_off = 0u; d.pub_off = 0u; d.msg_off = 0u; d.msg_sz = 0u; d.txn_idx = 0u;
  if( valid ) d = a.desc[ di ];
  uint64_t asz = a.arena_sz;
  bool ok = valid && (uint64_t)d.sig_off + 64u <= asz && (uint64_t)d.pub_off + 32u <= asz &&
            (uint64_t)d.msg_off + d.msg_sz <= asz;
  uint32_t lim_dw = (uint32_t)((asz + 3u) >> 2) + 1u;
  uint32_t R[ 8 ], A[ 8 ], k[ 8 ];
#pragma unroll
  for( int j=0; j<8; j++ ) { R[j] = 0u; A[j] = 0u; k[j] = 0u; }
  if( ok ) {
    load_words<8>( R, a.arena, d.sig_off, lim_dw );
    load_words<8>( A, a.arena, d.pub_off, lim_dw );
  }
  if( !ok ) d.msg_sz = 0u;                                         /* (every lane takes part in the wave's loop) */
  hash_ram<true>( k, R, A, a.arena, d.msg_off, d.msg_sz, lim_dw );
  if( ok ) {
    uint4 * o = (uint4 *)(a.k + 8u*di);
    o[0] = make_uint4( k[0], k[1], k[2], k[3] ); o[1] = make_uint4( k[4], k[5], k[6], k[7] );
  }
}

/* Key-table entry j (digit d != 0: entry |d|; d == 0: the identity record
   after the slots) of position p. */
__device__ __forceinline__ void ktab_fetch( uint32_t w[ 32 ], uint32_t const * ktab, uint64_t kcap, uint64_t slot,
                                            int p, int d ) {
  uint32_t e = (uint32_t)(d < 0 ? -d : d);
  uint32_t const * r = e ? ktab + slot * (uint64_t)FD_KTAB_WORDS + (uint64_t)(p*FD_KTAB_ENT + (int)e - 1) * 32u
                         : ktab + kcap * (uint64_t)FD_KTAB_WORDS;
  uint4 const * q = (uint4 const *)r;
#pragma unroll
  for( int j=0; j<8; j++ ) { uint4 v = q[j]; w[4*j] = v.x; w[4*j+1] = v.y; w[4*j+2] = v.z; w[4*j+3] = v.w; }
}

/* Signed w-bit digit p of a 256-bit scalar (w = FD_KTAB_WBITS divides 32),
   carry threaded by the caller (digits in [-2^(w-1), 2^(w-1)), the top one
   keeps its carry). */
__device__ __forceinline__ int nib_digit( uint32_t const x[ 8 ], int p, int * c ) {
  int const w = FD_KTAB_WBITS, per = 32 / FD_KTAB_WBITS;
  int d = (int)((x[p/per] >> (w*(p%per))) & ((1u << w) - 1u)) + *c;
  *c = d >= (1 << (w-1)) && p < FD_KTAB_POS-1;
  return d - (*c << w);
}

/* Verify with a cached key: the reference equation itself,
   [S]B + [k](-A) == R (fd_ed25519_user.c:208-228), as FD_KTAB_POS mixed additions
   from the key's comb table plus 16 from the fixed-base comb table -- no
   doublings, no lattice, no decode of A, no per-signature tables -- then
   the projective compare against the decoded R.  Codes follow the same
   check order as the main kernel (the key's decode / small-order status
   comes from the cache). */
extern "C" __global__ void __launch_bounds__( FD_VERIFY_BLOCK, FD_VERIFY_WAVES_PER_EU )
fd_ed25519_verify_cached_kernel( verify_args args ) {
  uint64_t gid = (uint64_t)blockIdx.x * FD_VERIFY_BLOCK + (uint64_t)threadIdx.x;
  uint64_t nn = (uint64_t)*args.cnt;
  if( (gid & ~(uint64_t)63) >= nn ) return;
  bool valid = gid < nn;
  uint64_t di = valid ? (uint64_t)args.idx[ gid ] : 0u;
  uint64_t slot = valid ? (uint64_t)args.slot[ gid ] : 0u;
  fd_ed25519_desc_t d; d.sig_off = 0u; d.pub_off = 0u; d.msg_off = 0u; d.msg_sz = 0u; d.txn_idx = 0u;
  if( valid ) d = args.desc[ di ];
  uint64_t asz = args.arena_sz;
  bool desc_ok = valid && (uint64_t)d.sig_off + 64u <= asz && (uint64_t)d.pub_off + 32u <= asz &&
                 (uint64_t)d.msg_off + d.msg_sz <= asz;
  uint32_t lim_dw = (uint32_t)((asz + 3u) >> 2) + 1u;
  uint32_t sig[ 16 ], pub[ 8 ];
#pragma unroll
  for( int j=0; j<16; j++ ) sig[j] = 0u;
#pragma unroll
  for( int j=0; j<8; j++ ) pub[j] = 0u;
  if( desc_ok ) {
    load_words<16>( sig, args.arena, d.sig_off, lim_dw );
    load_words<8> ( pub, args.arena, d.pub_off, lim_dw );
  }
  uint32_t st = valid ? args.kmeta[ slot * FD_KMETA_WORDS + 8u ] : 0u;
  bool bad_s = desc_ok && !sc_lt_l( sig + 8 );                           /* :157-159 */
  bool live  = desc_ok && !bad_s;
  uint32_t k[ 8 ];
#pragma unroll
  for( int j=0; j<8; j++ ) k[j] = 0u;
  if( live ) hash_ram<true>( k, sig, pub, args.arena, d.msg_off, d.msg_sz, lim_dw );   /* :203-206 */
  FE_FENCE();
  ge_p3 R;
  int smR;
  int okR = ge_decode_small( R, sig, !args.ref_codes, &smR );             /* :162 (R after A) */
  bool okA = (st & (args.ref_codes ? FD_KST_OK_REF : FD_KST_OK_AVX)) != 0u;
  int code;
  if     ( !desc_ok            ) code = FD_ED25519_GPU_CODE_BAD_DESC;
  else if( bad_s               ) code = FD_ED25519_ERR_SIG;
  else if( !okA                ) code = args.ref_codes ? FD_ED25519_ERR_PUBKEY : FD_ED25519_ERR_SIG;   /* :190-192 */
  else if( !okR                ) code = FD_ED25519_ERR_SIG;
  else if( st & FD_KST_SMALL   ) code = FD_ED25519_ERR_PUBKEY;                                        /* :193-195 */
  else if( smR                 ) code = FD_ED25519_ERR_SIG;                                           /* :196-198 */
  else                           code = 0;
  bool run = code == 0;
  if( __any( run ) ) {
    /* lanes not running the equation use slot 0 / digit 0 (valid memory) */
    uint64_t sl = run ? slot : 0u;
    uint32_t kk[ 8 ], ss[ 8 ];
#pragma unroll
    for( int j=0; j<8; j++ ) { kk[j] = run ? k[j] : 0u; ss[j] = run ? sig[8+j] : 0u; }
    ge_p3 acc; ge_identity( acc );
    uint32_t raw[ 32 ];
    int ck = 0;
    int dk = nib_digit( kk, 0, &ck );
    ktab_fetch( raw, args.ktab, args.kcap, sl, 0, dk );
#pragma unroll 1
    for( int p=0; p<FD_KTAB_POS; p++ ) {
      ge_precomp e;
      ctab_finish( e, raw, dk );
      if( p + 1 < FD_KTAB_POS ) { dk = nib_digit( kk, p + 1, &ck ); ktab_fetch( raw, args.ktab, args.kcap, sl, p + 1, dk ); }
      FE_FENCE();
      ge_madd( acc, acc, e, true );
      FE_FENCE();
    }
    /* + [S]B from the fixed-base comb table (signed 23-bit comb digits of
       S < l, fd_scalar_dev.h; lanes that do not run have S = 0) */
    uint32_t ys[ 8 ];
    comb_bias( ys, ss );
    int ds = comb_digit( ys, 0 );
    ctab_fetch( raw, args.ctab, 0, ds );
#pragma unroll 1
    for( int q=0; q<FD_CTAB_POS; q++ ) {
      ge_precomp e;
      ctab_finish( e, raw, ds );
      if( q + 1 < FD_CTAB_POS ) {
        /* the next digit by shifting ys down 23 bits (no dynamic register index) */
#pragma unroll
        for( int j=0; j<7; j++ ) ys[j] = __builtin_amdgcn_alignbit( ys[j+1], ys[j], 23u );
        ys[7] >>= 23;
        ds = (int)(ys[0] & ((1u << 23) - 1u)) - (q + 1 < 10 ? (1 << 22) : 0);
        ctab_fetch( raw, args.ctab, q + 1, ds );
      }
      FE_FENCE();
      ge_madd( acc, acc, e, q + 1 < FD_CTAB_POS );
      FE_FENCE();
    }
    if( run ) code = ge_eq_z1( acc, R ) ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;   /* :225-228 */
  }
  if( valid ) args.out[ di ] = (int8_t)code;
}

/* ------------------------------------------------------------------ frag parsing */

/* The verify tile's per-frag checks and field reads (fd_verify.c:92-115,
   fd_verify.h:49-60) on the GPU, one frag per lane, over a device copy of
   the batch's frag span; the same logic as frag_parse in fd_verify_stage.cpp
   (the host form), with one difference: a signature / pubkey / message
   region outside the copied span (impossible for fd_txn_parse output) is
   BAD_FRAG here. */
__device__ __forceinline__ uint32_t span_ld16( uint8_t const * p ) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

/* Exclusive prefix sum over the FD_FRAG_BLOCK threads of a workgroup
   (wavefront scan by lane shifts, then the four wave totals through LDS);
   *tot gets the workgroup's sum.  Every thread of the workgroup calls it. */
__device__ __forceinline__ uint32_t frag_block_scan( uint32_t x, uint32_t * wsum, uint32_t * tot ) {
  uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t v = x;
#pragma unroll
  for( uint32_t o=1u; o<64u; o<<=1 ) { uint32_t y = __shfl_up( v, o, 64 ); if( lane >= o ) v += y; }
  __syncthreads();                                   /* wsum free (a previous call's readers done) */
  if( lane == 63u ) wsum[ w ] = v;
  __syncthreads();
  uint32_t pre = 0u, all = 0u;
#pragma unroll
  for( uint32_t k=0; k<FD_FRAG_BLOCK/64u; k++ ) { pre += k < w ? wsum[ k ] : 0u; all += wsum[ k ]; }
  *tot = all;
  return pre + v - x;
}

/* Decoupled look-back (single-pass scan across tiles of FD_FRAG_BLOCK
   frags): tile t publishes its aggregate, then sums its predecessors' words
   64 at a time (one per lane) until one of them carries an inclusive
   prefix, and publishes its own.  Word: epoch (32) | status (2: 1
   aggregate, 2 inclusive prefix) | value (30); a word of an older epoch is
   "not yet".  Called by one whole wave; returns the exclusive prefix
   (uniform).  The wait is bounded (*late on expiry; the batch then fails). */
#define FD_LB_AGG    1ull
#define FD_LB_PREFIX 2ull
#define FD_LB_SPIN   (1u << 22)
__device__ __forceinline__ uint32_t frag_lookback( uint64_t * flag, uint64_t t, uint32_t agg, uint32_t epoch, int * late ) {
  uint32_t lane = threadIdx.x & 63u;
  uint64_t ep = (uint64_t)epoch << 32;
  if( t == 0u ) {
    if( lane == 0u ) __hip_atomic_store( flag, ep | (FD_LB_PREFIX << 30) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
    return 0u;
  }
  if( lane == 0u ) __hip_atomic_store( flag + t, ep | (FD_LB_AGG << 30) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  uint32_t excl = 0u, spin = 0u;
  int64_t top = (int64_t)t - 1;
  for(;;) {
    int64_t k = top - (int64_t)lane;             /* lane l reads predecessor top - l; none left: a prefix of 0 */
    uint64_t w = k >= 0 ? __hip_atomic_load( flag + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ) : (ep | (FD_LB_PREFIX << 30));
    uint64_t stt = (w >> 30) & 3ull;
    bool ready = (w & 0xffffffff00000000ull) == ep && stt != 0ull;
    uint64_t pre = __ballot( ready && stt >= FD_LB_PREFIX );   /* FD_LB_DONE (in-launch parse) is a prefix too */
    uint64_t need = pre ? ((pre & (~pre + 1ull)) << 1) - 1ull : ~0ull;   /* lanes up to the nearest prefix */
    if( __ballot( !ready ) & need ) {
      if( ++spin > FD_LB_SPIN ) { *late = 1; break; }
      __builtin_amdgcn_s_sleep( 1 );
      continue;
    }
    uint32_t v = ((need >> lane) & 1ull) ? (uint32_t)(w & 0x3fffffffull) : 0u;
#pragma unroll
    for( int o=32; o>=1; o>>=1 ) v += __shfl_xor( v, o );
    excl += v;
    if( pre ) break;
    top -= 64;
  }
  if( lane == 0u )
    __hip_atomic_store( flag + t, ep | (FD_LB_PREFIX << 30) | ((excl + agg) & 0x3fffffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  return excl;
}

/* The per-frag parse, the descriptor-index scan and the descriptors in one
   launch (round 4 ran parse + scan, then an emit launch; the fold of the
   codes now runs in the pipelined kernel's phase C).  Workgroup g takes
   tiles g, g + G, g + 2G, ... (G = the grid, at most one workgroup per CU,
   all co-resident): each tile scans its frags' signature counts, takes its
   base from the look-back over the tiles before it -- tile t's
   predecessors are earlier tiles of co-resident workgroups, each of which
   runs its tiles in order, so every wait ends whatever order the workgroups
   were dispatched in -- and every lane writes its frag's descriptors at
   base + its exclusive count; the last tile writes the batch's total.  Per
   frag: status, tag, first descriptor index, and the fold words (min key
   ~0, the descriptor count) the phase-C fold counts down. */
/* One frag's checks and fields (frag i of the batch; i >= n: BAD_FRAG, no
   descriptors): status, tag, signature count and the descriptor fields. */
struct frag_fields { int st; uint64_t tag; uint32_t cnt, so, po, mo, ms; };
__device__ __forceinline__ frag_fields frag_parse_one( fparse_args const & a, uint64_t i ) {
  frag_fields r; r.st = FD_TXN_VERIFY_BAD_FRAG; r.tag = 0u; r.cnt = 0u; r.so = 0u; r.po = 0u; r.mo = 0u; r.ms = 0u;
  fd_ed25519_gpu_frag_t f; f.off = 0xffffffffu; f.sz = 0u;
  if( i < a.n ) f = a.frag[ i ];
  uint64_t off = f.off, sz = f.sz;
  do {
    if( off > a.arena_sz || sz > a.arena_sz - off || sz < 2u ) break;          /* fd_verify.c:94-96 */
    if( off < a.span_lo || off + sz > a.span_lo + a.span_sz ) break;
    uint64_t ro = off - a.span_lo, re = ro + sz;                                /* the frag, span-relative */
    uint64_t psz = span_ld16( a.span + re - 2u );                               /* :98 */
    if( psz > 2086u ) break;                                                    /* :101-103 */
    uint64_t t = ro + psz + ((a.host_parity + off + psz) & 1u);                  /* :108 align_up( addr, 2 ) */
    if( t + 14u > re ) break;                    /* every field read lies inside the frag (fd_txn_parse output does) */
    uint8_t const * txn = a.span + t;
    if( span_ld16( txn + 12 ) >= psz ) break;                                   /* :112-115 */
    uint64_t c = txn[1];
    uint64_t s_ = ro + span_ld16( txn + 2 ), p_ = ro + span_ld16( txn + 10 ), m_ = span_ld16( txn + 4 );
    if( s_ + 8u > re ) break;
    uint8_t const * sg = a.span + s_;
#pragma unroll
    for( int b=7; b>=0; b-- ) r.tag = (r.tag << 8) | sg[b];
    if( m_ > psz || psz > sz ) break;
    if( !c || c > 16u ) { r.st = FD_TXN_VERIFY_FAILED; break; }                /* batch_sz 0 or > 16 -> ERR_SIG */
    if( c * FD_FRAG_SIG_BYTES > sz ) break;                                     /* more signatures than the frag holds */
    if( s_ + 64u*c > re || p_ + 32u*c > re ) break;
    r.st = 0; r.cnt = (uint32_t)c; r.so = (uint32_t)s_; r.po = (uint32_t)p_; r.mo = (uint32_t)(ro + m_); r.ms = (uint32_t)(psz - m_);
  } while( 0 );
  return r;
}

/* Descriptor stores and loads that are coherent across the XCDs inside one
   launch (agent-scope relaxed atomics: write-through stores, loads that do
   not hit a stale L2 line), for the pipelined kernel's in-launch parse: its
   phase-A waves read descriptors other workgroups -- on other XCDs, whose
   L2s are not coherent with this one -- wrote in the same launch.  No fence
   with a cache operation is needed: the data never sits dirty in an L2. */
__device__ __forceinline__ void desc_st_coh( fd_ed25519_desc_t * p, fd_ed25519_desc_t const & d ) {
  uint64_t lo = (uint64_t)d.sig_off | ((uint64_t)d.pub_off << 32);
  uint64_t hi = (uint64_t)d.msg_off | ((uint64_t)d.msg_sz << 32) | ((uint64_t)d.txn_idx << 48);
  __hip_atomic_store( (uint64_t *)p,     lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  __hip_atomic_store( (uint64_t *)p + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
}
__device__ __forceinline__ fd_ed25519_desc_t desc_ld_coh( fd_ed25519_desc_t const * p ) {
  uint64_t lo = __hip_atomic_load( (uint64_t *)p,     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  uint64_t hi = __hip_atomic_load( (uint64_t *)p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  fd_ed25519_desc_t d;
  d.sig_off = (uint32_t)lo; d.pub_off = (uint32_t)(lo >> 32);
  d.msg_off = (uint32_t)hi; d.msg_sz = (uint16_t)(hi >> 32); d.txn_idx = (uint16_t)(hi >> 48);
  return d;
}

/* Frag i's outputs: status, tag, first descriptor index, fold word, the
   host record of a frag without descriptors, and its descriptors
   (coherent stores for the in-launch parse). */
template<bool COH>
__device__ __forceinline__ void frag_write( fparse_args const & a, uint64_t i, frag_fields const & r, uint32_t first ) {
  if( i >= a.n ) return;
  a.status[ i ] = (int8_t)r.st; a.tag[ i ] = r.tag;
  if( COH ) __hip_atomic_store( a.first + i, first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  else      a.first[ i ] = first;
  a.fold[ i ] = r.cnt;
  if( r.st ) ((uint4 *)a.hrec)[ i ] = make_uint4( (uint32_t)r.tag, (uint32_t)(r.tag >> 32), (uint32_t)(int32_t)r.st, 0u );   /* no descriptors: final */
  for( uint32_t j=0; j<r.cnt && (uint64_t)first + j < a.desc_cap; j++ ) {
    fd_ed25519_desc_t d;
    d.sig_off = r.so + 64u*j; d.pub_off = r.po + 32u*j; d.msg_off = r.mo;
    d.msg_sz = (uint16_t)r.ms; d.txn_idx = (uint16_t)i;
    if( COH ) desc_st_coh( a.desc + first + j, d );
    else      a.desc[ first + j ] = d;
  }
}

extern "C" __global__ void __launch_bounds__( FD_FRAG_BLOCK )
fd_frag_parse_kernel( fparse_args a ) {
  __shared__ uint32_t wsum[ FD_FRAG_BLOCK / 64u ];
  __shared__ uint32_t s_base;
  uint64_t ntile = (a.n + FD_FRAG_BLOCK - 1u) / FD_FRAG_BLOCK;
  for( uint64_t tl=blockIdx.x; tl<ntile; tl+=gridDim.x ) {
    uint64_t i = tl * FD_FRAG_BLOCK + threadIdx.x;
    frag_fields r = frag_parse_one( a, i );
    uint32_t btot;
    uint32_t excl = frag_block_scan( r.cnt, wsum, &btot );                      /* (its first barrier frees s_base) */
    if( threadIdx.x < 64u ) {                                                   /* wave 0: the look-back */
      int late = 0;
      uint32_t base = frag_lookback( a.flag, tl, btot, a.epoch, &late );
      if( threadIdx.x == 0u ) {
        s_base = base;
        if( late && a.err ) __hip_atomic_store( a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
        if( tl == ntile - 1u ) *a.total = base + btot;
      }
    }
    __syncthreads();
    frag_write<false>( a, i, r, s_base + excl );
  }
}

/* The pipelined kernel's in-launch parse (frag batches, pipe_args.aparse):
   the four phase-A waves of every workgroup take the batch's tiles of 256
   frags from a counter, in order (tile IDs by one atomic add each, not by
   workgroup index), and parse each as fd_frag_parse_kernel does: the per-frag fields,
   the tile's scan, its base by the decoupled look-back, its descriptors.  A
   tile's look-back only waits on tiles taken before it, by workgroups that
   were running when they took them, so every wait ends whether or not the
   launch's workgroups are all resident at once (another kernel on the GPU,
   a grid above one workgroup per CU).  The four waves cannot use a
   workgroup barrier (the workgroup's phase-B / C waves never reach one): they
   meet on an LDS counter instead.  A tile's look-back word goes to
   FD_LB_DONE once all of its descriptors are stored.  Once no tile is left,
   wave 0 waits until the tiles holding the workgroup's descriptors
   [b0, b0 + 256) are DONE -- all taken by running workgroups, so they will
   be -- and returns the count its phase A may use (the batch's total if that
   ends inside the workgroup's range, else b0 + 256).  Waits are bounded; an
   expired wait fails the batch (fparse_args.err). */
#define FD_LB_DONE 3ull
__device__ __forceinline__ void wave4_meet( uint32_t * ctr, uint32_t gen, int lane, int * late ) {
  __builtin_amdgcn_fence( __ATOMIC_RELEASE, "workgroup" );
  if( lane == 0 ) __hip_atomic_fetch_add( ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP );
  uint32_t i;
  for( i=0; i<FD_LB_SPIN && __hip_atomic_load( ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP ) < 4u*gen; i++ )
    __builtin_amdgcn_s_sleep( 1 );
  if( i == FD_LB_SPIN ) *late = 1;
  __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "workgroup" );
}

__device__ __forceinline__ uint32_t pipe_aparse( fparse_args const & a, uint32_t * s_ap, int wv, int lane ) {
  int late = 0;
  uint32_t gen = 0u;
  uint64_t ntile = (a.n + FD_FRAG_BLOCK - 1u) / FD_FRAG_BLOCK;
  uint64_t ep = (uint64_t)a.epoch << 32;
  for(;;) {
    if( wv == 0 && lane == 0 )          /* one relaxed add per take: no retry loop on the shared word */
      s_ap[ 7 ] = (uint32_t)min( __hip_atomic_fetch_add( a.tctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ) - a.tbase,
                                 (uint64_t)ntile );
    wave4_meet( s_ap + 6, ++gen, lane, &late );                 /* the tile this workgroup takes */
    uint64_t tl = s_ap[ 7 ];
    if( tl >= ntile ) break;
    uint64_t i = tl * FD_FRAG_BLOCK + (uint64_t)(wv*64 + lane);
    frag_fields r = frag_parse_one( a, i );
    uint32_t v = r.cnt;
#pragma unroll
    for( uint32_t o=1u; o<64u; o<<=1 ) { uint32_t y = __shfl_up( v, o, 64 ); if( lane >= (int)o ) v += y; }
    if( lane == 63 ) s_ap[ wv ] = v;
    wave4_meet( s_ap + 6, ++gen, lane, &late );                 /* the four wave totals */
    uint32_t pre = 0u, all = 0u;
#pragma unroll
    for( int k=0; k<4; k++ ) { uint32_t t = s_ap[ k ]; pre += k < wv ? t : 0u; all += t; }
    if( wv == 0 ) {
      uint32_t base = frag_lookback( a.flag, tl, all, a.epoch, &late );
      if( lane == 0 ) { s_ap[ 4 ] = base; if( tl == ntile - 1u ) *a.total = base + all; }
    }
    wave4_meet( s_ap + 6, ++gen, lane, &late );                 /* the tile's base */
    uint32_t base = s_ap[ 4 ];
    frag_write<true>( a, i, r, base + pre + v - r.cnt );
    __builtin_amdgcn_s_waitcnt( 0x0F70 );                       /* vmcnt(0): this wave's stores are done */
    wave4_meet( s_ap + 6, ++gen, lane, &late );                 /* all four waves' stores */
    if( wv == 0 && lane == 0 )
      __hip_atomic_store( a.flag + tl, ep | (FD_LB_DONE << 30) | ((base + all) & 0x3fffffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  }
  /* wave 0: wait for the tiles that hold descriptors [b0, b0 + 256) */
  if( wv == 0 ) {
    uint64_t need = (uint64_t)blockIdx.x * FD_VERIFY_BLOCK + FD_VERIFY_BLOCK;
    uint32_t nn = 0u, spin = 0u;
    int64_t top = 0;
    while( ntile ) {
      int64_t k = top + lane;
      uint64_t w = k < (int64_t)ntile ? __hip_atomic_load( a.flag + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT ) : 0ull;
      bool done = (w & 0xffffffff00000000ull) == ep && ((w >> 30) & 3ull) == FD_LB_DONE;
      uint32_t P = (uint32_t)(w & 0x3fffffffull);
      uint64_t term = __ballot( done && (k == (int64_t)ntile - 1 || (uint64_t)P >= need) );
      uint64_t nd = __ballot( k < (int64_t)ntile && !done );
      uint64_t before = term ? (term & (~term + 1ull)) - 1ull : ~0ull;   /* lanes before the first terminal one */
      if( nd & before ) {
        if( ++spin > FD_LB_SPIN ) { late = 1; break; }
        __builtin_amdgcn_s_sleep( 1 );
        continue;
      }
      if( term ) {
        int f = __builtin_ctzll( term );
        uint32_t Pf = __shfl( P, f, 64 );
        nn = (uint64_t)Pf >= need ? (uint32_t)need : Pf;
        break;
      }
      top += 64;
    }
    if( lane == 0 ) s_ap[ 5 ] = nn;
  }
  wave4_meet( s_ap + 6, ++gen, lane, &late );
  if( late && lane == 0 && a.err ) __hip_atomic_store( a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM );
  return s_ap[ 5 ];
}

/* Each frag's verify code from its descriptors' codes, with
   fd_ed25519_verify_batch_single_msg's precedence (first phase-1 error,
   else ERR_MSG, else SUCCESS), for batches verified by the one-shot kernels
   (the pipelined kernel folds in its phase C); every frag's status and tag
   go straight into the host's page-locked staging. */
extern "C" __global__ void __launch_bounds__( FD_FRAG_BLOCK )
fd_frag_fold_kernel( fparse_args a ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= a.n ) return;
  int st = a.status[ i ];
  if( !st ) {
    uint64_t at = a.first[ i ], end = at + (a.fold[ i ] & 0xffu);
    int first = 0, any_msg = 0;
    for( uint64_t k=at; k<end; k++ ) {
      int c = a.code[ k ];
      if( c == FD_ED25519_ERR_MSG ) any_msg = 1;
      else if( c != FD_ED25519_SUCCESS && !first ) first = c;
    }
    st = first ? first : (any_msg ? FD_ED25519_ERR_MSG : FD_ED25519_SUCCESS);
  }
  uint64_t tag = a.tag[ i ];
  ((uint4 *)a.hrec)[ i ] = make_uint4( (uint32_t)tag, (uint32_t)(tag >> 32), (uint32_t)(int32_t)st, 0u );
}

/* Self-test kernel (tests only, fd_ed25519_gpu_test_lattice): the device
   lattice reduction on caller-supplied k, one per lane. */
extern "C" __global__ void fd_ed25519_lattice_test_kernel( uint32_t const * k, uint32_t * out, uint64_t n ) {
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


/* Self-test kernel (tests only, fd_ed25519_gpu_test_field): the device field
   and group operations on caller-supplied limbs, one operation per launch,
   one input per lane (a, b: 40 limbs each; out: 40 limbs), so the tests can
   hold the inline-asm device code limb for limb against the host build of
   the same headers at the documented bounds.
     0 fe_mul(a,b)  1 fe_sq(a)  2 fe_sq_neg(a)  3 fe_sq_seed(a,b)  4 fe_add(a,b)
     5 fe_sub(a,b)  6 fe_lshl1_add(a,b)  7 fe_cneg(a, b[0]&1)
     8 ge_dbl(a) with T  9 ge_add_cached(a, b) with T  (points: X,Y,Z,T limbs) */
extern "C" __global__ void __launch_bounds__( 64 )
fd_fe_test_kernel( int op, uint32_t const * a, uint32_t const * b, uint32_t * out, uint64_t n ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  uint32_t const * pa = a + i*40u;
  uint32_t const * pb = b + i*40u;
  uint32_t * po = out + i*40u;
  fe x, y, r;
#pragma unroll
  for( int j=0; j<10; j++ ) { x.v[j] = pa[j]; y.v[j] = pb[j]; r.v[j] = 0u; }
  if( op <= 7 ) {
    switch( op ) {
      case 0: fe_mul( r, x, y ); break;
      case 1: fe_sq( r, x ); break;
      case 2: fe_sq_neg( r, x ); break;
      case 3: fe_sq_seed( r, x, y ); break;
      case 4: fe_add( r, x, y ); break;
      case 5: fe_sub( r, x, y ); break;
      case 6: fe_lshl1_add( r, x, y ); break;
      default: fe_cneg( r, x, (pb[0] & 1u) != 0u ); break;
    }
#pragma unroll
    for( int j=0; j<10; j++ ) po[j] = r.v[j];
    return;
  }
  ge_p3 p, o;
#pragma unroll
  for( int j=0; j<10; j++ ) { p.X.v[j] = pa[j]; p.Y.v[j] = pa[10+j]; p.Z.v[j] = pa[20+j]; p.T.v[j] = pa[30+j]; }
  if( op == 8 ) ge_dbl( o, p, true );
  else {
    ge_cached q;
#pragma unroll
    for( int j=0; j<10; j++ ) { q.YpX.v[j] = pb[j]; q.YmX.v[j] = pb[10+j]; q.T2d.v[j] = pb[20+j]; q.Z2.v[j] = pb[30+j]; }
    ge_add_cached( o, p, q, true );
  }
#pragma unroll
  for( int j=0; j<10; j++ ) { po[j] = o.X.v[j]; po[10+j] = o.Y.v[j]; po[20+j] = o.Z.v[j]; po[30+j] = o.T.v[j]; }
}
