/* fd_sha512_dev.h -- per-lane SHA-512 for gfx950: the 8x64-bit state and
   the 16-word rolling message schedule live in VGPRs (64-bit adds as
   v_lshl_add_u64, rotates as v_alignbit_b32 pairs, Ch as v_bfi_b32, Maj and
   the three-way XORs as v_bitop3_b32).

   Replaces the verify-path use of fd_sha512_init/append/fini
   (src/ballet/sha512/fd_sha512.c:264-399; cores fd_sha512_core_ref :128-229
   and fd_sha512_core_avx2.S).  The verify kernel hashes R || A || M with no
   intermediate buffer: blocks are assembled on the fly from the signature
   and public-key registers and from the message bytes in HBM. */

#ifndef FD_SHA512_DEV_H
#define FD_SHA512_DEV_H

#include <stdint.h>

#if defined(__HIPCC__)
#define FD_SHA_FN __device__ __forceinline__
#define FD_SHA_CONST __constant__
#else
#define FD_SHA_FN static inline
#define FD_SHA_CONST static const
#endif

FD_SHA_CONST uint64_t fd_sha512_dev_K[ 80 ] = {
  0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,0x3956c25bf348b538ULL,
  0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,0xd807aa98a3030242ULL,0x12835b0145706fbeULL,
  0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,
  0xc19bf174cf692694ULL,0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,0x983e5152ee66dfabULL,
  0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,
  0x06ca6351e003826fULL,0x142929670a0e6e70ULL,0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,
  0x53380d139d95b3dfULL,0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,0xd192e819d6ef5218ULL,
  0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,
  0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,
  0x682e6ff3d6b2b8a3ULL,0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,0xca273eceea26619cULL,
  0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,
  0x113f9804bef90daeULL,0x1b710b35131c471bULL,0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,
  0x431d67c49c100d4cULL,0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL };

/* 64-bit rotate right by a compile-time n: two v_alignbit_b32 on the
   32-bit halves (the generic shift/shift/or form costs four 64-bit ops). */
FD_SHA_FN uint64_t sha_ror( uint64_t x, int n ) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if( n >= 32 ) { uint32_t t = lo; lo = hi; hi = t; n -= 32; }
  if( n == 0 ) return ((uint64_t)hi << 32) | lo;
  uint32_t rlo = __builtin_amdgcn_alignbit( hi, lo, (uint32_t)n );
  uint32_t rhi = __builtin_amdgcn_alignbit( lo, hi, (uint32_t)n );
  return ((uint64_t)rhi << 32) | rlo;
#else
  return (x >> n) | (x << (64 - n));
#endif
}

/* Ch(e,f,g) = (e & f) | (~e & g): one v_bfi_b32 per half (left to itself
   the compiler emits an and, a bfi and an extra 64-bit add per half).
   Maj(a,b,c) and the three-way XORs of the Sigma functions: one
   v_bitop3_b32 per half (gfx950's three-input bitwise op, truth tables 0xE8
   and 0x96 -- both symmetric, so the operand order does not matter) instead
   of two or three two-input ops. */
#if defined(__HIP_DEVICE_COMPILE__)
FD_SHA_FN uint32_t sha_bfi( uint32_t m, uint32_t x, uint32_t y ) {
  uint32_t r; asm( "v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(x), "v"(y) ); return r;
}
FD_SHA_FN uint32_t sha_x3( uint32_t a, uint32_t b, uint32_t c ) { return __builtin_amdgcn_bitop3_b32( a, b, c, 0x96 ); }
FD_SHA_FN uint32_t sha_mj( uint32_t a, uint32_t b, uint32_t c ) { return __builtin_amdgcn_bitop3_b32( a, b, c, 0xe8 ); }
/* The two halves as one 64-bit register pair, opaque to the optimiser:
   left visible, it splits the 64-bit add the pair feeds into an add of the
   zero-extended low half and one of the high half (two adds, two moves). */
FD_SHA_FN uint64_t sha_pair( uint32_t lo, uint32_t hi ) {
  uint64_t r = ((uint64_t)hi << 32) | lo;
  asm( "" : "+v"(r) );
  return r;
}
/* x >> n as one v_lshrrev_b64 (split into halves the compiler makes it a
   shift and an alignbit) */
FD_SHA_FN uint64_t sha_shr( uint64_t x, int n ) {
  uint64_t r = x >> n;
  asm( "" : "+v"(r) );
  return r;
}
FD_SHA_FN uint64_t sha_ch( uint64_t e, uint64_t f, uint64_t g ) {
  return sha_pair( sha_bfi( (uint32_t)e, (uint32_t)f, (uint32_t)g ),
                   sha_bfi( (uint32_t)(e >> 32), (uint32_t)(f >> 32), (uint32_t)(g >> 32) ) );
}
FD_SHA_FN uint64_t sha_maj( uint64_t a, uint64_t b, uint64_t c ) {
  return sha_pair( sha_mj( (uint32_t)a, (uint32_t)b, (uint32_t)c ),
                   sha_mj( (uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32) ) );
}
FD_SHA_FN uint64_t sha_xor3( uint64_t a, uint64_t b, uint64_t c ) {
  return sha_pair( sha_x3( (uint32_t)a, (uint32_t)b, (uint32_t)c ),
                   sha_x3( (uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32) ) );
}
#else
FD_SHA_FN uint64_t sha_shr ( uint64_t x, int n ) { return x >> n; }
FD_SHA_FN uint64_t sha_ch  ( uint64_t e, uint64_t f, uint64_t g ) { return (e & f) | (~e & g); }
FD_SHA_FN uint64_t sha_maj ( uint64_t a, uint64_t b, uint64_t c ) { return (a & b) | (a & c) | (b & c); }
FD_SHA_FN uint64_t sha_xor3( uint64_t a, uint64_t b, uint64_t c ) { return a ^ b ^ c; }
#endif

FD_SHA_FN void sha512_init_state( uint64_t h[ 8 ] ) {
  h[0]=0x6a09e667f3bcc908ULL; h[1]=0xbb67ae8584caa73bULL; h[2]=0x3c6ef372fe94f82bULL; h[3]=0xa54ff53a5f1d36f1ULL;
  h[4]=0x510e527fade682d1ULL; h[5]=0x9b05688c2b3e6c1fULL; h[6]=0x1f83d9abfb41bd6bULL; h[7]=0x5be0cd19137e2179ULL;
}

#define SHA_ROUND( a, b, c, d, e, f, g, hh, k, w ) do {                                               \
    uint64_t t1 = hh + sha_xor3( sha_ror( e, 14 ), sha_ror( e, 18 ), sha_ror( e, 41 ) ) + sha_ch( e, f, g ) + (k) + (w); \
    uint64_t t2 = sha_xor3( sha_ror( a, 28 ), sha_ror( a, 34 ), sha_ror( a, 39 ) ) + sha_maj( a, b, c );           \
    d += t1; hh = t1 + t2; } while( 0 )

/* One 128-byte block, W[16] big-endian words (clobbered).  16 rounds per
   loop trip, the eight working variables renamed at compile time (8-round
   macro groups), the schedule computed in place. */
FD_SHA_FN void sha512_compress( uint64_t h[ 8 ], uint64_t W[ 16 ] ) {
  uint64_t a=h[0], b=h[1], c=h[2], d=h[3], e=h[4], f=h[5], g=h[6], hh=h[7];
#pragma unroll 1
  for( int r=0; r<80; r+=16 ) {
    if( r ) {
#pragma unroll
      for( int i=0; i<16; i++ ) {
        uint64_t w15 = W[(i+1)&15], w2 = W[(i+14)&15];
        uint64_t s0 = sha_xor3( sha_ror( w15, 1 ), sha_ror( w15, 8 ), sha_shr( w15, 7 ) );
        uint64_t s1 = sha_xor3( sha_ror( w2, 19 ), sha_ror( w2, 61 ), sha_shr( w2, 6 ) );
        W[i] = W[i] + s0 + W[(i+9)&15] + s1;
      }
    }
#pragma unroll
    for( int i=0; i<16; i+=8 ) {
      SHA_ROUND( a, b, c, d, e, f, g, hh, fd_sha512_dev_K[ r+i   ], W[i  ] );
      SHA_ROUND( hh, a, b, c, d, e, f, g, fd_sha512_dev_K[ r+i+1 ], W[i+1] );
      SHA_ROUND( g, hh, a, b, c, d, e, f, fd_sha512_dev_K[ r+i+2 ], W[i+2] );
      SHA_ROUND( f, g, hh, a, b, c, d, e, fd_sha512_dev_K[ r+i+3 ], W[i+3] );
      SHA_ROUND( e, f, g, hh, a, b, c, d, fd_sha512_dev_K[ r+i+4 ], W[i+4] );
      SHA_ROUND( d, e, f, g, hh, a, b, c, fd_sha512_dev_K[ r+i+5 ], W[i+5] );
      SHA_ROUND( c, d, e, f, g, hh, a, b, fd_sha512_dev_K[ r+i+6 ], W[i+6] );
      SHA_ROUND( b, c, d, e, f, g, hh, a, fd_sha512_dev_K[ r+i+7 ], W[i+7] );
    }
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
}

FD_SHA_FN uint32_t sha_bswap32( uint32_t x ) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

#endif /* FD_SHA512_DEV_H */
