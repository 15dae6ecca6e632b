/* fd_sha256_dev.h -- per-lane SHA-256 for gfx950: the 8-word state and the
   16-word rolling message schedule live in VGPRs; rotates are single
   v_alignbit_b32, Ch / Maj bitfield inserts.

   Replaces, for the GPU callers, the reference's SHA-256 (fd_sha256_hash /
   the fd_sha256_batch_* API, src/ballet/sha256/fd_sha256.h, cores
   fd_sha256_core_ref / fd_sha256_core_shaext.S): the batched digest kernel
   (fd_sha256_batch_gpu) and the shred Merkle roots of the FEC resolver's
   signature check (src/disco/shred/fd_fec_resolver.c:334-399: the leaf over
   the shred's protected bytes, the proof climbed with 20-byte nodes,
   src/ballet/bmtree/fd_bmtree.c:385-420).  A message is an optional short
   constant prefix followed by bytes streamed from HBM; blocks are assembled
   on the fly, each block's dwords fetched one block ahead. */

#ifndef FD_SHA256_DEV_H
#define FD_SHA256_DEV_H

#include <stdint.h>

#if defined(__HIPCC__)
#define FD_S256_FN __device__ __forceinline__
#define FD_S256_CONST __constant__
#else
#define FD_S256_FN static inline
#define FD_S256_CONST static const
#endif

FD_S256_CONST uint32_t fd_sha256_dev_K[ 64 ] = {
  0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
  0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
  0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
  0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
  0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
  0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
  0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
  0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u };

FD_S256_FN uint32_t s256_ror( uint32_t x, int n ) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit( x, x, (uint32_t)n );
#else
  return (x >> n) | (x << (32 - n));
#endif
}

FD_S256_FN uint32_t s256_bswap( uint32_t x ) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

FD_S256_FN void sha256_init_state( uint32_t h[ 8 ] ) {
  h[0]=0x6a09e667u; h[1]=0xbb67ae85u; h[2]=0x3c6ef372u; h[3]=0xa54ff53au;
  h[4]=0x510e527fu; h[5]=0x9b05688cu; h[6]=0x1f83d9abu; h[7]=0x5be0cd19u;
}

/* Ch(e,f,g) = e ? f : g and Maj(a,b,c) = (a^b) ? c : b, as bitfield selects */
#define S256_ROUND( a, b, c, d, e, f, g, hh, k, w ) do {                                              \
    uint32_t t1 = hh + (s256_ror( e, 6 ) ^ s256_ror( e, 11 ) ^ s256_ror( e, 25 )) + ((e & f) | (~e & g)) + (k) + (w); \
    uint32_t m_ = a ^ b;                                                                              \
    uint32_t t2 = (s256_ror( a, 2 ) ^ s256_ror( a, 13 ) ^ s256_ror( a, 22 )) + ((m_ & c) | (~m_ & b));  \
    d += t1; hh = t1 + t2; } while( 0 )

/* One 64-byte block, W[16] big-endian words (clobbered): 16 rounds per loop
   trip with the working variables renamed at compile time, the schedule
   computed in place. */
FD_S256_FN void sha256_compress( uint32_t h[ 8 ], uint32_t W[ 16 ] ) {
  uint32_t a=h[0], b=h[1], c=h[2], d=h[3], e=h[4], f=h[5], g=h[6], hh=h[7];
#pragma unroll 1
  for( int r=0; r<64; r+=16 ) {
    if( r ) {
#pragma unroll
      for( int i=0; i<16; i++ ) {
        uint32_t w15 = W[(i+1)&15], w2 = W[(i+14)&15];
        uint32_t s0 = s256_ror( w15, 7 ) ^ s256_ror( w15, 18 ) ^ (w15 >> 3);
        uint32_t s1 = s256_ror( w2, 17 ) ^ s256_ror( w2, 19 ) ^ (w2 >> 10);
        W[i] = W[i] + s0 + W[(i+9)&15] + s1;
      }
    }
#pragma unroll
    for( int i=0; i<16; i+=8 ) {
      S256_ROUND( a, b, c, d, e, f, g, hh, fd_sha256_dev_K[ r+i   ], W[i  ] );
      S256_ROUND( hh, a, b, c, d, e, f, g, fd_sha256_dev_K[ r+i+1 ], W[i+1] );
      S256_ROUND( g, hh, a, b, c, d, e, f, fd_sha256_dev_K[ r+i+2 ], W[i+2] );
      S256_ROUND( f, g, hh, a, b, c, d, e, fd_sha256_dev_K[ r+i+3 ], W[i+3] );
      S256_ROUND( e, f, g, hh, a, b, c, d, fd_sha256_dev_K[ r+i+4 ], W[i+4] );
      S256_ROUND( d, e, f, g, hh, a, b, c, fd_sha256_dev_K[ r+i+5 ], W[i+5] );
      S256_ROUND( c, d, e, f, g, hh, a, b, fd_sha256_dev_K[ r+i+6 ], W[i+6] );
      S256_ROUND( b, c, d, e, f, g, hh, a, fd_sha256_dev_K[ r+i+7 ], W[i+7] );
    }
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
}

#if defined(__HIPCC__)
/* Raw dwords of block b of the stream that starts at arena byte `base`
   (dword (base >> 2) + 16 b + i, i < 17, clamped to [0, lim_dw]). */
__device__ __forceinline__ void s256_fetch( uint32_t raw[ 17 ], uint32_t const * a32, int64_t base, uint32_t b,
                                            uint32_t lim_dw ) {
  int64_t start = (base >> 2) + 16*(int64_t)b;
#pragma unroll
  for( int i=0; i<17; i++ ) {
    int64_t k = start + i;
    raw[i] = a32[ k < 0 ? 0u : (k > (int64_t)lim_dw ? lim_dw : (uint32_t)k) ];
  }
}

/* h = SHA-256( P || arena[doff, doff + dlen) ), P = plen (< 32) bytes given
   as big-endian words pw[0..7] (unused bytes zero).  The stream byte s sits
   at arena byte doff - plen + s; the words of the prefix bytes come from pw,
   the padding (0x80, zeros, the 64-bit bit length) is spliced in by masks.
   lim_dw: the last readable arena dword. */
__device__ __forceinline__ void sha256_span( uint32_t h[ 8 ], uint32_t const pw[ 8 ], uint32_t plen,
                                             uint8_t const * arena, uint64_t doff, uint32_t dlen, uint32_t lim_dw ) {
  sha256_init_state( h );
  uint32_t total = plen + dlen;
  uint32_t nblk = (total + 72u) >> 6;
  uint32_t const * a32 = (uint32_t const *)arena;
  int64_t base = (int64_t)doff - (int64_t)plen;
  uint32_t sh = (uint32_t)(base & 3);
  uint32_t nxt[ 17 ];
  s256_fetch( nxt, a32, base, 0u, lim_dw );
  for( uint32_t b=0; b<nblk; b++ ) {
    uint32_t raw[ 17 ];
#pragma unroll
    for( int i=0; i<17; i++ ) raw[i] = nxt[i];
    if( b + 1u < nblk ) s256_fetch( nxt, a32, base, b + 1u, lim_dw );
    uint32_t W[ 16 ];
#pragma unroll
    for( int j=0; j<16; j++ ) {
      int32_t s = (int32_t)(64u*b) + 4*j;
      uint32_t w = s256_bswap( __builtin_amdgcn_alignbyte( raw[j+1], raw[j], sh ) );
      /* prefix bytes (only in block 0: plen < 32) */
      if( b == 0u && j < 8 ) {
        int32_t pre = (int32_t)plen - s;
        uint32_t pm = pre >= 4 ? 0xffffffffu : (pre <= 0 ? 0u : ~(0xffffffffu >> (8*pre)));
        w = (pw[j] & pm) | (w & ~pm);
      }
      int32_t rem = (int32_t)total - s;
      uint32_t keep = rem >= 4 ? 0xffffffffu : (rem <= 0 ? 0u : ~(0xffffffffu >> (8*rem)));
      uint32_t pad  = (rem >= 0 && rem < 4) ? (0x80000000u >> (8*rem)) : 0u;
      w = (w & keep) | pad;
      if( b == nblk - 1u && j == 14 ) w = total >> 29;
      if( b == nblk - 1u && j == 15 ) w = total << 3;
      W[j] = w;
    }
    sha256_compress( h, W );
  }
}
#endif

#endif /* FD_SHA256_DEV_H */
