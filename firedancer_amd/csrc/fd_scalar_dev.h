/* fd_scalar_dev.h -- scalars mod l on 32-bit words, per lane.

   l = 2^252 + 27742317777372353535851937790883648493.
   Replaces fd_curve25519_scalar_validate (src/ballet/ed25519/
   fd_curve25519_scalar.h:57-73) and fd_curve25519_scalar_reduce
   (fd_curve25519_scalar.c:3-110).  The reference's wNAF recoding
   (fd_curve25519_scalar_wnaf, :277-360) is replaced by fixed-width signed
   windows (fd_scalar_recode_*), which keeps every lane of a wave on the
   same add schedule (no divergence), at the cost of a few more additions. */

#ifndef FD_SCALAR_DEV_H
#define FD_SCALAR_DEV_H

#include <stdint.h>

#if defined(__HIPCC__)
#define FD_SC_FN __device__ __forceinline__
#else
#define FD_SC_FN static inline
#endif

/* l as 8 LE words */
#define FD_L0 0x5cf5d3edu
#define FD_L1 0x5812631au
#define FD_L2 0xa2f79cd6u
#define FD_L3 0x14def9deu
#define FD_L7 0x10000000u

/* s <= l-1, i.e. s < l, as a 256-bit LE integer: the S check of
   fd_ed25519_verify (fd_ed25519_user.c:157-159).  Bits 253..255 of s are
   NOT masked (s >= 2^253 is rejected). */
FD_SC_FN int sc_lt_l( uint32_t const s[ 8 ] ) {
  uint32_t const l[ 8 ] = { FD_L0, FD_L1, FD_L2, FD_L3, 0u, 0u, 0u, FD_L7 };
  int lt = 0, eq = 1;
#pragma unroll
  for( int i=7; i>=0; i-- ) {
    lt |= eq & (s[i] < l[i]);
    eq &= (s[i] == l[i]);
  }
  return lt;
}

/* r = x mod l for a 512-bit x (16 LE words).  Barrett with b = 2^32, k = 8,
   mu = floor(2^512 / l) (derived constant, 9 words). */
FD_SC_FN void sc_reduce512( uint32_t r[ 8 ], uint32_t const x[ 16 ] ) {
  uint32_t const mu[ 9 ] = { 0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                             0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu };
  uint32_t const l[ 8 ] = { FD_L0, FD_L1, FD_L2, FD_L3, 0u, 0u, 0u, FD_L7 };
  /* q1 = floor(x / b^7): words 7..15 (9 words); q2 = q1*mu; q3 = floor(q2 / b^9) */
  uint32_t q2[ 18 ];
#pragma unroll
  for( int i=0; i<18; i++ ) q2[i] = 0u;
#pragma unroll
  for( int i=0; i<9; i++ ) {
    uint64_t c = 0;
#pragma unroll
    for( int j=0; j<9; j++ ) {
      uint64_t t = (uint64_t)x[7+i] * mu[j] + q2[i+j] + c;
      q2[i+j] = (uint32_t)t; c = t >> 32;
    }
    q2[i+9] = (uint32_t)c;
  }
  /* r2 = (q3 * l) mod b^9, q3 = q2[9..17] */
  uint32_t r2[ 9 ];
#pragma unroll
  for( int i=0; i<9; i++ ) r2[i] = 0u;
#pragma unroll
  for( int i=0; i<9; i++ ) {
    uint64_t c = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) {
      if( i+j<9 ) {
        uint64_t t = (uint64_t)q2[9+i] * l[j] + r2[i+j] + c;
        r2[i+j] = (uint32_t)t; c = t >> 32;
      }
    }
    if( i+8<9 ) r2[i+8] = (uint32_t)c;
  }
  /* r = (x mod b^9) - r2 mod b^9, then at most two subtractions of l */
  uint32_t t9[ 9 ];
  uint64_t br = 0;
#pragma unroll
  for( int i=0; i<9; i++ ) {
    uint64_t d = (uint64_t)x[i] - r2[i] - br;
    t9[i] = (uint32_t)d; br = (d >> 63) & 1u;
  }
#pragma unroll
  for( int it=0; it<2; it++ ) {
    /* t9 >= l ? subtract */
    uint32_t s9[ 9 ]; uint64_t b2 = 0;
#pragma unroll
    for( int i=0; i<9; i++ ) {
      uint64_t d = (uint64_t)t9[i] - (i<8 ? l[i] : 0u) - b2;
      s9[i] = (uint32_t)d; b2 = (d >> 63) & 1u;
    }
    int ge = (b2 == 0);
#pragma unroll
    for( int i=0; i<9; i++ ) t9[i] = ge ? s9[i] : t9[i];
  }
#pragma unroll
  for( int i=0; i<8; i++ ) r[i] = t9[i];
}

/* Signed fixed-window recoding.  s (< 2^253) = sum_i d_i 2^(w i) with
   d_i in [-2^(w-1), 2^(w-1)-1] for all but possibly the top digit.  The
   digits are emitted as (d + 2^(w-1)) biased bytes so they fit a u8. */
FD_SC_FN void sc_recode_w4( uint8_t out[ 64 ], uint32_t const s[ 8 ] ) {
  int c = 0;
#pragma unroll
  for( int i=0; i<64; i++ ) {
    int d = (int)((s[i>>3] >> (4*(i&7))) & 15u) + c;
    c = d >= 8;
    d -= c << 4;
    out[i] = (uint8_t)(d + 8);
  }
}

FD_SC_FN void sc_recode_w8( uint8_t out[ 32 ], uint32_t const s[ 8 ] ) {
  int c = 0;
#pragma unroll
  for( int i=0; i<32; i++ ) {
    int d = (int)((s[i>>2] >> (8*(i&3))) & 255u) + c;
    c = d >= 128;
    d -= c << 8;
    out[i] = (uint8_t)(d + 128);
  }
}

/* Signed radix-2^23 comb digits of w < l (the fixed-base comb table,
   fd_ed25519_gpu_abi.h FD_CTAB_*): y = w + sum_{k<10} 2^22 2^(23 k) (the
   recoding as a bias), then d_k = bits [23 k, 23 k + 23) of y minus 2^22
   for k < 10 (in [-2^22, 2^22)) and d_10 = y >> 230 unbiased (in
   [0, 2^22]: w < l = 2^252 + 2^124.4 and the bias is below 2^229 + 1, so
   y < 2^252 + 2^230); sum_k d_k 2^(23 k) = w. */
FD_SC_FN void comb_bias( uint32_t y[ 8 ], uint32_t const w[ 8 ] ) {
  uint32_t const b[ 8 ] = { 0x400000u, 0x2000u, 0x8000010u, 0x40000u, 0x200u, 0x800001u, 0x4000u, 0x20u };
  uint64_t c = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) { c += (uint64_t)w[j] + b[j]; y[j] = (uint32_t)c; c >>= 32; }
}

/* Digit k of a comb_bias'ed y (words lo = y[(23 k) >> 5], hi = the next word
   or 0 past the top, r = (23 k) & 31). */
FD_SC_FN int comb_digit_w( uint32_t lo, uint32_t hi, int k ) {
  int r = (23*k) & 31;
  uint32_t x = (uint32_t)((((uint64_t)hi << 32) | lo) >> r) & ((1u << 23) - 1u);
  return (int)x - (k < 10 ? (1 << 22) : 0);
}
FD_SC_FN int comb_digit( uint32_t const y[ 8 ], int k ) {
  int q = (23*k) >> 5;
  return comb_digit_w( y[q], q < 7 ? y[q+1] : 0u, k );
}


/* The verify kernels' recoding of the lattice scalars u, v (x < 2^(P+3)): the
   top digit at bit P (P = nbits - 3 of the wave's longest scalar, at least
   124: recode_p_top), so the Straus chain takes P doublings rather than the
   next multiple of four; windows 0 .. m-2 are 4-bit (bias 8 each), window
   m-1 = nw-2 is wn = P - 4 (m-1) bits (bias 2^(wn-1)), the top digit is
   y >> P; m = ceil(P / 4), nw = m + 1.  x < 2^(P+3) keeps the top digit <= 8
   (y < 8.77 2^P).  Pinned on the CPU through this code by
   tests/test_field_bounds.py::test_pipe_recoding. */
FD_SC_FN int recode_p_top( int nbits ) {
  int P = nbits - 3;
  P = P < 124 ? 124 : P;
  return P > 252 ? 252 : P;          /* 4 (FD_NDIG_MAX - 2) + 4: 64 windows */
}
FD_SC_FN void ybias_p( uint32_t y[ 8 ], uint32_t const x[ 8 ], int P ) {
  int m = (P + 3) >> 2, wn = P - 4*(m - 1), eb = 4*(m - 1) + wn - 1;
  uint64_t c = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) {
    int nb = m - 1 - 8*j;                           /* 4-bit biased nibbles in word j */
    uint32_t pat = nb >= 8 ? 0x88888888u : (nb <= 0 ? 0u : (0x88888888u & ((1u << (4*nb)) - 1u)));
    uint32_t ex = (eb >> 5) == j ? (1u << (eb & 31)) : 0u;
    c += (uint64_t)x[j] + pat + ex;
    y[j] = (uint32_t)c; c >>= 32;
  }
}
/* Digit i < nw-1 of a ybias_p scalar, biased: d_i + 8 in [0, 16]. */
FD_SC_FN uint32_t recode_p_low( uint32_t const y[ 8 ], int i, int P ) {
  int nw = ((P + 3) >> 2) + 1, wn = P - 4*(nw - 2);
  uint32_t db = (y[ i >> 3 ] >> (4*(i & 7))) & 15u;
  return i == nw-2 ? (db & ((1u << wn) - 1u)) + 8u - (1u << (wn - 1)) : db;
}
/* The top digit (i = nw-1, at bit P), biased. */
FD_SC_FN uint32_t recode_p_hi( uint32_t const y[ 8 ], int P ) {
  int q = P >> 5;
  uint64_t two = (uint64_t)y[ q ] | (q < 7 ? (uint64_t)y[ q + 1 ] << 32 : 0ull);
  return ((uint32_t)(two >> (P & 31)) & 15u) + 8u;
}

#endif /* FD_SCALAR_DEV_H */
