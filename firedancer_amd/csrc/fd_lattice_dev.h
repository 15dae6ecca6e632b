/* fd_lattice_dev.h -- halving the double-scalar multiplication of the
   verify equation by a short vector of the lattice {(u,v) : u = v k mod 8l}.

   The reference checks  [S]B - [k]A == R  (fd_ed25519_user.c:203-228) with
   one 253-bit scalar per point (fd_ed25519_double_scalar_mul_base,
   fd_curve25519.c:122-166: ~252 doublings).  Here, per lane:

     find (u, v), v odd, 0 < |v| < l, u = v k (mod 8l), |u|,|v| ~ 2^127
     w = v S mod l
     check  [w]B - [u]A - [v]R == O

   Exactness (no probabilistic step, no cofactor): let D = [S]B - [k]A - R.
   Every decoded point lies on the curve, whose group has order 8l, so
   [v k]A = [u]A, and B has order l, so [v S]B = [w]B; hence the checked
   point is [v]D.  gcd(v, 8l) = 1 (v odd, 0 < |v| < l, l prime), so
   [v]D == O  <=>  D == O  <=>  the reference's equation holds, for points
   of any order (mixed-order A/R included).  The double-scalar product then
   needs ~128 doublings instead of ~252 (after Pornin, "Optimized Lattice
   Basis Reduction In Dimension 2, and Fast Schnorr and EdDSA Signature
   Verification", 2020, here with modulus 8l so torsion cancels exactly).

   The short vector comes from the extended Euclidean algorithm on (8l, k),
   stopped at the first remainder below 2^128 (r_i |t_{i-1}| + r_{i-1} |t_i|
   = 8l bounds |t_i| < 2^127.01); quotients are estimated from f64
   approximations and always rounded DOWN, so every step is exact integer
   arithmetic and the estimate only decides how many steps are taken.  If
   t_i is even, (r_{i-1} - j r_i, t_{i-1} - j t_i) with a balancing j is
   used (t_{i-1} is then odd, consecutive t are coprime).  (u, v) = (k, 1)
   is always valid and is the fallback if the iteration cap is hit.

   Compiled for the device and, unchanged, for the host (tests/csrc). */

#ifndef FD_LATTICE_DEV_H
#define FD_LATTICE_DEV_H

#include <stdint.h>

#if defined(__HIPCC__)
#define FD_LT_FN __device__ __forceinline__
#else
#define FD_LT_FN static inline
#include <math.h>
#endif

#define FD_LAT_MAX_ITER 1024

/* 8l as 8 LE words */
#define FD_N8L0 0xe7ae9f68u
#define FD_N8L1 0xc09318d2u
#define FD_N8L2 0x17bce6b2u
#define FD_N8L3 0xa6f7cef5u
#define FD_N8L7 0x80000000u

FD_LT_FN double lat_f64( uint32_t const x[ 8 ] ) {
  double f = (double)x[7];
#pragma unroll
  for( int j=6; j>=0; j-- ) f = fma( f, 4294967296.0, (double)x[j] );
  return f;
}
FD_LT_FN double lat_f64_4( uint32_t const x[ 4 ] ) {
  double f = (double)x[3];
#pragma unroll
  for( int j=2; j>=0; j-- ) f = fma( f, 4294967296.0, (double)x[j] );
  return f;
}

/* a >= b, 8 words */
FD_LT_FN int lat_ge( uint32_t const a[ 8 ], uint32_t const b[ 8 ] ) {
  uint32_t br = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) {
    uint64_t d = (uint64_t)a[j] - b[j] - br;
    br = (uint32_t)(d >> 63);
  }
  return !br;
}

/* Conservative quotient estimate: returns (m, s) with 1 <= m 2^s <= floor(x/y),
   m < 2^32, assuming x >= y > 0 and xf, yf their f64 approximations
   (relative error <= 2^-50 each, so qf is within 2^-48 of x/y). */
FD_LT_FN uint32_t lat_qest( double xf, double yf, int * s ) {
  double q = (xf / yf) * (1.0 - 0x1p-40);
  *s = 0;
  if( q < 1.0 ) return 1u;
  if( q < 4294967296.0 ) return (uint32_t)q;
  int e = ilogb( q );                   /* q in [2^e, 2^(e+1)) */
  *s = e - 31;
  return (uint32_t)ldexp( q, -(e - 31) ); /* in [2^31, 2^32) */
}

/* x (n words) <<= s bits, 0 <= s < 32 n, truncated (select network, no
   dynamic register indexing). */
template<int N>
FD_LT_FN void lat_shl( uint32_t x[ N ], int s ) {
  int ws = s >> 5, bs = s & 31;
#pragma unroll
  for( int st=1; st<N; st<<=1 ) {
    bool on = (ws & st) != 0;
#pragma unroll
    for( int j=N-1; j>=0; j-- ) x[j] = on ? (j >= st ? x[j-st] : 0u) : x[j];
  }
  if( bs ) {
#pragma unroll
    for( int j=N-1; j>0; j-- ) x[j] = (x[j] << bs) | (x[j-1] >> (32 - bs));
    x[0] <<= bs;
  }
}

/* a -= (m 2^s) b ; t += (m 2^s) tb (t mod 2^(32 TN)).  Caller guarantees
   m 2^s <= floor(a / b). */
template<int TN>
FD_LT_FN void lat_submul( uint32_t a[ 8 ], uint32_t const b[ 8 ], uint32_t t[ TN ], uint32_t const tb[ TN ],
                          uint32_t m, int s ) {
  if( s == 0 ) {
    uint64_t c = 0; uint32_t br = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) {
      uint64_t p = (uint64_t)m * b[j] + c;
      c = p >> 32;
      uint64_t d = (uint64_t)a[j] - (uint32_t)p - br;
      a[j] = (uint32_t)d; br = (uint32_t)(d >> 63);
    }
    c = 0;
#pragma unroll
    for( int j=0; j<TN; j++ ) {
      uint64_t p = (uint64_t)m * tb[j] + t[j] + c;
      t[j] = (uint32_t)p; c = p >> 32;
    }
  } else {
    uint32_t mb[ 8 ], mt[ TN ];
    uint64_t c = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) { uint64_t p = (uint64_t)m * b[j] + c; mb[j] = (uint32_t)p; c = p >> 32; }
    /* the product's 9th word is dropped: m 2^s b <= a < 2^256, so every bit
       shifted past bit 255 (and that whole word) is zero */
    lat_shl<8>( mb, s );
    uint32_t br = 0;
#pragma unroll
    for( int j=0; j<8; j++ ) { uint64_t d = (uint64_t)a[j] - mb[j] - br; a[j] = (uint32_t)d; br = (uint32_t)(d >> 63); }
    c = 0;
#pragma unroll
    for( int j=0; j<TN; j++ ) { uint64_t p = (uint64_t)m * tb[j] + c; mt[j] = (uint32_t)p; c = p >> 32; }
    lat_shl<TN>( mt, s );
    c = 0;
#pragma unroll
    for( int j=0; j<TN; j++ ) { uint64_t p = (uint64_t)t[j] + mt[j] + c; t[j] = (uint32_t)p; c = p >> 32; }
  }
}

/* Any lane of the wave still active? (host: this lane) */
FD_LT_FN int lat_any( int p ) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __any( p );
#else
  return p;
#endif
}

/* Short lattice vector for k (8 LE words, k < l).  Outputs |u| and v (> 0)
   as 8 LE words each and the sign of u.  Returns the number of loop
   iterations (>= FD_LAT_MAX_ITER means the fallback (k, 1) was taken). */
FD_LT_FN int lat_short_vector( uint32_t const k[ 8 ], uint32_t u[ 8 ], uint32_t v[ 8 ], int * u_neg ) {
  uint32_t a[ 8 ] = { FD_N8L0, FD_N8L1, FD_N8L2, FD_N8L3, 0u, 0u, 0u, FD_N8L7 };
  uint32_t b[ 8 ];
  uint32_t ta[ 4 ] = { 0u, 0u, 0u, 0u }, tb[ 4 ] = { 1u, 0u, 0u, 0u };
#pragma unroll
  for( int j=0; j<8; j++ ) b[j] = k[j];
  int par = 0;                                    /* b = (-1)^par tb k, a = -(-1)^par ta k (mod 8l) */
  int active = (b[4] | b[5] | b[6] | b[7]) != 0u; /* b >= 2^128 */
  int it = 0;
  while( lat_any( active ) ) {
    if( active ) {
      if( lat_ge( a, b ) ) {
        int s; uint32_t m = lat_qest( lat_f64( a ), lat_f64( b ), &s );
        lat_submul<4>( a, b, ta, tb, m, s );
      }
      if( !lat_ge( a, b ) ) {
#pragma unroll
        for( int j=0; j<8; j++ ) { uint32_t x = a[j]; a[j] = b[j]; b[j] = x; }
#pragma unroll
        for( int j=0; j<4; j++ ) { uint32_t x = ta[j]; ta[j] = tb[j]; tb[j] = x; }
        par ^= 1;
      }
      active = (b[4] | b[5] | b[6] | b[7]) != 0u;
      if( ++it >= FD_LAT_MAX_ITER ) active = 0;
    }
  }
  if( it >= FD_LAT_MAX_ITER ) {
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = k[j]; v[j] = j == 0 ? 1u : 0u; }
    *u_neg = 0;
    return it;
  }
  if( tb[0] & 1u ) {
    /* (u, v) = (b, (-1)^par tb) */
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = b[j]; v[j] = j < 4 ? tb[j] : 0u; }
    *u_neg = par;
  } else {
    /* (u, v) = (a - j b, -(-1)^par (ta + j tb)), j ~ (a - ta) / (b + tb) */
    double af = lat_f64( a ), bf = lat_f64( b ), taf = lat_f64_4( ta ), tbf = lat_f64_4( tb );
    double jf = ((af - taf) / (bf + tbf)) * (1.0 - 0x1p-40);
    uint32_t jj = jf < 1.0 ? 0u : (jf < 4294967295.0 ? (uint32_t)jf : 0xffffffffu);
    /* clamp to floor(a/b) (only matters if the estimate is off) */
    if( jj ) {
      int s; uint32_t mq = lat_qest( af, bf, &s );
      if( s == 0 && mq < jj ) jj = mq;
    }
    uint32_t t8[ 8 ] = { ta[0], ta[1], ta[2], ta[3], 0u, 0u, 0u, 0u };
    uint32_t tb8[ 8 ] = { tb[0], tb[1], tb[2], tb[3], 0u, 0u, 0u, 0u };
    if( jj ) lat_submul<8>( a, b, t8, tb8, jj, 0 );
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = a[j]; v[j] = t8[j]; }
    *u_neg = par ^ 1;
  }
  return it;
}

#endif /* FD_LATTICE_DEV_H */
