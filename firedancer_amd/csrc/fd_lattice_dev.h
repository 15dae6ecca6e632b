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

/* f64 approximation of x >= 2^128 from its top six words (the two low
   words contribute < 2^-64 relative). */
FD_LT_FN double lat_f64_hi( uint32_t const x[ 8 ] ) {
  double f = (double)x[7];
#pragma unroll
  for( int j=6; j>=2; j-- ) f = fma( f, 4294967296.0, (double)x[j] );
  return f * 18446744073709551616.0;
}

/* 1/y to ~2^-52 relative: hardware reciprocal + two Newton steps. */
FD_LT_FN double lat_rcp( double y ) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp( y );
  r = r * fma( -y, r, 2.0 );
  r = r * fma( -y, r, 2.0 );
  return r;
#else
  return 1.0 / y;
#endif
}

/* a < b, 8 words */
FD_LT_FN int lat_lt( uint32_t const a[ 8 ], uint32_t const b[ 8 ] ) { return !lat_ge( a, b ); }

/* One Euclid half-step on (x, tx) by (y, ty), y >= 2^128, x > y on entry:
   x -= m y, tx += m ty with m the f64 quotient estimate (1 <= m <=
   floor(x/y)), repeated (rarely) until x < y.  xf/yf: f64 approximations
   of x/y on entry; xf is refreshed on exit. */
FD_LT_FN void lat_reduce( uint32_t x[ 8 ], uint32_t tx[ 4 ], uint32_t const y[ 8 ], uint32_t const ty[ 4 ],
                          double & xf, double yf, int act ) {
  double ry = lat_rcp( yf );
  double q = (xf * ry) * (1.0 - 0x1p-40);
  int big = act && q >= 4294967296.0;
  if( lat_any( big ) ) {
    if( big ) {                                   /* rare: quotient >= 2^32 */
      int s; uint32_t m = lat_qest( lat_f64( x ), lat_f64( y ), &s );
      lat_submul<4>( x, y, tx, ty, m, s );
    }
  }
  if( act && !big ) {
    uint32_t m = q < 1.0 ? 1u : (uint32_t)q;
    lat_submul<4>( x, y, tx, ty, m, 0 );
  }
  /* the estimate undershot (quotient close to an integer, or big): repeat */
  int more = act && lat_ge( x, y );
  while( lat_any( more ) ) {
    if( more ) {
      int s; uint32_t m = lat_qest( lat_f64( x ), lat_f64( y ), &s );
      lat_submul<4>( x, y, tx, ty, m, s );
    }
    more = more && lat_ge( x, y );
  }
  if( act ) xf = lat_f64_hi( x );
}

/* Short lattice vector for k (8 LE words, k < l).  Outputs |u| and v (> 0)
   as 8 LE words each and the sign of u.  Returns the number of half-steps
   (>= FD_LAT_MAX_ITER means the fallback (k, 1) was taken).

   Invariants: a tb + b ta = 8l; with the larger of (a, b) reduced by the
   smaller in alternation (no register swap), the one just reduced is
   r_{i+1} = (-1)^(i+1) t_{i+1} k (mod 8l) in Euclid's numbering, i.e. the
   pair's signs alternate.  Any m in [1, floor(x/y)] keeps the invariants. */
FD_LT_FN int lat_short_vector( uint32_t const k[ 8 ], uint32_t u[ 8 ], uint32_t v[ 8 ], int * u_neg ) {
  uint32_t a[ 8 ] = { FD_N8L0, FD_N8L1, FD_N8L2, FD_N8L3, 0u, 0u, 0u, FD_N8L7 };
  uint32_t b[ 8 ];
  uint32_t ta[ 4 ] = { 0u, 0u, 0u, 0u }, tb[ 4 ] = { 1u, 0u, 0u, 0u };
#pragma unroll
  for( int j=0; j<8; j++ ) b[j] = k[j];
  /* b = +tb k, a = -ta k (mod 8l) */
  int active = (b[4] | b[5] | b[6] | b[7]) != 0u;   /* b >= 2^128: keep going */
  int last = 1;                                     /* which of (a, b) holds r_i: 1 = b */
  int it = 0;
  double af = 0.0, bf = 0.0;
  if( active ) { af = lat_f64_hi( a ); bf = lat_f64_hi( b ); }
  while( lat_any( active ) ) {
    /* a -= q b: now a = r_{i+1} < b */
    lat_reduce( a, ta, b, tb, af, bf, active );
    if( active ) { last = 0; it++; active = ((a[4] | a[5] | a[6] | a[7]) != 0u) && it < FD_LAT_MAX_ITER; }
    if( !lat_any( active ) ) break;
    /* b -= q a */
    lat_reduce( b, tb, a, ta, bf, af, active );
    if( active ) { last = 1; it++; active = ((b[4] | b[5] | b[6] | b[7]) != 0u) && it < FD_LAT_MAX_ITER; }
  }
  if( it >= FD_LAT_MAX_ITER ) {
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = k[j]; v[j] = j == 0 ? 1u : 0u; }
    *u_neg = 0;
    return it;
  }
  /* (r, tr) = the remainder below 2^128 and its cofactor, (p, tp) = the
     previous remainder.  Sign: b-side values are +t k, a-side -t k; the
     cofactor magnitudes tb, ta carry those signs ((-1)^par in the swapped
     formulation: par = 1 when r sits in a). */
  uint32_t r[ 8 ], p[ 8 ], tr[ 4 ], tp[ 4 ];
#pragma unroll
  for( int j=0; j<8; j++ ) { r[j] = last ? b[j] : a[j]; p[j] = last ? a[j] : b[j]; }
#pragma unroll
  for( int j=0; j<4; j++ ) { tr[j] = last ? tb[j] : ta[j]; tp[j] = last ? ta[j] : tb[j]; }
  int par = !last;
  if( tr[0] & 1u ) {
    /* (u, v) = (r, (-1)^par tr) */
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = r[j]; v[j] = j < 4 ? tr[j] : 0u; }
    *u_neg = par;
  } else {
    /* (u, v) = (p - j r, -(-1)^par (tp + j tr)), j ~ (p - tp) / (r + tr) */
    double pf = lat_f64( p ), rf = lat_f64( r ), tpf = lat_f64_4( tp ), trf = lat_f64_4( tr );
    double jf = ((pf - tpf) / (rf + trf)) * (1.0 - 0x1p-40);
    uint32_t jj = jf < 1.0 ? 0u : (jf < 4294967295.0 ? (uint32_t)jf : 0xffffffffu);
    /* clamp to floor(p/r) (only matters if the estimate is off) */
    if( jj ) {
      int s; uint32_t mq = lat_qest( pf, rf, &s );
      if( s == 0 && mq < jj ) jj = mq;
    }
    uint32_t t8[ 8 ] = { tp[0], tp[1], tp[2], tp[3], 0u, 0u, 0u, 0u };
    uint32_t tr8[ 8 ] = { tr[0], tr[1], tr[2], tr[3], 0u, 0u, 0u, 0u };
    if( jj ) lat_submul<8>( p, r, t8, tr8, jj, 0 );
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = p[j]; v[j] = t8[j]; }
    *u_neg = par ^ 1;
  }
  return it;
}

#endif /* FD_LATTICE_DEV_H */
