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

/* FD_OPT_LATSTEP: the Lehmer step with a low-biased reciprocal (one
   quotient correction instead of two, one Newton step instead of two) and
   the exactness tests on S = q EB + EA (48 instead of 61 VALU a step).  It
   leaves every lane's remainder sequence, hence (u, v), unchanged. */
#ifndef FD_OPT_LATSTEP
#define FD_OPT_LATSTEP 1
#endif

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

/* 1/y rounded DOWN by ~2^-35 relative: the hardware reciprocal, relative
   error e (at most 2^-24.36 over 2^32 mantissas, tools/rcp_probe.hip,
   profiles/r06/rcp_probe.json; the argument needs e < 2^-18), and one
   Newton step whose constant carries the bias: r (2 - 2^-35 - y r) =
   (1/y)(1 - e^2 - 2^-35 (1 + e)), an underestimate by 2^-35 (1 -+ 2^-17)
   at most 2^-34.4.  A quotient q* below 2^27 is then floor(A
   lat_rcp_lo(B)) or one more (A lat_rcp_lo(B) > q* - 1 and, after the
   product's 2^-53 rounding, still below A/B). */
FD_LT_FN double lat_rcp_lo( double y ) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp( y );
  return r * fma( -y, r, 2.0 - 0x1p-35 );
#else
  return (1.0 / y) * (1.0 - 0x1p-35);
#endif
}


/* a < b, 8 words */
FD_LT_FN int lat_lt( uint32_t const a[ 8 ], uint32_t const b[ 8 ] ) { return !lat_ge( a, b ); }

/* 8-word x: word i selected by a lane-varying i in [2, 7] (select chain, no
   dynamic register indexing). */
FD_LT_FN uint32_t lat_word( uint32_t const x[ 8 ], int i ) {
  /* word i (2 <= i <= 7) by masks: a select chain over the array is folded
     back into an indexed load by the compiler, which puts x in scratch */
  uint32_t r = 0u;
#pragma unroll
  for( int j=2; j<8; j++ ) r |= x[j] & (0u - (uint32_t)(i == j));
  return r;
}

/* r = m x - n y (9-word two's complement, the caller knows the sign), m, n < 2^32 */
FD_LT_FN void lat_mxny( uint32_t r[ 9 ], uint32_t m, uint32_t const x[ 8 ], uint32_t n, uint32_t const y[ 8 ] ) {
  uint64_t cx = 0, cy = 0; uint32_t br = 0;
#pragma unroll
  for( int j=0; j<8; j++ ) {
    uint64_t px = (uint64_t)m * x[j] + cx; cx = px >> 32;
    uint64_t py = (uint64_t)n * y[j] + cy; cy = py >> 32;
    uint64_t d = (uint64_t)(uint32_t)px - (uint32_t)py - br;
    r[j] = (uint32_t)d; br = (uint32_t)(d >> 63);
  }
  r[8] = (uint32_t)cx - (uint32_t)cy - br;
}

/* r = neg ? -r : r (9 words), result known to fit 8 words */
FD_LT_FN void lat_cneg( uint32_t o[ 8 ], uint32_t const r[ 9 ], int neg ) {
  uint32_t msk = neg ? 0xffffffffu : 0u;
  uint32_t c = neg ? 1u : 0u;
#pragma unroll
  for( int j=0; j<8; j++ ) { uint64_t t = (uint64_t)(r[j] ^ msk) + c; o[j] = (uint32_t)t; c = (uint32_t)(t >> 32); }
}

/* One Lehmer round (Lehmer 1938; exact-quotient test with interval bounds):
   x > y >= 2^128.  The top 53 bits of x and the same bits of y (exact
   truncations X, Y: x/2^e in [X, X+1)) drive Euclid in f64; a step is taken
   only if its quotient is provably the true one given the truncation
   error, and the round stops once the new remainder might be below 2^128
   (the caller finishes the crossing exactly).  The accumulated 2x2
   matrix is then applied to (x, y) and the cofactors (tx, ty).  Returns
   the number of Euclid steps taken (0: no progress, take an exact step).
   Sign bookkeeping: with x = s tx k, y = -s ty k (mod 8l) on entry, the
   same holds on exit with s multiplied by (-1)^steps. */
FD_LT_FN int lat_lehmer( uint32_t x[ 8 ], uint32_t tx[ 4 ], uint32_t y[ 8 ], uint32_t ty[ 4 ], int act ) {
  int t = x[7] ? 7 : (x[6] ? 6 : (x[5] ? 5 : 4));
  uint32_t xt = lat_word( x, t ), xt1 = lat_word( x, t-1 ), xt2 = lat_word( x, t-2 );
  uint32_t yt = lat_word( y, t ), yt1 = lat_word( y, t-1 ), yt2 = lat_word( y, t-2 );
  int c = xt ? __builtin_clz( xt ) : 0;
  uint64_t X64 = ((((uint64_t)xt << 32) | xt1) << c) | (((uint64_t)xt2) >> (32 - c));
  uint64_t Y64 = ((((uint64_t)yt << 32) | yt1) << c) | (((uint64_t)yt2) >> (32 - c));
  double A = (double)(X64 >> 11), B = (double)(Y64 >> 11);
  int e0 = 32*t - 21 - c;                            /* x ~ A 2^e0 */
  double thr = ldexp( 1.0, 128 - e0 );               /* b >= 2^128  <=>  b/2^e0 >= thr */
  double a0 = 1.0, a1 = 0.0, b0 = 0.0, b1 = 1.0;     /* magnitudes of the 2x2 matrix */
  int j = 0;
  int go = act;
  /* branch-free step (selects, no divergent ifs): the branchy form kept
     every loop-carried double live in two register copies, ~20 moves a
     step; a lane that stopped computes on with its state held */
  while( lat_any( go ) ) {
#if FD_OPT_LATSTEP
    /* q from the low-biased reciprocal is the quotient or one less (a q
       that is off by more is >= 2^26 and fails the matrix bound below) */
    double q = floor( A * lat_rcp_lo( B ) );
    double R = fma( -q, B, A );
    int hi = R >= B;
    q = hi ? q + 1.0 : q; R = hi ? R - B : R;
    double EA = a0 + a1, EB = b0 + b1;
    double nb0 = fma( q, b0, a0 ), nb1 = fma( q, b1, a1 );
    /* S = nb0 + nb1 = q EB + EA; the tests below are the ones of the
       form without FD_OPT_LATSTEP rewritten with S, exact whenever S <
       2^26 (every operand is then an integer below 2^53) */
    double S = fma( q, EB, EA );
    int ok = go & (R >= S) & (B - R - EB > S) & (S < 67108864.0);
#else
    double q = floor( A * lat_rcp( B ) );
    double R = fma( -q, B, A );
    int lo = R < 0.0;
    q = lo ? q - 1.0 : q; R = lo ? R + B : R;
    int hi = R >= B;
    q = hi ? q + 1.0 : q; R = hi ? R - B : R;
    double EA = a0 + a1, EB = b0 + b1;
    double nb0 = fma( q, b0, a0 ), nb1 = fma( q, b1, a1 );
    double S = nb0 + nb1;
    /* exact iff q <= true quotient < q+1 for every x/2^e0, y/2^e0 in
       their truncation intervals; keep every quantity below 2^53 */
    int ok = go & (R - EA - q*EB >= 0.0) & (B - R - EA - (q + 1.0)*EB > 0.0) & (S < 67108864.0);
#endif
    A  = ok ? B   : A;  B  = ok ? R   : B;
    a0 = ok ? b0  : a0; a1 = ok ? b1  : a1;
    b0 = ok ? nb0 : b0; b1 = ok ? nb1 : b1;
    j += ok;
    /* stop once the new remainder might be < 2^128 (or shrank too far to steer) */
    go = ok & (R - S >= thr) & (R >= 67108864.0);
  }
  if( act && j ) {
    /* (x', y') = j even: (a0 x - a1 y, b1 y - b0 x); j odd: negated */
    uint32_t ua0 = (uint32_t)a0, ua1 = (uint32_t)a1, ub0 = (uint32_t)b0, ub1 = (uint32_t)b1;
    uint32_t rx[ 9 ], ry[ 9 ];
    lat_mxny( rx, ua0, x, ua1, y );
    lat_mxny( ry, ub1, y, ub0, x );
    uint32_t ntx[ 4 ], nty[ 4 ];
    uint64_t c1 = 0, c2 = 0;
#pragma unroll
    for( int i=0; i<4; i++ ) {
      uint64_t p1 = (uint64_t)ua0 * tx[i] + c1; uint64_t p1b = (uint64_t)ua1 * ty[i] + (uint32_t)p1;
      ntx[i] = (uint32_t)p1b; c1 = (p1 >> 32) + (p1b >> 32);
      uint64_t p2 = (uint64_t)ub0 * tx[i] + c2; uint64_t p2b = (uint64_t)ub1 * ty[i] + (uint32_t)p2;
      nty[i] = (uint32_t)p2b; c2 = (p2 >> 32) + (p2b >> 32);
    }
    lat_cneg( x, rx, j & 1 );
    lat_cneg( y, ry, j & 1 );
#pragma unroll
    for( int i=0; i<4; i++ ) { tx[i] = ntx[i]; ty[i] = nty[i]; }
  }
  return act ? j : 0;
}

/* One exact Euclid step on x > y: x -= m y (f64 estimate, repeated until
   x < y), then swap (x, tx) <-> (y, ty). */
FD_LT_FN void lat_exact_step( uint32_t x[ 8 ], uint32_t tx[ 4 ], uint32_t y[ 8 ], uint32_t ty[ 4 ], int act ) {
  int more = act;
  while( lat_any( more ) ) {
    if( more ) {
      int s; uint32_t m = lat_qest( lat_f64( x ), lat_f64( y ), &s );
      lat_submul<4>( x, y, tx, ty, m, s );
    }
    more = more && lat_ge( x, y );
  }
  if( act ) {
#pragma unroll
    for( int j=0; j<8; j++ ) { uint32_t q = x[j]; x[j] = y[j]; y[j] = q; }
#pragma unroll
    for( int j=0; j<4; j++ ) { uint32_t q = tx[j]; tx[j] = ty[j]; ty[j] = q; }
  }
}

/* Short lattice vector for k (8 LE words, k < l).  Outputs |u| and v (> 0)
   as 8 LE words each and the sign of u.  Returns the number of rounds and
   exact steps (>= FD_LAT_MAX_ITER means the fallback (k, 1) was taken).

   Invariants: x > y, x tx... : x ty + y tx = 8l (Euclid's identity for
   consecutive remainders), y = (-1)^par ty k and x = -(-1)^par tx k
   (mod 8l); each Lehmer round takes j exact Euclid steps at once (par
   advances by j), and the crossing below 2^128 is made by exact steps. */
FD_LT_FN int lat_short_vector( uint32_t const k[ 8 ], uint32_t u[ 8 ], uint32_t v[ 8 ], int * u_neg ) {
  uint32_t x[ 8 ] = { FD_N8L0, FD_N8L1, FD_N8L2, FD_N8L3, 0u, 0u, 0u, FD_N8L7 };
  uint32_t y[ 8 ];
  uint32_t tx[ 4 ] = { 0u, 0u, 0u, 0u }, ty[ 4 ] = { 1u, 0u, 0u, 0u };
#pragma unroll
  for( int j=0; j<8; j++ ) y[j] = k[j];
  int par = 0;
  int active = (y[4] | y[5] | y[6] | y[7]) != 0u;   /* y >= 2^128: keep going */
  int it = 0;
  while( lat_any( active ) ) {
    int jj = lat_lehmer( x, tx, y, ty, active );
    par ^= jj & 1;
    int need = active && jj == 0;
    if( lat_any( need ) ) { lat_exact_step( x, tx, y, ty, need ); par ^= need; }
    if( active ) { it++; active = ((y[4] | y[5] | y[6] | y[7]) != 0u) && it < FD_LAT_MAX_ITER; }
  }
  if( it >= FD_LAT_MAX_ITER ) {
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = k[j]; v[j] = j == 0 ? 1u : 0u; }
    *u_neg = 0;
    return it;
  }
  /* (r, tr) = (y, ty) the first remainder below 2^128, (p, tp) = (x, tx) */
  if( ty[0] & 1u ) {
    /* (u, v) = (r, (-1)^par tr) */
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = y[j]; v[j] = j < 4 ? ty[j] : 0u; }
    *u_neg = par;
  } else {
    /* (u, v) = (p - j r, -(-1)^par (tp + j tr)), j ~ (p - tp) / (r + tr) */
    double pf = lat_f64( x ), rf = lat_f64( y ), tpf = lat_f64_4( tx ), trf = lat_f64_4( ty );
    double jf = ((pf - tpf) / (rf + trf)) * (1.0 - 0x1p-40);
    uint32_t jj = jf < 1.0 ? 0u : (jf < 4294967295.0 ? (uint32_t)jf : 0xffffffffu);
    /* clamp to floor(p/r) (only matters if the estimate is off) */
    if( jj ) {
      int s; uint32_t mq = lat_qest( pf, rf, &s );
      if( s == 0 && mq < jj ) jj = mq;
    }
    uint32_t t8[ 8 ] = { tx[0], tx[1], tx[2], tx[3], 0u, 0u, 0u, 0u };
    uint32_t tr8[ 8 ] = { ty[0], ty[1], ty[2], ty[3], 0u, 0u, 0u, 0u };
    if( jj ) lat_submul<8>( x, y, t8, tr8, jj, 0 );
#pragma unroll
    for( int j=0; j<8; j++ ) { u[j] = x[j]; v[j] = t8[j]; }
    *u_neg = par ^ 1;
  }
  return it;
}

#endif /* FD_LATTICE_DEV_H */
