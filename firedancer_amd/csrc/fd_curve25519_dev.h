/* fd_curve25519_dev.h -- twisted Edwards group ops for gfx950 (a = -1,
   d = -121665/121666), one point per lane, extended coordinates.

   Replaces the verify-path group code of the reference:
     fd_ed25519_point_frombytes      src/ballet/ed25519/fd_curve25519.c:25-62
     fd_r43x6_ge_decode2 (AVX-512)   src/ballet/ed25519/avx512/fd_r43x6_ge.c:163-254
     fd_ed25519_partial_dbl          src/ballet/ed25519/ref/fd_curve25519.h:190-211
     fd_ed25519_point_add_with_opts  src/ballet/ed25519/ref/fd_curve25519.c:25-92
     fd_curve25519_into_precomputed  src/ballet/ed25519/ref/fd_curve25519.h:144-154
     fd_ed25519_affine_is_small_order src/ballet/ed25519/fd_curve25519.h:81-111
     fd_ed25519_point_eq_z1          src/ballet/ed25519/ref/fd_curve25519.h:132-139
   Limb-bound bookkeeping (R / M, see fd_f25519_dev.h) is noted per line. */

#ifndef FD_CURVE25519_DEV_H
#define FD_CURVE25519_DEV_H

#include "fd_f25519_dev.h"

/* Big group operations are compiled as real (non-inlined) device functions:
   it bounds the register allocator to one operation at a time (the kernel
   otherwise interleaves independent point ops and spills). */
#if defined(__HIPCC__)
#define FD_GE_FN __device__ __forceinline__
#else
#define FD_GE_FN static
#endif

struct ge_p3     { fe X, Y, Z, T; };          /* all R */
struct ge_cached { fe YpX, YmX, T2d, Z2; };   /* (Y+X, Y-X, 2dT, 2Z): 2dT in R, the others in M */
struct ge_precomp{ fe YpX, YmX, T2d; };       /* affine (Z=1) form of ge_cached */

/* d, 2d, sqrt(-1) in radix 2^25.5 (derived: d = -121665/121666 mod p) */
FD_FN void fe_const_d( fe & r ) {
  r.v[0]=0x35978a3u; r.v[1]=0x0d37284u; r.v[2]=0x3156ebdu; r.v[3]=0x06a0a0eu; r.v[4]=0x001c029u;
  r.v[5]=0x179e898u; r.v[6]=0x3a03cbbu; r.v[7]=0x1ce7198u; r.v[8]=0x2e2b6ffu; r.v[9]=0x1480db3u;
}
FD_FN void fe_const_d2( fe & r ) {
  r.v[0]=0x2b2f159u; r.v[1]=0x1a6e509u; r.v[2]=0x22add7au; r.v[3]=0x0d4141du; r.v[4]=0x0038052u;
  r.v[5]=0x0f3d130u; r.v[6]=0x3407977u; r.v[7]=0x19ce331u; r.v[8]=0x1c56dffu; r.v[9]=0x0901b67u;
}
FD_FN void fe_const_sqrtm1( fe & r ) {
  r.v[0]=0x20ea0b0u; r.v[1]=0x186c9d2u; r.v[2]=0x08f189du; r.v[3]=0x035697fu; r.v[4]=0x0bd0c60u;
  r.v[5]=0x1fbd7a7u; r.v[6]=0x2804c9eu; r.v[7]=0x1e16569u; r.v[8]=0x004fc1du; r.v[9]=0x0ae0c92u;
}

/* 1/d */
FD_FN void fe_const_invd( fe & r ) {
  r.v[0]=0x1c9f843u; r.v[1]=0x03c9db3u; r.v[2]=0x285c4bcu; r.v[3]=0x0c213cau; r.v[4]=0x02d775au;
  r.v[5]=0x1b9cf66u; r.v[6]=0x3108a66u; r.v[7]=0x1c86562u; r.v[8]=0x1214d5cu; r.v[9]=0x10241fbu;
}

FD_FN void ge_identity( ge_p3 & p ) { fe_set0( p.X ); fe_set1( p.Y ); fe_set1( p.Z ); fe_set0( p.T ); }

/* r = 2p (dbl-2008-hwcd, a=-1).  p.X,Y,Z in R.  T computed iff want_t.
   Operand order of the output products (here and in the additions): each
   premultiplied operand (x2 odd limbs of the first, x19 of the second) is
   computed once and shared by two products (the compiler merges them; the
   E/G-first order of the first change: -90 v_mul_lo_u32 and -65 shifts in
   the pair kernel, 0.674 vs 0.677 ms at 64K, profiles/r01/ab_operand_order.txt).
   Here and in ge_madd, F and H are the FIRST operands and E, G the second:
   F is then left uncarried (bound class "F" of fd_f25519_dev.h: its x19 would
   not fit 32 bits, its x2 does, and F x M column sums stay below 2^63),
   which drops one fe_carry per doubling / mixed addition.
   The formula wants G = YY-XX and E = (X+Y)^2-XX-YY; here both come out
   NEGATED at no subtraction of their own: G' = XX-YY (+2p) = -G, and
   E' = H + (-(X+Y)^2) with the square produced in complement form
   (fe_sq_neg: the negation is in the product's finish), so E' = -E is one
   limb-pair addition.  F = 2ZZ-G = 2ZZ+G' needs no 4p-G either.  Every
   output product then carries exactly one negated factor: X' = F E' = -X,
   Y' = H G' = -Y, Z' = F G' = -Z, T' = H E' = -T, i.e. (-X,-Y,-Z,-T), the
   same projective point as 2p. */
FD_GE_FN void ge_dbl( ge_p3 & r, ge_p3 const & p, bool want_t ) {
  fe XX, YY, ZZ, s, H, G, E, Fn;
  fe_sq( XX, p.X );                     /* R */
  FE_FENCE();
  fe_sq( YY, p.Y );                     /* R */
  FE_FENCE();
  fe_sq( ZZ, p.Z );                     /* R */
  FE_FENCE();
  fe_add( H, YY, XX );                  /* M   H = YY+XX, not carried: first operand only */
  fe_add( s, p.X, p.Y );                /* M */
  fe_sq_neg( E, s );                    /* N   -(X+Y)^2, complement form (limb 1 < 2^26) */
  FE_FENCE();
  fe_add( E, E, H );                    /* E'  = XX+YY-(X+Y)^2 = -2XY: a second operand only */
  fe_sub( G, XX, YY );                  /* M   G' = XX-YY+2p = -G */
  fe_lshl1_add( Fn, ZZ, G );            /* F   Fn = 2ZZ+G' = 2ZZ-G, not carried: first operand only */
  fe_mul( r.X, Fn, E );                 /* -X */
  FE_FENCE();
  fe_mul( r.Y, H, G );                  /* -Y */
  FE_FENCE();
  fe_mul( r.Z, Fn, G );                 /* -Z */
  FE_FENCE();
  if( want_t ) fe_mul( r.T, H, E );     /* -T */
  FE_FENCE();
}

/* r = p + q, q cached (projective).  p in R.  neg: add -q instead. */
FD_GE_FN void ge_add_cached( ge_p3 & r, ge_p3 const & p, ge_cached const & q, bool want_t ) {
  fe a, b, PP, MM, TT, D, E, F, G, H;
  fe_add( a, p.Y, p.X );                /* M */
  fe_sub( b, p.Y, p.X );                /* M */
  fe_mul( PP, a, q.YpX );
  FE_FENCE();
  fe_mul( MM, b, q.YmX );
  FE_FENCE();
  fe_mul( TT, p.T, q.T2d );
  FE_FENCE();
  fe_mul( D,  p.Z, q.Z2 );              /* 2 Z1 Z2 */
  FE_FENCE();
  fe_sub( E, PP, MM );                  /* M */
  fe_add( H, PP, MM );                  /* M */
  fe_add( G, D, TT );                   /* M */
  fe_sub( F, D, TT );                   /* M */
  fe_mul( r.X, E, F );
  FE_FENCE();
  fe_mul( r.Y, G, H );
  FE_FENCE();
  fe_mul( r.Z, G, F );
  FE_FENCE();
  if( want_t ) fe_mul( r.T, E, H );
  FE_FENCE();
}

/* r = p + q, q affine precomputed (Z2 = 1).  T2d may be given in M form
   (negated) -- it is only a multiplicand. */
FD_GE_FN void ge_madd( ge_p3 & r, ge_p3 const & p, ge_precomp const & q, bool want_t ) {
  fe a, b, PP, MM, TT, D, E, F, G, H;
  fe_add( a, p.Y, p.X );                /* M */
  fe_sub( b, p.Y, p.X );                /* M */
  fe_mul( PP, a, q.YpX );
  FE_FENCE();
  fe_mul( MM, b, q.YmX );
  FE_FENCE();
  fe_mul( TT, p.T, q.T2d );
  FE_FENCE();
  fe_add( D, p.Z, p.Z );                /* 2R */
  fe_sub( E, PP, MM );                  /* M */
  fe_add( H, PP, MM );                  /* M */
  fe_add( G, D, TT );                   /* 3R -> M */
  fe_sub( F, D, TT );                   /* F (4R + ...), not carried: first operand only */
  fe_mul( r.X, F, E );
  FE_FENCE();
  fe_mul( r.Y, H, G );
  FE_FENCE();
  fe_mul( r.Z, F, G );
  FE_FENCE();
  if( want_t ) fe_mul( r.T, H, E );
  FE_FENCE();
}

/* Cached form.  Y+X, Y-X and 2Z are left uncarried (M): every consumer
   (ge_add_cached, through vtab_finish's swap) uses them only as the second
   operand of fe_mul, which takes M.  T2d stays R (vtab_finish negates it). */
FD_FN void ge_to_cached( ge_cached & c, ge_p3 const & p ) {
  fe d2; fe_const_d2( d2 );
  fe_add( c.YpX, p.Y, p.X );
  fe_sub( c.YmX, p.Y, p.X );
  fe_mul( c.T2d, p.T, d2 );
  FE_FENCE();
  fe_add( c.Z2, p.Z, p.Z );
}

/* The extended point of a cached entry (Y+X, Y-X, 2dT, 2Z), scaled by 2:
   (Y+X - (Y-X), Y+X + Y-X, 2Z, 2dT / d) = (2X, 2Y, 2Z, 2T), the same
   projective point -- what identity + entry gives, for ~1/4 of an addition
   (the Straus chain's first window).  Y+X and Y-X may be M (the cached
   form's bound), so the difference takes a 4p bias; 2dT may be M (a
   negated entry); every output is carried to R. */
FD_FN void ge_from_cached( ge_p3 & r, ge_cached const & c ) {
  fe t;
  t.v[0] = c.YpX.v[0] + FE_4P0 - c.YmX.v[0];
#pragma unroll
  for( int i=1; i<10; i++ ) t.v[i] = c.YpX.v[i] + ((i&1) ? FE_4PO : FE_4PE) - c.YmX.v[i];
  fe_carry( r.X, t );
  fe_add( t, c.YpX, c.YmX );
  fe_carry( r.Y, t );
  fe_carry( r.Z, c.Z2 );
  fe invd; fe_const_invd( invd );
  fe_mul( r.T, c.T2d, invd );
  FE_FENCE();
}

/* 1/z = z^(p-2) = (z^(2^252-3))^8 * z^3 */
FD_GE_FN void fe_invert( fe & out, fe const & z ) {
  fe t, z2, z3;
  fe_pow22523( t, z );
  fe_sqn( t, t, 3 );
  fe_sq( z2, z ); fe_mul( z3, z2, z );
  FE_FENCE();
  fe_mul( out, t, z3 );
  FE_FENCE();
}

/* Point decompression.  w: 8 LE words of the 32-byte encoding.  Returns 1
   on success.  Semantics: y = w with bit 255 cleared
   (not reduced), u = y^2-1, v = dy^2+1, x = uv^3 (uv^7)^((p-5)/8); fail if
   neither vx^2 == u nor vx^2 == -u; x *= sqrt(-1) in the second case.
   avx512_rule: also fail on x == 0 with sign bit 1 (fd_r43x6_ge.c:139-140). */
FD_GE_FN int ge_decode_small( ge_p3 & P, uint32_t const w[ 8 ], bool avx512_rule, int * small );
FD_GE_FN int ge_decode( ge_p3 & P, uint32_t const w[ 8 ], bool avx512_rule ) { int sm; return ge_decode_small( P, w, avx512_rule, &sm ); }

/* ge_decode plus the order <= 8 test of the decoded point (*small;
   meaningful when the decode succeeds): x == 0 from the bytes of x the
   decode computes anyway, and y's canonical value in {0, y0, y1} read off
   the encoding: y is w with bit 255 cleared, so its canonical value is 0, y0
   or y1 iff that word string is 0, p, y0 or y1 (y0 + p and y1 + p are past
   2^255).  Equals ge_affine_small_order on the decoded point. */
FD_GE_FN int ge_decode_small( ge_p3 & P, uint32_t const w[ 8 ], bool avx512_rule, int * small ) {
  fe one, d, y, y2, u, v, v2, v3, v4, uv3, uv7, t, x, x2, vxx, chk;
  fe_set1( one ); fe_const_d( d );
  int sign = (int)(w[7] >> 31);
  fe_frombytes32( y, w );               /* R */
  fe_sq( y2, y );
  FE_FENCE();
  fe_sub( u, y2, one ); fe_carry( u, u );        /* R */
  fe_mul( v, y2, d ); v.v[0] += 1u; fe_carry( v, v ); /* R */
  FE_FENCE();
  fe_sq( v2, v );
  FE_FENCE();
  fe_mul( v3, v2, v );
  FE_FENCE();
  fe_sq( v4, v2 );
  FE_FENCE();
  fe_mul( uv3, u, v3 );
  FE_FENCE();
  fe_mul( uv7, uv3, v4 );
  FE_FENCE();
  fe_pow22523( t, uv7 );
  fe_mul( x, uv3, t );
  FE_FENCE();
  fe_sq( x2, x );
  FE_FENCE();
  fe_mul( vxx, v, x2 );                 /* R */
  FE_FENCE();
  fe_sub( chk, vxx, u ); fe_carry( chk, chk );
  int ok_pos = fe_is_zero( chk );
  fe_add( chk, vxx, u ); fe_carry( chk, chk );
  int ok_neg = fe_is_zero( chk );
  if( !ok_pos ) {
    fe sm1; fe_const_sqrtm1( sm1 );
    fe_mul( x, x, sm1 );
    FE_FENCE();
  }
  int ok = ok_pos | ok_neg;
  uint32_t xb[ 8 ]; fe_tobytes32( xb, x );
  int x_zero = !(xb[0]|xb[1]|xb[2]|xb[3]|xb[4]|xb[5]|xb[6]|xb[7]);
  if( avx512_rule && x_zero && sign ) ok = 0;
  if( (int)(xb[0] & 1u) != sign ) { fe nx; fe_neg( nx, x ); fe_carry( x, nx ); }
  P.X = x; P.Y = y; fe_set1( P.Z );
  fe_mul( P.T, x, y );
  FE_FENCE();
  {
    uint32_t const y0[ 8 ] = { 0x8f95e826u,0xb027b2c2u,0x89f4c345u,0xf098eff2u,0x05acdfd5u,0x3933c6d3u,0x880238b1u,0x05fc536du };
    uint32_t const y1[ 8 ] = { 0x706a17c7u,0x4fd84d3du,0x760b3cbau,0x0f67100du,0xfa53202au,0xc6cc392cu,0x77fdc74eu,0x7a03ac92u };
    uint32_t yo = 0u, ep = 0u, e0 = 0u, e1 = 0u;
#pragma unroll
    for( int i=0; i<8; i++ ) {
      uint32_t wi = i == 7 ? (w[7] & 0x7fffffffu) : w[i];
      uint32_t pi = i == 0 ? 0xffffffedu : (i == 7 ? 0x7fffffffu : 0xffffffffu);
      yo |= wi; ep |= wi ^ pi; e0 |= wi ^ y0[i]; e1 |= wi ^ y1[i];
    }
    *small = x_zero | (yo == 0u) | (ep == 0u) | (e0 == 0u) | (e1 == 0u);
  }
  return ok;
}

/* order <= 8 test for an affine point (x, y): x==0 | y==0 | y==y0 | y==y1
   (fd_curve25519.h:81-111; y0, y1 = y of the order-8 points). */
FD_FN int ge_affine_small_order( ge_p3 const & P ) {
  uint32_t xb[ 8 ], yb[ 8 ];
  fe_tobytes32( xb, P.X );
  fe_tobytes32( yb, P.Y );
  uint32_t const y0[ 8 ] = { 0x8f95e826u,0xb027b2c2u,0x89f4c345u,0xf098eff2u,0x05acdfd5u,0x3933c6d3u,0x880238b1u,0x05fc536du };
  uint32_t const y1[ 8 ] = { 0x706a17c7u,0x4fd84d3du,0x760b3cbau,0x0f67100du,0xfa53202au,0xc6cc392cu,0x77fdc74eu,0x7a03ac92u };
  uint32_t xo = 0, yo = 0, e0 = 0, e1 = 0;
#pragma unroll
  for( int i=0; i<8; i++ ) { xo |= xb[i]; yo |= yb[i]; e0 |= yb[i] ^ y0[i]; e1 |= yb[i] ^ y1[i]; }
  return (xo == 0u) | (yo == 0u) | (e0 == 0u) | (e1 == 0u);
}

/* X == x_R Z and Y == y_R Z (R affine) */
FD_FN int ge_eq_z1( ge_p3 const & P, ge_p3 const & R ) {
  fe t, dlt;
  fe_mul( t, R.X, P.Z ); fe_sub( dlt, P.X, t ); fe_carry( dlt, dlt );
  FE_FENCE();
  int ex = fe_is_zero( dlt );
  fe_mul( t, R.Y, P.Z ); fe_sub( dlt, P.Y, t ); fe_carry( dlt, dlt );
  FE_FENCE();
  int ey = fe_is_zero( dlt );
  return ex & ey;
}

#endif /* FD_CURVE25519_DEV_H */
