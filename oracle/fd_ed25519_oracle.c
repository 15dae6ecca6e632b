/* fd_ed25519_oracle.c -- TEST INFRASTRUCTURE ONLY (see fd_ed25519_oracle.h).

   Deliberately simple and independent of the GPU code: 4x64-bit limbs with
   unsigned __int128 products, generic square-and-multiply exponentiation,
   bit-serial double-and-add.  Slow (tens of microseconds per verify) but
   easy to audit against the reference semantics cited inline. */

#include "fd_ed25519_oracle.h"
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[ 4 ]; } fe;          /* value < 2^256, congruent mod p */
typedef struct { fe X, Y, Z, T; } ge;              /* extended twisted Edwards, x=X/Z, y=Y/Z, xy=T/Z */

/* ---------------------------------------------------------------- SHA-512
   FIPS 180-4; the reference's portable core is fd_sha512_core_ref
   (src/ballet/sha512/fd_sha512.c:128-229), init/append/fini :264-399. */

static uint64_t const K512[ 80 ] = {
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

static uint64_t ror64( uint64_t x, int n ) { return (x>>n) | (x<<(64-n)); }

static void
sha512_block( uint64_t h[ 8 ], uint8_t const * b ) {
  uint64_t w[ 80 ];
  for( int i=0; i<16; i++ ) {
    uint64_t x = 0; for( int j=0; j<8; j++ ) x = (x<<8) | b[ 8*i+j ];
    w[ i ] = x;
  }
  for( int i=16; i<80; i++ ) {
    uint64_t s0 = ror64( w[i-15], 1 ) ^ ror64( w[i-15], 8 ) ^ (w[i-15]>>7);
    uint64_t s1 = ror64( w[i-2], 19 ) ^ ror64( w[i-2], 61 ) ^ (w[i-2]>>6);
    w[ i ] = w[i-16] + s0 + w[i-7] + s1;
  }
  uint64_t a=h[0],bb=h[1],c=h[2],d=h[3],e=h[4],f=h[5],g=h[6],hh=h[7];
  for( int i=0; i<80; i++ ) {
    uint64_t t1 = hh + (ror64(e,14)^ror64(e,18)^ror64(e,41)) + ((e&f)^(~e&g)) + K512[i] + w[i];
    uint64_t t2 = (ror64(a,28)^ror64(a,34)^ror64(a,39)) + ((a&bb)^(a&c)^(bb&c));
    hh=g; g=f; f=e; e=d+t1; d=c; c=bb; bb=a; a=t1+t2;
  }
  h[0]+=a; h[1]+=bb; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=hh;
}

/* Hash of the concatenation p0[n0] || p1[n1] || p2[n2] without copying. */
static void
sha512_3( uint8_t const * p0, size_t n0, uint8_t const * p1, size_t n1, uint8_t const * p2, size_t n2,
          uint8_t out[ 64 ] ) {
  uint64_t h[ 8 ] = { 0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,0xa54ff53a5f1d36f1ULL,
                      0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL };
  uint8_t buf[ 128 ]; size_t fill = 0; uint64_t total = (uint64_t)(n0+n1+n2);
  uint8_t const * ps[ 3 ] = { p0, p1, p2 }; size_t ns[ 3 ] = { n0, n1, n2 };
  for( int s=0; s<3; s++ ) {
    for( size_t i=0; i<ns[s]; i++ ) {
      buf[ fill++ ] = ps[s][i];
      if( fill==128 ) { sha512_block( h, buf ); fill = 0; }
    }
  }
  buf[ fill++ ] = 0x80;
  if( fill>112 ) { memset( buf+fill, 0, 128-fill ); sha512_block( h, buf ); fill = 0; }
  memset( buf+fill, 0, 128-fill );
  uint64_t bits = total<<3;
  for( int j=0; j<8; j++ ) buf[ 127-j ] = (uint8_t)(bits>>(8*j));
  buf[ 119 ] = (uint8_t)(total>>61);
  sha512_block( h, buf );
  for( int i=0; i<8; i++ ) for( int j=0; j<8; j++ ) out[ 8*i+j ] = (uint8_t)(h[i]>>(56-8*j));
}

void fdo_sha512( uint8_t const * msg, size_t sz, uint8_t out[ 64 ] ) { sha512_3( msg, sz, NULL, 0, NULL, 0, out ); }

/* ---------------------------------------------------------------- scalars
   l = 2^252 + 27742317777372353535851937790883648493
   (src/ballet/ed25519/fd_curve25519_scalar.h:20-30). */

static uint64_t const Lw[ 4 ] = { 0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL };

/* S <= l-1 as a 256-bit little-endian integer (fd_curve25519_scalar.h:57-73) */
static int
scalar_ok( uint8_t const s[ 32 ] ) {
  for( int i=3; i>=0; i-- ) {
    uint64_t w; memcpy( &w, s+8*i, 8 );
    if( w<Lw[i] ) return 1;
    if( w>Lw[i] ) return 0;
  }
  return 0; /* s == l */
}

/* 512-bit mod l (fd_curve25519_scalar.c:3-110), bit-serial: r = 2r + bit mod l */
void
fdo_scalar_reduce( uint8_t out[ 32 ], uint8_t const in[ 64 ] ) {
  uint64_t r[ 4 ] = {0,0,0,0};
  for( int i=511; i>=0; i-- ) {
    uint64_t top = r[3]>>63;
    r[3] = (r[3]<<1) | (r[2]>>63); r[2] = (r[2]<<1) | (r[1]>>63);
    r[1] = (r[1]<<1) | (r[0]>>63); r[0] = (r[0]<<1) | (uint64_t)((in[i>>3]>>(i&7))&1);
    (void)top; /* r < l < 2^253 before the shift, so 2r+1 < 2^254: no overflow */
    int ge = 1;
    for( int k=3; k>=0; k-- ) { if( r[k]>Lw[k] ) { ge = 1; break; } if( r[k]<Lw[k] ) { ge = 0; break; } }
    if( ge ) {
      uint64_t br = 0;
      for( int k=0; k<4; k++ ) { u128 d = (u128)r[k] - Lw[k] - br; r[k] = (uint64_t)d; br = (uint64_t)(d>>64) & 1; }
    }
  }
  memcpy( out, r, 32 );
}

/* ---------------------------------------------------------------- field GF(2^255-19)
   Semantics of fd_f25519_* (src/ballet/ed25519/fd_f25519.h:46-253). */

static void fe_set( fe * r, uint64_t x ) { r->v[0]=x; r->v[1]=r->v[2]=r->v[3]=0; }

static void
fe_add( fe * r, fe const * a, fe const * b ) {
  u128 c = 0;
  for( int i=0; i<4; i++ ) { c += (u128)a->v[i] + b->v[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  while( c ) {                                   /* 2^256 == 38 mod p */
    u128 d = c*38; c = 0;
    for( int i=0; i<4; i++ ) { d += r->v[i]; r->v[i] = (uint64_t)d; d >>= 64; }
    c = d;
  }
}

static void
fe_sub( fe * r, fe const * a, fe const * b ) {
  uint64_t br = 0;
  for( int i=0; i<4; i++ ) { u128 d = (u128)a->v[i] - b->v[i] - br; r->v[i] = (uint64_t)d; br = (uint64_t)(d>>64)&1; }
  while( br ) {                                  /* wrapped by 2^256 == 38: take 38 back */
    uint64_t b2 = 0; u128 d = (u128)r->v[0] - 38; r->v[0] = (uint64_t)d; b2 = (uint64_t)(d>>64)&1;
    for( int i=1; i<4; i++ ) { d = (u128)r->v[i] - b2; r->v[i] = (uint64_t)d; b2 = (uint64_t)(d>>64)&1; }
    br = b2;
  }
}

static void
fe_mul( fe * r, fe const * a, fe const * b ) {
  uint64_t t[ 8 ] = {0};
  for( int i=0; i<4; i++ ) {
    u128 c = 0;
    for( int j=0; j<4; j++ ) { c += (u128)a->v[i]*b->v[j] + t[i+j]; t[i+j] = (uint64_t)c; c >>= 64; }
    t[i+4] = (uint64_t)c;
  }
  u128 c = 0;
  for( int i=0; i<4; i++ ) { c += (u128)t[i+4]*38 + t[i]; r->v[i] = (uint64_t)c; c >>= 64; }
  while( c ) {
    u128 d = c*38; c = 0;
    for( int i=0; i<4; i++ ) { d += r->v[i]; r->v[i] = (uint64_t)d; d >>= 64; }
    c = d;
  }
}

static void fe_sq( fe * r, fe const * a ) { fe_mul( r, a, a ); }

/* canonical value in [0,p) */
static void
fe_canon( uint64_t o[ 4 ], fe const * a ) {
  static uint64_t const Pw[ 4 ] = { 0xffffffffffffffedULL, 0xffffffffffffffffULL, 0xffffffffffffffffULL, 0x7fffffffffffffffULL };
  memcpy( o, a->v, 32 );
  for( int it=0; it<3; it++ ) {
    int ge = 1;
    for( int k=3; k>=0; k-- ) { if( o[k]>Pw[k] ) { ge=1; break; } if( o[k]<Pw[k] ) { ge=0; break; } }
    if( !ge ) break;
    uint64_t br = 0;
    for( int k=0; k<4; k++ ) { u128 d = (u128)o[k] - Pw[k] - br; o[k] = (uint64_t)d; br = (uint64_t)(d>>64)&1; }
  }
}

static int fe_is_zero( fe const * a ) { uint64_t o[4]; fe_canon( o, a ); return !(o[0]|o[1]|o[2]|o[3]); }
static int fe_eq( fe const * a, fe const * b ) { fe d; fe_sub( &d, a, b ); return fe_is_zero( &d ); }
static int fe_sgn( fe const * a ) { uint64_t o[4]; fe_canon( o, a ); return (int)(o[0]&1); }
static void fe_neg( fe * r, fe const * a ) { fe z; fe_set( &z, 0 ); fe_sub( r, &z, a ); }

/* a^e for a 256-bit exponent e (little-endian words) */
static void
fe_pow( fe * r, fe const * a, uint64_t const e[ 4 ] ) {
  fe acc; fe_set( &acc, 1 );
  for( int i=255; i>=0; i-- ) {
    fe_sq( &acc, &acc );
    if( (e[i>>6]>>(i&63))&1 ) fe_mul( &acc, &acc, a );
  }
  *r = acc;
}

static void
fe_inv( fe * r, fe const * a ) {    /* a^(p-2) (fd_f25519_inv, fd_f25519.c:61-103) */
  static uint64_t const e[ 4 ] = { 0xffffffffffffffebULL, 0xffffffffffffffffULL, 0xffffffffffffffffULL, 0x7fffffffffffffffULL };
  fe_pow( r, a, e );
}

static void
fe_pow22523( fe * r, fe const * a ) { /* a^((p-5)/8) = a^(2^252-3) (fd_f25519_pow22523, fd_f25519.c:10-59) */
  static uint64_t const e[ 4 ] = { 0xfffffffffffffffdULL, 0xffffffffffffffffULL, 0xffffffffffffffffULL, 0x0fffffffffffffffULL };
  fe_pow( r, a, e );
}

static void
fe_frombytes( fe * r, uint8_t const b[ 32 ] ) { /* bit 255 ignored, NOT reduced (fd_f25519_frombytes) */
  memcpy( r->v, b, 32 );
  r->v[3] &= 0x7fffffffffffffffULL;
}

static void
fe_tobytes( uint8_t b[ 32 ], fe const * a ) { uint64_t o[4]; fe_canon( o, a ); memcpy( b, o, 32 ); }

/* ---------------------------------------------------------------- constants, derived from definitions
   d = -121665/121666, sqrt(-1) = 2^((p-1)/4), base point y = 4/5, x even
   (values tabulated by the reference in table/fd_f25519_table_ref.c:38,43 and
   table/fd_curve25519_table_ref.c:8). */

static fe C_d, C_sqrtm1, C_one;
static ge C_B;
static int C_init = 0;

static int decode( ge * P, uint8_t const b[ 32 ], int flavor );

static void
consts_init( void ) {
  if( C_init ) return;
  fe a, b;
  fe_set( &C_one, 1 );
  fe_set( &a, 121665 ); fe_set( &b, 121666 );
  fe_inv( &b, &b ); fe_mul( &C_d, &a, &b ); fe_neg( &C_d, &C_d );
  static uint64_t const e[ 4 ] = { 0xfffffffffffffffbULL, 0xffffffffffffffffULL, 0xffffffffffffffffULL, 0x1fffffffffffffffULL };
  fe_set( &a, 2 ); fe_pow( &C_sqrtm1, &a, e );
  fe_set( &a, 4 ); fe_set( &b, 5 ); fe_inv( &b, &b ); fe_mul( &a, &a, &b );
  uint8_t yb[ 32 ]; fe_tobytes( yb, &a );
  C_init = 1;
  decode( &C_B, yb, FDO_FLAVOR_REF );
}

/* ---------------------------------------------------------------- group */

/* Point decompression.  Follows fd_ed25519_point_frombytes
   (src/ballet/ed25519/fd_curve25519.c:25-62): y taken unreduced with bit 255
   cleared, u = y^2-1, v = dy^2+1, x = uv^3 (uv^7)^((p-5)/8), fix by sqrt(-1)
   or fail, then select the sign.  AVX-512 flavor additionally fails on
   x==0 && sign==1 (src/ballet/ed25519/avx512/fd_r43x6_ge.c:139-140,231-232). */
static int
decode( ge * P, uint8_t const b[ 32 ], int flavor ) {
  fe y, u, v, v3, t, x, vxx, chk;
  fe_frombytes( &y, b );
  int sign = b[31]>>7;
  fe_sq( &u, &y ); fe_mul( &v, &u, &C_d ); fe_sub( &u, &u, &C_one ); fe_add( &v, &v, &C_one );
  fe_sq( &v3, &v ); fe_mul( &v3, &v3, &v );                 /* v^3 */
  fe_sq( &t, &v3 ); fe_mul( &t, &t, &v ); fe_mul( &t, &t, &u ); /* u v^7 */
  fe_pow22523( &t, &t );
  fe_mul( &x, &t, &v3 ); fe_mul( &x, &x, &u );              /* u v^3 (u v^7)^((p-5)/8) */
  fe_sq( &vxx, &x ); fe_mul( &vxx, &vxx, &v );
  fe_sub( &chk, &vxx, &u );
  if( !fe_is_zero( &chk ) ) {
    fe_add( &chk, &vxx, &u );
    if( !fe_is_zero( &chk ) ) return 0;
    fe_mul( &x, &x, &C_sqrtm1 );
  }
  if( flavor==FDO_FLAVOR_AVX512 && fe_is_zero( &x ) && sign ) return 0;
  if( fe_sgn( &x )!=sign ) fe_neg( &x, &x );
  P->X = x; P->Y = y; fe_set( &P->Z, 1 ); fe_mul( &P->T, &x, &y );
  return 1;
}

/* x==0 | y==0 | y==y0 | y==y1 (fd_ed25519_affine_is_small_order, fd_curve25519.h:81-111) */
static int
small_order( ge const * P ) {
  static uint8_t const y0b[ 32 ] = { 0x26,0xe8,0x95,0x8f,0xc2,0xb2,0x27,0xb0,0x45,0xc3,0xf4,0x89,0xf2,0xef,0x98,0xf0,
                                     0xd5,0xdf,0xac,0x05,0xd3,0xc6,0x33,0x39,0xb1,0x38,0x02,0x88,0x6d,0x53,0xfc,0x05 };
  static uint8_t const y1b[ 32 ] = { 0xc7,0x17,0x6a,0x70,0x3d,0x4d,0xd8,0x4f,0xba,0x3c,0x0b,0x76,0x0d,0x10,0x67,0x0f,
                                     0x2a,0x20,0x53,0xfa,0x2c,0x39,0xcc,0xc6,0x4e,0xc7,0xfd,0x77,0x92,0xac,0x03,0x7a };
  fe y0, y1; fe_frombytes( &y0, y0b ); fe_frombytes( &y1, y1b );
  return fe_is_zero( &P->X ) | fe_is_zero( &P->Y ) | fe_eq( &P->Y, &y0 ) | fe_eq( &P->Y, &y1 );
}

/* Unified addition, a=-1 (add-2008-hwcd-3; reference ref/fd_curve25519.c:25-92) */
static void
ge_add( ge * r, ge const * p, ge const * q ) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub( &a, &p->Y, &p->X ); fe_sub( &t, &q->Y, &q->X ); fe_mul( &a, &a, &t );
  fe_add( &b, &p->Y, &p->X ); fe_add( &t, &q->Y, &q->X ); fe_mul( &b, &b, &t );
  fe_mul( &c, &p->T, &q->T ); fe_mul( &c, &c, &C_d ); fe_add( &c, &c, &c );
  fe_mul( &d, &p->Z, &q->Z ); fe_add( &d, &d, &d );
  fe_sub( &e, &b, &a ); fe_sub( &f, &d, &c ); fe_add( &g, &d, &c ); fe_add( &h, &b, &a );
  fe_mul( &r->X, &e, &f ); fe_mul( &r->Y, &g, &h ); fe_mul( &r->T, &e, &h ); fe_mul( &r->Z, &f, &g );
}

/* Doubling (dbl-2008-hwcd; reference ref/fd_curve25519.h:190-211) */
static void
ge_dbl( ge * r, ge const * p ) {
  fe a, b, c, e, f, g, h, t;
  fe_sq( &a, &p->X ); fe_sq( &b, &p->Y ); fe_sq( &c, &p->Z ); fe_add( &c, &c, &c );
  fe_add( &h, &a, &b ); fe_add( &t, &p->X, &p->Y ); fe_sq( &t, &t ); fe_sub( &e, &h, &t );
  fe_sub( &g, &a, &b ); fe_add( &f, &c, &g );
  fe_mul( &r->X, &e, &f ); fe_mul( &r->Y, &g, &h ); fe_mul( &r->T, &e, &h ); fe_mul( &r->Z, &f, &g );
}

static void
ge_neg( ge * r, ge const * p ) { r->Y = p->Y; r->Z = p->Z; fe_neg( &r->X, &p->X ); fe_neg( &r->T, &p->T ); }

/* [n1]A + [n2]B, bit serial (fd_ed25519_double_scalar_mul_base, fd_curve25519.c:122-166, evaluates
   the same group element with a wNAF schedule) */
static void
dmul( ge * r, uint8_t const n1[ 32 ], ge const * A, uint8_t const n2[ 32 ] ) {
  ge acc; fe_set( &acc.X, 0 ); fe_set( &acc.Y, 1 ); fe_set( &acc.Z, 1 ); fe_set( &acc.T, 0 );
  for( int i=255; i>=0; i-- ) {
    ge_dbl( &acc, &acc );
    if( (n1[i>>3]>>(i&7))&1 ) ge_add( &acc, &acc, A );
    if( (n2[i>>3]>>(i&7))&1 ) ge_add( &acc, &acc, &C_B );
  }
  *r = acc;
}

/* X == x_R Z and Y == y_R Z (fd_ed25519_point_eq_z1, ref/fd_curve25519.h:132-139) */
static int
eq_z1( ge const * P, ge const * R ) {
  fe t;
  fe_mul( &t, &R->X, &P->Z ); if( !fe_eq( &t, &P->X ) ) return 0;
  fe_mul( &t, &R->Y, &P->Z ); if( !fe_eq( &t, &P->Y ) ) return 0;
  return 1;
}

/* ---------------------------------------------------------------- verify
   fd_ed25519_verify (src/ballet/ed25519/fd_ed25519_user.c:134-229).  Split in
   the reference's two phases so the batch wrapper can reuse them. */

typedef struct { ge A, R; uint8_t k[ 32 ]; } phase1_t;

static int
verify_phase1( phase1_t * s, uint8_t const * msg, size_t sz, uint8_t const sig[ 64 ], uint8_t const pub[ 32 ], int flavor ) {
  if( !scalar_ok( sig+32 ) ) return -1;                                     /* :157-159 ERR_SIG */
  int okA = decode( &s->A, pub, flavor );                                   /* :162 frombytes_2x, A first */
  if( !okA ) return flavor==FDO_FLAVOR_AVX512 ? -1 : -2;                    /* :190-192 (avx512 -1 | ref 1) */
  int okR = decode( &s->R, sig, flavor );
  if( !okR ) return -1;                                                     /* (avx512 -2 | ref 2) -> ERR_SIG */
  if( small_order( &s->A ) ) return -2;                                     /* :193-195 ERR_PUBKEY */
  if( small_order( &s->R ) ) return -1;                                     /* :196-198 ERR_SIG */
  uint8_t h[ 64 ];
  sha512_3( sig, 32, pub, 32, msg, sz, h );                                 /* :203-205 SHA512(R||A||M) */
  fdo_scalar_reduce( s->k, h );                                             /* :206 */
  return 0;
}

static int
verify_phase2( phase1_t * s, uint8_t const sig[ 64 ] ) {
  ge negA, Rc;
  ge_neg( &negA, &s->A );                                                   /* :215 */
  dmul( &Rc, s->k, &negA, sig+32 );                                         /* :216 [k](-A) + [S]B */
  return eq_z1( &Rc, &s->R ) ? 0 : -3;                                      /* :225-228 */
}

int
fdo_verify( uint8_t const * msg, size_t sz, uint8_t const sig[ 64 ], uint8_t const pub[ 32 ], int flavor ) {
  consts_init();
  phase1_t s;
  int err = verify_phase1( &s, msg, sz, sig, pub, flavor );
  if( err ) return err;
  return verify_phase2( &s, sig );
}

/* fd_ed25519_verify_batch_single_msg (fd_ed25519_user.c:231-309): n in [1,16],
   phase 1 for every j in order (first error wins), then phase 2 in order. */
int
fdo_verify_batch_single_msg( uint8_t const * msg, size_t sz, uint8_t const * sigs, uint8_t const * pubs,
                             size_t n, int flavor ) {
  consts_init();
  if( n==0 || n>16 ) return -1;
  phase1_t s[ 16 ];
  for( size_t j=0; j<n; j++ ) {
    int err = verify_phase1( &s[j], msg, sz, sigs+64*j, pubs+32*j, flavor );
    if( err ) return err;
  }
  for( size_t j=0; j<n; j++ ) {
    if( verify_phase2( &s[j], sigs+64*j ) ) return -3;
  }
  return 0;
}

typedef struct { uint32_t sig_off, pub_off, msg_off; uint16_t msg_sz, txn_idx; } fdo_desc_t;

void
fdo_verify_descs( uint8_t const * arena, void const * desc, size_t n, int8_t * out, int flavor ) {
  fdo_desc_t const * d = (fdo_desc_t const *)desc;
  for( size_t i=0; i<n; i++ )
    out[i] = (int8_t)fdo_verify( arena+d[i].msg_off, d[i].msg_sz, arena+d[i].sig_off, arena+d[i].pub_off, flavor );
}
