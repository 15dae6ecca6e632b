/* synth_sign.c -- workload generator for the benchmarks: the fixed-base
   scalar multiplication [s]B on edwards25519, encoded (RFC 8032 5.1.2),
   for many scalars on host threads.  tools/synth.py builds RFC 8032 Ed25519
   signatures from it (hashing and scalar arithmetic in Python), so the
   bench inputs do not come from the reference or the oracle.  Not part of
   the product; checked against the reference signer in tests/test_synth.py.

   Field: radix 2^51, five u64 limbs, unsigned __int128 products.  Points:
   extended twisted-Edwards coordinates (X:Y:Z:T), a = -1.  Scalar
   multiplication: 4-bit fixed windows over a 16-entry table of multiples of
   B, 4 doublings + 1 addition per window (not constant time: test data). */

#include <stdint.h>
#include <string.h>
#include <pthread.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[ 5 ]; } fe;
typedef struct { fe X, Y, Z, T; } ge;

#define M51 ((1ull << 51) - 1u)

static void fe_carry( fe * r ) {
  for( int k=0; k<2; k++ ) {
    uint64_t c;
    c = r->v[ 0 ] >> 51; r->v[ 0 ] &= M51; r->v[ 1 ] += c;
    c = r->v[ 1 ] >> 51; r->v[ 1 ] &= M51; r->v[ 2 ] += c;
    c = r->v[ 2 ] >> 51; r->v[ 2 ] &= M51; r->v[ 3 ] += c;
    c = r->v[ 3 ] >> 51; r->v[ 3 ] &= M51; r->v[ 4 ] += c;
    c = r->v[ 4 ] >> 51; r->v[ 4 ] &= M51; r->v[ 0 ] += 19u * c;
  }
}
static void fe_add( fe * r, fe const * a, fe const * b ) { for( int i=0; i<5; i++ ) r->v[ i ] = a->v[ i ] + b->v[ i ]; fe_carry( r ); }
/* a - b + 4p (limbwise 4p keeps every limb positive for carried inputs) */
static void fe_sub( fe * r, fe const * a, fe const * b ) {
  static const uint64_t p4[ 5 ] = { 4u * (M51 - 18u), 4u * M51, 4u * M51, 4u * M51, 4u * M51 };
  for( int i=0; i<5; i++ ) r->v[ i ] = a->v[ i ] + p4[ i ] - b->v[ i ];
  fe_carry( r );
}
static void fe_mul( fe * r, fe const * a, fe const * b ) {
  uint64_t const * x = a->v, * y = b->v;
  uint64_t y19[ 5 ]; for( int i=0; i<5; i++ ) y19[ i ] = 19u * y[ i ];
  u128 t[ 5 ];
  t[ 0 ] = (u128)x[0]*y[0] + (u128)x[1]*y19[4] + (u128)x[2]*y19[3] + (u128)x[3]*y19[2] + (u128)x[4]*y19[1];
  t[ 1 ] = (u128)x[0]*y[1] + (u128)x[1]*y[0]   + (u128)x[2]*y19[4] + (u128)x[3]*y19[3] + (u128)x[4]*y19[2];
  t[ 2 ] = (u128)x[0]*y[2] + (u128)x[1]*y[1]   + (u128)x[2]*y[0]   + (u128)x[3]*y19[4] + (u128)x[4]*y19[3];
  t[ 3 ] = (u128)x[0]*y[3] + (u128)x[1]*y[2]   + (u128)x[2]*y[1]   + (u128)x[3]*y[0]   + (u128)x[4]*y19[4];
  t[ 4 ] = (u128)x[0]*y[4] + (u128)x[1]*y[3]   + (u128)x[2]*y[2]   + (u128)x[3]*y[1]   + (u128)x[4]*y[0];
  for( int i=0; i<4; i++ ) { t[ i+1 ] += (uint64_t)(t[ i ] >> 51); t[ i ] &= M51; }
  uint64_t c = (uint64_t)(t[ 4 ] >> 51); t[ 4 ] &= M51;
  for( int i=0; i<5; i++ ) r->v[ i ] = (uint64_t)t[ i ];
  r->v[ 0 ] += 19u * c;
  fe_carry( r );
}
static void fe_inv( fe * r, fe const * a ) {          /* a^(p-2), p-2 = 2^255 - 21 */
  fe acc = *a, res;
  int first = 1;
  for( int i=254; i>=0; i-- ) {                       /* left-to-right square-and-multiply */
    int bit = (i == 2 || i == 4) ? 0 : 1;             /* 2^255-21 = 1...1101011 (bits 2 and 4 clear) */
    if( first ) { res = acc; first = 0; continue; }
    fe_mul( &res, &res, &res );
    if( bit ) fe_mul( &res, &res, &acc );
  }
  *r = res;
}
static void fe_tobytes( uint8_t out[ 32 ], fe const * a ) {
  fe t = *a; fe_carry( &t );
  /* subtract p if t >= p */
  uint64_t q = (t.v[ 0 ] + 19u) >> 51;
  q = (t.v[ 1 ] + q) >> 51; q = (t.v[ 2 ] + q) >> 51; q = (t.v[ 3 ] + q) >> 51; q = (t.v[ 4 ] + q) >> 51;
  t.v[ 0 ] += 19u * q;
  for( int i=0; i<4; i++ ) { t.v[ i+1 ] += t.v[ i ] >> 51; t.v[ i ] &= M51; }
  t.v[ 4 ] &= M51;
  uint64_t w[ 4 ] = { t.v[0] | (t.v[1] << 51), (t.v[1] >> 13) | (t.v[2] << 38),
                      (t.v[2] >> 26) | (t.v[3] << 25), (t.v[3] >> 39) | (t.v[4] << 12) };
  memcpy( out, w, 32 );
}
static void fe_frombytes( fe * r, uint8_t const in[ 32 ] ) {
  uint64_t w[ 4 ]; memcpy( w, in, 32 ); w[ 3 ] &= 0x7fffffffffffffffull;
  r->v[ 0 ] = w[0] & M51; r->v[ 1 ] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r->v[ 2 ] = ((w[1] >> 38) | (w[2] << 26)) & M51; r->v[ 3 ] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r->v[ 4 ] = w[3] >> 12;
}

static fe D2;   /* 2d */
static ge TAB[ 16 ];
static pthread_once_t once = PTHREAD_ONCE_INIT;

/* add-2008-hwcd-3 (a = -1) */
static void ge_add( ge * r, ge const * p, ge const * q ) {
  fe a, b, c, d, e, f, g, h, t;
  fe_sub( &a, &p->Y, &p->X ); fe_sub( &t, &q->Y, &q->X ); fe_mul( &a, &a, &t );
  fe_add( &b, &p->Y, &p->X ); fe_add( &t, &q->Y, &q->X ); fe_mul( &b, &b, &t );
  fe_mul( &c, &p->T, &q->T ); fe_mul( &c, &c, &D2 );
  fe_mul( &d, &p->Z, &q->Z ); fe_add( &d, &d, &d );
  fe_sub( &e, &b, &a ); fe_sub( &f, &d, &c ); fe_add( &g, &d, &c ); fe_add( &h, &b, &a );
  fe_mul( &r->X, &e, &f ); fe_mul( &r->Y, &g, &h ); fe_mul( &r->T, &e, &h ); fe_mul( &r->Z, &f, &g );
}
/* dbl-2008-hwcd (a = -1): E = (X+Y)^2 - A - B, G = B - A, F = G - C,
   H = -(A + B) */
static void ge_dbl( ge * r, ge const * p ) {
  fe a, b, c, e, f, g, h, t, zero = { { 0 } };
  fe_mul( &a, &p->X, &p->X ); fe_mul( &b, &p->Y, &p->Y );
  fe_mul( &c, &p->Z, &p->Z ); fe_add( &c, &c, &c );
  fe_add( &t, &p->X, &p->Y ); fe_mul( &t, &t, &t );
  fe_add( &h, &a, &b );
  fe_sub( &e, &t, &h );
  fe_sub( &g, &b, &a );
  fe_sub( &f, &g, &c );
  fe_sub( &h, &zero, &h );
  fe_mul( &r->X, &e, &f ); fe_mul( &r->Y, &g, &h ); fe_mul( &r->T, &e, &h ); fe_mul( &r->Z, &f, &g );
}

static void init_tables( void ) {
  /* d = -121665/121666 */
  fe n = { { 121665 } }, m = { { 121666 } }, zero = { { 0 } }, inv, d;
  fe_inv( &inv, &m ); fe_mul( &d, &n, &inv ); fe_sub( &d, &zero, &d );
  fe_add( &D2, &d, &d );
  /* B: y = 4/5, x even root -- use the standard encoding 0x58666...66 */
  uint8_t by[ 32 ]; memset( by, 0x66, 32 ); by[ 0 ] = 0x58;
  static const uint8_t bx[ 32 ] = {   /* x(B) little-endian */
    0x1a,0xd5,0x25,0x8f,0x60,0x2d,0x56,0xc9,0xb2,0xa7,0x25,0x95,0x60,0xc7,0x2c,0x69,
    0x5c,0xdc,0xd6,0xfd,0x31,0xe2,0xa4,0xc0,0xfe,0x53,0x6e,0xcd,0xd3,0x36,0x69,0x21 };
  ge b;
  fe_frombytes( &b.X, bx ); fe_frombytes( &b.Y, by );
  memset( &b.Z, 0, sizeof(fe) ); b.Z.v[ 0 ] = 1; fe_mul( &b.T, &b.X, &b.Y );
  memset( &TAB[ 0 ], 0, sizeof(ge) ); TAB[ 0 ].Y.v[ 0 ] = 1; TAB[ 0 ].Z.v[ 0 ] = 1;
  TAB[ 1 ] = b;
  for( int i=2; i<16; i++ ) ge_add( &TAB[ i ], &TAB[ i-1 ], &b );
}

static void scalarmult_base( uint8_t out[ 32 ], uint8_t const s[ 32 ] ) {
  ge r = TAB[ 0 ];
  for( int i=63; i>=0; i-- ) {
    for( int k=0; k<4; k++ ) ge_dbl( &r, &r );
    int nib = (s[ i >> 1 ] >> ((i & 1) * 4)) & 15;
    ge_add( &r, &r, &TAB[ nib ] );
  }
  fe zi, x, y;
  fe_inv( &zi, &r.Z ); fe_mul( &x, &r.X, &zi ); fe_mul( &y, &r.Y, &zi );
  uint8_t xb[ 32 ];
  fe_tobytes( out, &y ); fe_tobytes( xb, &x );
  out[ 31 ] |= (uint8_t)((xb[ 0 ] & 1) << 7);
}

typedef struct { uint8_t const * s; uint8_t * out; uint64_t lo, hi; } job_t;
static void * worker( void * arg ) {
  job_t * j = (job_t *)arg;
  for( uint64_t i=j->lo; i<j->hi; i++ ) scalarmult_base( j->out + 32u * i, j->s + 32u * i );
  return NULL;
}

/* out[32 i..] = encode([s_i]B) for n little-endian 32-byte scalars (any
   value < 2^256), on nthreads host threads. */
int
synth_scalarmult_base( uint8_t const * s, uint64_t n, uint8_t * out, int nthreads ) {
  pthread_once( &once, init_tables );
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > 64 ) nthreads = 64;
  pthread_t tid[ 64 ]; job_t job[ 64 ];
  for( int t=0; t<nthreads; t++ ) {
    job[ t ] = (job_t){ s, out, n * (uint64_t)t / (uint64_t)nthreads, n * (uint64_t)(t + 1) / (uint64_t)nthreads };
    pthread_create( &tid[ t ], NULL, worker, &job[ t ] );
  }
  for( int t=0; t<nthreads; t++ ) pthread_join( tid[ t ], NULL );
  return 0;
}
