// field_host_check.cpp -- TEST ONLY: compiles the device field header for the
// host so tests/test_field_bounds.py can drive fe_mul/fe_sq/... with limb
// vectors at the documented bounds and compare against Python big ints.
#include "../../firedancer_amd/csrc/fd_f25519_dev.h"
extern "C" {
void t_mul( uint32_t * h, uint32_t const * f, uint32_t const * g ) { fe a, b, r; for( int i=0;i<10;i++ ){a.v[i]=f[i];b.v[i]=g[i];} fe_mul( r, a, b ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_sq ( uint32_t * h, uint32_t const * f ) { fe a, r; for( int i=0;i<10;i++ ) a.v[i]=f[i]; fe_sq( r, a ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_sq_seed( uint32_t * h, uint32_t const * f, uint32_t const * g ) { fe a, b, r; for( int i=0;i<10;i++ ){a.v[i]=f[i];b.v[i]=g[i];} fe_sq_seed( r, a, b ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_sub4p( uint32_t * h, uint32_t const * f ) { fe a, r; for( int i=0;i<10;i++ ) a.v[i]=f[i]; fe_sub4p( r, a ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_sub( uint32_t * h, uint32_t const * f, uint32_t const * g ) { fe a, b, r; for( int i=0;i<10;i++ ){a.v[i]=f[i];b.v[i]=g[i];} fe_sub( r, a, b ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_carry( uint32_t * h, uint32_t const * f ) { fe a, r; for( int i=0;i<10;i++ ) a.v[i]=f[i]; fe_carry( r, a ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_tobytes( uint32_t * o, uint32_t const * f ) { fe a; for( int i=0;i<10;i++ ) a.v[i]=f[i]; fe_tobytes32( o, a ); }
void t_frombytes( uint32_t * h, uint32_t const * w ) { fe a; fe_frombytes32( a, w ); for( int i=0;i<10;i++ ) h[i]=a.v[i]; }
void t_sq_neg( uint32_t * h, uint32_t const * f ) { fe a, r; for( int i=0;i<10;i++ ) a.v[i]=f[i]; fe_sq_neg( r, a ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_add( uint32_t * h, uint32_t const * f, uint32_t const * g ) { fe a, b, r; for( int i=0;i<10;i++ ){a.v[i]=f[i];b.v[i]=g[i];} fe_add( r, a, b ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_lshl1_add( uint32_t * h, uint32_t const * f, uint32_t const * g ) { fe a, b, r; for( int i=0;i<10;i++ ){a.v[i]=f[i];b.v[i]=g[i];} fe_lshl1_add( r, a, b ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_cneg( uint32_t * h, uint32_t const * f, int neg ) { fe a, r; for( int i=0;i<10;i++ ) a.v[i]=f[i]; fe_cneg( r, a, neg != 0 ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
void t_pow22523( uint32_t * h, uint32_t const * f ) { fe a, r; for( int i=0;i<10;i++ ) a.v[i]=f[i]; fe_pow22523( r, a ); for( int i=0;i<10;i++ ) h[i]=r.v[i]; }
}
#include "../../firedancer_amd/csrc/fd_scalar_dev.h"
#include "../../firedancer_amd/csrc/fd_sha512_dev.h"
extern "C" {
void t_sc_reduce( uint32_t * r, uint32_t const * x ) { sc_reduce512( r, x ); }
int  t_sc_lt_l( uint32_t const * s ) { return sc_lt_l( s ); }
void t_recode4( uint8_t * o, uint32_t const * s ) { sc_recode_w4( o, s ); }
void t_recode8( uint8_t * o, uint32_t const * s ) { sc_recode_w8( o, s ); }
int  t_recode_p_top( int nbits ) { return recode_p_top( nbits ); }
void t_recode_p( uint8_t * o, uint32_t const * x, int P ) {    /* ybias_p's digits, biased */
  uint32_t y[ 8 ]; ybias_p( y, x, P );
  int nw = ((P + 3) >> 2) + 1;
  for( int i=0; i<nw-1; i++ ) o[i] = (uint8_t)recode_p_low( y, i, P );
  o[nw-1] = (uint8_t)recode_p_hi( y, P );
}
void t_sha_block( uint64_t * h, uint64_t * w ) { sha512_compress( h, w ); }
void t_comb_digits( int * d, uint32_t const * w ) {
  uint32_t y[ 8 ]; comb_bias( y, w );
  for( int k=0; k<11; k++ ) d[k] = comb_digit( y, k );
  /* the cached kernel's form: shift the biased scalar down 23 bits per digit */
  for( int k=1; k<11; k++ ) {
    for( int j=0; j<7; j++ ) y[j] = (uint32_t)((((uint64_t)y[j+1] << 32) | y[j]) >> 23);
    y[7] >>= 23;
    int dd = (int)(y[0] & ((1u << 23) - 1u)) - (k < 10 ? (1 << 22) : 0);
    if( dd != d[k] ) d[k] = 0x7fffffff;      /* disagreement flag */
  }
}
}
#include "../../firedancer_amd/csrc/fd_lattice_dev.h"
extern "C" {
int t_lattice( uint32_t const * k, uint32_t * u, uint32_t * v, int * u_neg ) { return lat_short_vector( k, u, v, u_neg ); }
}
#include "../../firedancer_amd/csrc/fd_curve25519_dev.h"
extern "C" {
/* p: X,Y,Z,T (40 limbs) -> r = 2p with T (40 limbs) */
void t_dbl( uint32_t * r, uint32_t const * p ) {
  ge_p3 a, o; for( int i=0;i<10;i++ ){ a.X.v[i]=p[i]; a.Y.v[i]=p[10+i]; a.Z.v[i]=p[20+i]; a.T.v[i]=p[30+i]; }
  ge_dbl( o, a, true );
  for( int i=0;i<10;i++ ){ r[i]=o.X.v[i]; r[10+i]=o.Y.v[i]; r[20+i]=o.Z.v[i]; r[30+i]=o.T.v[i]; }
}
int t_is_zero( uint32_t const * f ) { fe a; for( int i=0;i<10;i++ ) a.v[i]=f[i]; return fe_is_zero( a ); }
/* decode with the kernels' small-order flag, and the flag of the affine
   test on the decoded point (bytes of X and Y), for comparison */
int t_decode_small( uint32_t const * w, int avx512_rule, int * small, int * small_affine ) {
  ge_p3 P; int ok = ge_decode_small( P, w, avx512_rule != 0, small );
  *small_affine = ge_affine_small_order( P );
  return ok;
}
}
extern "C" {
/* The host build of fd_fe_test_kernel's operations (fd_ed25519_gpu_kern.hip):
   same op numbers, same 40-limb records, for a limb-exact comparison. */
void t_op( int op, uint32_t const * a, uint32_t const * b, uint32_t * out, uint64_t n ) {
  for( uint64_t i=0; i<n; i++ ) {
    uint32_t const * pa = a + i*40u; uint32_t const * pb = b + i*40u; uint32_t * po = out + i*40u;
    for( int j=0; j<40; j++ ) po[j] = 0u;
    fe x, y, r;
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
      for( int j=0; j<10; j++ ) po[j] = r.v[j];
      continue;
    }
    ge_p3 p, o;
    for( int j=0; j<10; j++ ) { p.X.v[j] = pa[j]; p.Y.v[j] = pa[10+j]; p.Z.v[j] = pa[20+j]; p.T.v[j] = pa[30+j]; }
    if( op == 8 ) ge_dbl( o, p, true );
    else {
      ge_cached q;
      for( int j=0; j<10; j++ ) { q.YpX.v[j] = pb[j]; q.YmX.v[j] = pb[10+j]; q.T2d.v[j] = pb[20+j]; q.Z2.v[j] = pb[30+j]; }
      ge_add_cached( o, p, q, true );
    }
    for( int j=0; j<10; j++ ) { po[j] = o.X.v[j]; po[10+j] = o.Y.v[j]; po[20+j] = o.Z.v[j]; po[30+j] = o.T.v[j]; }
  }
}
}
