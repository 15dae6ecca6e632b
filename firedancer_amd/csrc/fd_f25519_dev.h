/* fd_f25519_dev.h -- GF(2^255-19) arithmetic for gfx950, one field element
   per lane in ten 32-bit VGPRs (radix 2^25.5: limb i sits at bit
   ceil(25.5*i); even limbs hold 26 bits, odd limbs 25).

   Replaces fd_f25519_* (src/ballet/ed25519/fd_f25519.h:46-253; ref backend
   5x51 fiat-crypto ref/fd_f25519.h, AVX-512 backend 6x43 r43x6
   avx512/fd_f25519.h).  Design (measured on MI355X, tools/valu_probe.hip,
   profiles/r01_valu_probe.json):

   * v_mad_u64_u32 issues at the same rate as every other "half-rate"
     gfx950 VALU op (mul/mad/add3/alignbit/add_co/addc), ~4.4 cyc per wave
     instruction per SIMD at 8 waves/SIMD, while add/and/xor/lshr_b32 run at
     ~2.5.  A saturated 2^32-radix schoolbook needs an add-with-carry per
     MAC (64 mad + 64 addc per mul); radix 2^25.5 keeps every column sum
     below 2^64, so each MAC is ONE v_mad_u64_u32 and the column carry is
     folded into the next column's chain as its initial addend.
   * Per product: 100 mad (mul) / 55 mad (sqr), +19/x2 premultiplies, one
     64-bit shift + one AND per column.

   Limb bounds (checked by tests/test_field_bounds.py on the exact limb
   operations):
     "R"  (reduced)    even <= 2^26 + 2^11,     odd <= 2^25 + 2^16
     "M"  (mul input)  even <= 3*2^26 + 2^13, odd <= 3*2^25 + 2^18
   so any sum of up to three R values, and R + 2p - R, are valid M inputs.
     "F"  (first operand only) even <= 5*2^26 + 3*2^11, odd <= 5*2^25 + 3*2^16
   (e.g. 2R + R + 2p - R uncarried): fe_mul( h, F, M ) is exact with h in R
   (2*F fits 32 bits, column sums < 2^62.9); 19*F does not fit, so an F value
   is never the second operand of fe_mul nor an fe_sq input.
   fe_mul / fe_sq accept M inputs and return R; fe_sq_seed( h, f, s ) = f^2 + s
   likewise (s limbs < 2^31); fe_add of two R is M;
   fe_sub(R, R) is M; fe_carry(any limbs < 2^31) is R. */

#ifndef FD_F25519_DEV_H
#define FD_F25519_DEV_H

#include <stdint.h>

#if defined(__HIPCC__)
#define FD_FN __device__ __forceinline__
#else
#define FD_FN static inline
#endif

struct fe { uint32_t v[ 10 ]; };

#define FE_M26 0x3ffffffu
#define FE_M25 0x1ffffffu
/* column-0 addend of a complement-form product (fe_sq_neg): 18 + 2^51 */
#define FE_NEG_SEED ( 18ull + (1ull << 51) )

/* 2p and 4p in limb form (limb 0 of p is 2^26-19, others 2^26-1 / 2^25-1) */
#define FE_2P0  (2u*(0x3ffffffu-18u))
#define FE_2PE  (2u*0x3ffffffu)
#define FE_2PO  (2u*0x1ffffffu)

/* 32x32->64 multiply-accumulate (host path and single uses on the device,
   where the compiler emits one v_mad_u64_u32). */
FD_FN uint64_t mad64( uint32_t a, uint32_t b, uint64_t c ) { return (uint64_t)a * (uint64_t)b + c; }
FD_FN uint64_t col5( uint64_t c, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2, uint32_t b2,
                     uint32_t a3, uint32_t b3, uint32_t a4, uint32_t b4 ) {
  return c + (uint64_t)a0*b0 + (uint64_t)a1*b1 + (uint64_t)a2*b2 + (uint64_t)a3*b3 + (uint64_t)a4*b4;
}
#define COL10( c, a0,b0,a1,b1,a2,b2,a3,b3,a4,b4,a5,b5,a6,b6,a7,b7,a8,b8,a9,b9 ) \
  col5( col5( (c), a0,b0,a1,b1,a2,b2,a3,b3,a4,b4 ), a5,b5,a6,b6,a7,b7,a8,b8,a9,b9 )

/* Scheduling fence: keeps the machine scheduler from interleaving
   independent field products (which raises VGPR pressure past the
   occupancy target and spills). */
#if defined(__HIP_DEVICE_COMPILE__)
#define FE_FENCE() __builtin_amdgcn_sched_barrier( 0 )
#else
#define FE_FENCE() do {} while( 0 )
#endif

FD_FN void fe_set0( fe & r ) { for( int i=0; i<10; i++ ) r.v[i] = 0u; }
FD_FN void fe_set1( fe & r ) { r.v[0] = 1u; for( int i=1; i<10; i++ ) r.v[i] = 0u; }

/* Limb pairs.  Every limb stays below 2^31, so a 64-bit add (or a 64-bit
   shift left by one) of two limb pairs never carries out of the low limb:
   it is exactly two independent 32-bit operations, in ONE issue slot
   (v_lshl_add_u64 / v_lshlrev_b64 take the same slot as a v_add_u32 when
   several waves share the SIMD, profiles/r03/probes).  As asm: the compiler
   would otherwise split the 64-bit add back into two 32-bit ones (it may
   assume a carry between the halves). */
FD_FN uint64_t fe_pk( uint32_t lo, uint32_t hi ) { return (uint64_t)lo | ((uint64_t)hi << 32); }
#if defined(__HIP_DEVICE_COMPILE__)
FD_FN uint64_t pk_add( uint64_t a, uint64_t b ) {
  uint64_t r; asm( "v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b) ); return r;
}
FD_FN uint64_t pk_add_s( uint64_t a, uint64_t s ) {      /* s: a wave-uniform pair (SGPRs) */
  uint64_t r; asm( "v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "s"(s) ); return r;
}
FD_FN uint64_t pk_shl1_add( uint64_t a, uint64_t b ) {
  uint64_t r; asm( "v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(a), "v"(b) ); return r;
}
FD_FN uint64_t pk_shl1( uint64_t a ) {
  uint64_t r; asm( "v_lshlrev_b64 %0, 1, %1" : "=v"(r) : "v"(a) ); return r;
}
#else
FD_FN uint64_t pk_add( uint64_t a, uint64_t b ) { return a + b; }
FD_FN uint64_t pk_add_s( uint64_t a, uint64_t s ) { return a + s; }
FD_FN uint64_t pk_shl1_add( uint64_t a, uint64_t b ) { return (a << 1) + b; }
FD_FN uint64_t pk_shl1( uint64_t a ) { return a << 1; }
#endif
#define FE_PK( f, i ) fe_pk( (f).v[2*(i)], (f).v[2*(i)+1] )
#define FE_UNPK( r, i, x ) do { uint64_t _x = (x); (r).v[2*(i)] = (uint32_t)_x; (r).v[2*(i)+1] = (uint32_t)(_x >> 32); } while( 0 )

FD_FN void fe_add( fe & r, fe const & a, fe const & b ) {
#pragma unroll
  for( int i=0; i<5; i++ ) FE_UNPK( r, i, pk_add( FE_PK( a, i ), FE_PK( b, i ) ) );
}

/* r = a + 2p - b.  Requires b limbs <= 2p limbs (b in R).  On the device
   each limb is ONE v_sad_u32: |2p_i - b_i| + a_i, which is 2p_i - b_i + a_i
   since b_i <= 2p_i (and every value is below 2^31, so the signed and the
   unsigned readings of the difference agree) -- ten instructions instead of
   five bias pair-adds plus ten subtractions. */
FD_FN void fe_sub( fe & r, fe const & a, fe const & b ) {
#pragma unroll
  for( int i=0; i<10; i++ ) {
    uint32_t c = i == 0 ? FE_2P0 : ((i & 1) ? FE_2PO : FE_2PE);
#if defined(__HIP_DEVICE_COMPILE__)
    asm( "v_sad_u32 %0, %1, %2, %3" : "=v"(r.v[i]) : "s"(c), "v"(b.v[i]), "v"(a.v[i]) );
#else
    r.v[i] = c - b.v[i] + a.v[i];
#endif
  }
}

/* One parallel carry round: limbs < 2^31 in, R out. */
FD_FN void fe_carry( fe & r, fe const & a ) {
  uint32_t c[ 10 ];
#pragma unroll
  for( int i=0; i<10; i++ ) c[i] = a.v[i] >> ((i&1) ? 25 : 26);
  r.v[0] = (a.v[0] & FE_M26) + 19u*c[9];
#pragma unroll
  for( int i=1; i<10; i++ ) r.v[i] = (a.v[i] & ((i&1) ? FE_M25 : FE_M26)) + c[i-1];
}

FD_FN void fe_add_r( fe & r, fe const & a, fe const & b ) { fe t; fe_add( t, a, b ); fe_carry( r, t ); }
FD_FN void fe_sub_r( fe & r, fe const & a, fe const & b ) { fe t; fe_sub( t, a, b ); fe_carry( r, t ); }

/* 4p - a, limbwise nonnegative for a up to 2R (a in M from a sum of two R);
   the addend of fe_sq_seed that subtracts a */
#define FE_4P0  (4u*(0x3ffffffu-18u))
#define FE_4PE  (4u*0x3ffffffu)
#define FE_4PO  (4u*0x1ffffffu)
FD_FN void fe_sub4p( fe & r, fe const & a ) {
  r.v[0] = FE_4P0 - a.v[0];
#pragma unroll
  for( int i=1; i<10; i++ ) r.v[i] = ((i&1) ? FE_4PO : FE_4PE) - a.v[i];
}

/* r = 2a + b limbwise: one v_lshl_add_u64 per limb pair on the device
   (a's limbs below 2^31, so no bit crosses into the high limb). */
FD_FN void fe_lshl1_add( fe & r, fe const & a, fe const & b ) {
#pragma unroll
  for( int i=0; i<5; i++ ) FE_UNPK( r, i, pk_shl1_add( FE_PK( a, i ), FE_PK( b, i ) ) );
}

/* 2p - a (a in R) -> M */
FD_FN void fe_neg( fe & r, fe const & a ) {
  r.v[0] = FE_2P0 - a.v[0];
#pragma unroll
  for( int i=1; i<10; i++ ) r.v[i] = ((i&1) ? FE_2PO : FE_2PE) - a.v[i];
}

/* r = neg ? 2p - a : a (a in R) per lane: (a ^ m) + (m & (2p+1)) with
   m = neg ? ~0 : 0 is -a-1+2p+1 or a, one v_xad_u32 per limb (plus the
   mask and its three limb constants) instead of a negation and a select. */
FD_FN void fe_cneg( fe & r, fe const & a, bool neg ) {
  uint32_t m = neg ? ~0u : 0u;
  uint32_t c0 = m & (FE_2P0 + 1u), ce = m & (FE_2PE + 1u), co = m & (FE_2PO + 1u);
#pragma unroll
  for( int i=0; i<10; i++ ) {
    uint32_t c = i == 0 ? c0 : ((i & 1) ? co : ce);
#if defined(__HIP_DEVICE_COMPILE__)
    asm( "v_xad_u32 %0, %1, %2, %3" : "=v"(r.v[i]) : "v"(a.v[i]), "v"(m), "v"(c) );
#else
    r.v[i] = (a.v[i] ^ m) + c;
#endif
  }
}

/* Column finish: split the 64-bit column into its limb and carry the rest
   into the next column's accumulator. */
#define FE_COL_DONE( acc, out, sh, msk ) do { (out) = (uint32_t)(acc) & (msk); (acc) = (acc) >> (sh); } while( 0 )

#if defined(__HIP_DEVICE_COMPILE__)
/* Device: whole-product inline-asm MAC chains, single and two-way
   interleaved (fd_f25519_asm.h, generated by tools/gen_field_asm.py). */
#include "fd_f25519_asm.h"
#else
/* h = f*g.  Inputs in M, output in R. */
FD_FN void fe_mul( fe & h, fe const & f, fe const & g ) {
  uint32_t f0=f.v[0],f1=f.v[1],f2=f.v[2],f3=f.v[3],f4=f.v[4],f5=f.v[5],f6=f.v[6],f7=f.v[7],f8=f.v[8],f9=f.v[9];
  uint32_t g0=g.v[0],g1=g.v[1],g2=g.v[2],g3=g.v[3],g4=g.v[4],g5=g.v[5],g6=g.v[6],g7=g.v[7],g8=g.v[8],g9=g.v[9];
  uint32_t g1_19=19u*g1, g2_19=19u*g2, g3_19=19u*g3, g4_19=19u*g4, g5_19=19u*g5;
  uint32_t g6_19=19u*g6, g7_19=19u*g7, g8_19=19u*g8, g9_19=19u*g9;
  uint32_t f1_2=2u*f1, f3_2=2u*f3, f5_2=2u*f5, f7_2=2u*f7, f9_2=2u*f9;
  uint64_t a = 0;
  uint32_t h0,h1,h2,h3,h4,h5,h6,h7,h8,h9;
  a = COL10( a, f0,g0, f1_2,g9_19, f2,g8_19, f3_2,g7_19, f4,g6_19, f5_2,g5_19, f6,g4_19, f7_2,g3_19, f8,g2_19, f9_2,g1_19 );
  FE_COL_DONE( a, h0, 26, FE_M26 );
  a = COL10( a, f0,g1, f1,g0, f2,g9_19, f3,g8_19, f4,g7_19, f5,g6_19, f6,g5_19, f7,g4_19, f8,g3_19, f9,g2_19 );
  FE_COL_DONE( a, h1, 25, FE_M25 );
  a = COL10( a, f0,g2, f1_2,g1, f2,g0, f3_2,g9_19, f4,g8_19, f5_2,g7_19, f6,g6_19, f7_2,g5_19, f8,g4_19, f9_2,g3_19 );
  FE_COL_DONE( a, h2, 26, FE_M26 );
  a = COL10( a, f0,g3, f1,g2, f2,g1, f3,g0, f4,g9_19, f5,g8_19, f6,g7_19, f7,g6_19, f8,g5_19, f9,g4_19 );
  FE_COL_DONE( a, h3, 25, FE_M25 );
  a = COL10( a, f0,g4, f1_2,g3, f2,g2, f3_2,g1, f4,g0, f5_2,g9_19, f6,g8_19, f7_2,g7_19, f8,g6_19, f9_2,g5_19 );
  FE_COL_DONE( a, h4, 26, FE_M26 );
  a = COL10( a, f0,g5, f1,g4, f2,g3, f3,g2, f4,g1, f5,g0, f6,g9_19, f7,g8_19, f8,g7_19, f9,g6_19 );
  FE_COL_DONE( a, h5, 25, FE_M25 );
  a = COL10( a, f0,g6, f1_2,g5, f2,g4, f3_2,g3, f4,g2, f5_2,g1, f6,g0, f7_2,g9_19, f8,g8_19, f9_2,g7_19 );
  FE_COL_DONE( a, h6, 26, FE_M26 );
  a = COL10( a, f0,g7, f1,g6, f2,g5, f3,g4, f4,g3, f5,g2, f6,g1, f7,g0, f8,g9_19, f9,g8_19 );
  FE_COL_DONE( a, h7, 25, FE_M25 );
  a = COL10( a, f0,g8, f1_2,g7, f2,g6, f3_2,g5, f4,g4, f5_2,g3, f6,g2, f7_2,g1, f8,g0, f9_2,g9_19 );
  FE_COL_DONE( a, h8, 26, FE_M26 );
  a = COL10( a, f0,g9, f1,g8, f2,g7, f3,g6, f4,g5, f5,g4, f6,g3, f7,g2, f8,g1, f9,g0 );
  FE_COL_DONE( a, h9, 25, FE_M25 );
  /* a = carry out of limb 9 (< 2^39): times 19 back into limb 0, as one
     multiply-add with 19 * (a >> 32) in the addend's high word */
  a = mad64( (uint32_t)a, 19u, ((uint64_t)(19u*(uint32_t)(a>>32))<<32) | (uint64_t)h0 );
  h0 = (uint32_t)a & FE_M26;
  h1 += (uint32_t)(a >> 26);
  h.v[0]=h0; h.v[1]=h1; h.v[2]=h2; h.v[3]=h3; h.v[4]=h4; h.v[5]=h5; h.v[6]=h6; h.v[7]=h7; h.v[8]=h8; h.v[9]=h9;
}

/* h = f^2.  Input in M, output in R. */
FD_FN void fe_sq( fe & h, fe const & f ) {
  uint32_t f0=f.v[0],f1=f.v[1],f2=f.v[2],f3=f.v[3],f4=f.v[4],f5=f.v[5],f6=f.v[6],f7=f.v[7],f8=f.v[8],f9=f.v[9];
  uint32_t f0_2=2u*f0, f1_2=2u*f1, f2_2=2u*f2, f3_2=2u*f3, f4_2=2u*f4, f5_2=2u*f5, f6_2=2u*f6, f7_2=2u*f7;
  uint32_t f5_38=38u*f5, f6_19=19u*f6, f7_38=38u*f7, f8_19=19u*f8, f9_38=38u*f9;
  uint64_t a;
  uint32_t h0,h1,h2,h3,h4,h5,h6,h7,h8,h9;
  a = col5( (uint64_t)f0*f0, f1_2,f9_38, f2_2,f8_19, f3_2,f7_38, f4_2,f6_19, f5,f5_38 );
  FE_COL_DONE( a, h0, 26, FE_M26 );
  a = col5( a, f0_2,f1, f2,f9_38, f3_2,f8_19, f4,f7_38, f5_2,f6_19 );
  FE_COL_DONE( a, h1, 25, FE_M25 );
  a = mad64( f0_2,f2, col5( a, f1_2,f1, f3_2,f9_38, f4_2,f8_19, f5_2,f7_38, f6,f6_19 ) );
  FE_COL_DONE( a, h2, 26, FE_M26 );
  a = col5( a, f0_2,f3, f1_2,f2, f4,f9_38, f5_2,f8_19, f6,f7_38 );
  FE_COL_DONE( a, h3, 25, FE_M25 );
  a = mad64( f0_2,f4, col5( a, f1_2,f3_2, f2,f2, f5_2,f9_38, f6_2,f8_19, f7,f7_38 ) );
  FE_COL_DONE( a, h4, 26, FE_M26 );
  a = col5( a, f0_2,f5, f1_2,f4, f2_2,f3, f6,f9_38, f7_2,f8_19 );
  FE_COL_DONE( a, h5, 25, FE_M25 );
  a = mad64( f0_2,f6, col5( a, f1_2,f5_2, f2_2,f4, f3_2,f3, f7_2,f9_38, f8,f8_19 ) );
  FE_COL_DONE( a, h6, 26, FE_M26 );
  a = col5( a, f0_2,f7, f1_2,f6, f2_2,f5, f3_2,f4, f8,f9_38 );
  FE_COL_DONE( a, h7, 25, FE_M25 );
  a = mad64( f0_2,f8, col5( a, f1_2,f7_2, f2_2,f6, f3_2,f5_2, f4,f4, f9,f9_38 ) );
  FE_COL_DONE( a, h8, 26, FE_M26 );
  a = col5( a, f0_2,f9, f1_2,f8, f2_2,f7, f3_2,f6, f4_2,f5 );
  FE_COL_DONE( a, h9, 25, FE_M25 );
  a = mad64( (uint32_t)a, 19u, ((uint64_t)(19u*(uint32_t)(a>>32))<<32) | (uint64_t)h0 );
  h0 = (uint32_t)a & FE_M26;
  h1 += (uint32_t)(a >> 26);
  h.v[0]=h0; h.v[1]=h1; h.v[2]=h2; h.v[3]=h3; h.v[4]=h4; h.v[5]=h5; h.v[6]=h6; h.v[7]=h7; h.v[8]=h8; h.v[9]=h9;
}

/* h = f^2 + s (s limbwise, < 2^31 each, added to each column before its
   carry).  Input f in M, output in R. */
FD_FN void fe_sq_seed( fe & h, fe const & f, fe const & s ) {
  uint32_t f0=f.v[0],f1=f.v[1],f2=f.v[2],f3=f.v[3],f4=f.v[4],f5=f.v[5],f6=f.v[6],f7=f.v[7],f8=f.v[8],f9=f.v[9];
  uint32_t f0_2=2u*f0, f1_2=2u*f1, f2_2=2u*f2, f3_2=2u*f3, f4_2=2u*f4, f5_2=2u*f5, f6_2=2u*f6, f7_2=2u*f7;
  uint32_t f5_38=38u*f5, f6_19=19u*f6, f7_38=38u*f7, f8_19=19u*f8, f9_38=38u*f9;
  uint64_t a;
  uint32_t h0,h1,h2,h3,h4,h5,h6,h7,h8,h9;
  a = col5( (uint64_t)f0*f0 + s.v[0], f1_2,f9_38, f2_2,f8_19, f3_2,f7_38, f4_2,f6_19, f5,f5_38 );
  FE_COL_DONE( a, h0, 26, FE_M26 );
  a = col5( a + s.v[1], f0_2,f1, f2,f9_38, f3_2,f8_19, f4,f7_38, f5_2,f6_19 );
  FE_COL_DONE( a, h1, 25, FE_M25 );
  a = mad64( f0_2,f2, col5( a + s.v[2], f1_2,f1, f3_2,f9_38, f4_2,f8_19, f5_2,f7_38, f6,f6_19 ) );
  FE_COL_DONE( a, h2, 26, FE_M26 );
  a = col5( a + s.v[3], f0_2,f3, f1_2,f2, f4,f9_38, f5_2,f8_19, f6,f7_38 );
  FE_COL_DONE( a, h3, 25, FE_M25 );
  a = mad64( f0_2,f4, col5( a + s.v[4], f1_2,f3_2, f2,f2, f5_2,f9_38, f6_2,f8_19, f7,f7_38 ) );
  FE_COL_DONE( a, h4, 26, FE_M26 );
  a = col5( a + s.v[5], f0_2,f5, f1_2,f4, f2_2,f3, f6,f9_38, f7_2,f8_19 );
  FE_COL_DONE( a, h5, 25, FE_M25 );
  a = mad64( f0_2,f6, col5( a + s.v[6], f1_2,f5_2, f2_2,f4, f3_2,f3, f7_2,f9_38, f8,f8_19 ) );
  FE_COL_DONE( a, h6, 26, FE_M26 );
  a = col5( a + s.v[7], f0_2,f7, f1_2,f6, f2_2,f5, f3_2,f4, f8,f9_38 );
  FE_COL_DONE( a, h7, 25, FE_M25 );
  a = mad64( f0_2,f8, col5( a + s.v[8], f1_2,f7_2, f2_2,f6, f3_2,f5_2, f4,f4, f9,f9_38 ) );
  FE_COL_DONE( a, h8, 26, FE_M26 );
  a = col5( a + s.v[9], f0_2,f9, f1_2,f8, f2_2,f7, f3_2,f6, f4_2,f5 );
  FE_COL_DONE( a, h9, 25, FE_M25 );
  a = mad64( (uint32_t)a, 19u, ((uint64_t)(19u*(uint32_t)(a>>32))<<32) | (uint64_t)h0 );
  h0 = (uint32_t)a & FE_M26;
  h1 += (uint32_t)(a >> 26);
  h.v[0]=h0; h.v[1]=h1; h.v[2]=h2; h.v[3]=h3; h.v[4]=h4; h.v[5]=h5; h.v[6]=h6; h.v[7]=h7; h.v[8]=h8; h.v[9]=h9;
}

/* h = -f^2 in fe_finish_neg's complement form (fd_f25519_asm.h): the square
   of f plus FE_NEG_SEED, carried, then every limb taken from its mask
   (limb 1 from 2^26 - 1).  Input in M; output limbs like R except limb 1
   (up to 2^26). */
FD_FN void fe_sq_neg( fe & h, fe const & f ) {
  uint32_t f0=f.v[0],f1=f.v[1],f2=f.v[2],f3=f.v[3],f4=f.v[4],f5=f.v[5],f6=f.v[6],f7=f.v[7],f8=f.v[8],f9=f.v[9];
  uint32_t f0_2=2u*f0, f1_2=2u*f1, f2_2=2u*f2, f3_2=2u*f3, f4_2=2u*f4, f5_2=2u*f5, f6_2=2u*f6, f7_2=2u*f7;
  uint32_t f5_38=38u*f5, f6_19=19u*f6, f7_38=38u*f7, f8_19=19u*f8, f9_38=38u*f9;
  uint64_t c[ 10 ];
  c[0] = col5( (uint64_t)f0*f0 + FE_NEG_SEED, f1_2,f9_38, f2_2,f8_19, f3_2,f7_38, f4_2,f6_19, f5,f5_38 );
  c[1] = col5( c[0] >> 26, f0_2,f1, f2,f9_38, f3_2,f8_19, f4,f7_38, f5_2,f6_19 );
  c[2] = mad64( f0_2,f2, col5( c[1] >> 25, f1_2,f1, f3_2,f9_38, f4_2,f8_19, f5_2,f7_38, f6,f6_19 ) );
  c[3] = col5( c[2] >> 26, f0_2,f3, f1_2,f2, f4,f9_38, f5_2,f8_19, f6,f7_38 );
  c[4] = mad64( f0_2,f4, col5( c[3] >> 25, f1_2,f3_2, f2,f2, f5_2,f9_38, f6_2,f8_19, f7,f7_38 ) );
  c[5] = col5( c[4] >> 26, f0_2,f5, f1_2,f4, f2_2,f3, f6,f9_38, f7_2,f8_19 );
  c[6] = mad64( f0_2,f6, col5( c[5] >> 25, f1_2,f5_2, f2_2,f4, f3_2,f3, f7_2,f9_38, f8,f8_19 ) );
  c[7] = col5( c[6] >> 26, f0_2,f7, f1_2,f6, f2_2,f5, f3_2,f4, f8,f9_38 );
  c[8] = mad64( f0_2,f8, col5( c[7] >> 25, f1_2,f7_2, f2_2,f6, f3_2,f5_2, f4,f4, f9,f9_38 ) );
  c[9] = col5( c[8] >> 26, f0_2,f9, f1_2,f8, f2_2,f7, f3_2,f6, f4_2,f5 );
  uint64_t t = c[9] >> 25;
  uint64_t a = 19u*t + ((uint32_t)c[0] & FE_M26);
  for( int i=0; i<10; i++ ) h.v[i] = ~(uint32_t)c[i] & ((i&1) ? FE_M25 : FE_M26);
  h.v[0] = ~(uint32_t)a & FE_M26;
  h.v[1] += (1u << 25) - (uint32_t)(a >> 26);
}

FD_FN void fe_mul2( fe & h, fe const & f, fe const & g, fe & k, fe const & p, fe const & q ) { fe_mul( h, f, g ); fe_mul( k, p, q ); }
FD_FN void fe_sq2( fe & h, fe const & f, fe & k, fe const & p ) { fe_sq( h, f ); fe_sq( k, p ); }
#endif

FD_FN void fe_sqn( fe & h, fe const & f, int n ) {
  fe_sq( h, f );
#pragma unroll 1
  for( int i=1; i<n; i++ ) fe_sq( h, h );
}

/* 2 * f in one multiply-free pass (M in R out not guaranteed: use only on R inputs; result M) */
FD_FN void fe_dbl( fe & r, fe const & a ) { fe_add( r, a, a ); }

/* Canonical 8x32 little-endian words of f (fully reduced mod p). */
FD_FN void fe_tobytes32( uint32_t o[ 8 ], fe const & f ) {
  /* full carry chain to get limbs in range with the value < 2^255 + small */
  uint32_t h[ 10 ];
  for( int i=0; i<10; i++ ) h[i] = f.v[i];
  uint32_t c;
  for( int pass=0; pass<2; pass++ ) {
    for( int i=0; i<9; i++ ) { int s = (i&1) ? 25 : 26; c = h[i] >> s; h[i] &= (1u<<s)-1u; h[i+1] += c; }
    c = h[9] >> 25; h[9] &= FE_M25; h[0] += 19u*c;
  }
  /* now h < 2^255 + 2^26 roughly: compute q = (h + 19) >> 255 to subtract p once */
  uint32_t q = (h[0] + 19u) >> 26;
  for( int i=1; i<10; i++ ) q = (h[i] + q) >> ((i&1) ? 25 : 26);
  h[0] += 19u*q;
  for( int i=0; i<9; i++ ) { int s = (i&1) ? 25 : 26; c = h[i] >> s; h[i] &= (1u<<s)-1u; h[i+1] += c; }
  h[9] &= FE_M25;
  /* pack limbs at bit positions 0,26,51,77,102,128,153,179,204,230 */
  o[0] = h[0]        | (h[1] << 26);
  o[1] = (h[1] >> 6) | (h[2] << 19);
  o[2] = (h[2] >> 13)| (h[3] << 13);
  o[3] = (h[3] >> 19)| (h[4] << 6);
  o[4] = h[5]        | (h[6] << 25);
  o[5] = (h[6] >> 7) | (h[7] << 19);
  o[6] = (h[7] >> 13)| (h[8] << 12);
  o[7] = (h[8] >> 20)| (h[9] << 6);
}

/* f from 8 little-endian words, bit 255 ignored (NOT reduced mod p: values
   in [p, 2^255) are kept as-is, matching fd_f25519_frombytes). */
FD_FN void fe_frombytes32( fe & f, uint32_t const w[ 8 ] ) {
  f.v[0] =  w[0]                          & FE_M26;
  f.v[1] = ((w[0] >> 26) | (w[1] << 6))   & FE_M25;
  f.v[2] = ((w[1] >> 19) | (w[2] << 13))  & FE_M26;
  f.v[3] = ((w[2] >> 13) | (w[3] << 19))  & FE_M25;
  f.v[4] =  (w[3] >> 6)                   & FE_M26;
  f.v[5] =  w[4]                          & FE_M25;
  f.v[6] = ((w[4] >> 25) | (w[5] << 7))   & FE_M26;
  f.v[7] = ((w[5] >> 19) | (w[6] << 13))  & FE_M25;
  f.v[8] = ((w[6] >> 12) | (w[7] << 20))  & FE_M26;
  f.v[9] =  (w[7] >> 6)                   & FE_M25;
}

/* f == 0 (mod p) for f in R (every caller passes a product or an
   fe_carry result): one sequential carry pass leaves the limbs canonical
   unless the value reached 2^255 (R values are below 2^255 + 2^241 < 2p);
   below 2^255 the value is 0 (mod p) iff it is 0 or p, above it never.
   ~45 instructions instead of fe_tobytes32's ~130. */
FD_FN int fe_is_zero( fe const & f ) {
  uint32_t h[ 10 ];
#pragma unroll
  for( int i=0; i<10; i++ ) h[i] = f.v[i];
#pragma unroll
  for( int i=0; i<9; i++ ) { int s = (i&1) ? 25 : 26; h[i+1] += h[i] >> s; h[i] &= (1u<<s) - 1u; }
  uint32_t c9 = h[9] >> 25;
  h[9] &= FE_M25;
  uint32_t z = 0u, q = h[0] ^ (FE_M26 - 18u);          /* p's limbs: 2^26-19, then the masks */
#pragma unroll
  for( int i=0; i<10; i++ ) z |= h[i];
#pragma unroll
  for( int i=1; i<10; i++ ) q |= h[i] ^ ((i&1) ? FE_M25 : FE_M26);
  return (c9 == 0u) & ((z == 0u) | (q == 0u));
}

/* parity of the canonical value (fd_f25519_sgn) */
FD_FN int fe_sgn( fe const & f ) { uint32_t o[ 8 ]; fe_tobytes32( o, f ); return (int)(o[0] & 1u); }

FD_FN int fe_eq( fe const & a, fe const & b ) { fe d; fe_sub( d, a, b ); fe_carry( d, d ); return fe_is_zero( d ); }

/* a^(2^252-3) (replaces fd_f25519_pow22523, src/ballet/ed25519/fd_f25519.c:10-59) */
FD_FN void fe_pow22523( fe & out, fe const & z ) {
  fe t0, t1, t2;
  fe_sq( t0, z );                 /* 2 */
  fe_sqn( t1, t0, 2 );            /* 8 */
  fe_mul( t1, z, t1 );            /* 9 */
  fe_mul( t0, t0, t1 );           /* 11 */
  fe_sq( t0, t0 );                /* 22 */
  fe_mul( t0, t1, t0 );           /* 31 = 2^5-1 */
  fe_sqn( t1, t0, 5 );
  fe_mul( t0, t1, t0 );           /* 2^10-1 */
  fe_sqn( t1, t0, 10 );
  fe_mul( t1, t1, t0 );           /* 2^20-1 */
  fe_sqn( t2, t1, 20 );
  fe_mul( t1, t2, t1 );           /* 2^40-1 */
  fe_sqn( t1, t1, 10 );
  fe_mul( t0, t1, t0 );           /* 2^50-1 */
  fe_sqn( t1, t0, 50 );
  fe_mul( t1, t1, t0 );           /* 2^100-1 */
  fe_sqn( t2, t1, 100 );
  fe_mul( t1, t2, t1 );           /* 2^200-1 */
  fe_sqn( t1, t1, 50 );
  fe_mul( t0, t1, t0 );           /* 2^250-1 */
  fe_sqn( t0, t0, 2 );            /* 2^252-4 */
  fe_mul( out, t0, z );           /* 2^252-3 */
}

#endif /* FD_F25519_DEV_H */
