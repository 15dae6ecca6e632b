#!/usr/bin/env python3
"""gen_field_asm.py -- generates firedancer_amd/csrc/fd_f25519_asm.h, the
device (gfx950) field products of fd_f25519_dev.h as whole-product inline-asm
blocks: fe_mul / fe_sq (one product) and fe_mul2 / fe_sq2 (two independent
products with their instruction streams interleaved one-for-one, so each
product's dependent MAC chain has an independent instruction between
consecutive links).

Radix 2^25.5, ten limbs; column k of f*g is sum_i f_i g_{k-i} with the
wrapped terms (k-i < 0) multiplied by 19 and odd*odd terms by 2 (the
premultiplied operands are computed in C before the block).  Each column is a
chain of v_mad_u64_u32 into a 64-bit accumulator seeded with the previous
column's accumulator shifted right by the previous limb width.

Usage: gen_field_asm.py > firedancer_amd/csrc/fd_f25519_asm.h
"""


def mul_terms(k):
    t = []
    for i in range(10):
        j = k - i
        wrap = j < 0
        jj = j % 10
        two = (i & 1) and (jj & 1)
        t.append(("f%d_2" % i if two else "f%d" % i, "g%d_19" % jj if wrap else "g%d" % jj))
    return t


SQ_TERMS = [
    [("f0", "f0"), ("f1_2", "f9_38"), ("f2_2", "f8_19"), ("f3_2", "f7_38"), ("f4_2", "f6_19"), ("f5", "f5_38")],
    [("f0_2", "f1"), ("f2", "f9_38"), ("f3_2", "f8_19"), ("f4", "f7_38"), ("f5_2", "f6_19")],
    [("f1_2", "f1"), ("f3_2", "f9_38"), ("f4_2", "f8_19"), ("f5_2", "f7_38"), ("f6", "f6_19"), ("f0_2", "f2")],
    [("f0_2", "f3"), ("f1_2", "f2"), ("f4", "f9_38"), ("f5_2", "f8_19"), ("f6", "f7_38")],
    [("f1_2", "f3_2"), ("f2", "f2"), ("f5_2", "f9_38"), ("f6_2", "f8_19"), ("f7", "f7_38"), ("f0_2", "f4")],
    [("f0_2", "f5"), ("f1_2", "f4"), ("f2_2", "f3"), ("f6", "f9_38"), ("f7_2", "f8_19")],
    [("f1_2", "f5_2"), ("f2_2", "f4"), ("f3_2", "f3"), ("f7_2", "f9_38"), ("f8", "f8_19"), ("f0_2", "f6")],
    [("f0_2", "f7"), ("f1_2", "f6"), ("f2_2", "f5"), ("f3_2", "f4"), ("f8", "f9_38")],
    [("f1_2", "f7_2"), ("f2_2", "f6"), ("f3_2", "f5_2"), ("f4", "f4"), ("f9", "f9_38"), ("f0_2", "f8")],
    [("f0_2", "f9"), ("f1_2", "f8"), ("f2_2", "f7"), ("f3_2", "f6"), ("f4_2", "f5")],
]
MUL_INS = ["f%d" % i for i in range(10)] + ["g%d" % i for i in range(10)] + \
          ["g%d_19" % i for i in range(1, 10)] + ["f%d_2" % i for i in (1, 3, 5, 7, 9)]
SQ_INS = ["f%d" % i for i in range(10)] + ["f%d_2" % i for i in range(8)] + ["f5_38", "f6_19", "f7_38", "f8_19", "f9_38"]
SEEDS = ["s%d" % i for i in range(10)]


def stream(cols, ins, out_base, in_base, seeds=None, add0=None):
    """instruction list (strings) of one product; seeds: per-column 32-bit
    addends (input names), each added to its column's accumulator by one
    v_mad_u64_u32 with multiplier 1 before the column's carry moves on;
    add0: operand number of a 64-bit addend of column 0 (free: the column's
    first multiply-add takes it instead of 0)"""
    idx = {n: in_base + i for i, n in enumerate(ins)}
    ops = []
    for k, terms in enumerate(cols):
        o = out_base + k
        if k:
            ops.append("v_lshrrev_b64 %%%d, %d, %%%d" % (o, 26 if (k - 1) % 2 == 0 else 25, o - 1))
        for n, (a, b) in enumerate(terms):
            src2 = ("0" if add0 is None else "%%%d" % add0) if (k == 0 and n == 0) else "%%%d" % o
            ops.append("v_mad_u64_u32 %%%d, vcc, %%%d, %%%d, %s" % (o, idx[a], idx[b], src2))
        if seeds:
            ops.append("v_mad_u64_u32 %%%d, vcc, %%%d, 1, %%%d" % (o, idx[seeds[k]], o))
    return ops


def interleave(a, b):
    out = []
    for i in range(max(len(a), len(b))):
        if i < len(a):
            out.append(a[i])
        if i < len(b):
            out.append(b[i])
    return out


def asm_block(ops, outs, inps, sinps=()):
    body = '\\n\\t"\n       "'.join(ops)
    return '  asm( "%s"\n       : %s\n       : %s : "vcc" );\n' % (
        body, ", ".join('"=&v"(%s)' % o for o in outs),
        ", ".join(['"v"(%s)' % n for n in inps] + ['"s"(%s)' % n for n in sinps]))


PRE_MUL = '''  uint32_t {p}f0={F}.v[0],{p}f1={F}.v[1],{p}f2={F}.v[2],{p}f3={F}.v[3],{p}f4={F}.v[4],{p}f5={F}.v[5],{p}f6={F}.v[6],{p}f7={F}.v[7],{p}f8={F}.v[8],{p}f9={F}.v[9];
  uint32_t {p}g0={G}.v[0],{p}g1={G}.v[1],{p}g2={G}.v[2],{p}g3={G}.v[3],{p}g4={G}.v[4],{p}g5={G}.v[5],{p}g6={G}.v[6],{p}g7={G}.v[7],{p}g8={G}.v[8],{p}g9={G}.v[9];
  uint32_t {p}g1_19=19u*{p}g1, {p}g2_19=19u*{p}g2, {p}g3_19=19u*{p}g3, {p}g4_19=19u*{p}g4, {p}g5_19=19u*{p}g5;
  uint32_t {p}g6_19=19u*{p}g6, {p}g7_19=19u*{p}g7, {p}g8_19=19u*{p}g8, {p}g9_19=19u*{p}g9;
  uint32_t {p}f1_2=2u*{p}f1, {p}f3_2=2u*{p}f3, {p}f5_2=2u*{p}f5, {p}f7_2=2u*{p}f7, {p}f9_2=2u*{p}f9;
  uint64_t {p}c0,{p}c1,{p}c2,{p}c3,{p}c4,{p}c5,{p}c6,{p}c7,{p}c8,{p}c9;
'''
PRE_SQ = '''  uint32_t {p}f0={F}.v[0],{p}f1={F}.v[1],{p}f2={F}.v[2],{p}f3={F}.v[3],{p}f4={F}.v[4],{p}f5={F}.v[5],{p}f6={F}.v[6],{p}f7={F}.v[7],{p}f8={F}.v[8],{p}f9={F}.v[9];
  uint64_t {p}d01=pk_shl1(FE_PK({F},0)), {p}d23=pk_shl1(FE_PK({F},1)), {p}d45=pk_shl1(FE_PK({F},2)), {p}d67=pk_shl1(FE_PK({F},3));
  uint32_t {p}f0_2=(uint32_t){p}d01, {p}f1_2=(uint32_t)({p}d01>>32), {p}f2_2=(uint32_t){p}d23, {p}f3_2=(uint32_t)({p}d23>>32);
  uint32_t {p}f4_2=(uint32_t){p}d45, {p}f5_2=(uint32_t)({p}d45>>32), {p}f6_2=(uint32_t){p}d67, {p}f7_2=(uint32_t)({p}d67>>32);
  uint32_t {p}f5_38=38u*{p}f5, {p}f6_19=19u*{p}f6, {p}f7_38=38u*{p}f7, {p}f8_19=19u*{p}f8, {p}f9_38=38u*{p}f9;
  uint64_t {p}c0,{p}c1,{p}c2,{p}c3,{p}c4,{p}c5,{p}c6,{p}c7,{p}c8,{p}c9;
'''
FIN = '''  fe_finish( {H}, {p}c0,{p}c1,{p}c2,{p}c3,{p}c4,{p}c5,{p}c6,{p}c7,{p}c8,{p}c9 );
'''


def pre(tmpl, p, F, G=None):
    return tmpl.replace("{p}", p).replace("{F}", F).replace("{G}", G or "")


def main():
    mul_cols = [mul_terms(k) for k in range(10)]
    out = []
    out.append('''/* fd_f25519_asm.h -- GENERATED by tools/gen_field_asm.py; do not edit.
   Device (gfx950) field products for fd_f25519_dev.h: whole-product
   inline-asm MAC chains (one v_mad_u64_u32 per MAC), single and two-way
   interleaved (two independent products, one instruction of each in turn). */

#ifndef FD_F25519_ASM_H
#define FD_F25519_ASM_H

/* c >> 25 as one v_lshrrev_b64 (the compiler splits a 64-bit shift whose
   halves it reads separately into two 32-bit operations) */
__device__ __forceinline__ uint64_t fe_shr25( uint64_t c ) {
  uint64_t r; asm( "v_lshrrev_b64 %0, 25, %1" : "=v"(r) : "v"(c) ); return r;
}

/* (uint32_t)(a >> 26) for a < 2^58 as ONE v_alignbit_b32 (left to itself
   the compiler sometimes makes it a 64-bit shift plus a 64-bit add and a
   move, in the squaring loops) */
__device__ __forceinline__ uint32_t fe_hi26( uint64_t a ) {
  uint32_t r; asm( "v_alignbit_b32 %0, %1, %2, 26" : "=v"(r) : "v"((uint32_t)(a >> 32)), "v"((uint32_t)a) ); return r;
}

/* column accumulators -> limbs (R form): mask, then fold the carry out of
   limb 9 (< 2^38) times 19 into limbs 0/1 */
__device__ __forceinline__ void fe_finish( fe & h, uint64_t c0, uint64_t c1, uint64_t c2, uint64_t c3, uint64_t c4,
                                           uint64_t c5, uint64_t c6, uint64_t c7, uint64_t c8, uint64_t c9 ) {
  uint32_t h0 = (uint32_t)c0 & FE_M26, h1 = (uint32_t)c1 & FE_M25, h2 = (uint32_t)c2 & FE_M26, h3 = (uint32_t)c3 & FE_M25;
  uint32_t h4 = (uint32_t)c4 & FE_M26, h5 = (uint32_t)c5 & FE_M25, h6 = (uint32_t)c6 & FE_M26, h7 = (uint32_t)c7 & FE_M25;
  uint32_t h8 = (uint32_t)c8 & FE_M26, h9 = (uint32_t)c9 & FE_M25;
  uint64_t t = fe_shr25( c9 );
  /* 19 t + h0 as ONE v_mad_u64_u32: the high word of 19 t (t >> 32 < 2^7)
     goes into the high word of the 64-bit addend (h0 is below 2^26, so the
     sum is exact) */
  uint64_t add = ((uint64_t)(19u*(uint32_t)(t>>32)) << 32) | (uint64_t)h0;
  uint64_t a = (uint64_t)(uint32_t)t * 19u + add;
  h0 = (uint32_t)a & FE_M26;
  h1 += fe_hi26( a );
  h.v[0]=h0; h.v[1]=h1; h.v[2]=h2; h.v[3]=h3; h.v[4]=h4; h.v[5]=h5; h.v[6]=h6; h.v[7]=h7; h.v[8]=h8; h.v[9]=h9;
}

/* Complement finish: the limbs of K - h instead of h, where h is fe_finish's
   result and K has every limb at its mask except limb 1 at 2^26-1 (so limb
   1, which the final carry can push past 2^25, never goes negative):
   K = 2^255-1+2^51.  Each mask becomes one v_bfi_b32 (~c & mask).  With the
   product seeded by FE_NEG_SEED = 18+2^51 in column 0 the result is
   K - (x+18+2^51) = p - x = -x (mod p): a negated product for the price of
   one extra operation (limb 1's 2^25 - carry). */
__device__ __forceinline__ uint32_t fe_bfi_not( uint32_t c, uint32_t m ) {
  uint32_t r; asm( "v_bfi_b32 %0, %1, 0, %2" : "=v"(r) : "v"(c), "s"(m) ); return r;
}
__device__ __forceinline__ void fe_finish_neg( fe & h, uint64_t c0, uint64_t c1, uint64_t c2, uint64_t c3, uint64_t c4,
                                               uint64_t c5, uint64_t c6, uint64_t c7, uint64_t c8, uint64_t c9 ) {
  uint32_t h0 = (uint32_t)c0 & FE_M26;
  uint64_t t = fe_shr25( c9 );
  uint64_t add = ((uint64_t)(19u*(uint32_t)(t>>32)) << 32) | (uint64_t)h0;
  uint64_t a = (uint64_t)(uint32_t)t * 19u + add;
  h.v[0] = fe_bfi_not( (uint32_t)a, FE_M26 );
  h.v[1] = fe_bfi_not( (uint32_t)c1, FE_M25 ) + ((1u << 25) - fe_hi26( a ));
  h.v[2] = fe_bfi_not( (uint32_t)c2, FE_M26 ); h.v[3] = fe_bfi_not( (uint32_t)c3, FE_M25 );
  h.v[4] = fe_bfi_not( (uint32_t)c4, FE_M26 ); h.v[5] = fe_bfi_not( (uint32_t)c5, FE_M25 );
  h.v[6] = fe_bfi_not( (uint32_t)c6, FE_M26 ); h.v[7] = fe_bfi_not( (uint32_t)c7, FE_M25 );
  h.v[8] = fe_bfi_not( (uint32_t)c8, FE_M26 ); h.v[9] = fe_bfi_not( (uint32_t)c9, FE_M25 );
}
''')
    # fe_mul
    out.append("/* h = f*g.  Inputs in M, output in R. */\n")
    out.append("__device__ __forceinline__ void fe_mul( fe & h, fe const & f, fe const & g ) {\n")
    out.append(pre(PRE_MUL, "", "f", "g"))
    out.append(asm_block(stream(mul_cols, MUL_INS, 0, 10), ["c%d" % i for i in range(10)], MUL_INS))
    out.append(FIN.replace("{H}", "h").replace("{p}", ""))
    out.append("}\n\n")
    # fe_sq
    out.append("/* h = f^2.  Input in M, output in R (55 MACs). */\n")
    out.append("__device__ __forceinline__ void fe_sq( fe & h, fe const & f ) {\n")
    out.append(pre(PRE_SQ, "", "f"))
    out.append(asm_block(stream(SQ_TERMS, SQ_INS, 0, 10), ["c%d" % i for i in range(10)], SQ_INS))
    out.append(FIN.replace("{H}", "h").replace("{p}", ""))
    out.append("}\n\n")
    # fe_sq_neg
    out.append("/* h = -f^2 (mod p) in the complement form of fe_finish_neg: limbs like R\n"
               "   except limb 1 (up to 2^26).  Input in M. */\n")
    out.append("__device__ __forceinline__ void fe_sq_neg( fe & h, fe const & f ) {\n")
    out.append(pre(PRE_SQ, "", "f"))
    out.append("  uint64_t s0 = FE_NEG_SEED;\n")
    out.append(asm_block(stream(SQ_TERMS, SQ_INS, 0, 10, add0=10 + len(SQ_INS)), ["c%d" % i for i in range(10)], SQ_INS, ["s0"]))
    out.append(FIN.replace("{H}", "h").replace("{p}", "").replace("fe_finish", "fe_finish_neg"))
    out.append("}\n\n")
    # fe_sq_seed
    out.append("/* h = f^2 + s (limbwise addend s, limbs < 2^31, added to each column before\n"
               "   its carry: h comes out carried).  Input f in M, output in R. */\n")
    out.append("__device__ __forceinline__ void fe_sq_seed( fe & h, fe const & f, fe const & s ) {\n")
    out.append(pre(PRE_SQ, "", "f"))
    out.append("  uint32_t " + ", ".join("s%d=s.v[%d]" % (i, i) for i in range(10)) + ";\n")
    out.append(asm_block(stream(SQ_TERMS, SQ_INS + SEEDS, 0, 10, seeds=SEEDS), ["c%d" % i for i in range(10)], SQ_INS + SEEDS))
    out.append(FIN.replace("{H}", "h").replace("{p}", ""))
    out.append("}\n\n")
    # fe_mul2
    out.append("/* h = f*g and k = p*q, interleaved. */\n")
    out.append("__device__ __forceinline__ void fe_mul2( fe & h, fe const & f, fe const & g, fe & k, fe const & p, fe const & q ) {\n")
    out.append(pre(PRE_MUL, "a", "f", "g"))
    out.append(pre(PRE_MUL, "b", "p", "q"))
    ins_a = ["a" + n for n in MUL_INS]
    ins_b = ["b" + n for n in MUL_INS]
    ops = interleave(stream(mul_cols, MUL_INS, 0, 20), stream(mul_cols, MUL_INS, 10, 20 + len(MUL_INS)))
    out.append(asm_block(ops, ["ac%d" % i for i in range(10)] + ["bc%d" % i for i in range(10)], ins_a + ins_b))
    out.append(FIN.replace("{H}", "h").replace("{p}", "a"))
    out.append(FIN.replace("{H}", "k").replace("{p}", "b"))
    out.append("}\n\n")
    # fe_sq2
    out.append("/* h = f^2 and k = p^2, interleaved. */\n")
    out.append("__device__ __forceinline__ void fe_sq2( fe & h, fe const & f, fe & k, fe const & p ) {\n")
    out.append(pre(PRE_SQ, "a", "f"))
    out.append(pre(PRE_SQ, "b", "p"))
    ins_a = ["a" + n for n in SQ_INS]
    ins_b = ["b" + n for n in SQ_INS]
    ops = interleave(stream(SQ_TERMS, SQ_INS, 0, 20), stream(SQ_TERMS, SQ_INS, 10, 20 + len(SQ_INS)))
    out.append(asm_block(ops, ["ac%d" % i for i in range(10)] + ["bc%d" % i for i in range(10)], ins_a + ins_b))
    out.append(FIN.replace("{H}", "h").replace("{p}", "a"))
    out.append(FIN.replace("{H}", "k").replace("{p}", "b"))
    out.append("}\n\n")
    out.append("#endif /* FD_F25519_ASM_H */\n")
    print("".join(out), end="")


if __name__ == "__main__":
    main()
