#!/usr/bin/env python3
"""gen_mix_probe.py -- emits tools/mix_probe.hip (dev tool): how much SIMD
issue time gfx950 VALU instruction mixes take when up to three waves share a
SIMD, the question behind moving the field products' carries and x19
premultiplies from 64-bit / multiplier opcodes onto 32-bit ones.

768-thread workgroups, one per CU (256 of them): waves 0-3 run kind A, 4-7
kind B, 8-11 kind C (waves i, i+4, i+8 share SIMD i); kind -1 exits at once.
Each kind is one inline-asm loop over fixed registers (8 independent chains
per wave, ITERS iterations), so the compiler cannot reschedule or reallocate
it.  Run under rocprofv3 --pmc (tools/pmc_mix_probe.sh) for busy cycles per
SIMD; main() also prints each launch's HIP-event time.

Usage: gen_mix_probe.py > tools/mix_probe.hip
"""

CH = 8  # independent chains per wave


def acc(c):   # 64-bit accumulator of chain c
    return "v[%d:%d]" % (40 + 2 * c, 41 + 2 * c)


def lo(c):
    return "v%d" % (40 + 2 * c)


def hi(c):
    return "v%d" % (41 + 2 * c)


def x(c):     # 32-bit register of chain c
    return "v%d" % (60 + c)


def mad(c):
    return "v_mad_u64_u32 %s, s[70:71], v100, v101, %s" % (acc(c), acc(c))


def carry_old(c):
    return ["v_lshrrev_b64 %s, 26, %s" % (acc(c), acc(c))]


def carry_new(c):
    # lo first: it reads hi before hi is rewritten
    return ["v_alignbit_b32 %s, %s, %s, 26" % (lo(c), hi(c), lo(c)), "v_lshrrev_b32 %s, 26, %s" % (hi(c), hi(c))]


def m19_old(c):
    return ["v_mul_lo_u32 %s, %s, 19" % (x(c), x(c))]


def m19_new(c):
    # 19 y = 2 (8 y + y) + y, through v70 as the temp of this chain group
    return ["v_lshl_add_u32 v71, %s, 3, %s" % (x(c), x(c)), "v_lshl_add_u32 %s, v71, 1, %s" % (x(c), x(c))]


def fast3(c):
    return ["v_and_b32 %s, v102, %s" % (x(c), x(c)), "v_add_u32 %s, v103, %s" % (x(c), x(c)),
            "v_lshlrev_b32 %s, 1, %s" % (x(c), x(c))]


KINDS = {
    "mad": lambda c: [mad(c)],
    "add_u32": lambda c: ["v_add_u32 %s, v100, %s" % (x(c), x(c))],
    "and_b32": lambda c: ["v_and_b32 %s, v100, %s" % (x(c), x(c))],
    "alignbit": lambda c: ["v_alignbit_b32 %s, v100, %s, 7" % (x(c), x(c))],
    "lshrrev_b32": lambda c: ["v_lshrrev_b32 %s, 7, %s" % (x(c), x(c))],
    "lshlrev_b32": lambda c: ["v_lshlrev_b32 %s, 3, %s" % (x(c), x(c))],
    "lshl_add_u32": lambda c: ["v_lshl_add_u32 %s, %s, 3, v100" % (x(c), x(c))],
    "mul_u32_u24": lambda c: ["v_mul_u32_u24 %s, v100, %s" % (x(c), x(c))],
    "sub_u32": lambda c: ["v_sub_u32 %s, v100, %s" % (x(c), x(c))],
    "bfe_u32": lambda c: ["v_bfe_u32 %s, %s, 3, 26" % (x(c), x(c))],
    "lshrrev_b64": lambda c: carry_old(c),
    "mul_lo_u32": lambda c: ["v_mul_lo_u32 %s, v100, %s" % (x(c), x(c))],
    "lshl_add_u64": lambda c: ["v_lshl_add_u64 %s, %s, 0, v[100:101]" % (acc(c), acc(c))],
    "cndmask_e64": lambda c: ["v_cndmask_b32_e64 %s, v100, %s, s[72:73]" % (x(c), x(c))],
    # one column: 4 MACs then the carry to the next column
    "col_old": lambda c: [mad(c)] * 4 + carry_old(c),
    "col_new": lambda c: [mad(c)] * 4 + carry_new(c),
    # x19 premultiply alone
    "m19_old": lambda c: m19_old(c),
    "m19_new": lambda c: m19_new(c),
    # the doubling's measured mix (537 mad : 63 carries : 38 x19 : ~230 32-bit
    # ops), per chain: 8 mad, 1 carry, 1 x19 (every other chain), 3 32-bit ops
    "dbl_old": lambda c: [mad(c)] * 8 + carry_old(c) + (m19_old(c) if c % 2 == 0 else []) + fast3(c),
    "dbl_new": lambda c: [mad(c)] * 8 + carry_new(c) + (m19_new(c) if c % 2 == 0 else []) + fast3(c),
}
NAMES = list(KINDS)

# (A, B, C) kind triples to run; None = the role's waves exit at once
RUNS = [
    ("mad", None, None), ("mad", "mad", None), ("mad", "mad", "mad"),
    ("add_u32", None, None), ("add_u32", "add_u32", None), ("add_u32", "add_u32", "add_u32"),
    ("mad", "mad", "add_u32"), ("mad", "mad", "alignbit"), ("mad", "mad", "lshrrev_b32"),
    ("mad", "mad", "lshl_add_u32"), ("mad", "mad", "and_b32"), ("mad", "mad", "mul_u32_u24"),
    ("mad", "add_u32", "add_u32"), ("mad", "add_u32", None),
    ("lshl_add_u32", "lshl_add_u32", None), ("mul_u32_u24", "mul_u32_u24", None),
    ("lshrrev_b32", "lshrrev_b32", None), ("lshlrev_b32", "lshlrev_b32", None), ("sub_u32", "sub_u32", None),
    ("bfe_u32", "bfe_u32", None), ("and_b32", "and_b32", None), ("alignbit", "alignbit", None),
    ("lshrrev_b64", "lshrrev_b64", None), ("mul_lo_u32", "mul_lo_u32", None), ("lshl_add_u64", "lshl_add_u64", None),
    ("cndmask_e64", "cndmask_e64", None),
    ("col_old", "col_old", "col_old"), ("col_new", "col_new", "col_new"),
    ("col_old", "col_old", None), ("col_new", "col_new", None),
    ("m19_old", "m19_old", "m19_old"), ("m19_new", "m19_new", "m19_new"),
    ("dbl_old", "dbl_old", "dbl_old"), ("dbl_new", "dbl_new", "dbl_new"),
    ("dbl_old", "dbl_old", None), ("dbl_new", "dbl_new", None),
    ("dbl_old", None, None), ("dbl_new", None, None),
]

CLOBBER = ",".join('"v%d"' % r for r in list(range(40, 56)) + list(range(60, 72)) + list(range(100, 104)))


def kind_fn(i, name):
    body = []
    for c in range(CH):
        body += KINDS[name](c)
    lines = ["v_mov_b32 v100, %0", "v_mov_b32 v101, %1", "v_mov_b32 v102, %1", "v_mov_b32 v103, %0",
             "s_mov_b64 s[72:73], exec"]
    for c in range(CH):
        lines += ["v_mov_b32 %s, %%0" % lo(c), "v_mov_b32 %s, %%1" % hi(c), "v_mov_b32 %s, %%1" % x(c)]
    lines += ["s_mov_b32 s74, %2", "1:"] + body + ["s_sub_u32 s74, s74, 1", "s_cmp_lg_u32 s74, 0", "s_cbranch_scc1 1b"]
    fold = "".join("\n     \"v_xor_b32 %%0, %%0, %s\\n\"" % r for r in [lo(c) for c in range(CH)] + [x(c) for c in range(CH)])
    return ('__device__ __attribute__((noinline)) uint32_t k_%s( uint32_t a, uint32_t b, int iters ) {\n'
            '  uint32_t r;\n'
            '  asm volatile(\n%s\n    : : "v"(a), "v"(b), "s"(iters) : %s, "s70", "s71", "s72", "s73", "s74", "scc" );\n'
            '  asm volatile( "v_mov_b32 %%0, v60\\n"%s\n    : "=v"(r) : : %s );\n'
            '  return r;\n}\n') % (
        name, "\n".join('     "%s\\n"' % l for l in lines), CLOBBER, fold, CLOBBER)


def main():
    out = ['// mix_probe.hip -- GENERATED by tools/gen_mix_probe.py; do not edit (dev tool).',
           '#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>', '',
           '#define ITERS 2048', '']
    for i, n in enumerate(NAMES):
        out.append(kind_fn(i, n))
    out.append('__device__ uint32_t dispatch( int k, uint32_t a, uint32_t b ) {\n  switch( k ) {')
    for i, n in enumerate(NAMES):
        out.append('    case %d: return k_%s( a, b, ITERS );' % (i, n))
    out.append('    default: return 0u;\n  }\n}\n')
    out.append('''extern "C" __global__ void __launch_bounds__( 768 ) k_mix( uint32_t * out, uint32_t seed, int ka, int kb, int kc ) {
  int role = __builtin_amdgcn_readfirstlane( (int)threadIdx.x >> 8 );
  int k = role == 0 ? ka : role == 1 ? kb : kc;
  uint32_t r = dispatch( k, threadIdx.x ^ seed, seed * 7u + 1u );
  if( r == 0x12345678u ) out[ threadIdx.x ] = r;
}
''')
    out.append('static const char * NM[] = { %s };' % ", ".join('"%s"' % n for n in NAMES))
    runs = []
    for r in RUNS:
        runs.append("{%s}" % ",".join(str(NAMES.index(k)) if k else "-1" for k in r))
    out.append('static const int RUNS[][3] = { %s };' % ", ".join(runs))
    out.append('''
int main() {
  uint32_t * d; hipMalloc( &d, 1 << 16 );
  hipEvent_t e0, e1; hipEventCreate( &e0 ); hipEventCreate( &e1 );
  hipLaunchKernelGGL( k_mix, dim3( 256 ), dim3( 768 ), 0, 0, d, 7u, 0, 0, 0 );  /* warm the clock */
  hipLaunchKernelGGL( k_mix, dim3( 256 ), dim3( 768 ), 0, 0, d, 7u, 0, 0, 0 );
  hipDeviceSynchronize();
  for( auto & r : RUNS ) {
    float ms = 0.f;
    for( int rep=0; rep<2; rep++ ) {
      hipEventRecord( e0, 0 );
      hipLaunchKernelGGL( k_mix, dim3( 256 ), dim3( 768 ), 0, 0, d, 7u, r[0], r[1], r[2] );
      hipEventRecord( e1, 0 ); hipEventSynchronize( e1 ); hipEventElapsedTime( &ms, e0, e1 );
    }
    printf( "{\\"a\\": \\"%s\\", \\"b\\": \\"%s\\", \\"c\\": \\"%s\\", \\"ms\\": %.4f}\\n", r[0] >= 0 ? NM[ r[0] ] : "-",
            r[1] >= 0 ? NM[ r[1] ] : "-", r[2] >= 0 ? NM[ r[2] ] : "-", ms );
  }
  hipFree( d );
  return 0;
}''')
    print("\n".join(out))


if __name__ == "__main__":
    main()
