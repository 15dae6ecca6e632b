#!/usr/bin/env python3
"""asm_peephole.py -- gfx950 assembly rewrites applied between the compiler
and the assembler (firedancer_amd/Makefile):

  1. v_cndmask_b32_e32 D, S0, V1, vcc  ->  v_cndmask_b32_e64 D, S0, V1, vcc
     The VOP2 encoding of v_cndmask (implicit VCC) issues at ~19 cycles per
     instruction for a wave alone on its SIMD, the VOP3 encoding with VCC as
     an explicit operand at ~5.5 (tools/issue_probe.hip, profiles/r01/
     issue_probe.json).  Same operation, same operands; only rewritten when
     S0 is a register or an inline constant (VOP3 takes no literal here).

  (Rounds 1-3 also dropped the s_nop 0 the compiler places after each
  inline-asm block when the next instruction was on a whitelist; a
  same-process A/B in round 4 measured it within noise -- 0.5466 ms per
  pipelined step with the drop, 0.5457 without, profiles/r04/ab/
  ab_b2b_peephole_snop.log -- so the compiler's hazard padding now stays
  as it emits it.)

  2. Experimental rewrites for same-process A/Bs, off unless named in the
     environment variable FD_PEEP (comma-separated):
       add2   v_lshlrev_b32_e32 D, 1, S      ->  v_add_u32_e32 D, S, S
              (same result; the add is one of the opcodes two waves of a
              SIMD dual-issue, tools/gen_mix_probe.py)
       carry32 v_lshrrev_b64 v[a:a+1], s, v[b:b+1] -> v_alignbit_b32 va, vb+1, vb, s
              + v_lshrrev_b32 va+1, s, vb+1 (a 64-bit shift as two 32-bit ops)
       add3   v_lshl_add_u32 D, A, 1, B      ->  v_add3_u32 D, A, A, B

Usage: asm_peephole.py in.s out.s   (prints the rewrite counts to stderr)
"""
import os
import re
import sys

INLINE_FLOAT = {"0.5", "-0.5", "1.0", "-1.0", "2.0", "-2.0", "4.0", "-4.0", "0.15915494"}
def is_inline_or_reg(op):
    op = op.strip()
    if re.fullmatch(r"-?[vs]\d+", op) or re.fullmatch(r"[vs]\[\d+:\d+\]", op):
        return True
    if op in ("vcc_lo", "vcc_hi", "exec_lo", "exec_hi", "m0"):
        return True
    if op in INLINE_FLOAT:
        return True
    try:
        v = int(op, 0)
    except ValueError:
        return False
    return -16 <= v <= 64


def mnemonic(line):
    s = line.strip()
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        return None
    return s.split()[0]


PEEP = set(x for x in os.environ.get("FD_PEEP", "").split(",") if x)


def experimental(ln):
    """the FD_PEEP rewrites of one line: (new text, rewrite name or None)"""
    if "add2" in PEEP:
        m = re.match(r"^(\s*)v_lshlrev_b32_e32\s+(v\d+),\s*1,\s*(v\d+)\s*$", ln)
        if m:
            return "%sv_add_u32_e32 %s, %s, %s" % (m.group(1), m.group(2), m.group(3), m.group(3)), "add2"
    if "add3" in PEEP:
        m = re.match(r"^(\s*)v_lshl_add_u32\s+(v\d+),\s*(v\d+),\s*1,\s*(v\d+)\s*$", ln)
        if m:
            return "%sv_add3_u32 %s, %s, %s, %s" % (m.group(1), m.group(2), m.group(3), m.group(3), m.group(4)), "add3"
    if "carry32" in PEEP:
        m = re.match(r"^(\s*)v_lshrrev_b64\s+v\[(\d+):(\d+)\],\s*(\d+),\s*v\[(\d+):(\d+)\]\s*$", ln)
        if m:
            ind, a, s_, b = m.group(1), int(m.group(2)), int(m.group(4)), int(m.group(5))
            lo = "%sv_alignbit_b32 v%d, v%d, v%d, %d" % (ind, a, b + 1, b, s_)
            hi = "%sv_lshrrev_b32_e32 v%d, %d, v%d" % (ind, a + 1, s_, b + 1)
            # the low half first unless it overwrites the source's high half
            return (hi + "\n" + lo) if a == b + 1 else (lo + "\n" + hi), "carry32"
    return ln, None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    lines = open(src).read().split("\n")
    out = []
    n_cnd = 0
    n_exp = {}
    i = 0
    while i < len(lines):
        ln = lines[i]
        st = ln.strip()
        ln, k = experimental( ln )
        if k:
            n_exp[ k ] = n_exp.get( k, 0 ) + 1
        m = re.match(r"^(\s*)v_cndmask_b32_e32\s+(v\d+),\s*([^,]+),\s*(v\d+),\s*vcc\s*$", ln)
        if m and is_inline_or_reg(m.group(3)):
            ln = "%sv_cndmask_b32_e64 %s, %s, %s, vcc" % (m.group(1), m.group(2), m.group(3).strip(), m.group(4))
            n_cnd += 1
        out.append(ln)
        i += 1
    open(dst, "w").write("\n".join(out))
    sys.stderr.write("asm_peephole: %d v_cndmask_b32_e32 -> e64%s\n" % (
        n_cnd, "".join(", %d %s" % (v, k) for k, v in sorted(n_exp.items()))))


if __name__ == "__main__":
    main()
