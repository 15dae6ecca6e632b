#!/usr/bin/env python3
"""asm_peephole.py -- gfx950 assembly rewrites applied between the compiler
and the assembler (firedancer_amd/Makefile):

  1. v_cndmask_b32_e32 D, S0, V1, vcc  ->  v_cndmask_b32_e64 D, S0, V1, vcc
     The VOP2 encoding of v_cndmask (implicit VCC) issues at ~19 cycles per
     instruction for a wave alone on its SIMD, the VOP3 encoding with VCC as
     an explicit operand at ~5.5 (tools/issue_probe.hip, profiles/r01/
     issue_probe.json).  Same operation, same operands; only rewritten when
     S0 is a register or an inline constant (VOP3 takes no literal here).

  2. The s_nop 0 the compiler places after each inline-asm block (it cannot
     see inside asm and pads conservatively) is dropped when the block holds
     only v_mad_u64_u32 / v_lshrrev_b64 (the field-product chains of
     fd_f25519_dev.h) or the limb-pair / mask / negation helpers
     (v_lshl_add_u64, v_lshlrev_b64, v_bfi_b32, v_xad_u32) and the next instruction is a plain ALU op from the
     whitelist below -- the same pairs the compiler itself emits back to back
     with no wait state when it generates those instructions.

  3. Experimental rewrites for same-process A/Bs, off unless named in the
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
SAFE_AFTER_ASM = {
    "v_and_b32_e32", "v_and_b32_e64", "v_lshrrev_b64", "v_lshlrev_b64", "v_add_u32_e32", "v_add_u32_e64",
    "v_sub_u32_e32", "v_sub_u32_e64", "v_mad_u64_u32", "v_mov_b32_e32", "v_mov_b64_e32", "v_lshl_add_u64",
    "v_mul_lo_u32", "v_lshlrev_b32_e32", "v_lshrrev_b32_e32", "v_add3_u32", "v_alignbit_b32",
    "v_mul_u32_u24_e32", "v_mad_u32_u24", "v_or_b32_e32", "v_xor_b32_e32", "v_bfi_b32", "v_xad_u32",
    "v_lshl_add_u32", "v_cndmask_b32_e64", "v_bitop3_b32", "v_perm_b32",
}
ASM_BODY_OK = {"v_mad_u64_u32", "v_lshrrev_b64", "v_lshlrev_b64", "v_lshl_add_u64", "v_bfi_b32", "v_xad_u32"}


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
    n_cnd = n_nop = 0
    n_exp = {}
    i = 0
    in_asm = False
    asm_ok = True
    last_asm_end = -10
    while i < len(lines):
        ln = lines[i]
        st = ln.strip()
        if st.startswith(";;#ASMSTART"):
            in_asm, asm_ok = True, True
        elif st.startswith(";;#ASMEND"):
            in_asm = False
            last_asm_end = len(out)
            out.append(ln)
            i += 1
            # drop a following s_nop 0 when safe
            if asm_ok and i < len(lines) and lines[i].strip() == "s_nop 0":
                j = i + 1
                while j < len(lines) and mnemonic(lines[j]) is None and not lines[j].strip().endswith(":"):
                    j += 1
                if j < len(lines) and mnemonic(lines[j]) in SAFE_AFTER_ASM:
                    n_nop += 1
                    i += 1
            continue
        elif in_asm:
            m = mnemonic(ln)
            if m is not None and m not in ASM_BODY_OK:
                asm_ok = False
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
    sys.stderr.write("asm_peephole: %d v_cndmask_b32_e32 -> e64, %d s_nop after asm dropped%s\n" % (
        n_cnd, n_nop, "".join(", %d %s" % (v, k) for k, v in sorted(n_exp.items()))))


if __name__ == "__main__":
    main()
