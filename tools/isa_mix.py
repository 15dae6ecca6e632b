#!/usr/bin/env python3
"""isa_mix.py -- static instruction mix of one kernel in a built .s file, plus
the loop blocks (basic blocks that branch back to themselves) with their size.
Usage: isa_mix.py [kern.opt.s] [kernel-name]"""
import collections
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "firedancer_amd/build/prod/kern.opt.s"
kn = sys.argv[2] if len(sys.argv) > 2 else "fd_ed25519_verify_pipe_kernel"
s = open(src).read().split("\n")
start = [i for i, l in enumerate(s) if l.startswith(kn + ":")][0]
end = [i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end")][0]
blocks, name, cur = [], "entry", []
for l in s[start:end]:
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        blocks.append((name, cur)); name, cur = m.group(1), []; continue
    t = l.strip()
    if not t or t.startswith((".", ";", "/")) or t.endswith(":"):
        continue
    cur.append(t)
blocks.append((name, cur))
tot = collections.Counter(x.split()[0] for _, b in blocks for x in b)
valu = sum(v for k, v in tot.items() if k.startswith("v_"))
print("%s: %d instructions, %d VALU, %d s_nop" % (kn, sum(tot.values()), valu, tot["s_nop"]))
for name, b in blocks:
    if b and any(x.split()[-1] == name for x in b if x.startswith("s_cbranch")):
        c = collections.Counter(x.split()[0] for x in b)
        print("  loop %s: %d VALU (%d mad, %d mov)" % (name, sum(v for k, v in c.items() if k.startswith("v_")), c["v_mad_u64_u32"], c["v_mov_b32_e32"] + c["v_mov_b64_e32"]))
