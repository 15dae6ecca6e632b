#!/bin/bash
# Builds tools/bin/libvar_<name>.so for each "<name>=<-D flags>" argument
# (e.g. base="-DFD_OPT_EVENDBL=0") for same-process A/Bs (tools/ab_b2b.py),
# and prints the pipe kernel's VGPRs / spills for each.
set -e
cd "$(dirname "$0")/../firedancer_amd"
mkdir -p ../tools/bin
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  make -s VARIANT=var_$name EXTRA_DEFS="-DFD_DIAG_BUILD $defs" OUT=../tools/bin/libvar_$name.so ../tools/bin/libvar_$name.so 2>&1 | grep -v "hip-link\|asm_peephole" || true
  python3 - build/var_$name/kern.opt.s <<'PY'
import re, sys
s = open(sys.argv[1]).read()
for k in ("fd_ed25519_verify_pipe_kernel", "fd_ed25519_verify_kernel"):
    m = re.search(r"\.name:\s+" + k + r"\n(.*?)\.wavefront_size", s, re.S)
    blk = m.group(1) if m else ""
    g = lambda f: (re.search(r"\." + f + r":\s+(\d+)", blk) or [0, "?"])[1]
    print("  %-32s vgpr %s spill %s" % (k, g("vgpr_count"), g("vgpr_spill_count")))
PY
  echo "^ $name"
done
