#!/bin/bash
# Builds tools/bin/lib_<name>.so for each "<name>=<FD_PEEP list>" argument from
# the product build's compiled assembly (firedancer_amd/build/prod/kern.s) with
# the experimental peephole rewrites of tools/asm_peephole.py, for same-process
# A/Bs (tools/ab_libs.py).  "base=" builds the product rewrites only.
set -e
cd "$(dirname "$0")/../firedancer_amd"
make -s
mkdir -p ../tools/bin
for spec in "$@"; do
  name=${spec%%=*}; peep=${spec#*=}
  mkdir -p build/peep_$name
  cp -p build/prod/kern.s build/peep_$name/kern.s
  rm -f build/peep_$name/kern.opt.s
  FD_PEEP=$peep make -s VARIANT=peep_$name OUT=../tools/bin/lib_$name.so ../tools/bin/lib_$name.so
done
