#!/bin/bash
# Diagnostic: which cache holds the stale table lines when the
# variable-base table stores are nontemporal?  tests/test_pipe.py (golden
# sequences over consecutive pipelined launches) against each diagnostic
# build; a build whose codes are wrong fails its run, the script goes on.
mkdir -p gpurun_out
for v in nt ntl1 ntl2 ntl12; do
  FD_ED25519_GPU_LIB=tools/bin/libvar_$v.so timeout -k 10 300 python -u -m pytest tests/test_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/nt_$v.log)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
