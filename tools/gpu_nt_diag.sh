#!/bin/bash
# Diagnostic: the variable-base table stores nontemporal (nt)
# or at system scope (sc): golden parity over consecutive pipelined launches
# (tests/test_pipe.py, tests/test_gpu_parity.py) against each diagnostic
# build -- a build whose codes are wrong fails its run, the script goes on --
# then a back-to-back A/B of the step time against the product build.
mkdir -p gpurun_out
for v in ${NT_VARIANTS:-nt sc}; do
  FD_ED25519_GPU_LIB=tools/bin/libvar_$v.so timeout -k 10 400 python -u -m pytest tests/test_pipe.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/nt_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/nt_$v.log)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
AB_ROUNDS=16 timeout -k 10 300 python3 tools/ab_b2b.py tools/bin/lib_base.so $(for v in ${NT_VARIANTS:-nt sc}; do echo tools/bin/libvar_$v.so; done) 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_nt.log
