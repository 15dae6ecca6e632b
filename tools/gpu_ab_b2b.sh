#!/bin/bash
# One GPU call for kernel changes: field self-test and parity of the product
# build, then a back-to-back A/B (tools/ab_b2b.py) of $BASE against $LIBS,
# all in one process.  Stops at the first failure.
#   BASE=tools/bin/libvar_r3.so LIBS="tools/bin/libvar_cur.so ..." TAG=x tools/gpu_ab_b2b.sh
set -e
mkdir -p gpurun_out
T=${TAG:-ab}
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_field.py tests/test_gpu_parity.py tests/test_pipe.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 1; }
tail -2 gpurun_out/tests_$T.log
AB_ROUNDS=${AB_ROUNDS:-16} timeout -k 10 300 python3 tools/ab_b2b.py ${BASE:-tools/bin/libvar_base.so} ${LIBS} 20 > gpurun_out/b2b_$T.log 2>&1 || { tail -20 gpurun_out/b2b_$T.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b2b_$T.log
