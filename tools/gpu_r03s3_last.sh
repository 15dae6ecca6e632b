#!/bin/bash
# full -m gpu suite, the profile set, and a back-to-back A/B of the
# start-of-session build against the current one on the same box
set -e
mkdir -p gpurun_out
T=${TAG:-r03s3}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
bash tools/profile.sh $T
cut -c1-200 gpurun_out/prof_$T/bench_driver_form.json
AB_ROUNDS=16 timeout -k 10 400 python3 tools/ab_b2b.py tools/bin/libvar_base.so ${LIBS} firedancer_amd/libfd_ed25519_gpu.so 20 > gpurun_out/b2b_$T.log 2>&1 || { tail -20 gpurun_out/b2b_$T.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b2b_$T.log
