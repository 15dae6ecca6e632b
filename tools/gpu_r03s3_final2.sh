#!/bin/bash
# the profile set plus a back-to-back A/B of the start-of-session build on the same box
set -e
mkdir -p gpurun_out
T=${TAG:-r03s3}
bash tools/profile.sh $T
cat gpurun_out/prof_$T/bench_driver_form.json | cut -c1-200
AB_ROUNDS=16 timeout -k 10 400 python3 tools/ab_b2b.py tools/bin/libvar_base.so tools/bin/libvar_final.so 20 > gpurun_out/b2b_$T.log 2>&1 || { tail -20 gpurun_out/b2b_$T.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b2b_$T.log
