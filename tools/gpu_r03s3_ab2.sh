#!/bin/bash
set -e
mkdir -p gpurun_out
T=${TAG:-ab2}
timeout -k 10 120 python3 tools/gap_probe.py > gpurun_out/gap_probe_$T.log 2>&1 || { tail -20 gpurun_out/gap_probe_$T.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gap_probe_$T.log
AB_ROUNDS=24 timeout -k 10 400 python3 tools/ab_b2b.py tools/bin/libvar_base.so ${LIBS} 20 > gpurun_out/b2b_$T.log 2>&1 || { tail -20 gpurun_out/b2b_$T.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b2b_$T.log
