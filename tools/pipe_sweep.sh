#!/bin/bash
# Tuning sweep of the pipelined kernel (dev tool): chain windows in phase B
# (FD_ED25519_GPU_PIPE_KB) and wave priorities ("cba" digits,
# FD_ED25519_GPU_PIPE_PRIO); one quick_pipe run each, into gpurun_out/sweep.log.
set -o pipefail
out=gpurun_out/sweep.log
: > $out
for kb in ${KBS:-15}; do
  for pr in ${PRIOS:-000}; do
    echo "kb=$kb prio=$pr" >> $out
    FD_ED25519_GPU_PIPE_KB=$kb FD_ED25519_GPU_PIPE_PRIO=$pr timeout -k 5 100 python3 tools/quick_pipe.py 65536 pipe 30 >> $out 2>&1 || exit 1
  done
done
grep -v amdgpu $out
