#!/bin/bash
# r03: GPU parity of the working tree's build, then same-process A/Bs of
# tools/bin/lib_base.so (start of the change) vs the working build.
set -e
mkdir -p gpurun_out
T=${TAG:-r03ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
AB_MODE=pipe timeout -k 10 300 python3 tools/ab_libs.py tools/bin/lib_base.so ${AB_MID:-} firedancer_amd/libfd_ed25519_gpu.so > gpurun_out/ab_pipe_$T.log 2>&1 || { tail -30 gpurun_out/ab_pipe_$T.log; exit 1; }
cat gpurun_out/ab_pipe_$T.log | grep median
AB_MODE=pipe timeout -k 10 300 python3 tools/ab_libs.py firedancer_amd/libfd_ed25519_gpu.so ${AB_MID:-} tools/bin/lib_base.so > gpurun_out/ab_pipe2_$T.log 2>&1 || { tail -30 gpurun_out/ab_pipe2_$T.log; exit 1; }
cat gpurun_out/ab_pipe2_$T.log | grep median
timeout -k 10 300 python3 tools/ab_libs.py tools/bin/lib_base.so firedancer_amd/libfd_ed25519_gpu.so > gpurun_out/ab_oneshot_$T.log 2>&1 || { tail -30 gpurun_out/ab_oneshot_$T.log; exit 1; }
cat gpurun_out/ab_oneshot_$T.log | grep median
