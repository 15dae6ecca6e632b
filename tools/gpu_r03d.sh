#!/bin/bash
# r03: start-of-round vs current kernel A/B (same process), precompile GPU tests, shred bench.
set -e
mkdir -p gpurun_out
T=${TAG:-r03d}
AB_MODE=pipe timeout -k 10 300 python3 tools/ab_libs.py tools/bin/lib_r03start.so firedancer_amd/libfd_ed25519_gpu.so > gpurun_out/ab_$T.log 2>&1 || { tail -30 gpurun_out/ab_$T.log; exit 1; }
cat gpurun_out/ab_$T.log
timeout -k 10 300 python -u -m pytest tests/test_precompile.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$T.log
timeout -k 10 300 python3 bench.py --path shred --steps 20 --warmup 3 > gpurun_out/shred_$T.json 2> gpurun_out/shred_$T.err || { tail -20 gpurun_out/shred_$T.err; exit 1; }
cat gpurun_out/shred_$T.json
