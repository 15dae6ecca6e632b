#!/bin/bash
# One GPU call: the -m gpu suite, then the 1-GPU bench (driver defaults), then
# optional extras.  Every GPU step has its own limit; stop at the first failure.
set -e
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
