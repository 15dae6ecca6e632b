#!/bin/bash
# r03: the -m gpu suite, then the working build's driver-form bench and its
# profile set (tools/gpu_r03f.sh).
set -e
mkdir -p gpurun_out
T=${TAG:-r03g}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
PTAG=${PTAG:-r03c} bash tools/gpu_r03f.sh
