#!/bin/bash
# r03 session 3: the whole -m gpu suite, then the profile set (tools/profile.sh)
set -e
mkdir -p gpurun_out
T=${TAG:-r03s3}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$T.log
bash tools/profile.sh $T
cat gpurun_out/prof_$T/bench_driver_form.json
