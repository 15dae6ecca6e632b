#!/bin/bash
# r03: the remaining GPU tests, the driver-form bench, the verify-stage A/B.
set -e
mkdir -p gpurun_out
T=${TAG:-r03c}
timeout -k 10 600 python -u -m pytest tests/test_verify_stage.py tests/test_async_pipe.py tests/test_gossip.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$T.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail -20 gpurun_out/bench_$T.err; exit 1; }
cat gpurun_out/bench_$T.json
timeout -k 10 400 python3 tools/bench_verify_stage.py --frags 262144 --no-cpu > gpurun_out/stage_$T.json 2> gpurun_out/stage_$T.err || { tail -20 gpurun_out/stage_$T.err; exit 1; }
cat gpurun_out/stage_$T.json
