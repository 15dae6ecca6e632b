#!/bin/bash
# r03: the other configs on the working build -- config 3 (1M, variable
# messages), config 4 (adversarial golden mix), 2,048 hot keys, the async
# verify stage (262K frags) -- each its own JSON line in gpurun_out/.
set -e
mkdir -p gpurun_out
T=${TAG:-r03cfg}
timeout -k 10 300 python3 bench.py --config 3 --steps 10 --warmup 5 --no-cpu > gpurun_out/c3_$T.json 2> gpurun_out/c3_$T.err || { tail -20 gpurun_out/c3_$T.err; exit 1; }
cat gpurun_out/c3_$T.json | cut -c1-300
timeout -k 10 300 python3 bench.py --config 4 --no-cpu > gpurun_out/c4_$T.json 2> gpurun_out/c4_$T.err || { tail -20 gpurun_out/c4_$T.err; exit 1; }
cat gpurun_out/c4_$T.json | cut -c1-300
timeout -k 10 300 python3 bench.py --hot-keys 2048 --no-cpu > gpurun_out/hot_$T.json 2> gpurun_out/hot_$T.err || { tail -20 gpurun_out/hot_$T.err; exit 1; }
cat gpurun_out/hot_$T.json | cut -c1-300
timeout -k 10 400 python3 tools/bench_verify_stage.py ${STAGE_ARGS:---frags 262144 --no-cpu} > gpurun_out/stage_$T.json 2> gpurun_out/stage_$T.err || { tail -20 gpurun_out/stage_$T.err; exit 1; }
cat gpurun_out/stage_$T.json | cut -c1-400
