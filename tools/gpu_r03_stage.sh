#!/bin/bash
# r03: where the async verify stage's time goes -- kernel + memory-copy trace
# of tools/bench_verify_stage.py (few steps), into gpurun_out/stage_prof.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/stage_prof -o st -- python3 tools/bench_verify_stage.py --frags 262144 --no-cpu --steps 3 --warmup 1 > gpurun_out/stage_prof.json 2> gpurun_out/stage_prof.err || { tail -20 gpurun_out/stage_prof.err; exit 1; }
cut -c1-300 gpurun_out/stage_prof.json
ls gpurun_out/stage_prof
