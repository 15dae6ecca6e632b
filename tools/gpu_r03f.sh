#!/bin/bash
# r03: the working build's driver-form bench, then its profile set
# (kernel trace + PMC passes) into gpurun_out/prof_<PTAG>.
set -e
mkdir -p gpurun_out
P=${PTAG:-r03b}
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_$P.json 2> gpurun_out/bench_driver_$P.err || { tail -20 gpurun_out/bench_driver_$P.err; exit 1; }
cat gpurun_out/bench_driver_$P.json
bash tools/profile.sh $P
