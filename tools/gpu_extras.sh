#!/bin/bash
# One GPU call for the secondary lines of a round's numbers: config 4 (the
# adversarial golden mix), config 2 with hot keys, and the verify stage at
# 262K and 1M frags.  Stops at the first failure.
set -e
O=gpurun_out/extras
mkdir -p $O
timeout -k 10 300 python3 bench.py --config 4 --steps 20 --warmup 5 --no-cpu > $O/c4.json 2> $O/c4.err
timeout -k 10 300 python3 bench.py --hot-keys 2048 --steps 20 --warmup 5 --no-cpu > $O/hot2048.json 2> $O/hot2048.err
for F in 262144 1048576; do
  timeout -k 10 600 python3 -u tools/bench_verify_stage.py --frags $F --steps 5 --warmup 1 --no-cpu --async-batch 35000 > $O/stage_$F.json 2> $O/stage_$F.err
done
echo done > $O/DONE
