#!/bin/bash
# The bench lines DESIGN.md §5 quotes (one GPU call): config 2 pipelined
# (default) and one-launch, config 3, config 4, hot keys; into
# gpurun_out/matrix_<tag>/.
set -e
TAG=${1:-r02}
OUT=gpurun_out/matrix_$TAG
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }; tail -1 $OUT/$name.json | cut -c1-200; }
run c2_pipe --no-cpu
run c2_launch --pipeline 0 --no-cpu
run c3_pipe --config 3 --steps 10 --warmup 3 --no-cpu
run c3_launch --config 3 --pipeline 0 --steps 10 --warmup 3 --no-cpu
run c4_pipe --config 4 --no-cpu
run hot2048 --hot-keys 2048 --no-cpu
