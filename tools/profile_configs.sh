#!/bin/bash
# rocprofv3 kernel-trace summaries of the non-default bench configurations
# (config 3 one-launch, config 4 pipelined, hot keys), into
# gpurun_out/prof_cfg_<tag>/ (dev tool; DESIGN.md §5 numbers).
set -e
TAG=${1:-r02}
OUT=gpurun_out/prof_cfg_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
prof() { local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o kt -- python3 bench.py --no-cpu "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
  tail -1 $OUT/$name.json | cut -c1-160; }
prof c3 --config 3 --steps 10 --warmup 3
prof c4 --config 4
prof hot2048 --hot-keys 2048
echo done > $OUT/DONE
