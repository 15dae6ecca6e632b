#!/bin/bash
# Config 3 (1M signatures, Uniform{0..1232}-B) on the current build: the
# one-launch form (default) and the pipelined form at several phase-B
# window counts, driver-form runs (--steps 20 --warmup 5), one bench process
# each.
set -e
mkdir -p gpurun_out/c3
run() {  # tag, env..., args
  local t=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --config 3 --steps 20 --warmup 5 --no-cpu $C3ARGS > gpurun_out/c3/$t.json 2> gpurun_out/c3/$t.err || { tail -5 gpurun_out/c3/$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.2f M/s  %.3f ms/step' % (d['value']/1e6, d['ms_per_step']))" gpurun_out/c3/$t.json $t
}
run oneshot FD_X=0
C3ARGS="--pipeline 1"
for kb in ${KBS:-8 4 2}; do run pipe_kb$kb FD_ED25519_GPU_PIPE_KB=$kb; done
