#!/bin/bash
# Same-box A/B of the verify stage (tools/bench_verify_stage.py, 1M frags)
# under two environment settings, alternating: AB_ENV_A / AB_ENV_B are
# "VAR=VALUE" strings (empty: none).  Stops at the first failure.
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for side in A B; do
    v=AB_ENV_$side; envs=${!v}
    env $envs timeout -k 10 300 python3 -u tools/bench_verify_stage.py --frags 1048576 --steps 5 --warmup 1 --no-cpu --async-batch ${AB:-35000} > gpurun_out/stage_ab_${side}_$r.json 2> gpurun_out/stage_ab_${side}_$r.err || { tail -20 gpurun_out/stage_ab_${side}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['async_device_parse']; print(sys.argv[2], '[%s]' % sys.argv[3], 'reg %.1f pageable %.1f streaming %.1f M sigs/s' % (a['registered']['sigs_per_s']/1e6, a['pageable']['sigs_per_s']/1e6, a['streaming']['sigs_per_s']/1e6))" gpurun_out/stage_ab_${side}_$r.json $side "$envs"
  done
done
