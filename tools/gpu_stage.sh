#!/bin/bash
# One GPU call for the verify stage: its GPU tests, then the stage bench at
# $FRAGS frags (default 262144 and 1048576).  Stops at the first failure.
set -e
mkdir -p gpurun_out
T=${TAG:-stage}
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_verify_stage.py tests/test_multidev.py tests/test_offload.py tests/test_async_pipe.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -40 gpurun_out/tests_$T.log; exit 1; }
tail -2 gpurun_out/tests_$T.log
for F in ${FRAGS:-262144 1048576}; do
  timeout -k 10 600 python3 -u tools/bench_verify_stage.py --frags $F --steps 5 --warmup 1 --no-cpu --async-batch ${AB:-35000} > gpurun_out/stage_${T}_$F.json 2> gpurun_out/stage_${T}_$F.err || { tail -20 gpurun_out/stage_${T}_$F.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['async_device_parse']; print(sys.argv[1], 'reg %.1f M sigs/s, pageable %.1f M sigs/s, streaming %.1f M sigs/s' % (a['registered']['sigs_per_s']/1e6, a['pageable']['sigs_per_s']/1e6, a['streaming']['sigs_per_s']/1e6)); print(json.dumps(a['registered']))" gpurun_out/stage_${T}_$F.json
done
