#!/bin/bash
# r03: the async / stage / offload GPU tests, then the verify-stage bench, on
# the working build.
set -e
mkdir -p gpurun_out
T=${TAG:-r03st}
timeout -k 10 400 python -u -m pytest tests/test_async_pipe.py tests/test_verify_stage.py tests/test_offload.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
timeout -k 10 400 python3 tools/bench_verify_stage.py --frags ${FRAGS:-262144} --no-cpu > gpurun_out/stage_$T.json 2> gpurun_out/stage_$T.err || { tail -20 gpurun_out/stage_$T.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/stage_$T.json').readline())
print('sync', d['value'], 'async pipe', d['async_device_parse']['frags_per_s'], d['async_device_parse']['host_calls'], 'registered', d['async_device_parse']['registered_frags_per_s'], 'oneshot', d['async_device_parse_oneshot']['frags_per_s'])"
