#!/bin/bash
# r03 session 3: field self-test + parity of the current build, back-to-back
# A/B of tools/bin/libvar_*.so against tools/bin/libvar_base.so, kernel trace.
set -e
mkdir -p gpurun_out
T=${TAG:-ab}
timeout -k 10 400 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_parity.py tests/test_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 1; }
tail -2 gpurun_out/tests_$T.log
timeout -k 10 300 python3 tools/ab_b2b.py tools/bin/libvar_base.so ${LIBS} 20 > gpurun_out/b2b_$T.log 2>&1 || { tail -20 gpurun_out/b2b_$T.log; exit 1; }
grep -v amdgpu.ids gpurun_out/b2b_$T.log
if [ -n "$TRACE" ]; then
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$T -o tr -- python3 bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/trace_$T.json 2> gpurun_out/trace_$T.err || { tail -20 gpurun_out/trace_$T.err; exit 1; }
cat gpurun_out/trace_$T.json
python3 tools/trace_gaps.py $(find gpurun_out/trace_$T -name '*kernel_trace.csv' | head -1)
fi
