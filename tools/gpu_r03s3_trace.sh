#!/bin/bash
# kernel trace of the bench (launch durations and the gaps between them)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_gap -o tr -- python3 bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/trace_gap_bench.json 2> gpurun_out/trace_gap.err || { tail -20 gpurun_out/trace_gap.err; exit 1; }
cat gpurun_out/trace_gap_bench.json
python3 tools/trace_gaps.py $(find gpurun_out/trace_gap -name '*kernel_trace.csv' | head -1)
