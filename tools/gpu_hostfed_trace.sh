#!/bin/bash
# Kernel + copy trace of bench.py --path host-fed (where the host-fed
# config-2 stream loses time against the device-resident step).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/hostfed_trace -o tr -- python3 bench.py --path host-fed > gpurun_out/hostfed_trace.json 2> gpurun_out/hostfed_trace.err || { tail -20 gpurun_out/hostfed_trace.err; exit 1; }
cat gpurun_out/hostfed_trace.json
