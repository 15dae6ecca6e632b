#!/bin/bash
# One GPU call: bench.py --path host-fed (configs 2 and 3 from host memory).
set -e
mkdir -p gpurun_out
T=${TAG:-hostfed}
timeout -k 10 900 python3 -u bench.py --path host-fed > gpurun_out/hostfed_$T.json 2> gpurun_out/hostfed_$T.err || { tail -20 gpurun_out/hostfed_$T.err; exit 1; }
cat gpurun_out/hostfed_$T.json
