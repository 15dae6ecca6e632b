#!/bin/bash
# r03: per-wave timeline of the working build (stamps variant) and each pipe
# phase alone under PMC, into gpurun_out/.
set -e
mkdir -p gpurun_out
T=${TAG:-r03tl}
FD_ED25519_GPU_LIB=tools/bin/lib_stamps_run.so timeout -k 10 200 python3 tools/timeline.py 65536 30 gpurun_out/timeline_$T.json > gpurun_out/timeline_$T.txt 2>&1 || { tail -20 gpurun_out/timeline_$T.txt; exit 1; }
cat gpurun_out/timeline_$T.txt
timeout -k 10 200 bash tools/pmc_split.sh
