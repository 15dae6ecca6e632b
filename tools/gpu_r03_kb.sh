#!/bin/bash
# r03: phase-B window sweep of the working build (one process) and its PMC
# issue / mix counters (tools/pmc_pipe.sh passes), into gpurun_out/.
set -e
mkdir -p gpurun_out
T=${TAG:-r03kb}
timeout -k 10 300 python3 tools/pipe_knob_ab.py ${KBS:-6:000 7:000 8:000 9:000 10:000} > gpurun_out/kb_$T.log 2>&1 || { tail -30 gpurun_out/kb_$T.log; exit 1; }
cat gpurun_out/kb_$T.log | grep median
[ -n "$NOPMC" ] && exit 0
timeout -k 10 400 bash tools/pmc_pipe.sh
cat gpurun_out/pmc_pipe/issue.txt gpurun_out/pmc_pipe/mix.txt gpurun_out/pmc_pipe/gr.txt
