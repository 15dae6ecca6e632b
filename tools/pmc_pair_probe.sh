#!/bin/bash
# tools/bin/pair_probe under rocprofv3 issue counters -> gpurun_out/pair_probe.sum (dev tool)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pair_probe -o pmc -- tools/bin/pair_probe > gpurun_out/pair_probe.txt 2>&1
python3 tools/pmc_probe.py gpurun_out/pair_probe/pmc_counter_collection.csv | grep k_pair > gpurun_out/pair_probe.sum
paste -d' ' <(grep '"a"' gpurun_out/pair_probe.txt) <(awk 'NR%2==0' gpurun_out/pair_probe.sum)
