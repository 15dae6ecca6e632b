#!/bin/bash
# tools/bin/bank_probe under rocprofv3 issue counters (dev tool)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/bank_probe -o pmc -- tools/bin/bank_probe > gpurun_out/bank_probe.txt 2>&1
python3 tools/pmc_probe.py gpurun_out/bank_probe/pmc_counter_collection.csv | grep k_
