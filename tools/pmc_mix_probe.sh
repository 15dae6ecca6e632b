#!/bin/bash
# tools/bin/mix_probe (built here by tools/Makefile) under rocprofv3 issue
# counters -> gpurun_out/mix_probe.txt + .sum (dev tool)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 60 tools/bin/mix_probe > gpurun_out/mix_probe_plain.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/mix_probe -o pmc -- tools/bin/mix_probe > gpurun_out/mix_probe.txt 2>&1
python3 tools/pmc_probe.py gpurun_out/mix_probe/pmc_counter_collection.csv | grep k_mix > gpurun_out/mix_probe.sum
paste -d' ' <(grep '"a"' gpurun_out/mix_probe.txt) <(awk 'NR>2 && NR%2==0' gpurun_out/mix_probe.sum) > gpurun_out/mix_probe.joined
cat gpurun_out/mix_probe.joined
