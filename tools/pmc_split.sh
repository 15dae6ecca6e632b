#!/bin/bash
# VALU instructions and busy cycles of each pipe phase alone (quick_pipe.py
# split: phase A launch, phase B drain step, phase C drain step, repeated),
# into gpurun_out/pmc_split.sum (dev tool).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_split -o pmc -- python3 tools/quick_pipe.py 65536 split 4 > gpurun_out/pmc_split.txt 2>&1
python3 tools/pmc_probe.py gpurun_out/pmc_split/pmc_counter_collection.csv | grep pipe > gpurun_out/pmc_split.sum
tail -9 gpurun_out/pmc_split.sum
