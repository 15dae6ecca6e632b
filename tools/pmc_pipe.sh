#!/bin/bash
# Counters of the pipelined verify kernel at 64K (tools/quick_pipe.py pipe):
# icache, SQ wait/issue split, instruction mix.  One rocprofv3 pass per group.
set -e
OUT=gpurun_out/pmc_pipe
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
pass() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$tag -o pmc -- python3 tools/quick_pipe.py 65536 ${MODE:-pipe} 10 > /dev/null 2> $OUT/$tag.err
  python3 tools/pmc_summary.py $OUT/$tag/pmc_counter_collection.csv > $OUT/$tag.txt
}
pass ic SQC_ICACHE_MISSES SQC_ICACHE_HITS
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES
pass gr GRBM_GUI_ACTIVE GRBM_COUNT
pass mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_BRANCH
echo done > $OUT/DONE
