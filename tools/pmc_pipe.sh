#!/bin/bash
# Counters of the pipelined verify kernel at 64K (tools/quick_pipe.py pipe),
# one steady-state launch (the middle dispatch): issue (single / dual VALU
# issue cycles), instruction mix, waits, icache, clock.  One rocprofv3 pass
# per group, into gpurun_out/pmc_pipe/<tag>.txt.
set -e
OUT=gpurun_out/pmc_pipe
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
pass() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$tag -o pmc -- python3 tools/quick_pipe.py 65536 ${MODE:-pipe} 10 > /dev/null 2> $OUT/$tag.err
  python3 tools/pmc_summary.py $OUT/$tag/pmc_counter_collection.csv mid > $OUT/$tag.txt
}
pass issue SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY
pass mix SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY
pass gr GRBM_GUI_ACTIVE GRBM_COUNT
pass ic SQC_ICACHE_MISSES SQC_ICACHE_HITS
echo done > $OUT/DONE
