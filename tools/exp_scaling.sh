#!/bin/bash
# Why does a second wave per SIMD (128K batch) gain so little?  The single-lane
# verify kernel at 64K (one wave per SIMD) and 128K (two): SQ, icache, clock and
# instruction-mix counters, one rocprofv3 pass per counter group, each under its
# own time limit.  Output: gpurun_out/exp_scaling/*.
set -e
OUT=gpurun_out/exp_scaling
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export FD_ED25519_GPU_PAIR=0
pass() {  # tag n counters...
  local tag=$1 n=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/${tag}_$n -o pmc -- python3 tools/quick_perf.py $n > /dev/null 2> $OUT/${tag}_$n.err
  python3 tools/pmc_summary.py $OUT/${tag}_$n/pmc_counter_collection.csv > $OUT/${tag}_$n.txt
}
for n in 65536 131072; do
  pass sq $n SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES
  pass ic $n SQC_ICACHE_MISSES SQC_ICACHE_HITS
  pass gr $n GRBM_GUI_ACTIVE GRBM_COUNT
  pass if $n SQ_IFETCH SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH
done
echo done > $OUT/DONE
