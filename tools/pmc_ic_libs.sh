#!/bin/bash
# Instruction-cache and wait counters of the pipelined verify launch for
# several builds of the library (FD_ED25519_GPU_LIB), one rocprofv3 pass per
# counter group and library; prints the middle (steady-state) dispatch.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ic
for L in ${IC_LIBS:-tools/bin/lib_base.so}; do
  b=$(basename $L .so)
  echo "== $b"
  FD_ED25519_GPU_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/ic/$b.a -o pmc -- python3 tools/quick_pipe.py 65536 pipe 20 > gpurun_out/ic/$b.a.out 2> gpurun_out/ic/$b.a.err
  python3 tools/pmc_summary.py gpurun_out/ic/$b.a/pmc_counter_collection.csv mid
  FD_ED25519_GPU_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_IFETCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/ic/$b.b -o pmc -- python3 tools/quick_pipe.py 65536 pipe 20 > gpurun_out/ic/$b.b.out 2> gpurun_out/ic/$b.b.err
  python3 tools/pmc_summary.py gpurun_out/ic/$b.b/pmc_counter_collection.csv mid
done
