#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root).  Every GPU step
# has its own time limit; the script stops at the first failure.
#   tools/profile.sh <tag>   -> gpurun_out/prof_<tag>/...
#   CFG="--config 3" tools/profile.sh <tag>   profiles another bench configuration
set -e
TAG=${1:-r03}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="bench.py --no-cpu $CFG"
timeout -k 10 240 python3 bench.py $CFG > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 240 python3 bench.py $CFG --steps 20 --warmup 5 > $OUT/bench_driver_form.json 2> $OUT/bench_driver_form.err
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $BENCH > $OUT/kt_bench.json 2> $OUT/kt.err
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py $CFG --steps 3 --warmup 1 --no-cpu > /dev/null 2> $OUT/pmc_fetch.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py $CFG --steps 3 --warmup 1 --no-cpu > /dev/null 2> $OUT/pmc_write.err
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/pmc_sq -o pmc -- python3 bench.py $CFG --steps 3 --warmup 1 --no-cpu > /dev/null 2> $OUT/pmc_sq.err
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_issue -o pmc -- python3 bench.py $CFG --steps 3 --warmup 1 --no-cpu > /dev/null 2> $OUT/pmc_issue.err
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_grbm -o pmc -- python3 bench.py $CFG --steps 3 --warmup 1 --no-cpu > /dev/null 2> $OUT/pmc_grbm.err
echo done > $OUT/DONE
