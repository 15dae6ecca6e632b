#!/bin/bash
# The one GPU-box runner (run through gpurun from the repo root; chain steps
# with &&).  Every GPU step has its own time limit; output under gpurun_out/.
#
#   tools/gpu.sh test [pytest args]     -m gpu tests (default: all of tests/), product library
#                                       or $FD_ED25519_GPU_LIB
#   tools/gpu.sh ab A.so B.so ...       back-to-back A/B of library builds in one process
#                                       (tools/ab_b2b.py, codes checked); $TAG names the log
#   tools/gpu.sh bytes A.so B.so ...    per build: FETCH_SIZE, WRITE_SIZE and GRBM/SQ passes over
#                                       steady-state pipe launches -> gpurun_out/bytes_$TAG.jsonl
#   tools/gpu.sh bench [bench args]     one bench.py line -> gpurun_out/bench_$TAG.json
#   tools/gpu.sh profile [bench args]   kernel trace + PMC set of bench.py -> gpurun_out/prof_$TAG/
#   tools/gpu.sh stage [args]           verify-stage bench (tools/bench_verify_stage.py; default 1M frags)
#   tools/gpu.sh stagetrace             kernel + copy trace of the stage bench -> gpurun_out/stagetr_$TAG/
#   tools/gpu.sh hostfedtrace           kernel + copy trace of bench.py --path host-fed (+ the process's maps at exit)
#   tools/gpu.sh run SECONDS CMD...     any other command under its own time limit
set -e
mkdir -p gpurun_out
T=${TAG:-x}
cmd=$1; shift
case "$cmd" in
  test)
    timeout -k 10 ${TLIM:-900} python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
      > gpurun_out/tests_$T.log 2>&1 || { tail -40 gpurun_out/tests_$T.log; exit 1; }
    tail -3 gpurun_out/tests_$T.log ;;
  ab)
    AB_ROUNDS=${AB_ROUNDS:-16} timeout -k 10 400 python3 tools/ab_b2b.py "$@" 20 > gpurun_out/ab_$T.log 2>&1 \
      || { tail -20 gpurun_out/ab_$T.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/ab_$T.log ;;
  bytes)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    : > gpurun_out/bytes_$T.jsonl
    for L in "$@"; do
      b=$(basename $L .so); o=gpurun_out/bytes_$T/$b; mkdir -p $o
      for pass in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
        p=${pass%% *}
        AB_ROUNDS=2 timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $o/$p -o pmc -- \
          python3 tools/ab_b2b.py $L 20 > $o/$p.out 2> $o/$p.err
      done
      python3 tools/pmc_med.py --tag $b $o/*/pmc_counter_collection.csv | tee -a gpurun_out/bytes_$T.jsonl
    done ;;
  bench)
    timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err \
      || { tail -20 gpurun_out/bench_$T.err; exit 1; }
    cat gpurun_out/bench_$T.json ;;
  profile)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    o=gpurun_out/prof_$T; mkdir -p $o
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o kt -- python3 bench.py --no-cpu "$@" \
      > $o/kt_bench.json 2> $o/kt.err
    for pass in "FETCH_SIZE" "WRITE_SIZE" \
                "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY" \
                "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_THREAD_CYCLES_VALU" \
                "GRBM_GUI_ACTIVE GRBM_COUNT"; do
      p=${pass%% *}
      timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $o/pmc_$p -o pmc -- \
        python3 bench.py --no-cpu --steps 20 --warmup 5 "$@" > /dev/null 2> $o/pmc_$p.err
    done
    echo done > $o/DONE ;;
  stage)
    timeout -k 10 400 python3 -u tools/bench_verify_stage.py ${@:---frags 1048576 --steps 5 --warmup 1 --no-cpu --async-batch 35000} \
      > gpurun_out/stage_$T.json 2> gpurun_out/stage_$T.err || { tail -20 gpurun_out/stage_$T.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['async_device_parse']; print('reg %.1f M sigs/s, pageable %.1f M sigs/s, streaming %.1f M sigs/s' % (a['registered']['sigs_per_s']/1e6, a['pageable']['sigs_per_s']/1e6, a['streaming']['sigs_per_s']/1e6))" gpurun_out/stage_$T.json ;;
  stagetrace)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/stagetr_$T -o tr -- \
      python3 tools/bench_verify_stage.py --frags 1048576 --steps 3 --warmup 1 --no-cpu --async-batch 35000 \
      > gpurun_out/stagetr_$T.json 2> gpurun_out/stagetr_$T.err || { tail -20 gpurun_out/stagetr_$T.err; exit 1; } ;;
  hostfedtrace)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    FD_MAPS_OUT=gpurun_out/hostfed_maps_$T.txt timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace --stats \
      --output-format csv -d gpurun_out/hostfedtr_$T -o tr -- python3 bench.py --path host-fed \
      > gpurun_out/hostfedtr_$T.json 2> gpurun_out/hostfedtr_$T.err || { tail -30 gpurun_out/hostfedtr_$T.err; exit 1; }
    cat gpurun_out/hostfedtr_$T.json ;;
  run)
    lim=$1; shift
    timeout -k 10 $lim "$@" ;;
  *) echo "unknown command $cmd" >&2; exit 2 ;;
esac
