#!/bin/bash
# The one GPU-box runner (run through gpurun from the repo root; chain steps
# with &&).  Every GPU step has its own time limit; output under gpurun_out/.
#
#   tools/gpu.sh test [pytest args]     -m gpu tests (default: all of tests/), product library
#                                       or $FD_ED25519_GPU_LIB
#   tools/gpu.sh ab A.so B.so ...       back-to-back A/B of library builds in one process
#                                       (tools/ab_b2b.py, codes checked); $TAG names the log
#   tools/gpu.sh bytes A.so B.so ...    per build: FETCH_SIZE, WRITE_SIZE, read requests by size and GRBM/SQ passes over
#                                       steady-state pipe launches -> gpurun_out/bytes_$TAG.jsonl
#   tools/gpu.sh phasebytes [--reps N]  each pipe phase's bytes alone (tools/phase_bytes.py) -> gpurun_out/phasebytes_$TAG.json
#   tools/gpu.sh bench [bench args]     one bench.py line -> gpurun_out/bench_$TAG.json
#   tools/gpu.sh profile [bench args]   bench lines, kernel trace + PMC set of bench.py -> gpurun_out/prof_$TAG/
#                                       (then tools/summarize_profile.py gpurun_out/prof_$TAG profiles/rNN)
#   tools/gpu.sh offload                the two-process offload link run (server + client)
#   tools/gpu.sh stage [args]           verify-stage bench (tools/bench_verify_stage.py; default 1M frags)
#   tools/gpu.sh stagetrace             kernel + copy trace of the stage bench -> gpurun_out/stagetr_$TAG/
#   tools/gpu.sh hostfedtrace           kernel + copy trace of bench.py --path host-fed (+ the process's maps at exit)
#   tools/gpu.sh abstage "A:" "B:ENV=v" same-process A/B of stage settings (tools/ab_stage.py)
#   tools/gpu.sh clock 2|3              in-kernel clock stamps of config 2 / 3 (stamps build)
#   tools/gpu.sh crashctl MODE          exit-SIGSEGV control run (tools/crash_control.py) under the trace flags
#   tools/gpu.sh box                    the box's GPU: serial, power cap and draw, temperatures, clocks
#                                       (read-only rocm-smi / amd-smi queries) -> gpurun_out/box_$TAG.txt
#   tools/gpu.sh power [bench args]     bench.py in the background; rocm-smi power / clock samples every
#                                       0.4 s and one amd-smi metric dump once it draws > 1 kW
#                                       -> gpurun_out/power_$TAG.txt, amdsmi_$TAG.txt, bench_$TAG.json
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
      for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
                  "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
        p=${pass%% *}
        AB_ROUNDS=2 timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $o/$p -o pmc -- \
          python3 tools/ab_b2b.py $L 20 > $o/$p.out 2> $o/$p.err
      done
      python3 tools/pmc_med.py --tag $b $o/*/pmc_counter_collection.csv | tee -a gpurun_out/bytes_$T.jsonl
    done ;;
  phasebytes)
    # each pipe phase alone (tools/phase_bytes.py): FETCH, WRITE and read-request-size passes
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    o=gpurun_out/phasebytes_$T; mkdir -p $o
    for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
                "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
      p=${pass%% *}
      timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $o/$p -o pmc -- python3 tools/phase_bytes.py "$@" \
        > $o/$p.out 2> $o/$p.err
    done
    python3 tools/phase_bytes.py --summarize $o/*/pmc_counter_collection.csv | tee gpurun_out/phasebytes_$T.json ;;
  bench)
    timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err \
      || { tail -20 gpurun_out/bench_$T.err; exit 1; }
    cat gpurun_out/bench_$T.json ;;
  profile)
    # the layout tools/summarize_profile.py reads; the kernel trace runs 2,000 timed steps so its
    # --stats average is the steady state (the prime / warm-up launches at a ramping clock are few)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    o=gpurun_out/prof_$T; mkdir -p $o
    timeout -k 10 300 python3 bench.py "$@" > $o/bench.json 2> $o/bench.err
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 "$@" > $o/bench_driver_form.json 2> $o/bench_driver_form.err
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o kt -- \
      python3 bench.py --no-cpu --steps 2000 --warmup 50 "$@" > $o/kt_bench.json 2> $o/kt.err
    for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" \
                "sq SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY" \
                "issue SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_ANY" \
                "grbm GRBM_GUI_ACTIVE GRBM_COUNT"; do
      p=${pass%% *}; c=${pass#* }
      timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $o/pmc_$p -o pmc -- \
        python3 bench.py --no-cpu --steps 20 --warmup 5 "$@" > /dev/null 2> $o/pmc_$p.err
    done
    echo done > $o/DONE ;;
  stage)
    timeout -k 10 400 python3 -u tools/bench_verify_stage.py ${@:---frags 1048576 --steps 5 --warmup 1 --no-cpu --async-batch 36000} \
      > gpurun_out/stage_$T.json 2> gpurun_out/stage_$T.err || { tail -20 gpurun_out/stage_$T.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); a=d['async_device_parse']; r=a['registered']; print('reg %.1f M sigs/s (median of %d runs %.1f, %.1f-%.1f), pageable %.1f M sigs/s, streaming %.1f M sigs/s' % (r['sigs_per_s']/1e6, r['runs'], r['sigs_per_s_median']/1e6, r['sigs_per_s_min_max'][0]/1e6, r['sigs_per_s_min_max'][1]/1e6, a['pageable']['sigs_per_s']/1e6, a['streaming']['sigs_per_s']/1e6))" gpurun_out/stage_$T.json ;;
  stagetrace)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/stagetr_$T -o tr -- \
      python3 tools/bench_verify_stage.py --frags 1048576 --steps 3 --warmup 1 --no-cpu --async-batch 36000 \
      > gpurun_out/stagetr_$T.json 2> gpurun_out/stagetr_$T.err || { tail -20 gpurun_out/stagetr_$T.err; exit 1; } ;;
  hostfedtrace)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    FD_MAPS_OUT=gpurun_out/hostfed_maps_$T.txt timeout -k 10 900 rocprofv3 --kernel-trace --memory-copy-trace --stats \
      --output-format csv -d gpurun_out/hostfedtr_$T -o tr -- python3 bench.py --path host-fed \
      > gpurun_out/hostfedtr_$T.json 2> gpurun_out/hostfedtr_$T.err || { tail -30 gpurun_out/hostfedtr_$T.err; exit 1; }
    cat gpurun_out/hostfedtr_$T.json ;;
  offload)
    # the server (owns the GPU) in the background, the client (no GPU) in front
    NAME=/fdvo_e2e_$$
    timeout -k 10 300 ./firedancer_amd/fd_verify_offload_server --name $NAME --batch ${BATCH:-65536} --threads ${THREADS:-16} \
      > gpurun_out/offload_server_$T.json 2> gpurun_out/offload_server_$T.err &
    SRV=$!
    for i in $(seq 600); do grep -q ready gpurun_out/offload_server_$T.json 2>/dev/null && break; kill -0 $SRV 2>/dev/null || break; sleep 0.2; done
    timeout -k 10 240 python3 tools/bench_offload.py --name $NAME ${CLIENT_ARGS} > gpurun_out/offload_client_$T.json \
      2> gpurun_out/offload_client_$T.err || { kill $SRV; wait $SRV; exit 1; }
    wait $SRV
    cat gpurun_out/offload_client_$T.json gpurun_out/offload_server_$T.json ;;
  clock)
    # in-kernel clock stamps (stamps build) for bench config $1 (2: pipe kernel, 3: single-lane kernel)
    FD_ED25519_GPU_LIB=tools/bin/libfd_ed25519_gpu_stamps.so timeout -k 10 300 python3 tools/clock_stamps.py --config $1 \
      > gpurun_out/clock_c$1_$T.json 2> gpurun_out/clock_c$1_$T.err || { tail -20 gpurun_out/clock_c$1_$T.err; exit 1; }
    cat gpurun_out/clock_c$1_$T.json ;;
  crashctl)
    # the exit-time SIGSEGV control (tools/crash_control.py MODE) under the host-fed trace's profiler flags
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    FD_MAPS_OUT=gpurun_out/crashctl_$1_maps.txt timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
      --output-format csv -d gpurun_out/crashctl_$1 -o tr -- python3 tools/crash_control.py $1 \
      > gpurun_out/crashctl_$1.out 2> gpurun_out/crashctl_$1.err; echo "crashctl $1 rc=$?"; tail -3 gpurun_out/crashctl_$1.err ;;
  abstage)
    timeout -k 10 600 python3 -u tools/ab_stage.py "$@" > gpurun_out/abstage_$T.log 2>&1 || { tail -20 gpurun_out/abstage_$T.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/abstage_$T.log ;;
  box)
    { timeout -k 10 60 rocm-smi --showserial -M -P -t -c; timeout -k 10 60 amd-smi static --limit; } \
      > gpurun_out/box_$T.txt 2>&1 || true
    grep -v "^$" gpurun_out/box_$T.txt | grep -iv "warning" | head -80 ;;
  power)
    : > gpurun_out/power_$T.txt
    timeout -k 10 300 python3 bench.py --no-cpu "$@" > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err &
    P=$!; n=0
    for i in $(seq 1 600); do
      sleep 0.4
      kill -0 $P 2>/dev/null || break
      echo "T$i" >> gpurun_out/power_$T.txt
      timeout -k 5 20 rocm-smi -P -c -t >> gpurun_out/power_$T.txt 2>&1 || true
      w=$(tail -25 gpurun_out/power_$T.txt | grep -oE "Power \(W\): [0-9.]+" | tail -1 | awk '{print int($3)}')
      if [ -n "$w" ] && [ "$w" -gt 1000 ]; then
        n=$((n+1)); [ $n = 6 ] && { timeout -k 5 30 amd-smi metric > gpurun_out/amdsmi_$T.txt 2>&1 || true; }
      fi
    done
    wait $P
    grep -E "SOCKET_POWER|PPT_VIOLATION_ACTIVITY" gpurun_out/amdsmi_$T.txt 2>/dev/null || true
    tail -c 300 gpurun_out/bench_$T.json ;;
  run)
    lim=$1; shift
    timeout -k 10 $lim "$@" ;;
  *) echo "unknown command $cmd" >&2; exit 2 ;;
esac
