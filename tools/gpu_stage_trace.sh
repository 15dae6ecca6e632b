set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/stage_trace -o tr -- python3 tools/bench_verify_stage.py --frags 1048576 --steps 3 --warmup 1 --no-cpu --async-batch 35000 > gpurun_out/stage_trace.json 2> gpurun_out/stage_trace.err || { tail -20 gpurun_out/stage_trace.err; exit 1; }
ls -R gpurun_out/stage_trace | head
