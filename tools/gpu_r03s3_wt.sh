#!/bin/bash
# r03 session 3: write-through stores of the next launch's data (A/B, back to
# back) and a kernel trace of the bench (inter-launch gaps).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_b2b.py firedancer_amd/libfd_ed25519_gpu.so tools/bin/libvar_wt.so tools/bin/libvar_wtt.so 20 > gpurun_out/b2b_wt.log 2>&1 || { tail -20 gpurun_out/b2b_wt.log; exit 1; }
cat gpurun_out/b2b_wt.log | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_gap -o tr -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/trace_gap_bench.json 2> gpurun_out/trace_gap.err || { tail -20 gpurun_out/trace_gap.err; exit 1; }
cat gpurun_out/trace_gap_bench.json
