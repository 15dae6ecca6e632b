set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s3e.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s3e.log; exit 1; }
tail -2 gpurun_out/gpu_tests_s3e.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_new.so tools/bin/lib_ainb.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_pipe_s3e.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_ainb.so tools/bin/lib_new.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_pipe_s3e.log
timeout -k 10 200 python3 tools/pipe_knob_ab.py 12:000 11:000 13:000 14:000 12:000 2>&1 | grep -v amdgpu.ids | tee gpurun_out/knob_s3e.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_s3e.json 2> gpurun_out/bench_s3e.err || { tail -20 gpurun_out/bench_s3e.err; exit 1; }
cat gpurun_out/bench_s3e.json
