set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pipe.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_lsort_tests.log 2>&1 || { tail -40 gpurun_out/pipe_lsort_tests.log; exit 1; }
tail -1 gpurun_out/pipe_lsort_tests.log
echo "config 3 messages" | tee -a gpurun_out/ab_lsort_s3.log
AB_MSG=var timeout -k 10 300 python3 tools/pipe_knob_ab.py 12:000:1 12:000:0 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_lsort_s3.log
echo "config 2 messages" | tee -a gpurun_out/ab_lsort_s3.log
timeout -k 10 300 python3 tools/pipe_knob_ab.py 12:000:1 12:000:0 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_lsort_s3.log
timeout -k 10 300 python3 tools/pipe_knob_ab.py 12:000:0 12:000:1 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_lsort_s3.log
timeout -k 10 300 python3 bench.py --config 3 --pipeline 1 --steps 10 --warmup 3 --no-cpu 2>/dev/null | tail -1 | cut -c1-200 | tee -a gpurun_out/ab_lsort_s3.log
timeout -k 10 300 python3 bench.py --config 3 --steps 10 --warmup 3 --no-cpu 2>/dev/null | tail -1 | cut -c1-200 | tee -a gpurun_out/ab_lsort_s3.log
