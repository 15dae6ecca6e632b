set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_order_tests.log 2>&1 || { tail -30 gpurun_out/pipe_order_tests.log; exit 1; }
tail -1 gpurun_out/pipe_order_tests.log
timeout -k 10 300 python3 tools/pipe_knob_ab.py 8:000:1:012 8:000:1:102 8:000:1:021 8:000:1:120 8:000:1:201 8:000:1:210 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/order_sweep_s3.log
timeout -k 10 300 python3 tools/pipe_knob_ab.py 8:000:1:210 8:000:1:201 8:000:1:120 8:000:1:021 8:000:1:102 8:000:1:012 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/order_sweep_s3.log
