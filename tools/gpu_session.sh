set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s3c.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s3c.log; exit 1; }
tail -2 gpurun_out/gpu_tests_s3c.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_base.so tools/bin/lib_new.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_pipe_s3c.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_new.so tools/bin/lib_base.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_pipe_s3c.log
timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_base.so tools/bin/lib_new.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_oneshot_s3c.log
IC_LIBS="tools/bin/lib_base.so tools/bin/lib_rina.so tools/bin/lib_new.so" bash tools/pmc_ic_libs.sh 2>&1 | tee gpurun_out/ic_s3c.log
