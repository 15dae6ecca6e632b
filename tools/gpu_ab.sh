#!/bin/bash
# One GPU call for a kernel change: parity of the built library, then an A/B
# of tools/bin/lib_base.so against tools/bin/lib_new.so (pipelined and
# one-shot launches, both in one process).  Stops at the first failure.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${AB_TESTS:-tests/test_gpu_parity.py tests/test_pipe.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py ${AB_LIBS:-tools/bin/lib_base.so tools/bin/lib_new.so} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_pipe.log
timeout -k 10 200 python3 tools/ab_libs.py ${AB_LIBS:-tools/bin/lib_base.so tools/bin/lib_new.so} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_oneshot.log
