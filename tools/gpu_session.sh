set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_multi_tests.log 2>&1 || { tail -40 gpurun_out/pipe_multi_tests.log; exit 1; }
tail -1 gpurun_out/pipe_multi_tests.log
for md in 0 0x201 0x301 0x101; do
echo "mode $md" | tee -a gpurun_out/quick_multi_s3z.log
FD_ED25519_GPU_PIPE_MODE=$md timeout -k 10 200 python3 tools/quick_multi.py 65536 96 3 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/quick_multi_s3z.log
done
