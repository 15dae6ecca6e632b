set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_we3.log 2>&1 || { tail -40 gpurun_out/gpu_tests_we3.log; exit 1; }
tail -1 gpurun_out/gpu_tests_we3.log
for r in 1 2; do
for L in we2 we3; do
echo -n "$L " | tee -a gpurun_out/c3_we_s3.log
FD_ED25519_GPU_LIB=tools/bin/lib_$L.so timeout -k 10 300 python3 bench.py --config 3 --steps 10 --warmup 3 --no-cpu 2>/dev/null | tail -1 | cut -c1-140 | tee -a gpurun_out/c3_we_s3.log
done
done
