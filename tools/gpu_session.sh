set -e
mkdir -p gpurun_out
for r in 1 2; do
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_t0.so tools/bin/lib_t1.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_ntstore_s3.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_t1.so tools/bin/lib_t0.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_ntstore_s3.log
done
