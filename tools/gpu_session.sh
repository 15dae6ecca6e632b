set -e
mkdir -p gpurun_out
for r in 1 2; do
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_noorder.so tools/bin/lib_cur.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_order_s3.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_cur.so tools/bin/lib_noorder.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_order_s3.log
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu 2>/dev/null | cut -c1-160 | tee -a gpurun_out/ab_order_s3.log
