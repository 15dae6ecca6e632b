set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s3j.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s3j.log; exit 1; }
tail -1 gpurun_out/gpu_tests_s3j.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s3j.log 2>&1 || { tail -20 gpurun_out/smoke_s3j.log; exit 1; }
tail -1 gpurun_out/smoke_s3j.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_s3j.json 2> gpurun_out/bench_driver_s3j.err || { tail -20 gpurun_out/bench_driver_s3j.err; exit 1; }
cut -c1-200 gpurun_out/bench_driver_s3j.json
bash tools/profile_configs.sh r02s3j
