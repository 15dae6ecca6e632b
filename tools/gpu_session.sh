set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s3s.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s3s.log; exit 1; }
tail -1 gpurun_out/gpu_tests_s3s.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s3s.log 2>&1 || { tail -20 gpurun_out/smoke_s3s.log; exit 1; }
tail -1 gpurun_out/smoke_s3s.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_s3s.json 2> gpurun_out/bench_driver_s3s.err || { tail -20 gpurun_out/bench_driver_s3s.err; exit 1; }
cut -c1-220 gpurun_out/bench_driver_s3s.json
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_torchrun_s3s.json 2> gpurun_out/bench_torchrun_s3s.err || { tail -20 gpurun_out/bench_torchrun_s3s.err; exit 1; }
cut -c1-220 gpurun_out/bench_torchrun_s3s.json
