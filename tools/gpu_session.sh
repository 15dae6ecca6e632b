set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s2a.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s2a.log; exit 1; }
tail -3 gpurun_out/gpu_tests_s2a.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_s2a.json 2> gpurun_out/bench_s2a.err || { tail -20 gpurun_out/bench_s2a.err; exit 1; }
cat gpurun_out/bench_s2a.json
