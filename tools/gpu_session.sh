set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s3v.log 2>&1 || { tail -40 gpurun_out/gpu_tests_s3v.log; exit 1; }
tail -1 gpurun_out/gpu_tests_s3v.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s3v.log 2>&1 || { tail -20 gpurun_out/smoke_s3v.log; exit 1; }
tail -1 gpurun_out/smoke_s3v.log
bash tools/profile.sh r02s3v
bash tools/profile_configs.sh r02s3v
