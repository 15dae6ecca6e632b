set -e
mkdir -p gpurun_out
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s3h.log 2>&1 || { tail -20 gpurun_out/smoke_s3h.log; exit 1; }
tail -1 gpurun_out/smoke_s3h.log
bash tools/profile.sh r02s3
bash tools/profile_configs.sh r02s3
