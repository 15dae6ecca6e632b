set -e
mkdir -p gpurun_out
bash tools/profile.sh r02s3k
FD_ED25519_GPU_LIB=tools/bin/libfd_ed25519_gpu_stamps.so timeout -k 10 200 python3 tools/timeline.py 65536 30 gpurun_out/timeline_s3k.json > gpurun_out/timeline_s3k.log 2>&1 || true
echo done
