set -e
mkdir -p gpurun_out
timeout -k 10 200 python3 -c "
import time, ctypes, torch
torch.cuda.init()
for L in ('tools/bin/lib_new.so', 'tools/bin/lib_comb23.so', 'tools/bin/lib_new.so', 'tools/bin/lib_comb23.so'):
    lib = ctypes.CDLL(L); lib.fd_ed25519_gpu_new.restype = ctypes.c_void_p; lib.fd_ed25519_gpu_new.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    lib.fd_ed25519_gpu_delete.argtypes = [ctypes.c_void_p]
    t = time.perf_counter(); c = lib.fd_ed25519_gpu_new(1, 65536); dt = time.perf_counter() - t; assert c; lib.fd_ed25519_gpu_delete(c)
    print(L, 'context creation %.3f s' % dt, flush=True)
" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ctx_time_s3u.log
for r in 1 2 3; do
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_new.so tools/bin/lib_comb23.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_comb23_s3u.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_comb23.so tools/bin/lib_new.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_comb23_s3u.log
done
