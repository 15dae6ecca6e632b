set -e
mkdir -p gpurun_out
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_new.so tools/bin/lib_xcomb11.so tools/bin/lib_xbigcomb.so 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_bigcomb_s3r.log
AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py tools/bin/lib_xbigcomb.so tools/bin/lib_xcomb11.so tools/bin/lib_new.so 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/ab_bigcomb_s3r.log
