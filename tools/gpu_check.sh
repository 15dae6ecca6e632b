#!/bin/bash
# Quick GPU iteration: parity tests, timing at several batch sizes, one PMC pass.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/check_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/check_pytest.log; exit 1; }
tail -2 gpurun_out/check_pytest.log
timeout -k 10 200 python -u tools/quick_perf.py ${PERF_SIZES:-65536 131072 262144} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/check_perf.log
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/check_pmc -o pmc -- python3 tools/quick_perf.py 65536 > /dev/null 2> gpurun_out/check_pmc.err
  python3 tools/pmc_summary.py gpurun_out/check_pmc/pmc_counter_collection.csv
fi
