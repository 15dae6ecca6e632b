set -e
mkdir -p gpurun_out/pmc_c3b
timeout -k 10 400 python -u -m pytest tests/test_gpu_scenarios.py -x -v --timeout 300 --timeout-method thread > gpurun_out/scen_s3.log 2>&1 || { tail -30 gpurun_out/scen_s3.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/scen_s3.log | tail -8
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_c3b/sq -o pmc -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu > /dev/null 2> gpurun_out/pmc_c3b/sq.err
echo ok
