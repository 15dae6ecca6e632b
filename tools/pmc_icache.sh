set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ic
for n in 65536 131072; do
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/ic/a_$n -o pmc -- python3 tools/quick_perf.py $n > /dev/null 2> gpurun_out/ic/a_$n.err
  python3 tools/pmc_summary.py gpurun_out/ic/a_$n/pmc_counter_collection.csv
  timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVES --output-format csv -d gpurun_out/ic/b_$n -o pmc -- python3 tools/quick_perf.py $n > /dev/null 2> gpurun_out/ic/b_$n.err
  python3 tools/pmc_summary.py gpurun_out/ic/b_$n/pmc_counter_collection.csv
done
