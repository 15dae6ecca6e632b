set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for w in 1 2 4; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/probe_w$w -o pmc -- tools/bin/fe_probe2_w$w > gpurun_out/probe_w$w.txt 2>&1
  python3 tools/pmc_probe.py gpurun_out/probe_w$w/pmc_counter_collection.csv > gpurun_out/probe_w$w.sum
done
cat gpurun_out/probe_w*.sum
