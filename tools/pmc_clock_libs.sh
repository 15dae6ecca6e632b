#!/bin/bash
# Clock and wait counters of the pipelined verify launch per library build
# (FD_ED25519_GPU_LIB): effective clock = GRBM_GUI_ACTIVE / XCDs / duration.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/clk
for L in ${CLK_LIBS:-tools/bin/lib_base.so}; do
  b=$(basename $L .so)
  for rep in 1 2; do
    FD_ED25519_GPU_LIB=$L timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/clk/$b.$rep -o pmc -- python3 tools/quick_pipe.py 65536 pipe 40 > gpurun_out/clk/$b.$rep.out 2> gpurun_out/clk/$b.$rep.err
    python3 - gpurun_out/clk/$b.$rep/pmc_counter_collection.csv $b <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "pipe_kernel" in r["Kernel_Name"]]
by = {}
for r in rows:
    d = by.setdefault(r["Dispatch_Id"], {"dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
ds = list(by.values())[10:-5]
ghz = [d["GRBM_GUI_ACTIVE"] / 8 / d["dur"] / 1e6 for d in ds]
print("%-10s n=%d dur %.4f ms  clock %.3f GHz  VALU %.1fM  wait_any/wave_cyc %.3f  wait_inst/wave_cyc %.3f" % (
    sys.argv[2], len(ds), statistics.median(d["dur"] for d in ds), statistics.median(ghz),
    statistics.median(d["SQ_INSTS_VALU"] for d in ds) / 1e6,
    statistics.median(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"] for d in ds),
    statistics.median(d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"] for d in ds)))
PY
  done
done
