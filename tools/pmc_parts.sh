#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVES of the lattice and SHA-512 kernels alone (tools/part_costs.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/parts
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/parts/p -o pmc -- python3 tools/part_costs.py > gpurun_out/parts/out.txt 2> gpurun_out/parts/err.txt
python3 - <<'PY'
import csv
by = {}
for r in csv.DictReader(open("gpurun_out/parts/p/pmc_counter_collection.csv")):
    d = by.setdefault(r["Dispatch_Id"], {"k": r["Kernel_Name"][:40]})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
for d in by.values():
    if "lattice" in d["k"] or "sha512" in d["k"]:
        print("%-40s waves %6d  VALU/wave %8.0f" % (d["k"], d["SQ_WAVES"], d["SQ_INSTS_VALU"] / d["SQ_WAVES"]))
PY
