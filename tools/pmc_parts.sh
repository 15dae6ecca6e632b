#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVES of the lattice and SHA-512 kernels alone
# (tools/part_costs.py), for each library in PARTS_LIBS (default: the in-tree one).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/parts
for L in ${PARTS_LIBS:-firedancer_amd/libfd_ed25519_gpu.so}; do
  b=$(basename $L .so)
  FD_ED25519_GPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/parts/$b -o pmc -- python3 tools/part_costs.py > gpurun_out/parts/$b.out.txt 2> gpurun_out/parts/$b.err.txt
  B=$b python3 - <<'PY'
import csv, os
by = {}
for r in csv.DictReader(open("gpurun_out/parts/%s/pmc_counter_collection.csv" % os.environ["B"])):
    d = by.setdefault(r["Dispatch_Id"], {"k": r["Kernel_Name"][:40]})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
seen = set()
for d in by.values():
    if ("lattice" in d["k"] or "sha512" in d["k"]) and d["k"] not in seen:
        seen.add(d["k"])
        print("%-14s %-40s waves %6d  VALU/wave %8.0f" % (os.environ["B"], d["k"], d["SQ_WAVES"], d["SQ_INSTS_VALU"] / d["SQ_WAVES"]))
PY
done
