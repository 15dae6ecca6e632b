#!/usr/bin/env python3
"""Per-dispatch issue summary of a rocprofv3 counter CSV (dev tool): for each
kernel dispatch, VALU wave-instructions per SIMD, busy cycles per SIMD
(SQ_BUSY_CU_CYCLES is in quad-cycles, summed over the 1024 SIMDs' CUs as
rocprofv3 reports it), cycles per VALU instruction, dual-issue share.

  pmc_probe.py pmc_counter_collection.csv"""
import csv, sys, collections
by = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    d = by.setdefault(r["Dispatch_Id"], {"kernel": r["Kernel_Name"][:40],
                                         "dur_us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
for d in by.values():
    v = d.get("SQ_INSTS_VALU", 0.0) / 1024.0
    busy = 4.0 * d.get("SQ_BUSY_CU_CYCLES", 0.0) / 1024.0
    out = {"kernel": d["kernel"], "dur_us": round(d["dur_us"], 1), "valu_per_simd": round(v),
           "busy_cyc_per_simd": round(busy), "cyc_per_valu": round(busy / v, 3) if v else None,
           "dual_frac": round(d.get("SQ_ACTIVE_INST_VALU2", 0.0) / max(d.get("SQ_INSTS_VALU", 1.0), 1.0), 4),
           "int64_frac": round(d.get("SQ_INSTS_VALU_INT64", 0.0) / max(d.get("SQ_INSTS_VALU", 1.0), 1.0), 3),
           "int32_frac": round(d.get("SQ_INSTS_VALU_INT32", 0.0) / max(d.get("SQ_INSTS_VALU", 1.0), 1.0), 3)}
    if "GRBM_GUI_ACTIVE" in d:
        out["ghz"] = round(d["GRBM_GUI_ACTIVE"] / 8.0 / (d["dur_us"] * 1e3), 3)
    print(out)
