"""Print the last verify-kernel dispatch's counters from a rocprofv3 counter CSV
(the single-lane, pair or cached verify kernel, whichever the run launched)."""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if "verify" in r["Kernel_Name"] and "kernel" in r["Kernel_Name"] and "kcache" not in r["Kernel_Name"]]
by = {}
for r in rows:
    d = by.setdefault(r["Dispatch_Id"], {"kernel": r["Kernel_Name"],
                                         "dur_ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                                         "grid": r["Grid_Size"], "vgpr": r["VGPR_Count"]})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
last = list(by.values())[-1]
print({k: v for k, v in last.items()})
