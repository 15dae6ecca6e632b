"""Print one verify-kernel dispatch's counters from a rocprofv3 counter CSV
(the single-lane, pair, pipe or cached verify kernel, whichever the run
launched): the last one, or with "mid" as the second argument the middle one
(a steady-state launch of a pipelined run, whose last launches drain it)."""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if "verify" in r["Kernel_Name"] and "kernel" in r["Kernel_Name"] and "kcache" not in r["Kernel_Name"]]
by = {}
for r in rows:
    d = by.setdefault(r["Dispatch_Id"], {"kernel": r["Kernel_Name"],
                                         "dur_ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                                         "grid": r["Grid_Size"], "vgpr": r["VGPR_Count"]})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
disp = list(by.values())
last = disp[len(disp) // 2] if len(sys.argv) > 2 and sys.argv[2] == "mid" else disp[-1]
print({k: v for k, v in last.items()})
