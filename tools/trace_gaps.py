"""trace_gaps.py -- launch gaps from a rocprofv3 --kernel-trace CSV: for the
named kernel, the duration of each dispatch and the idle time between the end
of one dispatch and the start of the next (consecutive dispatches of that
kernel only).  Usage: trace_gaps.py kernel_trace.csv [kernel-name]"""
import csv
import statistics
import sys

path = sys.argv[1]
kn = sys.argv[2] if len(sys.argv) > 2 else "fd_ed25519_verify_pipe_kernel"
rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(kn)]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
gap_b2b = [g for g in gap if g < 50.0]       # back-to-back launches (not host pauses)
print("%s: %d dispatches, duration median %.1f us (min %.1f max %.1f)" % (
    kn, len(rows), statistics.median(dur), min(dur), max(dur)))
if gap_b2b:
    print("gap between back-to-back dispatches: median %.2f us, p10 %.2f, p90 %.2f (%d of %d gaps < 50 us)" % (
        statistics.median(gap_b2b), sorted(gap_b2b)[len(gap_b2b) // 10], sorted(gap_b2b)[9 * len(gap_b2b) // 10],
        len(gap_b2b), len(gap)))
