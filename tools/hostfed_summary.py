"""hostfed_summary.py -- summary of `tools/gpu.sh hostfedtrace` (rocprofv3
--kernel-trace --memory-copy-trace of bench.py --path host-fed): per kernel
and copy kind the calls and mean duration, and for the last async stream
(config 2 from a page-locked arena, 64 batches of 64K): the pipe kernel's
median duration, the median gap between consecutive pipe launches, and the
share of the H2D copy time that overlaps a pipe launch.

  python3 tools/hostfed_summary.py gpurun_out/hostfedtr_TAG [--out summary.json]
"""
import argparse
import csv
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--out")
ap.add_argument("--batches", type=int, default=64)
a = ap.parse_args()
kt = list(csv.DictReader(open(os.path.join(a.dir, "tr_kernel_trace.csv"))))
ct = list(csv.DictReader(open(os.path.join(a.dir, "tr_memory_copy_trace.csv"))))


def span(r):
    return int(r["Start_Timestamp"]), int(r["End_Timestamp"])


stats = {}
for r in kt:
    s, e = span(r)
    stats.setdefault(r["Kernel_Name"], []).append((e - s) / 1e3)
for r in ct:
    s, e = span(r)
    stats.setdefault(r["Direction"], []).append((e - s) / 1e3)
out = {"calls_mean_us": {k: {"calls": len(v), "mean_us": round(statistics.mean(v), 2)} for k, v in stats.items()}}
pipe = sorted((span(r) for r in kt if r["Kernel_Name"].startswith("fd_ed25519_verify_pipe_kernel")))
last = pipe[-(a.batches + 2):]                     # the registered stream's launches and its two drains
t0, t1 = last[0][0], last[-1][1]
h2d = [span(r) for r in ct if r["Direction"] == "MEMORY_COPY_HOST_TO_DEVICE" and t0 <= span(r)[0] <= t1]
cp_total = sum(e - s for s, e in h2d)
cp_over = 0
for s, e in h2d:
    for ps, pe in last:
        cp_over += max(0, min(e, pe) - max(s, ps))
gaps = [(b[0] - a_[1]) / 1e3 for a_, b in zip(last, last[1:])]
out["registered_stream"] = {
    "pipe_launches": len(last), "pipe_median_us": round(statistics.median((e - s) / 1e3 for s, e in last), 1),
    "gap_median_us": round(statistics.median(gaps), 2), "gap_p90_us": round(sorted(gaps)[9 * len(gaps) // 10], 2),
    "h2d_copies": len(h2d), "h2d_busy_us_per_batch": round(cp_total / 1e3 / a.batches, 1),
    "h2d_share_overlapping_a_pipe_launch": round(cp_over / cp_total, 3) if cp_total else None,
    "wall_us_per_batch": round((t1 - t0) / 1e3 / a.batches, 1)}
s = json.dumps(out, indent=1)
print(s)
if a.out:
    open(a.out, "w").write(s + "\n")
