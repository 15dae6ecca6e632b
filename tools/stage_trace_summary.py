"""stage_trace_summary.py -- summary of `tools/gpu.sh stagetrace` (rocprofv3
--kernel-trace --memory-copy-trace of tools/bench_verify_stage.py): per
kernel the median duration; over the streamed batches, the median time from
one pipe launch's start to the next, the median idle gap between a pipe
launch's end and the next launch on the device (a parse launch when the
parse has a launch of its own, else the next pipe launch), and how far
before the previous pipe launch's end each batch's H2D copies finished.

  python3 tools/stage_trace_summary.py gpurun_out/stagetr_TAG [--out summary.json] [--note TEXT]
"""
import argparse
import csv
import json
import os
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--out")
ap.add_argument("--note", default="")
a = ap.parse_args()
kt = sorted(csv.DictReader(open(os.path.join(a.dir, "tr_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
ct = sorted(csv.DictReader(open(os.path.join(a.dir, "tr_memory_copy_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
PIPE, PARSE = "fd_ed25519_verify_pipe_kernel", "fd_frag_parse_kernel"


def se(r):
    return int(r["Start_Timestamp"]), int(r["End_Timestamp"])


med = {}
for r in kt:
    s, e = se(r)
    med.setdefault(r["Kernel_Name"], []).append((e - s) / 1e3)
out = {"medians_us": {k: round(statistics.median(v), 2) for k, v in med.items() if k in (PIPE, PARSE)},
       "launches": {k: len(v) for k, v in med.items()}}
dev = [r for r in kt if r["Kernel_Name"] in (PIPE, PARSE)]
pipes = [se(r) for r in dev if r["Kernel_Name"] == PIPE]
# streamed: consecutive pipe launches less than 2 ms apart (not host pauses between runs)
p2p = [(b[0] - a_[0]) / 1e3 for a_, b in zip(pipes, pipes[1:]) if b[0] - a_[0] < 2_000_000]
gaps = []
for x, y in zip(dev, dev[1:]):
    if x["Kernel_Name"] == PIPE:
        g = (se(y)[0] - se(x)[1]) / 1e3
        if g < 1000:
            gaps.append(g)
out["pipe_to_pipe_start_median_us"] = round(statistics.median(p2p), 1) if p2p else None
out["pipe_end_to_next_launch_gap_median_us"] = round(statistics.median(gaps), 2) if gaps else None
out["per_batch_overhead_us"] = (round(statistics.median(p2p) - out["medians_us"][PIPE], 1) if p2p else None)
# each H2D copy's end against the end of the last pipe launch that started before the copy began
lead = []
h2d = [se(r) for r in ct if r["Direction"] == "MEMORY_COPY_HOST_TO_DEVICE"]
for s, e in h2d:
    prev = [p for p in pipes if p[0] <= s]
    if prev and prev[-1][1] >= e:
        lead.append((prev[-1][1] - e) / 1e3)
out["h2d_copies_ending_inside_a_pipe_launch"] = len(lead)
out["h2d_lead_before_pipe_end_median_us"] = round(statistics.median(lead), 1) if lead else None
out["note"] = a.note
s = json.dumps(out, indent=1)
print(s)
if a.out:
    open(a.out, "w").write(s + "\n")
